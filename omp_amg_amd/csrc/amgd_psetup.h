/*
 * amgd_psetup.h -- the partitioned multi-GPU setup (amgd_psetup.c) as seen by the
 * one-GPU driver's entry points (amgd_setup.c): amgd_setup_device / amgd_hier_export /
 * amgd_hier_free run it when the library communicator is in partitioned mode.
 */
#ifndef AMGD_PSETUP_H
#define AMGD_PSETUP_H
#include <stdint.h>

#include "amg_setup.h"
#include "omp_amg_amd.h"

typedef struct amgd_phier amgd_phier;
/* this rank's COO entries (global indices, any rows; every rank's together are the
   matrix, duplicates summed in rank order) -> the partitioned hierarchy */
int amgd_psetup_body(uint64_t nz, const uint32_t *dAi, const uint32_t *dAj, const double *dAv,
                     amgd_phier **out, amgd_stats *st);
/* the whole hierarchy (gathered) on every rank */
int amgd_phier_export(const amgd_phier *h, struct amg_setup_data *data);
void amgd_phier_free(amgd_phier **h);
void amgd_phier_free_host(amgd_phier **h);   /* after an unwind: host structs only */
void amgd_phier_info(const amgd_phier *h, uint32_t *nlevels, uint32_t *r0, uint32_t *r1);
#endif
