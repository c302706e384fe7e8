/*
 * crs.h -- gslib coarse-solver interface (reference crs.h:8-21), AMG flavour.
 *
 *   crs_setup(n, id, nz, Ai, Aj, A, null_space, comm) builds the AMG hierarchy
 *   of the assembled matrix on the GPU (the path of reference amg.c:475 before
 *   its hand-off to the solve phase) and keeps it resident in HBM.
 *   crs_free releases it.  crs_solve / crs_stats (the V-cycle, amg.c:114-208)
 *   belong to the solve phase, which this library does not implement yet:
 *   they print a diagnostic and abort.
 *
 * `struct comm` is gslib's (comm.h:85-88) for a non-MPI build: {uint id, np; int c}.
 * np > 1: rank comm->id passes its local rows over the library's own communicator
 * (omp_amg_amd.h amgd_comm_init_rccl / _host, same rank and size); by default the
 * setup is row-partitioned -- each rank keeps its row blocks of the hierarchy and the
 * matrix is never gathered; amgd_comm_set_partitioned(0) selects the
 * replicated mode (matrix gathered to every rank, row-sharded kernels).
 * On failure (communicator mismatch, out of HBM) crs_setup returns NULL and
 * amgd_error() holds the reason; the reference exits the process instead.
 * amgd_crs_export (omp_amg_amd.h) copies the kept hierarchy out.
 */
#ifndef OMP_AMG_AMD_CRS_H
#define OMP_AMG_AMD_CRS_H

#include "amg_setup.h"

#ifdef __cplusplus
extern "C" {
#endif

struct comm { amg_uint id, np; int c; };
struct crs_data;

struct crs_data *crs_setup(amg_uint n, const unsigned long *id, amg_uint nz, const amg_uint *Ai,
                           const amg_uint *Aj, const double *A, amg_uint null_space,
                           const struct comm *comm);
void crs_solve(double *x, struct crs_data *data, double *b);
void crs_stats(struct crs_data *data);
void crs_free(struct crs_data *data);

#ifdef __cplusplus
}
#endif
#endif
