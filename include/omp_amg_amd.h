/*
 * omp_amg_amd.h -- device-resident entry points of libomp_amg_amd.so.
 *
 * The drop-in host ABI (amg_setup.h) copies COO in and the hierarchy out over
 * PCIe.  Callers that already hold the matrix in HBM (the bench, a GPU solver)
 * use these: COO already on the device in, hierarchy kept in HBM, optional
 * export into a host `struct amg_setup_data`.
 *
 * Reference interface replaced: amg_setup() (amg_setup.h:5), split at the
 * host/device boundary.
 */
#ifndef OMP_AMG_AMD_H
#define OMP_AMG_AMD_H

#include <stddef.h>
#include <stdint.h>
#include "amg_setup.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct amgd_hier amgd_hier;

/* per-phase device times (ms) and work counters of the last setup */
typedef struct {
  double t_total_ms, t_build_ms, t_coarsen_ms, t_smoother_ms, t_interp_ms, t_rap_ms, t_copy_ms;
  double rap_kernel_ms;          /* fused/ordered SpGEMM kernels inside RAP, event-timed */
  uint64_t rap_out_nnz;          /* sum over levels of nnz(A_{l+1}) */
  uint64_t rap_bytes;            /* algorithmic HBM bytes of the RAP SpGEMMs */
  uint64_t rows0, nnz0;
  uint32_t nlevels, ub_events;   /* ub_events: inputs outside the reference's defined domain */
  size_t peak_bytes;
} amgd_stats;

int amgd_init(int device);                       /* 0 = ok; <0 = no usable HIP device */
/* release every device buffer, event and the stream of the library (hierarchies
   not yet freed become invalid); amgd_init may be called again afterwards */
void amgd_shutdown(void);
/* Global dot products (PCG, Lanczos): 1 = summed in the reference's left-to-right
   order (default; hierarchy bit-identical to the reference), 0 = fixed-order tree
   (faster; differs in the last bits, which the reference's chaotic constraint
   solve can amplify -- DESIGN.md "Parity").  Env AMGD_FAST_DOTS=1 sets 0. */
void amgd_set_exact_dots(int on);
const char *amgd_error(void);
/* device pointers in, hierarchy out (kept in HBM).  flags: bit0 = also keep host copies */
int amgd_setup_device(uint64_t nz, const uint32_t *dAi, const uint32_t *dAj, const double *dAv,
                      amgd_hier **out, int flags);
int amgd_hier_export(const amgd_hier *h, struct amg_setup_data *data);  /* D2H into the ABI struct */
void amgd_hier_free(amgd_hier **h);
void amgd_get_stats(amgd_stats *st);
/* device scratch helpers for ctypes callers (bench/tests) */
void *amgd_dev_alloc(size_t bytes);
void amgd_dev_free(void *p);
void amgd_dev_upload(void *d, const void *h, size_t n);
void amgd_dev_download(void *h, const void *d, size_t n);

#ifdef __cplusplus
}
#endif
#endif
