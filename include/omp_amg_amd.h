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
  double spmv_kernel_ms;         /* whole-matrix long-row SpMV kernels (k_spmv_pipe), event-timed */
  uint64_t spmv_bytes;           /* their bytes with x gathered once per entry */
  uint64_t spmv_bytes_strict;    /* their algorithmic HBM bytes: x read once per product */
  uint64_t spmv_launches, rap_launches;   /* kernel launches behind spmv_/rap_kernel_ms */
  /* the long-row SpMV per shape: RW = 4 / 16 / 64 rows per wavefront (k_spmv_pipe<.., RW>) */
  double spmv_rw_ms[3];
  uint64_t spmv_rw_bytes_strict[3], spmv_rw_launches[3];
  /* the first AMGD_UB_LOG reference-undefined events: site (1 find_support theta -> 0, 2 one-row R,
     3 a sweep removed nothing, 4 selections past nnz(R) + nc, 5 skeleton stalled) and level */
  uint8_t ub_site[8], ub_level[8];
} amgd_stats;
#define AMGD_UB_LOG 8

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
/* the hierarchy crs_setup (crs.h) keeps in HBM, copied into the ABI struct -- the same
   layout amg_setup fills; free with free_data */
struct crs_data;
int amgd_crs_export(const struct crs_data *crs, struct amg_setup_data *data);
/* ---- multi-GPU: row-sharded setup over the GPUs of one node (DESIGN.md "Multi-GPU") ----
   Every rank calls amgd_setup_device on the same matrix; the row-independent heavy
   kernels (SpGEMMs, Q factors) are split by work across the ranks and completed by
   an in-place allgatherv, so every rank ends with the same, bit-identical hierarchy.
   No reference interface corresponds: the reference's setup is serial
   (amg_setup.c:60); crs_setup's comm (crs.h:15) is where a caller passes its ranks. */
int amgd_comm_rccl_uid(unsigned char uid[128]);     /* rank 0: fresh RCCL unique id */
int amgd_comm_init_rccl(int rank, int size, const unsigned char uid[128]);
/* host transport: bufs[b] is a device buffer whose range s holds bytes
   [offs[b*(size+1)+s], offs[b*(size+1)+s+1]); rank `rank` fills its range, the callback
   must leave every range filled on every rank.  Returns 0 on success. */
typedef int (*amgd_allgatherv_fn)(void *user, int nbuf, void *const *bufs, const uint64_t *offs,
                                  int rank, int size);
int amgd_comm_init_host(int rank, int size, amgd_allgatherv_fn fn, void *user);
int amgd_comm_init_sim(int nshards);   /* one process computes all shards in turn (tests) */
void amgd_comm_free(void);             /* back to one GPU */
int amgd_comm_size(void);
int amgd_comm_rank(void);
/* Partitioned mode (the north_star layout): with a multi-process
   communicator (RCCL or host), amgd_setup_device takes each rank's OWN entries (global
   indices; every rank's entries together are the matrix, duplicates summed in rank order),
   routes them to the owners of their rows (contiguous equal row blocks of level 0, every
   coarser level inheriting the owners), and builds a hierarchy of which each rank holds
   only its row blocks: rows of A, Af, W and AfP of every level and of every intermediate;
   products fetch the halo rows they reference, transposes exchange row pieces, vectors
   stay whole.  amgd_hier_export gathers the whole hierarchy to every rank (bit-identical
   to the one-GPU hierarchy).  amgd_comm_set_partitioned(1) after amgd_comm_init_* turns
   it on for amgd_setup_device; crs_setup with np > 1 runs partitioned unless
   amgd_comm_set_partitioned(0) chose the round-2 replicated mode; amg_setup always takes
   the whole matrix on the calling process (amg_setup.h:5) and runs the one-GPU setup
   there.  amgd_comm_free resets the choice. */
void amgd_comm_set_partitioned(int on);
int amgd_comm_partitioned(void);
/* Collective-consistency guard (also AMGD_COMM_CHECK=1): before every collective the
   ranks exchange (sequence number, kind, call site, sizes) and abort naming both ranks'
   call sites on a mismatch; an out-of-HBM on one rank inside a setup is announced the
   same way and every rank's setup returns -2 (without the guard it aborts the job).
   1 on, 0 off, -1 back to the environment.  amgd_comm_guard_calls: record exchanges so far. */
void amgd_comm_set_check(int on);
uint64_t amgd_comm_guard_calls(void);
/* scale of the per-op minimum work below which an op runs unsharded (1 = default, 0 = always shard) */
void amgd_comm_set_min_work(double scale);
void amgd_comm_stats(uint64_t *calls, uint64_t *bytes, double *ms);
void amgd_comm_stats_reset(void);

/* device scratch helpers for ctypes callers (bench/tests) */
void *amgd_dev_alloc(size_t bytes);
void amgd_dev_free(void *p);
void amgd_dev_upload(void *d, const void *h, size_t n);
void amgd_dev_download(void *h, const void *d, size_t n);
void amgd_dev_sync(void);                        /* wait for the library stream */

#ifdef __cplusplus
}
#endif
#endif
