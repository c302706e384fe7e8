/*
 * amgd_part.h -- row-partitioned matrices and their distributed operations
 * (partitioned mode, amgd_psetup.c).
 *
 * Every index space of the setup (a level's rows, its F points, its C points) is split
 * into N contiguous ranges, one per rank: `apart`.  The split of level 0 is equal row
 * counts; every other space inherits it: the F (C) points of level l keep the rank of
 * their row, and the C points of level l are the rows of level l+1 -- so a row never
 * changes rank and the matrices of a level meet on the same ranks.
 *
 * A `pmat` holds rows [r0, r1) = rp->split[me..me+1] of a global matrix as an ordinary
 * dcsr (rn = r1 - r0, row offsets from 0, GLOBAL column indices), plus the row and
 * column partitions.  Vectors stay whole on every rank (8 B per row); a product whose
 * rows are local completes its output vector with one allgatherv of the row segments.
 * The exchange before a product X = A*B is the halo: the rows of B that the local rows
 * of A reference, fetched from their owners with one alltoallv and laid next to the
 * local rows in a global-row view (row offsets for every global row, the others empty)
 * -- so the one-GPU kernels run unchanged on the same rows with the same operands and
 * produce the same bits.
 */
#ifndef AMGD_PART_H
#define AMGD_PART_H

#include "amgd.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int N;              /* ranks */
  uint32_t n;         /* size of the index space */
  uint32_t *split;    /* host, N + 1 entries: rank p owns [split[p], split[p+1]) */
} apart;

typedef struct {
  dcsr *m;            /* local rows, global columns */
  const apart *rp;    /* row space */
  const apart *cp;    /* column space */
} pmat;

apart *apart_even(uint32_t n, int N);                      /* equal row counts */
/* the sub-space of the entries with mask != 0 (each keeps its owner): split'[p] = #mask
   before split[p] (mask: whole u8 vector, device) */
apart *apart_induced(const apart *P, const uint8_t *mask);
void apart_free(apart **P);
static inline uint32_t apart_lo(const apart *P, int me) { return P->split[me]; }
static inline uint32_t apart_hi(const apart *P, int me) { return P->split[me + 1]; }

pmat *pm_new(dcsr *m, const apart *rp, const apart *cp);  /* takes m over */
void pm_free(pmat **A);
pmat *pm_copy(const pmat *A);

/* whole vector from its row segments: v[split[p] .. split[p+1]) of rank p (elem bytes each) */
void pm_allgather_vec(void *v, size_t elem, const apart *P);
/* z_i for listed rows i (the list may differ in order between ranks, not in content):
   each rank holds the values of the listed rows it owns; afterwards every rank holds all */
void pm_list_sync(double *z, const uint32_t *list, uint32_t n, const apart *P);
/* the same for nv vectors (each its list and partition) in one exchange */
void pm_list_sync_n(int nv, double *const *z, const uint32_t *const *list, const uint32_t *n,
                    const apart *const *P);
/* every rank's `bytes` (device) and one u64 to every rank, concatenated in rank order (the
   returned device buffer, amgd_free it): len[p] bytes of rank p, users[p] its value.  One
   collective while the shares fit the call site's adaptive eager slot (a pm_eager kept by
   the caller, zero-initialised; every rank adapts it alike). */
typedef struct { uint64_t slot, gen; } pm_eager;
void pm_eager_new_setup(void);   /* every partitioned setup starts from the default slots */
char *pm_allgather_dyn(pm_eager *e, const void *mine, uint64_t bytes, uint64_t user, uint64_t *len,
                       uint64_t *users, uint64_t *total);

/* global-row view of A: row offsets for all rp->n rows (rows of other ranks empty),
   the same col / a arrays.  pm_gview_free releases the offsets only. */
dcsr pm_gview(const pmat *A);
void pm_gview_free(dcsr *g);
/* a matrix produced on the global-row view (rows of other ranks empty) -> local rows */
dcsr *pm_localize(dcsr *G, uint32_t r0, uint32_t r1);

/* vector-valued row ops: computed on the local rows, completed on every rank */
void pm_spmv(const pmat *M, const double *x, double *z, double alpha, const double *y, double beta,
             const uint8_t *f);
void pm_colsum(const pmat *Mt, double *z);                 /* row sums of Mt (= sum(M,1)) */
void pm_spmvt(const pmat *Mt, const double *x, double *z); /* Mt rows times x */
void pm_diag(const pmat *A, double *D);
void pm_rowsum_sq_inv(const pmat *A, double *s);
double pm_fro_minus_eye(const pmat *A);

/* matrix-valued row ops (same row partition) */
pmat *pm_mpm(double alpha, const pmat *A, double beta, const pmat *B);
pmat *pm_mxmpoint(const pmat *A, const pmat *B);
pmat *pm_drop_zeros(const pmat *A);
pmat *pm_rows_masked(const pmat *A, const uint8_t *mask);  /* mask: whole vector */
pmat *pm_sub_mat(const pmat *A, const uint8_t *vr, const uint8_t *vc, const apart *rp_out,
                 const apart *cp_out);
pmat *pm_transpose(const pmat *A);                          /* rows partitioned like A->cp */
void pm_diag_op(pmat *A, const double *D, int op);          /* DPLUS / DMINUS (global view) */
void pm_diag_op2(pmat *A, const double *Dl, const double *Dr, int op);  /* whole vectors */

/* X = A*B with B's halo rows fetched; pattern = 1: amgd_spgemm_pattern */
pmat *pm_spgemm(const pmat *A, const pmat *B, int pattern);
/* B's rows referenced by the columns of L (local rows), beside B's own, in a global-row
   view (row offsets for all B->rp->n rows).  B->m->col == NULL: values only (E->col NULL).
   Free with pm_ext_free. */
dcsr *pm_halo_rows(const pmat *B, const dcsr *L);
void pm_ext_free(dcsr **E);
int pm_ext_is_view(const dcsr *E);   /* 1: one rank, E aliases B's arrays (no copy) */

/* this rank's COO entries (global indices) to the owners of their rows (P); returns the
   count received, the arrays in source-rank order (free with amgd_free) */
uint64_t pm_route_coo(uint64_t nz, const uint32_t *I, const uint32_t *J, const double *V, const apart *P,
                      uint32_t **Io, uint32_t **Jo, double **Vo);
dcsr *pm_gather_full(const pmat *A);
dcsr *pm_gather_pattern(const pmat *A);     /* row offsets and columns only (a = NULL) */
/* level-0 build helpers: max(I)+1, max(J)+1 over this rank's entries; a[i] += v (mod 2^32);
   out[i] = row i of T is not empty */
void amgd_max_ij(uint64_t nz, const uint32_t *I, const uint32_t *J, uint32_t *mx);
void amgd_vadd_u32(uint32_t *a, uint64_t n, uint32_t v);
void amgd_nonempty_rows(const dcsr *T, uint8_t *out);                        /* every row on every rank */
/* kpos of each local W_skel entry: the position of its row in its column's support
   (WtE: W_skel^T rows referenced by the local rows, global-row view) */
uint32_t *pm_kpos(const pmat *Wskel, const dcsr *WtE);
/* entries (ri[t], cj[t]) of the own rows := 0 */
void pm_zero_entries(pmat *M, const uint32_t *ri, const uint32_t *cj, uint64_t n);
/* out[i] = ordered sum of row i of M for the listed rows (whole list), completed everywhere */
void pm_list_rowsum(const pmat *M, const uint32_t *list, uint32_t n, double *out);
/* rows la of A into oa and rows lb of B into ob (n each), one exchange */
void pm_list_rowsum2(const pmat *A, const uint32_t *la, double *oa, const pmat *B, const uint32_t *lb,
                     double *ob, uint32_t n);
/* the own rows of the whole COO (ri, cj, 1) as a partitioned CSR */
pmat *pm_coo_ones(const uint32_t *ri, const uint32_t *cj, uint64_t n, const apart *rp, const apart *cp);

#ifdef __cplusplus
}
#endif
#endif
