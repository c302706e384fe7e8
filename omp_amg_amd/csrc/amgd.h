/*
 * amgd.h -- the thin internal C ABI between the host setup driver (amgd_setup.c,
 * plain C) and the hand-written HIP kernels (amgd_*.hip).  No HIP or torch type
 * appears here: device memory is passed as plain pointers, matrices as `dcsr`.
 *
 * Device CSR layout in HBM (DESIGN.md "Data layout"):
 *   ro  : u64[rn+1]  row offsets (64-bit: coarse operators exceed 2^32 nnz at scale)
 *   col : u32[nnz]   column indices, ascending within a row (reference invariant)
 *   a   : f64[nnz]   values
 * Masks (C/F sets, strength filters) are u8 {0,1} arrays; the reference keeps
 * them as doubles (amg_setup.c:175-180) but every use is a !=0 test or a
 * multiply by 0/1 of a non-negative value, which the u8 form reproduces exactly.
 */
#ifndef AMGD_H
#define AMGD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint32_t rn, cn;
  uint64_t nnz;
  uint64_t *ro;
  uint32_t *col;
  double *a;
} dcsr;

/* ---------------- runtime (amgd_rt.hip) ---------------- */
int amgd_rt_init(int device);            /* idempotent; 0 on success */
const char *amgd_last_error(void);
void amgd_set_error(const char *msg);
void *amgd_alloc(size_t bytes);          /* arena; out of HBM: unwinds to amgd_try, else aborts */
void *amgd_alloc_f64(size_t bytes);      /* the same, for arrays of doubles (AMGD_POISON=1: NaN-filled) */
void amgd_set_poison(int on);
void amgd_set_hbm_cap(size_t bytes);     /* cap on live bytes (tests; 0: none) */
/* run fn(arg); if an allocation runs out of HBM inside it, every block allocated since
   the call is released and -2 returned (amgd_last_error() has the text) */
int amgd_try(int (*fn)(void *), void *arg);
void amgd_spmv_split_clear(void);        /* drop every cached SpMV shard split */
/* reset the per-call module state a setup sets and clears around its kernels (SpGEMM
   pattern mode / timer slot, Q-factor reuse pointers, component-split depth): called at the
   start of every setup and after an unwound one */
void amgd_reset_call_state(void);
void amgd_sparse_reset_state(void);
void amgd_interp_reset_state(void);
void amgd_free(void *p);
uint32_t amgd_max_row_len(const dcsr *M);   /* longest row of a pinned matrix, else UINT32_MAX */
void amgd_rowmax_pin(const dcsr *M);           /* pattern fixed until unpinned / freed */
void amgd_rowmax_unpin(const dcsr *M);
void amgd_spmv_split_forget(const void *ro);   /* drop cached SpMV shard splits of a freed buffer */
/* partitioned-setup diagnostics (tests): interp_lmop calls on gathered data / with a dirty
   prefix; eager exchanges / those that took the second round; forced rare paths */
void amgd_part_stats(uint64_t *out2);
void amgd_spmv_tab_stats(uint64_t *out3);       /* gather-table builds, tiles, direct tiles */
void amgd_spmv_set_tab(int on);
void amgd_part_set_force_gather(int on);
void pm_eager_stats(uint64_t *calls, uint64_t *second);
void pm_eager_force_slot(int64_t bytes);
void amgd_rt_shutdown(void);             /* free everything; pointers become invalid */
void amgd_pool_release(void);            /* return every cached block to the driver */
size_t amgd_pool_bytes_in_use(void);
size_t amgd_pool_peak_bytes(void);
void amgd_pool_peak_reset(void);
size_t amgd_pool_ipeak_take(void);        /* peak since the last call, then reset */          /* peak := bytes in use now (start of a setup) */
void amgd_pool_stats(uint64_t *nmalloc, double *gbytes, double *ms, uint64_t *nrelease);
void amgd_h2d(void *d, const void *h, size_t n);
void amgd_d2h(void *h, const void *d, size_t n);
void amgd_d2d(void *d, const void *s, size_t n);
void amgd_memset(void *d, int v, size_t n);
void amgd_sync(void);
double amgd_wtime(void);
void *amgd_stream(void);                 /* hipStream_t of the library */
void amgd_set_stream(void *stream);
/* event timers on the library stream, for kernel-level throughput */
void amgd_timer_start(int slot);
void amgd_timer_stop(int slot);
void amgd_timer_start2(int slot, int slot2);   /* two slots timing the same interval */
void amgd_timer_stop2(int slot, int slot2);
double amgd_timer_ms(int slot);          /* accumulated, syncs */
void amgd_timer_reset(void);
void amgd_spgemm_set_timer(int slot);     /* SpGEMM numeric kernels timed on slot (-1: off) */

dcsr *dcsr_new(uint32_t rn, uint32_t cn, uint64_t nnz);
void dcsr_free(dcsr **A);
dcsr *dcsr_copy(const dcsr *A);
dcsr *dcsr_empty_like_pattern(const dcsr *A);   /* same ro/col, fresh a */

/* kernel-route counters (which default paths a setup took; read by the parity tests
   at sizes where the default routing engages) */
enum { AMGD_R_SPMV_PIPE, AMGD_R_MV_LONG, AMGD_R_SG_TINY, AMGD_R_SG_KSEQ, AMGD_R_SG_WWIN,
       AMGD_R_SG_WWIN_SYM, AMGD_R_SG_LONG, AMGD_R_CS_INC, AMGD_R_FS_INC, AMGD_R_SG_ROW,
       AMGD_R_MV_RW4, AMGD_R_QF_REUSE, AMGD_R_LMOP_WAVE, AMGD_R_MV_RW16, AMGD_R_MV_RW64,
       AMGD_R_QF_T512, AMGD_R_QF_T1024, AMGD_R_MV_PAIR, AMGD_R_FS_AMX, AMGD_R_MV_TAB, AMGD_R_SG_SYMREUSE, AMGD_R_SPAT_INC, AMGD_R_SG_DRSORT, AMGD_R_N };
extern uint64_t amgd_route_ctr[32];
#define amgd_route_hit(r) (amgd_route_ctr[(r)]++)

/* scans: counts[0..n-1] -> exclusive prefix in counts[0..n], returns total */
uint64_t amgd_scan_u64(uint64_t *counts, uint64_t n);
uint32_t amgd_scan_u32(uint32_t *counts, uint64_t n);
/* compaction map for a u8 mask: map[i] = rank of i among set entries (or ~0) */
uint32_t amgd_mask_rank(const uint8_t *mask, uint32_t n, uint32_t *map);

/* AMGD_PHASES=1 phase profile (amgd_setup.c): time of the phase just ended on a level */
enum { PH_COARSEN, PH_SMOOTH, PH_IPRE, PH_QF, PH_W0, PH_SPAT, PH_LMOP, PH_PCG, PH_W, PH_AFW, PH_R,
       PH_FS, PH_FS_MV, PH_FS_MAX, PH_FS_SEL, PH_EXP, PH_EXP_R0, PH_FINAL, PH_RAP, PH_N };
void amgd_ph_mark(int lvl, int id);      /* -1: restart the clock */
void amgd_ph_report(uint32_t nlevels);

/* ---------------- row sharding over GPUs (amgd_comm.hip) ---------------- */
int amgd_nshards(void);                          /* 1: sharding off */
int amgd_comm_procs(void);                       /* processes of the communicator (sim: 1) */
void amgd_my_shards(int *first, int *last);      /* shard ranges this process computes */
int amgd_shard_worth(uint64_t work, uint64_t min_work);
/* contiguous ranges of equal work: split_h[0..N] from an exclusive prefix of n+1 entries */
void amgd_shard_split(const uint64_t *prefix, uint32_t n, uint32_t *split_h);
/* Collectives.  Each records its call site (file:line of the outermost caller) for the
   collective-consistency guard (AMGD_COMM_CHECK=1 / amgd_comm_set_check): before every
   collective the ranks exchange (sequence number, kind, call site, offsets signature,
   send lengths) in a fixed-size record and abort naming both ranks' sites on any
   mismatch -- a rank-local skip or a size disagreement cannot go unnoticed (RCCL would
   hang or corrupt).  The same record carries an out-of-HBM on one rank to all of them,
   so every rank unwinds its setup together (amgd_comm_fail_agree). */
void amgd_comm_site(const char *file, int line);
int amgd_comm_fail_agree(void);    /* 1: every rank was told of this rank's failure */
void amgd_comm_site_report(void);  /* AMGD_COMM_SITES=1: collectives per call site (stderr) */
/* range s of buffer b = bytes [off[b*(N+1)+s], off[b*(N+1)+s+1]), completed on every rank */
void amgd_allgatherv_(int nbuf, void *const *bufs, const uint64_t *off);
#define amgd_allgatherv(...) (amgd_comm_site(__FILE__, __LINE__), amgd_allgatherv_(__VA_ARGS__))
void amgd_allgather_u64_(uint64_t *vals_h);      /* vals_h[s] of the own shards -> all */
#define amgd_allgather_u64(...) (amgd_comm_site(__FILE__, __LINE__), amgd_allgather_u64_(__VA_ARGS__))
void amgd_gather_u64_at(const uint64_t *a, const uint32_t *idx_h, int n, uint64_t *out_h);

/* partitioned mode (amgd_psetup.c): ranks own row blocks; amgd_nshards() is 1 there */
int amgd_comm_partitioned(void);
void amgd_comm_suspend_partition(int on);
int amgd_comm_part_default(void);
int amgd_comm_part_get(void);          /* raw flag: -1 unset, 0 off, 1 on */
void amgd_comm_part_set(int v);
/* calls, bytes of: data allgatherv, alltoallv, small u64 allgathers (since the last reset) */
void amgd_comm_stats_kind(uint64_t *out6);
int amgd_pcomm_rank(void);
int amgd_pcomm_size(void);
void amgd_pcomm_allgather_u64_(uint64_t *vals_h, int m);  /* vals_h[N*m]: own m -> all */
#define amgd_pcomm_allgather_u64(...) (amgd_comm_site(__FILE__, __LINE__), amgd_pcomm_allgather_u64_(__VA_ARGS__))
/* rank sends send[soff[p]..soff[p+1]) to p, receives p's into recv[roff[p]..roff[p+1]) (bytes) */
void amgd_pcomm_alltoallv_(const void *send, const uint64_t *soff, void *recv, const uint64_t *roff);
#define amgd_pcomm_alltoallv(...) (amgd_comm_site(__FILE__, __LINE__), amgd_pcomm_alltoallv_(__VA_ARGS__))
/* nb such exchanges (buffers b = 0..nb-1) in one collective */
void amgd_pcomm_alltoallv_n_(int nb, const void *const *send, const uint64_t *const *soff, void *const *recv,
                             const uint64_t *const *roff);
#define amgd_pcomm_alltoallv_n(...) (amgd_comm_site(__FILE__, __LINE__), amgd_pcomm_alltoallv_n_(__VA_ARGS__))

/* ---------------- reductions (return host values, sync) ---------------- */
void amgd_set_exact(int on);     /* 1: reference-order (sequential) dots -- default; 0: tree */
int amgd_get_exact(void);
double amgd_dot(const double *a, const double *b, uint64_t n);
double amgd_norm2(const double *a, uint64_t n);
double amgd_max_first(const double *a, uint64_t n, uint64_t *idx);  /* first argmax */
double amgd_max_first2(const double *a, const double *b, uint64_t n, uint64_t *idx, double *maxb);
uint64_t amgd_count_gt(const double *a, uint64_t n, double thr, double *maxv);
double amgd_fro_minus_eye(const dcsr *A);                          /* ||A - I||_F^2 */

/* ---------------- sparse (amgd_sparse.hip) ---------------- */
dcsr *amgd_build_csr(uint64_t nz, const uint32_t *Ai, const uint32_t *Aj, const double *Av);
dcsr *amgd_coo2csr(uint64_t nz, const uint32_t *I, const uint32_t *J, const double *V,
                   uint32_t rn, uint32_t cn, int drop_zero);
dcsr *amgd_sub_mat(const dcsr *A, const uint8_t *vr, const uint8_t *vc);
dcsr *amgd_transpose(const dcsr *A, uint64_t **perm_out);
dcsr *amgd_drop_zeros(const dcsr *A);                      /* exactly-zero entries removed */
dcsr *amgd_rows_masked(const dcsr *A, const uint8_t *mask);  /* rows with mask==0 emptied */
dcsr *amgd_cols_masked(const dcsr *A, const uint8_t *mask);  /* entries with mask[col]==0 dropped */
uint64_t *amgd_perm_inverse(const uint64_t *p, uint64_t n);  /* q[p[t]] = t */
dcsr *amgd_spgemm(const dcsr *A, const dcsr *B);           /* A*B, reference semantics */
/* pattern of A*B, values unspecified nonzeros (operands with all values > 0) */
dcsr *amgd_spgemm_pattern(const dcsr *A, const dcsr *B);
/* the next one-GPU product: 1 keeps its symbolic phase, 2 takes the kept one when both
   operand patterns match (else runs in full); drop frees a kept state */
void amgd_spgemm_sym_next(int mode);
void amgd_spgemm_sym_drop(void);
void amgd_spgemm_sym_stats(uint64_t *kept, uint64_t *reused);
/* the constraint operator's pattern grown from the previous iteration's (amgd_setup.c) */
void amgd_spat_set_inc(int on);
void amgd_spat_stats(uint64_t *out3);     /* incremental, whole, same pattern */
void amgd_spat_forget(void);
dcsr *amgd_mpm(double alpha, const dcsr *A, double beta, const dcsr *B);
dcsr *amgd_mxmpoint(const dcsr *A, const dcsr *B);
/* z = (y ? alpha*y + beta*t : beta*t) [* f] with t = M x summed in column order */
void amgd_spmv(const dcsr *M, const double *x, double *z, double alpha, const double *y,
               double beta, const uint8_t *f);
/* z[list[r]] = row list[r] of M times x (x == NULL: row sums), left to right */
void amgd_spmv_rows(const dcsr *M, const uint32_t *list, uint32_t n, const double *x, double *z);
/* z = M^T x, per column in ascending row order; Mt = transpose(M) */
void amgd_spmvt(const dcsr *Mt, const double *x, double *z);
void amgd_colsum(const dcsr *Mt, double *z);   /* sum(M,1) via Mt */
void amgd_diag(const dcsr *A, double *D);
enum { AMGD_DPLUS = 0, AMGD_DMINUS = 1, AMGD_DMULT = 2, AMGD_MULTD = 3,
       AMGD_SCALE2 = 4, AMGD_SCALE_ABS = 5, AMGD_SCALE2_ABS = 6, AMGD_SCALE_ABS_T = 7 };
void amgd_diag_op(dcsr *A, const double *D, int op);
/* fused: SCALE2 a=(a*Dl[i])*Dr[col]; SCALE_ABS a=|a*Dl[i]|*Dr[col]; SCALE2_ABS a=|(a*Dl[i])*Dr[col]|;
   SCALE_ABS_T a=|a*Dl[col]|*Dr[i] (SCALE_ABS of the transpose, entry by entry) */
void amgd_diag_op2(dcsr *A, const double *Dl, const double *Dr, int op);
void amgd_vals_abs(dcsr *A);
void amgd_vals_sqr(dcsr *A);
void amgd_vals_scale(dcsr *A, double s);
void amgd_rowsum_sq_inv(const dcsr *A, double *s);     /* s_i = 1/sum_j a_ij^2 (row order) */
uint64_t amgd_to_host_cols(const dcsr *A, unsigned long *h_ro, unsigned long *h_col, double *h_a);

/* ---------------- vectors (amgd_vec.hip) ---------------- */
enum {
  AMGD_V_FILL, AMGD_V_INV, AMGD_V_SQRT, AMGD_V_MUL, AMGD_V_ADD, AMGD_V_SUB, AMGD_V_DIV
};
void amgd_vfill(double *a, uint64_t n, double v);
void amgd_vop(double *c, const double *a, const double *b, uint64_t n, int op); /* c = a op b */
void amgd_vunary(double *a, uint64_t n, int op);                                /* a = op(a) */
void amgd_vscale(double *a, uint64_t n, double s);                              /* a = a*s */
void amgd_u8_to_f64(const uint8_t *m, double *d, uint64_t n);
void amgd_compact_ids(const unsigned long *id, const uint8_t *vc, uint32_t n,
                      unsigned long *idc, unsigned long *idf);
void amgd_lanczos_step(const double *r, double rbeta_inv, double *qk, double *qkm1, uint64_t n);
void amgd_lanczos_resid(double *r, const double *Aqk, const double *qk, double alpha,
                        double *qkm1, double beta, uint64_t n);
/* pcg pieces */
void amgd_pcg_p(double *p, const double *z, double beta, uint64_t n);
void amgd_pcg_xrz(double *x, double *r, double *z, const double *p, const double *w,
                  const double *M, double alpha, uint64_t n);
void amgd_vmul_dot_prep(double *z, const double *M, const double *r, uint64_t n);
double amgd_dot3(const double *M, const double *b, uint64_t n);  /* sum (M.*b).*b */

/* ---------------- coarsening (amgd_coarsen.hip) ---------------- */
void amgd_coarsen_w(const double *w1, const double *w2, double *w, uint32_t n);
void amgd_coarsen_mask1(const double *w, double ctol2, const double *g, uint8_t *mask,
                        double *x, uint32_t n);
void amgd_mat_max(const dcsr *S, const dcsr *St, const uint8_t *f, const double *x, double tol,
                  double *amax_tmp, double *y);
void amgd_mat_amax(const dcsr *S, const uint8_t *f, double tol, double *amax);
void amgd_mat_max_gather(const dcsr *St, const uint8_t *f, const double *x, const double *amax,
                         double *y);
void amgd_coarsen_mask2(double *g, const double *m, uint8_t *mask, double *x, uint32_t n);
void amgd_coarsen_mask3(const double *m, uint8_t *mask, uint8_t *vc, uint8_t *vf, double *vfd,
                        uint32_t n, uint32_t *anyvc);
/* incremental sweeps (amgd_coarsen.hip): a stage of radius R runs on the rows
   within R hops of the last sweep's new C points -- the prefix cum[R] of the BFS
   list (list mode) or the rows i with fs[i] - fb <= R (filter mode); rows = NULL
   runs the full kernels */
typedef struct {
  const uint32_t *list;   /* BFS rows in hop order (list mode) or NULL */
  uint32_t cum[8];        /* rows within r hops */
  const uint32_t *fs;     /* row stamps (filter mode) */
  uint32_t fb;            /* 8 * sweep */
} amgd_csrows;
int amgd_cs_grow(const dcsr *S, const dcsr *St, uint32_t *front, uint32_t *cnt_d,
                 uint32_t *stamp, uint32_t base8, uint32_t limit, uint32_t *cum);
/* partitioned mode: one BFS hop of amgd_cs_grow, and the claim of another rank's hop rows */
void amgd_cs_hop1(const dcsr *S, const dcsr *St, uint32_t *front, uint32_t *cnt_d, int r, uint32_t *stamp,
                  uint32_t base8, uint32_t limit);
void amgd_cs_claim_ext(const uint32_t *ids, uint64_t n, uint32_t *stamp, uint32_t base8, int r,
                       uint32_t *front, uint32_t hi0, uint32_t *cntr);
void amgd_spmv_filt(const dcsr *M, const double *x, double *z, const uint8_t *f,
                    const uint32_t *fs, uint32_t fb, uint32_t fr);
void amgd_mat_amax_filt(const dcsr *S, const uint8_t *f, double tol, double *amax,
                        const uint32_t *fs, uint32_t fb, uint32_t fr);
void amgd_mat_max_gather_filt(const dcsr *St, const uint8_t *f, const double *x,
                              const double *amax, double *y, const uint32_t *fs, uint32_t fb,
                              uint32_t fr);
void amgd_cs_spmv(const dcsr *S, const double *x, double *z, const uint8_t *f,
                  const amgd_csrows *rows, uint32_t R);
void amgd_cs_w_mask1(uint32_t n, const double *w1, const double *w2, double *w, double ctol2,
                     const double *g, uint8_t *ma, double *x1, const amgd_csrows *rows,
                     uint32_t R);
void amgd_cs_amax(const dcsr *S, const uint8_t *f, double tol, double *amax,
                  const amgd_csrows *rows, uint32_t R);
void amgd_cs_gather(const dcsr *St, const uint8_t *f, const double *x, const double *amax,
                    double *y, const amgd_csrows *rows, uint32_t R);
void amgd_cs_mask2(uint32_t n, const double *g, const double *m1, const uint8_t *ma, uint8_t *mb,
                   double *x2, const amgd_csrows *rows, uint32_t R);
void amgd_cs_mask3(uint32_t n, const double *m2, const uint8_t *mb, uint8_t *vc, uint8_t *vf,
                   double *vfd, uint32_t *anyvc, uint32_t *d0, uint32_t *d0cnt, uint32_t *stamp,
                   uint32_t next_base8, const amgd_csrows *rows, uint32_t R);

/* ---------------- interpolation (amgd_interp.hip) ---------------- */
dcsr *amgd_min_skel(const dcsr *R);
/* Q factors of A restricted to each row-support of Wt (packed upper triangles) */
double *amgd_qfactor(const dcsr *Wt, const dcsr *A, uint64_t **qoff_out, uint64_t *qtotal);
/* the same, copying the factor of every support identical to the previous call's (Wp, Qp,
   qpoff: that call's Wt, factors and offsets; NULL: factor everything) */
double *amgd_qfactor_reuse(const dcsr *Wt, const dcsr *A, uint64_t **qoff_out, uint64_t *qtotal,
                           const dcsr *Wp, const double *Qp, const uint64_t *qpoff);
void amgd_qfactor_reuse_stats(uint64_t *reused, uint64_t *factored);
void amgd_qapply(const dcsr *Wt, const double *Q, const uint64_t *qoff, const dcsr *Bt,
                 const double *u, const double *lambda, double *out);
/* S := interp_lmop contributions (S pattern = W_skel*W_skel'); kpos from amgd_lmop_kpos */
int amgd_lmop(dcsr *S, const dcsr *Wskel, const uint32_t *kpos, const dcsr *Wt, const double *Q,
              const uint64_t *qoff, const double *u);
uint32_t *amgd_lmop_kpos(const dcsr *Wt, const uint64_t *perm);
void amgd_lmop_stats(uint64_t *out);   /* fast, general, dirty-prefix calls, misses, pruned supports */
void amgd_lmop_stats_reset(void);
void amgd_lmop_set_mode(int m);        /* 0: row-pull fast path where exact, 1: general walk */
void amgd_lmop_spill_detect(int on);   /* partitioned mode: flag walks past the view's last row */
int amgd_lmop_spilled(void);
/* partitioned mode: [0, d) already added to S (the dirty prefix walked on the whole S
   pattern); amgd_lmop then adds [d, nc) only.  0: off */
void amgd_lmop_set_prefix(uint32_t d);
/* amgd_lmop_general keeps the values of S positions [lo, hi) only, in a (NULL: off) */
void amgd_lmop_set_window(double *a, uint64_t lo, uint64_t hi);
/* the exact (sp_add-walk) contributions of the coarse points [cb, ce) added to S */
void amgd_lmop_general(dcsr *S, const dcsr *Wt, const double *Q, const uint64_t *qoff, const double *u,
                       uint32_t cb, uint32_t ce);
void amgd_lmop_classify_view(const dcsr *Wt, uint32_t *dend, uint32_t *cmin);
uint64_t amgd_lmop_qq_bytes(void);    /* QQ^t bytes of the last amgd_lmop call */
int amgd_lmop_missed(void);            /* a clean contribution missed (prefix mode); clears */
void amgd_qfactor_set_sparse(int m);   /* huge supports: 0 dense, 1 sparse first, 2 tiny capacity */
void amgd_qfactor_stats(unsigned long *st); /* [sparse, dense fallback, split] since the last call */
/* one find_support sweep: select/remove, then re-sum rs (rows) and sumR (columns) that lost
   an entry */
uint32_t amgd_fs_select(const dcsr *Rl, const dcsr *Rt, const uint64_t *perm, double *rs,
                        const double *w, double *sumR, double thr,
                        uint32_t *sel_i, uint32_t *sel_j, uint32_t *nremoved);
/* the same over rows c0.. of R' (w, sumR at c0; sel_j global); perm NULL: R untouched;
   resum 0: rs / sumR not re-summed (partitioned mode) */
void amgd_list_rowsum(const dcsr *M, const uint32_t *list, uint32_t n, double *out, int long_rows);
uint32_t amgd_fs_select_ex(const dcsr *Rl, const dcsr *Rt, const uint64_t *perm, double *rs,
                           const double *w, double *sumR, double thr, uint32_t *sel_i,
                           uint32_t *sel_j, uint32_t *nremoved, uint32_t c0, int resum);
/* incremental sweeps: distinct columns of the listed rows of M (stamp/tag dedupe);
   returns the count, > cap when the list overflowed */
int amgd_spmv_amax(const dcsr *M, const double *x, double *z, uint64_t *amx);
uint32_t amgd_fs_select_amx(const dcsr *Rl, const dcsr *Rt, const uint64_t *perm, double *rs,
                            const double *w, double *sumR, double thr, const uint64_t *amx,
                            uint32_t *sel_i, uint32_t *sel_j, uint32_t *nremoved);
uint32_t amgd_fs_expand(const dcsr *M, const uint32_t *list, uint32_t n, uint32_t *stamp,
                        uint32_t tag, uint32_t *out, uint32_t cap);
/* partitioned mode: ids of another rank's expansion claimed into out (have: entries so far) */
uint32_t amgd_fs_claim_ext(const uint32_t *ids, uint64_t n, uint32_t *stamp, uint32_t tag, uint32_t *out,
                           uint32_t have, uint32_t cap);
uint8_t *amgd_bad_rows(const dcsr *ns, uint32_t *nbad);
uint64_t amgd_expand_pick(const dcsr *Xf, const uint8_t *bad, uint32_t **pi, uint32_t **pj);
void amgd_skel_binarize(dcsr *A, int mode);
void amgd_scale_diag_match(dcsr *W, const double *v, const double *wuc);
void amgd_csc_gemv(const dcsr *Rt, const uint64_t *perm, const double *a, const double *x,
                   double *z);
/* misc vector kernels */
void amgd_vdiv_guard(double *r, const double *num, const double *den, uint64_t n); /* r=num/den, 0 where den==0 */
void amgd_alpha_update(double *alpha, const double *Dc, const double *w2, uint64_t n);
void amgd_u8_not(const uint8_t *a, uint8_t *b, uint64_t n);
void amgd_u8_nonzero(const double *a, uint8_t *m, uint64_t n);
uint64_t amgd_u8_count(const uint8_t *m, uint64_t n);
void amgd_vcompact(double *dst, const double *src, const uint8_t *mask, uint64_t n);
void amgd_vexpand_add(double *dst, const double *src, const uint8_t *mask, uint64_t n);
void amgd_vzero_where(double *a, const uint8_t *mask_keep, uint64_t n);
void amgd_ids_iota(unsigned long *id, uint64_t n);

#ifdef __cplusplus
}
#endif
#endif
