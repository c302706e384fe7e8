/*
 * amgd_testapi.c -- kernel-level test hooks of libomp_amg_amd.so.
 *
 * Exposes single device primitives on host CSR inputs so tests/test_gpu_*.py
 * can check each HIP kernel against a host restatement of the reference
 * operation it replaces (mxm, transpose, mpm, mxmpoint, apply_M, min_skel,
 * coarsen).  Not used by the setup path itself.
 */
#include <stdlib.h>
#include <string.h>

#include "amgd.h"

#define API __attribute__((visibility("default")))

typedef struct { uint32_t rn, cn; uint64_t nnz; uint64_t *ro; uint32_t *col; double *a; } hcsr;

static dcsr *up(const hcsr *H) {
  dcsr *A = dcsr_new(H->rn, H->cn, H->nnz);
  amgd_h2d(A->ro, H->ro, ((size_t)H->rn + 1) * 8);
  amgd_h2d(A->col, H->col, H->nnz * 4);
  amgd_h2d(A->a, H->a, H->nnz * 8);
  return A;
}
static void down(const dcsr *A, hcsr *H) {
  H->rn = A->rn; H->cn = A->cn; H->nnz = A->nnz;
  H->ro = (uint64_t *)malloc(((size_t)A->rn + 1) * 8);
  H->col = (uint32_t *)malloc(A->nnz * 4 + 4);
  H->a = (double *)malloc(A->nnz * 8 + 8);
  amgd_d2h(H->ro, A->ro, ((size_t)A->rn + 1) * 8);
  amgd_d2h(H->col, A->col, A->nnz * 4);
  amgd_d2h(H->a, A->a, A->nnz * 8);
}

/* op: 0 spgemm(A,B)  1 transpose(A)  2 mpm(alpha,A,beta,B)  3 mxmpoint(A,B)  4 min_skel(A)
       20 spgemm_pattern(A,B) */
API int amgd_test_csr(int op, const hcsr *HA, const hcsr *HB, double alpha, double beta, hcsr *HX) {
  if (amgd_rt_init(0) != 0) return -1;
  dcsr *A = up(HA), *B = HB ? up(HB) : NULL, *X = NULL;
  switch (op) {
    case 0: X = amgd_spgemm(A, B); break;
    case 1: X = amgd_transpose(A, NULL); break;
    case 2: X = amgd_mpm(alpha, A, beta, B); break;
    case 3: X = amgd_mxmpoint(A, B); break;
    case 4: X = amgd_min_skel(A); break;
    case 20: X = amgd_spgemm_pattern(A, B); break;
    case 5: {                     /* Q factors of the supports (rows of A) on B; X.a = packed Q */
      uint64_t tot = 0, *qoff = NULL;
      double *Q = amgd_qfactor(A, B, &qoff, &tot);
      X = (dcsr *)malloc(sizeof(dcsr));
      X->rn = A->rn; X->cn = 0; X->nnz = tot; X->ro = qoff; X->a = Q;
      X->col = (uint32_t *)amgd_alloc(tot * 4 + 4);
      amgd_memset(X->col, 0, tot * 4 + 4);
      break;
    }
    case 6: {                     /* expand_support picks on every row of A: X = pattern (ones) */
      uint8_t *all = (uint8_t *)amgd_alloc((size_t)A->rn + 1);
      amgd_memset(all, 1, (size_t)A->rn + 1);
      uint32_t *pi = NULL, *pj = NULL;
      uint64_t np = amgd_expand_pick(A, all, &pi, &pj);
      double *ones = (double *)amgd_alloc(np * 8 + 8);
      amgd_vfill(ones, np, 1.0);
      X = amgd_coo2csr(np, pi, pj, ones, A->rn, A->cn, 1);
      amgd_free(all); amgd_free(pi); amgd_free(pj); amgd_free(ones);
      break;
    }
    case 7: {                     /* Q application: Q = qfactor(A, B); X = A's pattern with
                                     values qapply(A, Q, B, u, lambda), u / lambda generated */
      uint64_t tot = 0, *qoff = NULL;
      double *Q = amgd_qfactor(A, B, &qoff, &tot);
      double *u = (double *)amgd_alloc((size_t)A->rn * 8 + 8);
      double *lam = (double *)amgd_alloc((size_t)A->cn * 8 + 8);
      double *hu = (double *)malloc((size_t)A->rn * 8 + 8), *hl = (double *)malloc((size_t)A->cn * 8 + 8);
      for (uint32_t i = 0; i < A->rn; i++) hu[i] = 0.5 + (double)(i % 3);
      for (uint32_t j = 0; j < A->cn; j++) hl[j] = 1.0 / (1.0 + (double)(j % 7));
      amgd_h2d(u, hu, (size_t)A->rn * 8);
      amgd_h2d(lam, hl, (size_t)A->cn * 8);
      free(hu); free(hl);
      X = dcsr_empty_like_pattern(A);
      amgd_qapply(A, Q, qoff, B, u, lam, X->a);
      amgd_free(Q); amgd_free(qoff); amgd_free(u); amgd_free(lam);
      break;
    }
    default: return -2;
  }
  down(X, HX);
  dcsr_free(&A); dcsr_free(&B); dcsr_free(&X);
  return 0;
}

/* z = alpha*y + beta*(A x) (y may be NULL) */
API int amgd_test_spmv(const hcsr *HA, const double *x, double alpha, const double *y, double beta, double *z) {
  if (amgd_rt_init(0) != 0) return -1;
  dcsr *A = up(HA);
  double *dx = (double *)amgd_alloc((size_t)HA->cn * 8 + 8), *dz = (double *)amgd_alloc((size_t)HA->rn * 8 + 8);
  double *dy = NULL;
  amgd_h2d(dx, x, (size_t)HA->cn * 8);
  if (y) { dy = (double *)amgd_alloc((size_t)HA->rn * 8 + 8); amgd_h2d(dy, y, (size_t)HA->rn * 8); }
  amgd_spmv(A, dx, dz, alpha, dy, beta, NULL);
  amgd_d2h(z, dz, (size_t)HA->rn * 8);
  amgd_free(dx); amgd_free(dz); if (dy) amgd_free(dy);
  dcsr_free(&A);
  return 0;
}

/* z = alpha*y + beta*(A x), f row mask, through the gather-table kernel: the matrix is
   pinned (amgd_rowmax_pin builds its tiles) for the product and unpinned after; amx != NULL:
   the fused-selection form (alpha 0, beta 1, no y / f) with each row's first largest
   product.  stats (3): table builds, tiles, direct tiles of this call. */
API int amgd_test_spmv_tab(const hcsr *HA, const double *x, double alpha, const double *y, double beta,
                           const uint8_t *f, double *z, uint64_t *amx, uint64_t *stats) {
  if (amgd_rt_init(0) != 0) return -1;
  dcsr *A = up(HA);
  double *dx = (double *)amgd_alloc((size_t)HA->cn * 8 + 8), *dz = (double *)amgd_alloc((size_t)HA->rn * 8 + 8);
  double *dy = NULL;
  uint8_t *df = NULL;
  uint64_t *dm = NULL;
  amgd_h2d(dx, x, (size_t)HA->cn * 8);
  if (y) { dy = (double *)amgd_alloc((size_t)HA->rn * 8 + 8); amgd_h2d(dy, y, (size_t)HA->rn * 8); }
  if (f) { df = (uint8_t *)amgd_alloc((size_t)HA->rn + 8); amgd_h2d(df, f, (size_t)HA->rn); }
  uint64_t s0[3], s1[3];
  amgd_spmv_tab_stats(s0);
  amgd_rowmax_pin(A);
  if (amx) {
    dm = (uint64_t *)amgd_alloc((size_t)HA->rn * 8 + 8);
    if (!amgd_spmv_amax(A, dx, dz, dm)) { amgd_rowmax_unpin(A); return -2; }
    amgd_d2h(amx, dm, (size_t)HA->rn * 8);
  } else {
    amgd_spmv(A, dx, dz, alpha, dy, beta, df);
  }
  amgd_spmv_tab_stats(s1);
  for (int q = 0; q < 3; q++) stats[q] = s1[q] - s0[q];
  amgd_d2h(z, dz, (size_t)HA->rn * 8);
  amgd_rowmax_unpin(A);
  amgd_free(dx); amgd_free(dz); if (dy) amgd_free(dy); if (df) amgd_free(df); if (dm) amgd_free(dm);
  dcsr_free(&A);
  return 0;
}
API void amgd_test_spmv_tab_on(int on) { amgd_spmv_set_tab(on); }
/* exact sums' resolution: 1 one wavefront per sum (default), 0 one 1024-thread block, -1 env */
extern void amgd_set_resolve_wave(int on);
API void amgd_test_resolve_wave(int on) { amgd_set_resolve_wave(on); }

/* build_csr on host COO (u32 indices) */
API int amgd_test_build(uint64_t nz, const uint32_t *I, const uint32_t *J, const double *V, hcsr *HX) {
  if (amgd_rt_init(0) != 0) return -1;
  uint32_t *di = (uint32_t *)amgd_alloc(nz * 4 + 4), *dj = (uint32_t *)amgd_alloc(nz * 4 + 4);
  double *dv = (double *)amgd_alloc(nz * 8 + 8);
  amgd_h2d(di, I, nz * 4); amgd_h2d(dj, J, nz * 4); amgd_h2d(dv, V, nz * 8);
  dcsr *X = amgd_build_csr(nz, di, dj, dv);
  down(X, HX);
  dcsr_free(&X);
  amgd_free(di); amgd_free(dj); amgd_free(dv);
  return 0;
}

/* sqrt / div / 1/x on a host vector, to check IEEE rounding of the device math */
API int amgd_test_math(int op, uint64_t n, const double *a, const double *b, double *out) {
  if (amgd_rt_init(0) != 0) return -1;
  double *da = (double *)amgd_alloc(n * 8 + 8), *db = (double *)amgd_alloc(n * 8 + 8);
  amgd_h2d(da, a, n * 8);
  amgd_h2d(db, b, n * 8);
  if (op == 0) amgd_vunary(da, n, AMGD_V_SQRT);
  else if (op == 1) amgd_vunary(da, n, AMGD_V_INV);
  else amgd_vop(da, da, db, n, AMGD_V_DIV);
  amgd_d2h(out, da, n * 8);
  amgd_free(da); amgd_free(db);
  return 0;
}

/* exact dot: mode 0 a.b, 1 a.a, 2 (a.*b).*b; plain=1 uses the one-lane loop */
extern void amgd_set_seq_plain(int on);
API double amgd_test_dot(int mode, uint64_t n, const double *a, const double *b, int plain, int exact) {
  if (amgd_rt_init(0) != 0) return 0.0 / 0.0;
  double *da = (double *)amgd_alloc(n * 8 + 8), *db = (double *)amgd_alloc(n * 8 + 8);
  amgd_h2d(da, a, n * 8);
  amgd_h2d(db, b, n * 8);
  int old = amgd_get_exact();
  amgd_set_exact(exact);
  amgd_set_seq_plain(plain);
  double r = mode == 0 ? amgd_dot(da, db, n) : mode == 1 ? amgd_dot(da, NULL, n) : amgd_dot3(da, db, n);
  amgd_set_seq_plain(0);
  amgd_set_exact(old);
  amgd_free(da); amgd_free(db);
  return r;
}

API void amgd_test_free(hcsr *H) {
  free(H->ro); free(H->col); free(H->a);
  H->ro = NULL; H->col = NULL; H->a = NULL;
}

/* interp_lmop path control and counters: [fast, general, dirty-prefix, misses] */
API void amgd_test_lmop_mode(int m) { amgd_lmop_set_mode(m); }
/* supports of at least n points take the pruned general walk (0: never, -1: env/default) */
extern void amgd_lmop_set_prune(int n);
API void amgd_test_lmop_prune(int n) { amgd_lmop_set_prune(n); }
API void amgd_test_lmop_stats(uint64_t *out, int reset) {
  amgd_lmop_stats(out);
  if (reset) amgd_lmop_stats_reset();
}

/* huge-support Q factor: mode (0 dense, 1 sparse first, 2 sparse with a tiny
   capacity, which forces the dense fallback) and [sparse, fallback] counters */
API void amgd_test_qf_sparse(int m) { amgd_qfactor_set_sparse(m); }
API void amgd_test_qf_stats(uint64_t *out) {
  unsigned long st[3];
  amgd_qfactor_stats(st);
  out[0] = st[0];
  out[1] = st[1];
  out[2] = st[2];
}

/* whole-matrix SpMVs that ran row-sharded (multi-GPU) since the library loaded */
extern uint64_t amgd_spmv_shard_calls(void);
/* cols_masked(A, mask) and transpose(rows_masked(B, mask)) for the same mask: equal */
API int amgd_test_cols_masked(const hcsr *HA, const uint8_t *hmask, hcsr *HX) {
  if (amgd_rt_init(0) != 0) return -1;
  dcsr *A = up(HA);
  uint8_t *m = (uint8_t *)amgd_alloc((size_t)A->cn + 1);
  amgd_h2d(m, hmask, A->cn);
  dcsr *X = amgd_cols_masked(A, m);
  down(X, HX);
  dcsr_free(&X); dcsr_free(&A);
  amgd_free(m);
  return 0;
}
void amgd_qfactor_set_reuse(int on);
API void amgd_test_qf_reuse(int on) { amgd_qfactor_set_reuse(on); }
void amgd_lmop_set_small(int n);
API void amgd_test_lmop_small(int n) { amgd_lmop_set_small(n); }
void amgd_lmop_set_wave(int n);
API void amgd_test_lmop_wave(int n) { amgd_lmop_set_wave(n); }
void amgd_spgemm_set_pattern(int on);
API void amgd_test_sg_pattern(int on) { amgd_spgemm_set_pattern(on); }
/* Q factors taken by copy from the previous iteration / factored, since the last call */
API void amgd_test_qf_reuse_stats(uint64_t *out) {
  static uint64_t r0 = 0, f0 = 0;
  uint64_t r, f;
  amgd_qfactor_reuse_stats(&r, &f);
  out[0] = r - r0; out[1] = f - f0;
  r0 = r; f0 = f;
}
/* cap on live device bytes (0: none): the out-of-HBM path without filling 288 GB */
API void amgd_test_hbm_cap(uint64_t bytes) { amgd_set_hbm_cap((size_t)bytes); }
API uint64_t amgd_test_pool_inuse(void) { return amgd_pool_bytes_in_use(); }

/* one bare partitioned-mode collective (the collective guard's tests): kind 0 an allgatherv
   of `bytes` per rank, 1 an alltoallv of `bytes` to every peer (expecting `expect` bytes
   from each); returns 0 */
API int amgd_test_comm(int kind, uint64_t bytes, uint64_t expect) {
  const int N = amgd_pcomm_size(), me = amgd_pcomm_rank();
  uint64_t *so = (uint64_t *)malloc(8 * ((size_t)N + 1)), *ro = (uint64_t *)malloc(8 * ((size_t)N + 1));
  for (int p = 0; p <= N; p++) { so[p] = bytes * p; ro[p] = (kind ? expect : bytes) * p; }
  char *sb = (char *)amgd_alloc(bytes * N + 16), *rb = (char *)amgd_alloc(ro[N] + 16);
  amgd_memset(sb, me + 1, bytes * N);
  if (kind == 0) {
    void *b = sb;
    amgd_allgatherv(1, &b, so);
  } else {
    amgd_pcomm_alltoallv(sb, so, rb, ro);
  }
  amgd_sync();
  amgd_free(sb); amgd_free(rb);
  free(so); free(ro);
  return 0;
}
/* kernel-route counters since the last reset (out: AMGD_R_N entries) */
API void amgd_test_route_stats(uint64_t *out, int reset) {
  for (int r = 0; r < AMGD_R_N; r++) out[r] = amgd_route_ctr[r];
  if (reset) memset(amgd_route_ctr, 0, sizeof amgd_route_ctr);
}
API uint64_t amgd_test_spmv_shard_calls(void) { return amgd_spmv_shard_calls(); }

/* SpGEMM kernel family: 1 = flat-enumeration kernels only, 0 = automatic */
extern void amgd_qapply_set_huge(int n);
API void amgd_test_qa_huge(int n) { amgd_qapply_set_huge(n); }
extern void amgd_spmv_set_rw(int rw);
API void amgd_test_spmv_rw(int rw) { amgd_spmv_set_rw(rw); }
extern void amgd_spmv_set_pair(int on);
extern void amgd_spmv_set_rw_bounds(int lo, int hi);
extern void amgd_set_d2h_poll(int on);
extern void amgd_fs_set_amx(int on);
API void amgd_test_fs_amx(int on) { amgd_fs_set_amx(on); }
extern void amgd_qa_set_tile(int t);
API void amgd_test_qa_tile(int t) { amgd_qa_set_tile(t); }
API void amgd_test_d2h_poll(int on) { amgd_set_d2h_poll(on); }
/* partitioned setup: [interp_lmop calls on gathered data, calls with a dirty prefix,
   eager exchanges, eager exchanges that took the exact second round] of the last setup(s) */
API void amgd_test_part_stats(uint64_t *out) {
  amgd_part_stats(out);
  pm_eager_stats(out + 2, out + 3);
}
/* forced rare paths: every interp_lmop on gathered data; a fixed eager slot (bytes, 0: adaptive) */
API void amgd_test_part_force(int lmop_gather, int64_t eager_slot) {
  amgd_part_set_force_gather(lmop_gather);
  pm_eager_force_slot(eager_slot);
}
API void amgd_test_spmv_rw_bounds(int lo, int hi) { amgd_spmv_set_rw_bounds(lo, hi); }
API void amgd_test_spmv_pair(int on) { amgd_spmv_set_pair(on); }
extern void amgd_qfactor_set_coop_lds(int m);
API void amgd_test_qf_coop_lds(int m) { amgd_qfactor_set_coop_lds(m); }
/* huge supports factored per connected component (1, default) or whole (0); -1: env */
extern void amgd_qfactor_set_split(int on);
API void amgd_test_qf_split(int on) { amgd_qfactor_set_split(on); }
/* long-row thresholds: listed products (k_rows_exact) and find_support's expand / select;
   0 disables, -1 restores the environment / default (4096) */
extern void amgd_spmv_set_long(int64_t n);
extern void amgd_fs_set_long(int64_t n);
API void amgd_test_mv_long(int64_t n) { amgd_spmv_set_long(n); }
API void amgd_test_fs_long(int64_t n) { amgd_fs_set_long(n); }
extern void amgd_spgemm_force_flat(int on);
API void amgd_test_spgemm_flat(int on) { amgd_spgemm_force_flat(on); }
/* windowed (k_sg_wwin) routing of wide rows: 0 = hash kernels only; > 0 = every wide row windowed
   (routing width 1024..16384); -1 = default (2048, rows with >= 48 products per window) */
extern void amgd_set_seg_split(int on);
API void amgd_test_seg_split(int on) { amgd_set_seg_split(on); }
extern void amgd_set_dot_split(int on);
API void amgd_test_dot_split(int on) { amgd_set_dot_split(on); }
extern void amgd_set_dot_spec_min(int chunks);
API void amgd_test_dot_spec_min(int chunks) { amgd_set_dot_spec_min(chunks); }
extern void amgd_spgemm_set_dr_sort(int on);
API void amgd_test_spgemm_dr_sort(int on) { amgd_spgemm_set_dr_sort(on); }
API void amgd_test_spat_inc(int on) { amgd_spat_set_inc(on); }
API void amgd_test_spat_stats(uint64_t *out3) { amgd_spat_stats(out3); }
API void amgd_test_spgemm_sym(int mode) { if (mode < 0) amgd_spgemm_sym_drop(); else amgd_spgemm_sym_next(mode); }
API void amgd_test_spgemm_sym_stats(uint64_t *kept, uint64_t *reused) { amgd_spgemm_sym_stats(kept, reused); }
extern void amgd_spgemm_set_win(int w);
API void amgd_test_spgemm_win(int w) { amgd_spgemm_set_win(w); }
/* SpMV: row count from which the lane-per-row kernel runs, for whole-matrix and
   listed-row products alike (0 = always, -1 = environment / default) */
extern void amgd_spmv_set_sl_min(int64_t n);
API void amgd_test_spmv_sl_min(int64_t n) { amgd_spmv_set_sl_min(n); }
/* amgd_spmv with every option: x NULL = ordered row sums, y / f optional (f: u8 row mask) */
API int amgd_test_spmv_f(const hcsr *HA, const double *x, double alpha, const double *y, double beta,
                         const uint8_t *f, double *z) {
  if (amgd_rt_init(0) != 0) return -1;
  dcsr *A = up(HA);
  double *dx = NULL, *dy = NULL, *dz = (double *)amgd_alloc((size_t)HA->rn * 8 + 8);
  uint8_t *df = NULL;
  if (x) { dx = (double *)amgd_alloc((size_t)HA->cn * 8 + 8); amgd_h2d(dx, x, (size_t)HA->cn * 8); }
  if (y) { dy = (double *)amgd_alloc((size_t)HA->rn * 8 + 8); amgd_h2d(dy, y, (size_t)HA->rn * 8); }
  if (f) { df = (uint8_t *)amgd_alloc((size_t)HA->rn + 8); amgd_h2d(df, f, HA->rn); }
  amgd_spmv(A, dx, dz, alpha, dy, beta, df);
  amgd_d2h(z, dz, (size_t)HA->rn * 8);
  if (dx) amgd_free(dx);
  if (dy) amgd_free(dy);
  if (df) amgd_free(df);
  amgd_free(dz);
  dcsr_free(&A);
  return 0;
}

/* amgd_spmv_rows: z[list[r]] = (A x)[list[r]] (x NULL: row sums); other rows of z keep
   their input values */
API int amgd_test_spmv_rows(const hcsr *HA, const uint32_t *list, uint32_t n, const double *x, double *z) {
  if (amgd_rt_init(0) != 0) return -1;
  dcsr *A = up(HA);
  double *dx = NULL, *dz = (double *)amgd_alloc((size_t)HA->rn * 8 + 8);
  uint32_t *dl = (uint32_t *)amgd_alloc((size_t)n * 4 + 8);
  if (x) { dx = (double *)amgd_alloc((size_t)HA->cn * 8 + 8); amgd_h2d(dx, x, (size_t)HA->cn * 8); }
  amgd_h2d(dz, z, (size_t)HA->rn * 8);
  amgd_h2d(dl, list, (size_t)n * 4);
  amgd_spmv_rows(A, dl, n, dx, dz);
  amgd_d2h(z, dz, (size_t)HA->rn * 8);
  if (dx) amgd_free(dx);
  amgd_free(dz); amgd_free(dl);
  dcsr_free(&A);
  return 0;
}

/* SpMV micro-benchmark: a generated matrix (amgd_bench_matrix), reps products timed
   with HIP events on the library stream; with_x = 0: ordered row sums (no gather).
   Returns ms per product and the matrix's nnz. */
extern dcsr *amgd_bench_matrix(uint32_t rn, uint32_t cn, uint32_t len0, uint32_t len1, uint32_t gap);
API double amgd_test_spmv_bench(uint32_t rn, uint32_t cn, uint32_t len0, uint32_t len1, uint32_t gap,
                                int with_x, int reps, uint64_t *nnz) {
  if (amgd_rt_init(0) != 0) return -1;
  dcsr *A = amgd_bench_matrix(rn, cn, len0, len1, gap);
  double *x = (double *)amgd_alloc((size_t)cn * 8 + 8), *z = (double *)amgd_alloc((size_t)rn * 8 + 8);
  amgd_vfill(x, cn, 0.5);
  amgd_spmv(A, with_x ? x : NULL, z, 0.0, NULL, 1.0, NULL);   /* warm */
  amgd_timer_reset();
  for (int r = 0; r < reps; r++) {
    amgd_timer_start(7);
    amgd_spmv(A, with_x ? x : NULL, z, 0.0, NULL, 1.0, NULL);
    amgd_timer_stop(7);
  }
  double ms = amgd_timer_ms(7) / reps;
  *nnz = A->nnz;
  amgd_free(x); amgd_free(z);
  dcsr_free(&A);
  return ms;
}
