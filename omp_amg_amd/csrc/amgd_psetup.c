/*
 * amgd_psetup.c -- host driver (C) of the PARTITIONED multi-GPU setup
 * (amgd_part.h for the data layout).
 *
 * The same level loop as amgd_setup.c (reference amg_setup.c:60-400) with every matrix
 * held as row blocks: rank p owns rows [split[p], split[p+1]) of each level's A, Af, W and
 * AfP and of every intermediate (R, R', W_skel, the constraint operator S, Q factors of
 * its coarse points ...).  Vectors are kept whole on every rank, so the reference-order
 * dots, maxima and every host decision (coarsening norm bound, Lanczos, PCG, the
 * find_support loop) are computed identically everywhere without a collective.  The
 * exchanges are the ones the rows need:
 *   - a product's output rows complete the whole vector (allgatherv of row segments);
 *   - X = A*B fetches the rows of B the local rows of A reference (halo, alltoallv);
 *   - transposes send each rank the pieces of its rows (alltoallv), concatenated in
 *     rank = ascending-row order, which is the stable transpose of amg_setup.c:2000;
 *   - the Q factors fetch the Af rows of their supports, interp_lmop the supports and
 *     Q factors of the coarse points its rows meet;
 *   - find_support's selections are allgathered and each rank removes its own entries.
 * Every row is computed by the one-GPU kernels from the same row data, so the hierarchy
 * is bit-identical to the one-GPU one (tests/test_gpu_partition.py).
 *
 * Not partitioned (each rank computes the whole, identically): the per-sweep vector
 * arithmetic and reductions.  The one-GPU driver's shortcuts run here too, on row blocks:
 * the incremental coarsening / find_support sweeps (list mode across the ranks), the
 * transposed product forms X = (B'A')' where A has long columns (p_spgemm_via_t, the
 * same rule on the global mean rows) and the transposed R chain of the interpolation.
 * interp_lmop's walks past the end of a row (amg_setup.c:1665-1677) are handled by the
 * dirty prefix (p_lmop_prefix) and, as a counted fallback, on gathered data.
 */
#define _POSIX_C_SOURCE 200809L
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "amgd.h"
#include "amgd_hostmath.h"
#include "amgd_part.h"
#include "amgd_psetup.h"

static double *dalloc(uint64_t n) { return (double *)amgd_alloc_f64(n * 8 + 8); }
static double *dones(uint64_t n) { double *p = dalloc(n); amgd_vfill(p, n, 1.0); return p; }
static double *dzeros(uint64_t n) { double *p = dalloc(n); amgd_vfill(p, n, 0.0); return p; }

static int g_me, g_N;
static uint64_t g_ub;
static amgd_stats *g_pst;             /* the stats being filled (ub sites) */
static int g_plvl;
static void ub_note(int site) {      /* site codes: amgd_setup.c ub_note */
  if (g_ub < AMGD_UB_LOG) { g_pst->ub_site[g_ub] = (uint8_t)site; g_pst->ub_level[g_ub] = (uint8_t)g_plvl; }
  g_ub++;
}
#define UB(site) ub_note(site)
static void ph(int id) { amgd_ph_mark(g_plvl, id); }     /* AMGD_PHASES=1 time table */
static int g_verbose = -1;
static int verbose(void) {
  if (g_verbose < 0) { const char *e = getenv("AMGD_VERBOSE"); g_verbose = e && *e && *e != '0'; }
  return g_verbose && g_me == 0;
}
static uint64_t g_lmop_full;        /* interp_lmop calls done on gathered data */
static uint64_t g_lmop_prefix;      /* interp_lmop calls with a dirty prefix walked on the whole S pattern */
/* AMGD_PART_LMOP_GATHER=1 / amgd_part_force(1, ..): every interp_lmop of a partitioned setup
   takes the gathered path (tests: the rare fallback exercised at every level) */
static int g_force_gather = -1;
static int force_gather(void) {
  if (g_force_gather < 0) { const char *e = getenv("AMGD_PART_LMOP_GATHER"); g_force_gather = e && *e ? atoi(e) : 0; }
  return g_force_gather;
}
void amgd_part_set_force_gather(int on) { g_force_gather = on; }
void amgd_part_stats(uint64_t *out) {       /* lmop gathered calls, lmop prefix calls */
  out[0] = g_lmop_full;
  out[1] = g_lmop_prefix;
}

/* sum / OR / max of one u64 per rank, identical on every rank */
static uint64_t all_sum(uint64_t v) {
  uint64_t *a = (uint64_t *)calloc((size_t)g_N, 8);
  a[g_me] = v;
  amgd_pcomm_allgather_u64(a, 1);
  uint64_t s = 0;
  for (int p = 0; p < g_N; p++) s += a[p];
  free(a);
  return s;
}
static uint64_t all_max(uint64_t v) {
  uint64_t *a = (uint64_t *)calloc((size_t)g_N, 8);
  a[g_me] = v;
  amgd_pcomm_allgather_u64(a, 1);
  uint64_t s = 0;
  for (int p = 0; p < g_N; p++) s = a[p] > s ? a[p] : s;
  free(a);
  return s;
}
static uint64_t gnnz(const pmat *A) { return all_sum(A->m->nnz); }
/* the global nnz of two matrices in one exchange */
static void gnnz2(const pmat *A, const pmat *B, uint64_t *na, uint64_t *nb) {
  uint64_t *a = (uint64_t *)calloc(2ull * g_N, 8);
  a[2 * g_me] = A->m->nnz;
  a[2 * g_me + 1] = B->m->nnz;
  amgd_pcomm_allgather_u64(a, 2);
  *na = *nb = 0;
  for (int p = 0; p < g_N; p++) { *na += a[2 * p]; *nb += a[2 * p + 1]; }
  free(a);
}

/* X = A*B, or as X = (B'*A')' where the one-GPU driver takes that form (amgd_setup.c
   spgemm_via_t: A' has long rows -- mean >= 64 and >= twice B's -- so the transposed
   product runs on the k-sequential kernels); the rule reads global means, so every rank
   takes the same form.  Same products in the same k order either way: bit-identical.
   tr != NULL: the transposed product is returned as it comes (*tr = 1). */
static pmat *p_spgemm_via_t(const pmat *A, const pmat *At, const pmat *B, const pmat *Bt, int *tr) {
  int t = 0;
  if (At && Bt) {
    uint64_t nat, nb;
    gnnz2(At, B, &nat, &nb);
    const uint64_t avg_at = At->rp->n ? nat / At->rp->n : 0, avg_b = B->rp->n ? nb / B->rp->n : 0;
    t = !(avg_at < 64 || avg_at < 2 * avg_b);
  }
  if (tr) *tr = t;
  if (!t) return pm_spgemm(A, B, 0);
  pmat *Xt = pm_spgemm(Bt, At, 0);
  if (tr) return Xt;
  pmat *X = pm_transpose(Xt);
  pm_free(&Xt);
  return X;
}

/* ------------------------------------------------------------------------ */
/* coarsen (amg_setup.c:2737): full sweeps, whole vectors                     */
/* ------------------------------------------------------------------------ */
static pmat *p_strength(const pmat *A) {
  const uint32_t n = A->rp->n;
  double *D = dalloc(n);
  pm_diag(A, D);
  amgd_vunary(D, n, AMGD_V_SQRT);
  amgd_vunary(D, n, AMGD_V_INV);
  pmat *S = pm_copy(A);
  pm_diag_op2(S, D, D, AMGD_SCALE2_ABS);
  pm_diag(S, D);
  pm_diag_op(S, D, AMGD_DMINUS);
  amgd_free(D);
  return S;
}
/* amgd_cs_grow across the ranks: every hop expands the own rows of the frontier (global
   views: the other rows are empty here), then the ranks' new rows are exchanged and
   claimed, so all ranks hold the same hop sets; 0 when a hop passes `limit` (the same
   decision everywhere: it reads the union's counts) */
static int p_cs_grow(const dcsr *gS, const dcsr *gSt, uint32_t *front, uint32_t *cnt_d, uint32_t *stamp,
                     uint32_t base8, uint32_t limit, uint32_t *cum) {
  /* one exchange per hop while the shares fit; one slot state per hop, since a hop's share
     is like the same hop's of the previous sweep (the front grows hop by hop within one) */
  static pm_eager eg[7];
  uint32_t c[8];
  uint64_t *len = (uint64_t *)calloc((size_t)g_N, 8), *usr = (uint64_t *)calloc((size_t)g_N, 8);
  int ok = 1;
  for (int r = 1; r <= 6 && ok; r++) {
    amgd_d2h(c, cnt_d, 32);
    uint32_t hi = 0;
    for (int q = 0; q < r; q++) hi += c[q];
    if (hi > limit) { ok = 0; break; }
    amgd_cs_hop1(gS, gSt, front, cnt_d, r, stamp, base8, limit);
    amgd_d2h(c, cnt_d, 32);
    uint64_t tot = 0;
    char *ids = pm_allgather_dyn(&eg[r], front + hi, 4ull * c[r], c[r], len, usr, &tot);
    for (int p = 0, at = 0; p < g_N; at += (int)len[p], p++)
      if (p != g_me && len[p])
        amgd_cs_claim_ext((const uint32_t *)(ids + at), len[p] / 4, stamp, base8, r, front, hi, cnt_d + r);
    amgd_free(ids);
  }
  free(len); free(usr);
  if (!ok) return 0;
  amgd_d2h(c, cnt_d, 32);
  uint32_t t = 0, cu[7];
  for (int r = 0; r <= 6; r++) {
    t += c[r];
    cu[r] = t;
    if (t > limit) return 0;
  }
  for (int r = 0; r <= 6; r++) cum[r] = cu[r];
  return 1;
}

/* Incremental sweeps as on one GPU (amgd_coarsen.hip: after the first sweep only the rows
   within 6 hops of the last sweep's new C points change).  Either mode of the one-GPU
   driver, by its rule (AMGD_CS_LIST_NNZ, on the global nnz): list mode -- every stage runs
   its list kernel on the global views (the other ranks' rows come out empty) -- or the
   block filter -- the stage kernels on the own rows, recomputing the 256-row blocks that
   hold a dirty row.  Then the owners' values of the dirty rows are exchanged
   (pm_list_sync): the same values a full sweep gives.  AMGD_CS_INC=0: full sweeps. */
static void p_coarsen(const pmat *A, uint8_t *vc, double ctol) {
  const uint32_t n = A->rp->n, r0 = A->rp->split[g_me];
  pmat *S = p_strength(A);
  pmat *St = pm_transpose(S);
  uint8_t *vf = (uint8_t *)amgd_alloc(n + 1), *ma = (uint8_t *)amgd_alloc(n + 1), *mb = (uint8_t *)amgd_alloc(n + 1);
  double *vfd = dones(n), *g = dalloc(n), *w1 = dalloc(n), *w2a = dalloc(n), *w2 = dalloc(n);
  double *w = dalloc(n), *x1 = dalloc(n), *x2 = dalloc(n), *m1 = dalloc(n), *m2 = dalloc(n), *amax = dalloc(n);
  uint32_t *anyvc = (uint32_t *)amgd_alloc(4), *stamp = (uint32_t *)amgd_alloc(4ull * n + 4);
  uint32_t *front[2], *cnt[2];
  for (int q = 0; q < 2; q++) {
    front[q] = (uint32_t *)amgd_alloc(4ull * n + 4);
    cnt[q] = (uint32_t *)amgd_alloc(64);
  }
  const char *e1 = getenv("AMGD_CS_INC"), *e2 = getenv("AMGD_CS_MIN_ROWS");
  const uint64_t min_rows = e2 && *e2 ? strtoull(e2, NULL, 10) : 65536;
  const uint64_t nnzS = gnnz(S);
  const int inc = !(e1 && *e1 && atoi(e1) == 0) && n >= min_rows && nnzS + gnnz(St) <= 64ull * n;
  const char *e3 = getenv("AMGD_CS_LIST_NNZ");
  const int list_mode = nnzS <= (uint64_t)(e3 && *e3 ? atoi(e3) : 12) * n;
  const uint32_t limit = n / 4;
  dcsr gS, gSt;
  if (inc) { gS = pm_gview(S); gSt = pm_gview(St); }
  amgd_memset(vc, 0, n);
  amgd_memset(vf, 1, n);
  amgd_memset(anyvc, 0, 4);
  amgd_memset(stamp, 0, 4ull * n);
  amgd_memset(cnt[0], 0, 64);
  int it = 0, cur = 0;
  for (;;) {
    it++;
    amgd_csrows rows_, *rows = NULL, lrows;
    if (inc && it > 1 && p_cs_grow(&gS, &gSt, front[cur], cnt[cur], stamp, 8u * it, limit, rows_.cum)) {
      rows_.list = list_mode ? front[cur] : NULL;
      rows_.fs = stamp;
      rows_.fb = 8u * it;
      rows = &rows_;
      lrows = rows_;                       /* the block filter on the own rows */
      lrows.fs = stamp + r0;
      amgd_route_hit(AMGD_R_CS_INC);
    }
    const uint32_t *L = front[cur];        /* the dirty rows by hop, in either mode */
#define PSYNC(v, R) pm_list_sync((v), L, rows->cum[(R)], S->rp)
    /* Amax (rows within 1 hop) depends on vf alone, fixed during the sweep: it is formed
       beside g, and both travel in one exchange */
#define PSYNC2(v1, v2, R)                                                            \
  do {                                                                               \
    double *zz_[2] = {(v1), (v2)};                                                   \
    const uint32_t *ll_[2] = {L, L};                                                 \
    const uint32_t nn_[2] = {rows->cum[(R)], rows->cum[(R)]};                        \
    const apart *pp_[2] = {S->rp, S->rp};                                            \
    pm_list_sync_n(2, zz_, ll_, nn_, pp_);                                           \
  } while (0)
    if (rows && !rows->list) {
      amgd_cs_spmv(S->m, vfd, g + r0, vf + r0, &lrows, 1);
      amgd_cs_amax(S->m, vf, 0.1, amax + r0, &lrows, 1);
      PSYNC2(g, amax, 1);
      amgd_cs_spmv(S->m, g, w1 + r0, vf + r0, &lrows, 2);   PSYNC(w1, 2);
      amgd_cs_spmv(S->m, w1, w2a + r0, vf + r0, &lrows, 3); PSYNC(w2a, 3);
      amgd_cs_spmv(S->m, w2a, w2 + r0, vf + r0, &lrows, 4); PSYNC(w2, 4);
    } else if (rows) {
      amgd_cs_spmv(&gS, vfd, g, vf, rows, 1);
      amgd_cs_amax(&gS, vf, 0.1, amax, rows, 1);
      PSYNC2(g, amax, 1);
      amgd_cs_spmv(&gS, g, w1, vf, rows, 2);   PSYNC(w1, 2);
      amgd_cs_spmv(&gS, w1, w2a, vf, rows, 3); PSYNC(w2a, 3);
      amgd_cs_spmv(&gS, w2a, w2, vf, rows, 4); PSYNC(w2, 4);
    } else {
      /* g = vf.*(S*vf) and Amax (vf alone: formed here, used after the bound test) in one
         exchange of their row segments */
      amgd_spmv(S->m, vfd, g + r0, 0.0, NULL, 1.0, vf + r0);
      amgd_mat_amax(S->m, vf, 0.1, amax + r0);
      {
        void *b2[2] = {g, amax};
        uint64_t *o2 = (uint64_t *)malloc(2 * ((size_t)g_N + 1) * 8);
        for (int p = 0; p <= g_N; p++) o2[p] = o2[g_N + 1 + p] = 8ull * S->rp->split[p];
        if (g_N > 1) amgd_allgatherv(2, b2, o2);
        free(o2);
      }
      pm_spmv(S, g, w1, 0.0, NULL, 1.0, vf);            /* w1  = vf.*(S*g)   */
      pm_spmv(S, w1, w2a, 0.0, NULL, 1.0, vf);          /* w2a = vf.*(S*w1)  */
      pm_spmv(S, w2a, w2, 0.0, NULL, 1.0, vf);          /* w2  = vf.*(S*w2a) */
    }
    amgd_cs_w_mask1(n, w1, w2, w, ctol * ctol, g, ma, x1, rows, 4);
    uint64_t mi = 0;
    double wm = 0;
    double w1m = amgd_max_first2(w1, w, n, &mi, &wm);
    double b = (w1m < wm) ? sqrt(w1m) : sqrt(wm);
    if (b <= ctol) {
      uint32_t any = 0;
      amgd_d2h(&any, anyvc, 4);
      if (!any) { uint8_t one = 1; amgd_h2d(vc + mi, &one, 1); }
      if (verbose()) printf("  coarsen: %d sweeps, norm bound = %f\n", it, b);
      break;
    }
    if (rows && !rows->list) {
      amgd_cs_gather(St->m, vf + r0, x1, amax, m1 + r0, &lrows, 5);  PSYNC(m1, 5);
      amgd_cs_mask2(n, g, m1, ma, mb, x2, rows, 5);
      amgd_cs_gather(St->m, vf + r0, x2, amax, m2 + r0, &lrows, 6);  PSYNC(m2, 6);
    } else if (rows) {
      amgd_cs_gather(&gSt, vf, x1, amax, m1, rows, 5);        PSYNC(m1, 5);
      amgd_cs_mask2(n, g, m1, ma, mb, x2, rows, 5);
      amgd_cs_gather(&gSt, vf, x2, amax, m2, rows, 6);        PSYNC(m2, 6);
    } else {
      /* (Amax: whole since the first exchange of the sweep) */
      amgd_mat_max_gather(St->m, vf + r0, x1, amax, m1 + r0);
      pm_allgather_vec(m1, 8, St->rp);
      amgd_cs_mask2(n, g, m1, ma, mb, x2, NULL, 5);
      amgd_mat_max_gather(St->m, vf + r0, x2, amax, m2 + r0);
      pm_allgather_vec(m2, 8, St->rp);
    }
#undef PSYNC
#undef PSYNC2
    const int nx = cur ^ 1;
    amgd_memset(cnt[nx], 0, 64);
    amgd_cs_mask3(n, m2, mb, vc, vf, vfd, anyvc, front[nx], cnt[nx], stamp, 8u * it + 8, rows, 6);
    cur = nx;
  }
  if (inc) { pm_gview_free(&gS); pm_gview_free(&gSt); }
  pm_free(&S); pm_free(&St);
  amgd_free(vf); amgd_free(ma); amgd_free(mb); amgd_free(vfd); amgd_free(g); amgd_free(w1);
  amgd_free(w2a); amgd_free(w2); amgd_free(w); amgd_free(x1); amgd_free(x2); amgd_free(m1);
  amgd_free(m2); amgd_free(amax); amgd_free(anyvc); amgd_free(stamp);
  for (int q = 0; q < 2; q++) { amgd_free(front[q]); amgd_free(cnt[q]); }
}

/* ------------------------------------------------------------------------ */
/* Lanczos (amg_setup.c:2435), PCG (amg_setup.c:2242)                         */
/* ------------------------------------------------------------------------ */
/* the value of a 1 x 1 matrix (on the rank owning row 0) */
static double p_a00(const pmat *A) {
  double v = 0;
  if (A->m->rn && A->m->nnz) amgd_d2h(&v, A->m->a, 8);
  uint64_t *a = (uint64_t *)calloc((size_t)g_N, 8);
  memcpy(&a[g_me], &v, 8);
  amgd_pcomm_allgather_u64(a, 1);
  int owner = 0;
  for (int p = 0; p < g_N; p++) if (A->rp->split[p + 1] > A->rp->split[p]) { owner = p; break; }
  memcpy(&v, &a[owner], 8);
  free(a);
  return v;
}
#define KMAX 299
static uint32_t p_lanczos(const pmat *A, double *out) {
  const uint32_t rn = A->rp->n;
  double *rh = (double *)malloc((size_t)rn * 8 + 8);
  for (uint32_t i = 0; i < rn; i++) rh[i] = (double)rand() / (double)RAND_MAX;
  double *r = dalloc(rn);
  amgd_h2d(r, rh, (size_t)rn * 8);
  free(rh);
  double l[KMAX + 2], y[KMAX + 2], d[KMAX + 2], v[KMAX + 2];
  double beta = amgd_norm2(r, rn), beta2 = beta * beta, change;
  beta = sqrt(beta2);
  uint32_t k = 0;
  {
    double fr = pm_fro_minus_eye(A), fro = sqrt(fr), fro2 = fro * fro;
    fro = sqrt(fro2);
    if (fro < 1e-11) { l[0] = 1; l[1] = 1; y[0] = 0; y[1] = 0; k = 2; change = 0.0; }
    else change = 1.0;
  }
  if (rn == 1) {
    const double a00 = p_a00(A);
    l[0] = a00; l[1] = a00; y[0] = 0; y[1] = 0; k = 2; change = 0.0;
  }
  double *qk = dzeros(rn), *qkm1 = dalloc(rn), *Aqk = dalloc(rn);
  while (k < KMAX && (change > 1e-5 || y[0] > 1e-3 || y[k - 1] > 1e-3)) {
    k++;
    amgd_lanczos_step(r, 1. / beta, qk, qkm1, rn);
    pm_spmv(A, qk, Aqk, 0, NULL, 1, NULL);
    double alpha = amgd_dot(qk, Aqk, rn);
    amgd_lanczos_resid(r, Aqk, qk, alpha, qkm1, beta, rn);
    if (k == 1) { l[0] = alpha; y[0] = 1; }
    else {
      double l0 = l[0], lkm2 = l[k - 2];
      d[0] = 0;
      for (uint32_t i = 1; i < k; i++) d[i] = l[i - 1];
      d[k] = 0;
      v[0] = alpha;
      for (uint32_t i = 1; i < k; i++) v[i] = beta * y[i - 1];
      tdeig(l, y, d, v, (int)k - 1);
      change = fabs(l0 - l[0]) + fabs(lkm2 - l[k - 1]);
    }
    beta = amgd_norm2(r, rn);
    beta2 = beta * beta;
    beta = sqrt(beta2);
    if (beta == 0) break;
  }
  uint32_t n = 0;
  for (uint32_t i = 0; i < k; i++) if (y[i] < 0.01) out[n++] = l[i];
  amgd_free(r); amgd_free(qk); amgd_free(qkm1); amgd_free(Aqk);
  return n;
}

static double g_pcg_rho, g_pcg_stop;
static uint32_t p_pcg(double *x, const pmat *A, double *r, const double *M, double tol, const double *b) {
  const uint32_t rn = A->rp->n;
  amgd_vfill(x, rn, 0.0);
  if (rn == 0) return 0;
  double *p = dzeros(rn), *z = dalloc(rn), *w = dalloc(rn);
  amgd_vmul_dot_prep(z, M, r, rn);
  double rho = amgd_dot(r, z, rn);
  double rho_0 = amgd_dot3(M, b, rn);
  double rho_stop = tol * tol * rho_0, rho_old = 1, alpha, beta;
  uint32_t n = rn <= 100 ? rn : 100, k = 0;
  while (rho > rho_stop && k < n) {
    k++;
    beta = rho / rho_old;
    amgd_pcg_p(p, z, beta, rn);
    pm_spmv(A, p, w, 0, NULL, 1, NULL);
    alpha = amgd_dot(p, w, rn);
    alpha = rho / alpha;
    amgd_pcg_xrz(x, r, z, p, w, M, alpha, rn);
    rho_old = rho;
    rho = amgd_dot(r, z, rn);
  }
  g_pcg_rho = rho;
  g_pcg_stop = rho_stop;
  amgd_free(p); amgd_free(z); amgd_free(w);
  return k;
}

/* ------------------------------------------------------------------------ */
/* interpolation pieces                                                      */
/* ------------------------------------------------------------------------ */
typedef struct {
  pmat *Wt;            /* W_skel^T: rows = coarse points of this rank */
  double *Q;           /* packed Q factors of those coarse points */
  uint64_t *qoff, qtot;
  pmat *S, *W0, *W0t;
  dcsr *Qbuf;          /* when set, Q points into it (the halo view of interp_lmop) */
} pfactor;
/* the buffer a factor's Q lives in */
static void q_release(double *Q, dcsr **Qbuf) {
  if (*Qbuf) pm_ext_free(Qbuf);
  else if (Q) amgd_free(Q);
}
static void pfactor_free(pfactor *f) {
  pm_free(&f->Wt);
  q_release(f->Q, &f->Qbuf);
  if (f->qoff) amgd_free(f->qoff);
  pm_free(&f->S); pm_free(&f->W0); pm_free(&f->W0t);
}

/* AMGD_PHASES=1: per level the pool peak (GB) inside coarsen / smoother / the parts of the
   interpolation / RAP on every rank (stderr) -- where a rank's HBM peak sits */
enum { PK_COARSEN, PK_SMOOTH, PK_INTERP, PK_RAP, PK_QF, PK_WEIGHTS, PK_AFW_R, PK_EXPAND, PK_LMOP, PK_N };
static const char *pk_name[PK_N] = {"coarsen", "smoother", "interp", "rap", "qfactor", "weights", "AfW_R", "expand", "lmop"};
static int g_pph = -1;
static uint32_t g_pklvl;
static double g_pk[64][PK_N];
static void pk_mark(uint32_t level, int ph) {
  if (g_pph < 0) { const char *e = getenv("AMGD_PHASES"); g_pph = e && *e && *e != '0'; }
  if (!g_pph || level >= 64) return;
  const double pk = amgd_pool_ipeak_take() / 1e9;
  if (pk > g_pk[level][ph]) g_pk[level][ph] = pk;
}
static void pk_report(uint32_t nl) {
  if (g_pph <= 0) return;
  fprintf(stderr, "rank %d pool peak GB per level:", g_me);
  for (int p = 0; p < PK_N; p++) fprintf(stderr, " %8s", pk_name[p]);
  fprintf(stderr, "\n");
  for (uint32_t l = 0; l < nl && l < 64; l++) {
    fprintf(stderr, "rank %d L%u", g_me, l);
    for (int p = 0; p < PK_N; p++) fprintf(stderr, " %8.3f", g_pk[l][p]);
    fprintf(stderr, "\n");
  }
  fprintf(stderr, "rank %d interp_lmop calls on gathered data: %lu\n", g_me, (unsigned long)g_lmop_full);
  uint64_t k[6];
  amgd_comm_stats_kind(k);
  fprintf(stderr, "rank %d exchanges: allgatherv %lu calls %.3f GB, alltoallv %lu calls %.3f GB received, "
          "u64 allgathers %lu calls\n", g_me, (unsigned long)k[0], k[1] / 1e9, (unsigned long)k[2], k[3] / 1e9,
          (unsigned long)k[4]);
  memset(g_pk, 0, sizeof g_pk);
}

/* interp_lmop (amg_setup.c:1589) on the own rows of S.  The supports and Q factors of the
   coarse points those rows meet are fetched (halo) and the one-GPU paths run on global-row
   views of the own rows of S and W_skel.  The dirty coarse points (a zero skeleton weight:
   their sp_add walks leave the row, amg_setup.c:1665-1677, and may run into the next
   rank's rows) form a prefix [0, D) of the coarse points; their contributions are walked on
   every rank over the whole S pattern with the supports and Q factors of [0, D) only, each
   rank keeping its rows' values, and the clean points [D, nc) -- sums that stay in their
   row -- follow on the views.  Only a walk of the views running past the rank's last row
   (a clean contribution missing its column) falls back to the whole operator. */
static dcsr prefix_view(const dcsr *M, uint32_t r0, uint32_t D, apart *Pd, const apart *P) {
  /* the rows of M (local rows from r0) below global row D, and the partition of [0, D) */
  dcsr v = *M;
  const uint32_t r1 = r0 + M->rn;
  v.rn = D <= r0 ? 0 : (D >= r1 ? M->rn : D - r0);
  v.nnz = 0;
  if (v.rn) amgd_d2h(&v.nnz, M->ro + v.rn, 8);
  Pd->N = P->N;
  Pd->n = D;
  for (int p = 0; p <= P->N; p++) Pd->split[p] = P->split[p] < D ? P->split[p] : D;
  return v;
}
static void p_lmop_prefix(pmat *S, const pfactor *f, const pmat *qp, const double *u, uint32_t D) {
  const apart *Pc = f->Wt->rp;
  uint32_t *spl = (uint32_t *)malloc(2 * sizeof(uint32_t) * (Pc->N + 1));
  apart Pd[2] = {{0, 0, spl}, {0, 0, spl + Pc->N + 1}};
  dcsr wv = prefix_view(f->Wt->m, Pc->split[g_me], D, &Pd[0], Pc);
  dcsr qv = prefix_view(qp->m, Pc->split[g_me], D, &Pd[1], Pc);
  pmat wp = {&wv, &Pd[0], f->Wt->cp}, qq = {&qv, &Pd[1], Pc};
  dcsr *WtD = pm_gather_full(&wp), *QD = pm_gather_full(&qq);
  /* the whole S pattern (row offsets, columns); the values of the own rows only */
  dcsr sv = *S->m;
  sv.a = NULL;
  pmat sp = {&sv, S->rp, S->cp};
  dcsr *Sf = pm_gather_pattern(&sp);
  const uint32_t r0 = S->rp->split[g_me];
  uint64_t off = 0;
  amgd_d2h(&off, Sf->ro + r0, 8);
  amgd_memset(S->m->a, 0, S->m->nnz * 8);
  amgd_lmop_set_window(S->m->a, off, off + S->m->nnz);
  amgd_lmop_general(Sf, WtD, QD->a, QD->ro, u, 0, D);
  amgd_lmop_set_window(NULL, 0, 0);
  if (g_pph > 0 && g_me == 0)
    fprintf(stderr, "rank 0 L%u lmop prefix D=%u: whole S pattern %.3f GB, supports %.3f GB, Q %.3f GB\n", g_pklvl,
            D, (Sf->nnz * 4.0 + Sf->rn * 8.0) / 1e9, WtD->nnz * 12.0 / 1e9, QD->nnz * 12.0 / 1e9);
  dcsr_free(&Sf); dcsr_free(&WtD); dcsr_free(&QD);
  free(spl);
}
static void p_lmop(pmat *S, const pmat *Wskel, pfactor *f, const double *u) {
  dcsr *WtE = pm_halo_rows(f->Wt, Wskel->m);
  /* the Q factors as a matrix whose row c holds Q_c (offsets qoff): halo rows of it */
  dcsr qm;
  qm.rn = f->Wt->m->rn;
  qm.cn = 1;
  qm.nnz = f->qtot;
  qm.ro = f->qoff;
  qm.col = NULL;                                      /* values only */
  qm.a = f->Q;
  pmat qp = {&qm, f->Wt->rp, f->Wt->cp};
  /* the dirty prefix: every dirty point of every rank (its own coarse points) lies below D */
  uint32_t dl, cl;
  amgd_lmop_classify_view(f->Wt->m, &dl, &cl);
  dl = dl ? f->Wt->rp->split[g_me] + dl : 0;
  const uint32_t D = (uint32_t)all_max(dl);
  if (D) {
    g_lmop_prefix++;
    p_lmop_prefix(S, f, &qp, u, D);
    amgd_lmop_set_prefix(D);
  }
  dcsr *QE = pm_halo_rows(&qp, Wskel->m);
  const int qview = pm_ext_is_view(QE);      /* one rank: QE is the factor's own buffer */
  if (!qview) {
    /* the own Q factors now sit in the view too (a contiguous copy at the own rows):
       the factor keeps that copy and its own buffer goes, instead of two copies of the
       own share through interp_lmop's peak */
    uint64_t o = 0;
    amgd_d2h(&o, QE->ro + f->Wt->rp->split[g_me], 8);
    q_release(f->Q, &f->Qbuf);
    f->Q = QE->a + o;
    f->Qbuf = QE;
    qm.a = f->Q;
  }
  uint32_t *kpos = pm_kpos(Wskel, WtE);
  dcsr gS = pm_gview(S), gW = pm_gview(Wskel);
  const int last = S->rp->split[g_me + 1] == S->rp->n;
  amgd_lmop_spill_detect(!last);
  amgd_lmop(&gS, &gW, kpos, WtE, QE->a, QE->ro, u);
  if (g_pph > 0 && g_me == 0)
    fprintf(stderr, "rank 0 L%u lmop views: S %.3f GB, W_skel %.3f GB, supports %.3f GB (%lu own), Q %.3f GB "
            "(%lu own), QQ %.3f GB\n", g_pklvl, S->m->nnz * 12.0 / 1e9, Wskel->m->nnz * 12.0 / 1e9,
            WtE->nnz * 12.0 / 1e9, (unsigned long)f->Wt->m->nnz, QE->nnz * 12.0 / 1e9, (unsigned long)f->qtot,
            amgd_lmop_qq_bytes() / 1e9);
  const int st = (last ? 0 : amgd_lmop_spilled()) | amgd_lmop_missed();
  amgd_lmop_spill_detect(0);
  amgd_lmop_set_prefix(0);
  pm_gview_free(&gS);
  pm_gview_free(&gW);
  if (all_max((uint64_t)st) != 0 || force_gather()) {
    g_lmop_full++;
    dcsr *Sf = pm_gather_full(S), *Wsf = pm_gather_full(Wskel), *Qf = pm_gather_full(&qp);
    uint64_t *perm = NULL;
    dcsr *Wtf = amgd_transpose(Wsf, &perm);
    uint32_t *kp = amgd_lmop_kpos(Wtf, perm);
    amgd_free(perm);
    amgd_comm_suspend_partition(1);
    amgd_lmop(Sf, Wsf, kp, Wtf, Qf->a, Qf->ro, u);
    amgd_comm_suspend_partition(0);
    const uint32_t r0 = S->rp->split[g_me];
    uint64_t off = 0;
    amgd_d2h(&off, Sf->ro + r0, 8);
    if (S->m->nnz) amgd_d2d(S->m->a, Sf->a + off, 8 * S->m->nnz);
    amgd_free(kp);
    dcsr_free(&Sf); dcsr_free(&Wsf); dcsr_free(&Wtf); dcsr_free(&Qf);
  }
  amgd_free(kpos);
  pm_ext_free(&WtE);
  if (qview) pm_ext_free(&QE);
  amgd_free(qm.col);
  pk_mark(g_pklvl, PK_LMOP);
}

static void p_solve_constraint(double *lam, const pmat *W_skel, pfactor *fac, const pmat *W0,
                               const double *alpha, const double *u, const double *v, double tol) {
  const uint32_t nf = W_skel->rp->n, nc = W_skel->cp->n;
  double *au2 = dalloc(nc);
  amgd_vop(au2, u, u, nc, AMGD_V_MUL);
  amgd_vop(au2, au2, alpha, nc, AMGD_V_MUL);
  if (!fac->S) {
    pmat *Wn = pm_drop_zeros(W_skel), *Wnt = pm_drop_zeros(fac->Wt);
    fac->S = pm_spgemm(Wn, Wnt, 1);
    pm_free(&Wn); pm_free(&Wnt);
    ph(PH_SPAT);
    p_lmop(fac->S, W_skel, fac, au2);
    ph(PH_LMOP);
  }
  pmat *S = fac->S;
  double *resid = dalloc(nf), *d = dalloc(nf);
  pm_spmv(W0, u, resid, 1.0, v, -1.0, NULL);
  pm_diag(S, d);
  uint8_t *dl = (uint8_t *)amgd_alloc(nf + 1);
  amgd_u8_nonzero(d, dl, nf);
  uint64_t ncond = amgd_u8_count(dl, nf);
  double *q = dalloc(ncond), *xx = dalloc(ncond);
  if (ncond != nf) {
    amgd_vzero_where(lam, dl, nf);
    apart *Pc = apart_induced(S->rp, dl);
    pmat *S2 = pm_sub_mat(S, dl, dl, Pc, Pc);
    double *rc = dalloc(nf), *dc = dalloc(nf), *lc = dalloc(nf);
    amgd_vcompact(rc, resid, dl, nf);
    amgd_vcompact(dc, d, dl, nf);
    amgd_vcompact(lc, lam, dl, nf);
    pm_spmv(S2, lc, q, 1., rc, -1., NULL);
    amgd_vunary(dc, ncond, AMGD_V_INV);
    const uint32_t its = p_pcg(xx, S2, q, dc, tol, rc);
    if (verbose())
      printf("   constraint: %lu of %u rows, pcg %u its, rho %.9e stop %.9e\n", (unsigned long)ncond, nf, its,
             g_pcg_rho, g_pcg_stop), fflush(stdout);
    amgd_vexpand_add(lam, xx, dl, nf);
    amgd_free(rc); amgd_free(dc); amgd_free(lc);
    pm_free(&S2);
    apart_free(&Pc);
  } else {
    pm_spmv(S, lam, q, 1., resid, -1., NULL);
    amgd_vunary(d, nf, AMGD_V_INV);
    const uint32_t its = p_pcg(xx, S, q, d, tol, resid);
    if (verbose())
      printf("   constraint: %u of %u rows, pcg %u its, rho %.9e stop %.9e\n", nf, nf, its, g_pcg_rho, g_pcg_stop),
          fflush(stdout);
    amgd_vop(lam, lam, xx, nf, AMGD_V_ADD);
  }
  amgd_free(au2); amgd_free(resid); amgd_free(d); amgd_free(dl); amgd_free(q); amgd_free(xx);
  ph(PH_PCG);
}

/* solve_weights (amg_setup.c:1437) */
static pmat *p_qapply(const pfactor *f, const pmat *Amt, const double *au, const double *lam) {
  pmat *Wt = pm_new(dcsr_empty_like_pattern(f->Wt->m), f->Wt->rp, f->Wt->cp);
  const uint32_t c0 = f->Wt->rp->split[g_me];
  amgd_qapply(f->Wt->m, f->Q, f->qoff, Amt->m, au + c0, lam, Wt->m->a);
  return Wt;
}
static pmat *p_solve_weights(const pmat **W0, double *lam, const pmat *W_skel, pfactor *fac, const pmat *Amt,
                             const double *alpha, const double *u, const double *v, double tol, pmat **Wt_out) {
  const uint32_t nf = W_skel->rp->n, nc = W_skel->cp->n;
  double *au = dalloc(nc), *zeros = dzeros(nf);
  amgd_vop(au, alpha, u, nc, AMGD_V_MUL);
  if (!fac->W0) {
    fac->W0t = p_qapply(fac, Amt, au, zeros);
    fac->W0 = pm_transpose(fac->W0t);
    ph(PH_W0);
  }
  *W0 = fac->W0;
  p_solve_constraint(lam, W_skel, fac, *W0, alpha, u, v, tol);
  pmat *Wt = p_qapply(fac, Amt, au, lam);
  pmat *W = pm_transpose(Wt);
  if (Wt_out) *Wt_out = Wt;
  else pm_free(&Wt);
  amgd_free(au); amgd_free(zeros);
  ph(PH_W);
  return W;
}

/* find_support (amg_setup.c:1260): full sweeps; selections per coarse point on the rank
   owning it, gathered, and each rank removes the selected entries of its own rows of R */
typedef struct { const double *rs, *w, *tmp, *w2; } pfs_first;
static uint32_t p_fs_select(pmat *Rl, pmat *Rt, double *rs, const double *w, double *sumR, double thr,
                            uint32_t *si, uint32_t *sj, uint32_t *nremoved) {
  static pm_eager eg;
  const uint32_t c0 = Rt->rp->split[g_me], nl = Rt->m->rn;
  uint32_t *lb = (uint32_t *)amgd_alloc(12ull * nl + 16);
  uint32_t *li = lb, *lj = lb + 2ull * nl + 2;         /* li has room for [rows | columns] */
  uint32_t rem = 0;
  const uint32_t h = amgd_fs_select_ex(Rl->m, Rt->m, NULL, rs, w + c0, sumR + c0, thr, li, lj, &rem, c0, 0);
  if (h) amgd_d2d(li + h, lj, 4ull * h);                 /* [rows | columns] of the selections */
  /* every rank's selections and its "removed" flag in one exchange */
  uint64_t *len = (uint64_t *)calloc((size_t)g_N, 8), *usr = (uint64_t *)calloc((size_t)g_N, 8), tb = 0;
  char *all = pm_allgather_dyn(&eg, li, 8ull * h, rem, len, usr, &tb);
  uint64_t tot = 0, remall = 0, at = 0;
  for (int p = 0; p < g_N; p++) {
    const uint64_t hp = len[p] / 8;
    if (hp) {
      amgd_d2d(si + tot, all + at, 4 * hp);
      amgd_d2d(sj + tot, all + at + 4 * hp, 4 * hp);
    }
    tot += hp;
    at += len[p];
    remall += usr[p];
  }
  amgd_free(all);
  free(len); free(usr);
  pm_zero_entries(Rl, si, sj, tot);
  if (remall) pm_list_rowsum2(Rl, si, rs, Rt, sj, sumR, (uint32_t)tot);
  amgd_free(lb);
  *nremoved = (uint32_t)(remall ? 1 : 0);
  return (uint32_t)tot;
}
/* amgd_fs_expand across the ranks: the own listed rows' neighbours (global view), then
   the union of the ranks' lists; > cap when any rank's list or the union overflowed */
static uint32_t p_fs_expand(const dcsr *gM, const uint32_t *list, uint32_t n, uint32_t *stamp, uint32_t tag,
                            uint32_t *out, uint32_t cap, pm_eager *eg) {
  const uint32_t h = amgd_fs_expand(gM, list, n, stamp, tag, out, cap);
  uint64_t *len = (uint64_t *)calloc((size_t)g_N, 8), *usr = (uint64_t *)calloc((size_t)g_N, 8), tb = 0;
  /* an overflowed list (h > cap) is incomplete: only its count travels */
  char *ids = pm_allgather_dyn(eg, out, h > cap ? 0 : 4ull * h, h, len, usr, &tb);
  uint32_t res = h;
  int over = 0;
  for (int p = 0; p < g_N; p++) if (usr[p] > cap) over = 1;
  if (over) res = cap + 1;
  else
    for (int p = 0, at = 0; p < g_N; at += (int)len[p], p++)
      if (p != g_me && len[p]) res = amgd_fs_claim_ext((const uint32_t *)(ids + at), len[p] / 4, stamp, tag, out, res, cap);
  amgd_free(ids);
  free(len); free(usr);
  return res;
}

static pmat *p_find_support(const pmat *R, pmat *Rt, double goal, const pfs_first *f1) {
  const uint32_t nf = R->rp->n, nc = R->cp->n;
  pmat *Rl = pm_copy(R);
  double *onec = dones(nc), *rs = dalloc(nf), *w = dalloc(nc), *w2 = dalloc(nc), *tmp = dalloc(nf);
  double *vv = dalloc(nc), *sumR = dalloc(nc);
  const uint64_t cap = gnnz(R) + nc + 16;      /* the one-GPU driver's guard (UB) */
  uint64_t ns = 0;
  /* the selection lists are whole on every rank: grown as they fill instead of sized
     nnz(R) up front (that would replicate an nnz-sized buffer on every rank) */
  uint64_t room = 4ull * nc + 64;
  uint32_t *si = (uint32_t *)amgd_alloc(room * 4), *sj = (uint32_t *)amgd_alloc(room * 4);
  double theta = 0.5;
  int it = 0;
  if (f1) amgd_d2d(rs, f1->rs, (size_t)nf * 8);
  else pm_spmv(Rl, onec, rs, 0., NULL, 1., NULL);
  pm_colsum(Rt, sumR);
  /* incremental sweeps as on one GPU (amgd_setup.c find_support): the listed products run
     on global views of R and R' (own rows only) and the owners' values are exchanged */
  const char *e_inc = getenv("AMGD_FS_INC");
  const int fs_mode = e_inc && *e_inc ? atoi(e_inc) : 1;
  const int fs_inc = fs_mode == 2 || (fs_mode == 1 && nf >= 4096);
  const uint32_t cap_c = nc / 4 + 1, cap_r = nf / 4 + 1;
  uint32_t *st_r = NULL, *st_c = NULL, *L1 = NULL, *L2 = NULL, *L3 = NULL, tag = 0;
  dcsr gRl, gRt;
  if (fs_inc) {
    st_r = (uint32_t *)amgd_alloc((size_t)nf * 4 + 4);
    st_c = (uint32_t *)amgd_alloc((size_t)nc * 4 + 4);
    amgd_memset(st_r, 0, (size_t)nf * 4);
    amgd_memset(st_c, 0, (size_t)nc * 4);
    L1 = (uint32_t *)amgd_alloc((size_t)cap_c * 4 + 4);
    L2 = (uint32_t *)amgd_alloc((size_t)cap_r * 4 + 4);
    L3 = (uint32_t *)amgd_alloc((size_t)cap_c * 4 + 4);
    gRl = pm_gview(Rl);
    gRt = pm_gview(Rt);
  }
  uint64_t prev_off = 0;
  uint32_t prev_nsel = 0;
  ph(PH_FS);
  for (;;) {
    it++;
    int done = 0;
    if (fs_inc && it > 1 && prev_nsel <= cap_c) {
      static pm_eager egx[3];          /* the three expansions' own slot states */
      const uint32_t n1 = p_fs_expand(&gRl, si + prev_off, prev_nsel, st_c, ++tag, L1, cap_c, &egx[0]);
      if (n1 <= cap_c) {
        const uint32_t n2 = p_fs_expand(&gRt, L1, n1, st_r, ++tag, L2, cap_r, &egx[1]);
        if (n2 <= cap_r) {
          const uint32_t n3 = p_fs_expand(&gRl, L2, n2, st_c, ++tag, L3, cap_c, &egx[2]);
          if (n3 <= cap_c) {
            amgd_spmv_rows(&gRt, L1, n1, rs, w);           /* w  on C1 */
            pm_list_sync(w, L1, n1, Rt->rp);
            amgd_spmv_rows(&gRl, L2, n2, w, tmp);          /* tmp on D2 */
            pm_list_sync(tmp, L2, n2, Rl->rp);
            amgd_spmv_rows(&gRt, L3, n3, tmp, w2);         /* w2 on C3 */
            pm_list_sync(w2, L3, n3, Rt->rp);
            done = 1;
            amgd_route_hit(AMGD_R_FS_INC);
          }
        }
      }
    }
    if (!done && it == 1 && f1) {
      amgd_d2d(w, f1->w, (size_t)nc * 8);
      amgd_d2d(tmp, f1->tmp, (size_t)nf * 8);
      amgd_d2d(w2, f1->w2, (size_t)nc * 8);
      done = 1;
    }
    if (!done) {
      pm_spmvt(Rt, rs, w);
      pm_spmv(Rl, w, tmp, 0., NULL, 1., NULL);
      pm_spmvt(Rt, tmp, w2);
    }
    ph(PH_FS_MV);
    amgd_vdiv_guard(vv, w2, w, nc);
    double mv = amgd_max_first(vv, nc, NULL), mw = mv;
    ph(PH_FS_MAX);
    if (mv < goal || mw < goal) break;
    while (mw <= (1 + theta) * goal && theta > 0) theta = theta / 2.;
    if (theta == 0) { UB(1); break; }
    if (nf <= 1) { UB(2); break; }
    uint32_t nrem = 0;
    if (ns + nc + 16 > room) {                  /* a sweep selects at most nc entries */
      const uint64_t r2 = 2 * room + nc + 16;
      uint32_t *a = (uint32_t *)amgd_alloc(r2 * 4), *b = (uint32_t *)amgd_alloc(r2 * 4);
      if (ns) { amgd_d2d(a, si, ns * 4); amgd_d2d(b, sj, ns * 4); }
      amgd_free(si); amgd_free(sj);
      si = a; sj = b; room = r2;
    }
    const uint32_t nsel = p_fs_select(Rl, Rt, rs, w, sumR, (1 + theta) * goal, si + ns, sj + ns, &nrem);
    ph(PH_FS_SEL);
    prev_off = ns;
    prev_nsel = nsel;
    ns += nsel;
    if (nrem == 0) { UB(3); break; }
    if (ns + nc > cap) { UB(4); break; }
  }
  pmat *Sk = pm_coo_ones(si, sj, ns, R->rp, R->cp);
  if (verbose()) printf("    find_support: %d sweeps, %lu entries\n", it, (unsigned long)ns);
  if (fs_inc) {
    pm_gview_free(&gRl); pm_gview_free(&gRt);
    amgd_free(st_r); amgd_free(st_c); amgd_free(L1); amgd_free(L2); amgd_free(L3);
  }
  pm_free(&Rl); pm_free(&Rt);
  amgd_free(onec); amgd_free(rs); amgd_free(w); amgd_free(w2); amgd_free(tmp); amgd_free(vv);
  amgd_free(sumR); amgd_free(si); amgd_free(sj);
  return Sk;
}

typedef struct {
  const pmat *Af, *AfT, *W0, *W0t, *Ar;
  const double *Dfsqrti, *Dcs;
} pr0_ctx;
static pmat *p_r0_rows(const pr0_ctx *c, const uint8_t *bad) {
  pmat *Afb = pm_rows_masked(c->Af, bad);
  /* (Af on the bad rows)' only where the transposed product will be taken (amgd_setup.c
     r0_rows: mean row nnz(Afb) / cols(Af) >= 64 and >= twice W0's), by a column mask of Af' */
  uint64_t nab, nw0;
  gnnz2(Afb, c->W0, &nab, &nw0);
  const uint64_t avg_at = c->Af->cp->n ? nab / c->Af->cp->n : 0, avg_b = c->W0->rp->n ? nw0 / c->W0->rp->n : 0;
  pmat *AfbT = NULL;
  if (avg_at >= 64 && avg_at >= 2 * avg_b)
    AfbT = c->AfT ? pm_new(amgd_cols_masked(c->AfT->m, bad), c->AfT->rp, c->AfT->cp) : pm_transpose(Afb);
  pmat *AfW0 = p_spgemm_via_t(Afb, AfbT, c->W0, c->W0t, NULL);
  pm_free(&Afb);
  pm_free(&AfbT);
  pmat *Arb = pm_rows_masked(c->Ar, bad);
  pmat *Arhat0 = pm_mpm(1., AfW0, 1., Arb);
  pm_free(&AfW0); pm_free(&Arb);
  pm_diag_op2(Arhat0, c->Dfsqrti, c->Dcs, AMGD_SCALE_ABS);   /* |Dfsqrti*X|*Dcs in place */
  return Arhat0;
}
/* expand_support (amg_setup.c:907) */
static pmat *p_expand_support(const pmat *W_skel, const pmat *R, pmat *Rt, const pr0_ctx *r0c, double gamma,
                              const pfs_first *f1) {
  const uint32_t nf = W_skel->rp->n, r0 = W_skel->rp->split[g_me];
  pmat *M = p_find_support(R, Rt, gamma, f1);
  ph(PH_FS);
  pmat *ns = pm_mpm(1., M, 1., W_skel);
  pm_free(&M);
  uint32_t nb_local = 0;
  uint8_t *badl = amgd_bad_rows(ns->m, &nb_local);
  const uint64_t nbad = all_sum(nb_local);
  if (nbad == 0) {
    amgd_skel_binarize(ns->m, 0);
    amgd_free(badl);
    ph(PH_EXP);
    return ns;
  }
  uint8_t *bad = (uint8_t *)amgd_alloc(nf + 8);
  amgd_memset(bad, 0, nf);
  if (ns->m->rn) amgd_d2d(bad + r0, badl, ns->m->rn);
  amgd_free(badl);
  pm_allgather_vec(bad, 1, W_skel->rp);
  if (verbose()) printf("    expand_support: %lu bad rows of %u\n", (unsigned long)nbad, nf);
  ph(PH_EXP);
  pmat *R0 = p_r0_rows(r0c, bad);
  ph(PH_EXP_R0);
  pmat *R0W = pm_mxmpoint(R0, W_skel);
  pmat *Xf = pm_mpm(1., R0, -1., R0W);
  pm_free(&R0W); pm_free(&R0);
  uint32_t *pi = NULL, *pj = NULL;
  uint64_t np = amgd_expand_pick(Xf->m, bad + r0, &pi, &pj);
  double *ones = dones(np);
  pmat *N = pm_new(amgd_coo2csr(np, pi, pj, ones, W_skel->m->rn, W_skel->m->cn, 1), W_skel->rp, W_skel->cp);
  pmat *out = pm_mpm(1., ns, 1., N);
  amgd_skel_binarize(out->m, 1);
  pm_free(&N); pm_free(&ns); pm_free(&Xf);
  amgd_free(ones); amgd_free(pi); amgd_free(pj); amgd_free(bad);
  ph(PH_EXP);
  return out;
}


static pmat *p_interpolation(const pmat *Af, const pmat *AfT, const pmat *Ac, const pmat *Ar, const pmat *ArT,
                             double gamma2, double tol) {
  const uint32_t rnf = Af->rp->n, cnc = Ac->rp->n;
  double *Df = dalloc(rnf), *Dfinv = dalloc(rnf);
  pm_diag(Af, Df);
  amgd_d2d(Dfinv, Df, (size_t)rnf * 8);
  amgd_vunary(Dfinv, rnf, AMGD_V_INV);
  double *uc = dones(cnc), *tmp = dalloc(rnf), *v = dalloc(rnf), *b = dones(rnf);
  pm_spmv(Ar, uc, tmp, 0, NULL, -1, NULL);              /* tmp = -Ar*uc */
  p_pcg(v, Af, tmp, Df, 1e-16, b);
  double *Dc = dalloc(cnc), *Dcinv = dalloc(cnc);
  pm_diag(Ac, Dc);
  amgd_d2d(Dcinv, Dc, (size_t)cnc * 8);
  amgd_vunary(Dcinv, cnc, AMGD_V_INV);
  pmat *ArD = pm_copy(Ar);
  amgd_vals_sqr(ArD->m);
  pm_diag_op2(ArD, Dfinv, Dcinv, AMGD_SCALE2);
  pmat *W_skel = pm_new(amgd_min_skel(ArD->m), Ar->rp, Ar->cp);   /* row-local: one entry per row */
  pm_free(&ArD);
  double *lam = dzeros(rnf), *alpha = dalloc(cnc);
  amgd_d2d(alpha, Dc, (size_t)cnc * 8);
  double *Dfsqrti = Dfinv;
  amgd_vunary(Dfsqrti, rnf, AMGD_V_SQRT);
  pmat *Amt = pm_transpose(Ar);                          /* -Ar' */
  amgd_vals_scale(Amt->m, -1.0);
  double *Dcs = dalloc(cnc), *w1 = dalloc(cnc), *w2 = dalloc(cnc), *onesc = dones(cnc), *r = dalloc(cnc);
  double *rs1 = dalloc(rnf);
  pmat *W = NULL;
  uint64_t prev_nnz = (uint64_t)-1;
  pmat *prevWt = NULL;
  double *prevQ = NULL;
  dcsr *prevQbuf = NULL;
  uint64_t *prevQoff = NULL;
  ph(PH_IPRE);
  for (;;) {
    pfactor fac;
    memset(&fac, 0, sizeof fac);
    fac.Wt = pm_transpose(W_skel);
    dcsr *AfE = pm_halo_rows(Af, fac.Wt->m);             /* the Af rows of the supports */
    fac.Q = amgd_qfactor_reuse(fac.Wt->m, AfE, &fac.qoff, &fac.qtot, prevWt ? prevWt->m : NULL, prevQ, prevQoff);
    pm_ext_free(&AfE);
    pk_mark(g_pklvl, PK_QF);
    ph(PH_QF);
    if (prevWt) {
      pm_free(&prevWt); q_release(prevQ, &prevQbuf); amgd_free(prevQoff);
      prevQ = NULL; prevQoff = NULL;
    }
    const pmat *W0;
    pmat *Wtmp_t = NULL;
    pmat *Wtmp = p_solve_weights(&W0, lam, W_skel, &fac, Amt, alpha, uc, v, tol, &Wtmp_t);
    pk_mark(g_pklvl, PK_WEIGHTS);
    /* Arhat = Af*W + Ar, R = |Dfsqrti*Arhat|*Dcs and R' -- in transposed form when Af*W
       runs as (W'*Af')' (the one-GPU chain, amgd_setup.c interpolation: entry-wise steps
       on the transposes, only R transposed back) */
    int trp = 0;
    pmat *AfWx = p_spgemm_via_t(Af, AfT, Wtmp, Wtmp_t, &trp);
    pmat *R, *Rt;
    if (!trp) {
      pmat *Arhat = pm_mpm(1., AfWx, 1., Ar);
      pm_free(&AfWx);
      pm_free(&Wtmp_t);
      ph(PH_AFW);
      pmat *Arr = pm_mpm(1.0, Arhat, 1.0, Ar);
      pmat *ArW = pm_mxmpoint(Wtmp, Arr);
      pm_free(&Arr);
      pmat *ArWt = pm_transpose(ArW);
      pm_colsum(ArWt, Dcs);
      pm_free(&ArW); pm_free(&ArWt);
      amgd_vop(Dcs, Dcs, Dc, cnc, AMGD_V_ADD);
      amgd_vunary(Dcs, cnc, AMGD_V_INV);
      amgd_vunary(Dcs, cnc, AMGD_V_SQRT);
      R = Arhat;                                         /* |Dfsqrti*Arhat|*Dcsqrti, in place */
      pm_diag_op2(R, Dfsqrti, Dcs, AMGD_SCALE_ABS);
      Rt = pm_transpose(R);
    } else {
      pmat *ArhatT = pm_mpm(1., AfWx, 1., ArT);          /* (Af*W + Ar)' */
      pm_free(&AfWx);
      ph(PH_AFW);
      pmat *ArrT = pm_mpm(1.0, ArhatT, 1.0, ArT);
      pmat *ArWT = pm_mxmpoint(Wtmp_t, ArrT);            /* (W.*Arr)' */
      pm_free(&ArrT); pm_free(&Wtmp_t);
      pm_colsum(ArWT, Dcs);                              /* sum(W.*(Arhat+Ar), 1) */
      pm_free(&ArWT);
      amgd_vop(Dcs, Dcs, Dc, cnc, AMGD_V_ADD);
      amgd_vunary(Dcs, cnc, AMGD_V_INV);
      amgd_vunary(Dcs, cnc, AMGD_V_SQRT);
      Rt = ArhatT;                                       /* R' = |Dfsqrti*Arhat|*Dcsqrti, transposed */
      pm_diag_op2(Rt, Dfsqrti, Dcs, AMGD_SCALE_ABS_T);
      R = pm_transpose(Rt);
    }
    pm_spmv(R, onesc, rs1, 0., NULL, 1., NULL);
    pm_spmvt(Rt, rs1, w1);
    pm_spmv(R, w1, tmp, 0., NULL, 1., NULL);
    pm_spmvt(Rt, tmp, w2);
    amgd_vdiv_guard(r, w2, w1, cnc);
    double maxr = 0;
    uint64_t n = amgd_count_gt(r, cnc, gamma2, &maxr);
    double w1m = amgd_max_first(w1, cnc, NULL);
    pk_mark(g_pklvl, PK_AFW_R);
    ph(PH_R);
    const uint64_t wsk = gnnz(W_skel);
    if (verbose())
      printf("   %lu nzs, %lu cols > %g, worst = %g\n", (unsigned long)wsk, (unsigned long)n, sqrt(gamma2),
             sqrt(maxr)), fflush(stdout);
    int stalled = prev_nnz == wsk;
    if (stalled) UB(5);
    prev_nnz = wsk;
    if (n == 0 || w1m <= gamma2 || stalled) {
      pm_free(&Rt);
      W = p_solve_weights(&W0, lam, W_skel, &fac, Amt, alpha, uc, v, 1e-16, NULL);
      double *wuc = dalloc(rnf);
      pm_spmv(W, uc, wuc, 0., NULL, 1., NULL);
      dcsr g = pm_gview(W);                              /* the diagonal match reads row ids */
      amgd_scale_diag_match(&g, v, wuc);
      pm_gview_free(&g);
      amgd_free(wuc);
      pm_free(&Wtmp);
      pm_free(&R);
      pfactor_free(&fac);
      ph(PH_FINAL);
      break;
    }
    amgd_alpha_update(alpha, Dc, w2, cnc);
    pr0_ctx r0c = {Af, AfT, W0, fac.W0t, Ar, Dfsqrti, Dcs};
    const pfs_first f1 = {rs1, w1, tmp, w2};
    pmat *nsk = p_expand_support(W_skel, R, Rt, &r0c, gamma2, &f1);
    pk_mark(g_pklvl, PK_EXPAND);
    pm_free(&W_skel);
    W_skel = nsk;
    pm_free(&Wtmp);
    pm_free(&R);
    prevWt = fac.Wt; prevQ = fac.Q; prevQoff = fac.qoff; prevQbuf = fac.Qbuf;
    fac.Wt = NULL; fac.Q = NULL; fac.qoff = NULL; fac.Qbuf = NULL;
    pfactor_free(&fac);
  }
  pm_free(&W_skel); pm_free(&Amt);
  amgd_free(Df); amgd_free(Dfinv); amgd_free(uc); amgd_free(tmp); amgd_free(v); amgd_free(b);
  amgd_free(Dc); amgd_free(Dcinv); amgd_free(lam); amgd_free(alpha); amgd_free(Dcs);
  amgd_free(w1); amgd_free(w2); amgd_free(onesc); amgd_free(r); amgd_free(rs1);
  return W;
}

/* ------------------------------------------------------------------------ */
/* hierarchy                                                                 */
/* ------------------------------------------------------------------------ */
typedef struct {
  pmat *A, *Af, *W, *AfP;
  uint8_t *vc;                 /* whole */
  double *D;                   /* whole (F points) */
  unsigned long *idc, *idf;    /* whole */
  double m, rho;
  apart *Pn, *Pf;              /* rows of A (owned by this level), F points */
} plevel;
struct amgd_phier {
  uint32_t nlevels, cap, n0;
  plevel *lv;
  unsigned long *id;
  int nullspace;
  double tolc, gamma;
};

static void add_time(double *acc, double *t0) {
  amgd_sync();
  double t = amgd_wtime();
  *acc += (t - *t0) * 1e3;
  *t0 = t;
}

__attribute__((visibility("hidden"))) int amgd_psetup_body(uint64_t nz, const uint32_t *dAi,
                                                           const uint32_t *dAj, const double *dAv,
                                                           amgd_phier **out, amgd_stats *st) {
  g_me = amgd_pcomm_rank();
  g_N = amgd_pcomm_size();
  pm_eager_new_setup();
  g_ub = 0;
  g_pst = st;
  g_plvl = 0;
  g_lmop_full = 0;
  g_lmop_prefix = 0;
  (void)amgd_pool_ipeak_take();
  amgd_sync();
  double t_start = amgd_wtime(), t0 = t_start;
  /* level 0: the global size, the even split, the entries to the owners of their rows,
     build_csr's empty-row / -column removal with the whole mask (amg_setup.c:3612) */
  uint32_t mx[2] = {0, 0};
  amgd_max_ij(nz, dAi, dAj, mx);
  const uint32_t n_in = (uint32_t)all_max(mx[0] > mx[1] ? mx[0] : mx[1]);
  apart *P0 = apart_even(n_in, g_N);
  uint32_t *I = NULL, *J = NULL;
  double *V = NULL;
  const uint64_t m = pm_route_coo(nz, dAi, dAj, dAv, P0, &I, &J, &V);
  const uint32_t r0 = P0->split[g_me], nl = P0->split[g_me + 1] - r0;
  amgd_vadd_u32(I, m, (uint32_t)(0u - r0));
  dcsr *T = amgd_coo2csr(m, I, J, V, nl, n_in, 1);
  amgd_free(I); amgd_free(J); amgd_free(V);
  uint8_t *zr = (uint8_t *)amgd_alloc((size_t)n_in + 8);
  amgd_nonempty_rows(T, zr + r0);
  pm_allgather_vec(zr, 1, P0);
  amgd_phier *h = (amgd_phier *)calloc(1, sizeof(amgd_phier));
  *out = h;
  h->cap = 64;
  h->lv = (plevel *)calloc(h->cap, sizeof(plevel));
  apart *Pn = apart_induced(P0, zr);
  pmat *Tp = pm_new(T, P0, P0);
  pmat *A = pm_sub_mat(Tp, zr, zr, Pn, Pn);
  pm_free(&Tp);
  amgd_free(zr);
  apart_free(&P0);
  add_time(&st->t_build_ms, &t0);
  const double tol = 0.5, ctol = 0.7, itol = 1e-4;
  const double gamma2 = 1. - sqrt(1. - tol), gamma = sqrt(gamma2);
  h->tolc = ctol;
  h->gamma = gamma;
  h->n0 = Pn->n;
  h->id = (unsigned long *)amgd_alloc((size_t)Pn->n * 8 + 8);
  amgd_ids_iota(h->id, Pn->n);
  st->rows0 = Pn->n;
  st->nnz0 = gnnz(A);
  uint32_t level = 0;
  for (;;) {
    if (level + 1 >= h->cap) {
      h->cap *= 2;
      h->lv = (plevel *)realloc(h->lv, h->cap * sizeof(plevel));
      memset(h->lv + h->cap / 2, 0, (h->cap / 2) * sizeof(plevel));
    }
    plevel *L = &h->lv[level];
    const uint32_t n = Pn->n;
    g_plvl = (int)level;
    L->A = A;
    L->Pn = Pn;
    if (verbose()) printf("Level %u, dim(A) = %u, nnz(A)/dim(A) = %f\n", level + 1, n,
                          n ? (double)gnnz(A) / n : 0.0), fflush(stdout);
    if (n <= 1) {
      const double a0 = n ? p_a00(A) : 0.0;
      h->nullspace = a0 < 1e-9 ? 1 : 0;
      break;
    }
    uint8_t *vc = (uint8_t *)amgd_alloc(n + 1), *vf = (uint8_t *)amgd_alloc(n + 1);
    ph(-1);
    p_coarsen(A, vc, ctol);
    amgd_u8_not(vc, vf, n);
    L->vc = vc;
    ph(PH_COARSEN);
    add_time(&st->t_coarsen_ms, &t0);
    pk_mark(level, PK_COARSEN);
    apart *Pf = apart_induced(Pn, vf), *Pc = apart_induced(Pn, vc);
    L->Pf = Pf;
    pmat *Af = pm_sub_mat(A, vf, vf, Pf, Pf);
    const uint32_t rnf = Pf->n;
    double *s = dalloc(rnf), *D = dalloc(rnf);
    pm_rowsum_sq_inv(Af, s);
    pm_diag(Af, D);
    amgd_vop(D, D, s, rnf, AMGD_V_MUL);
    amgd_free(s);
    if (rnf >= 2) {
      double *Dh = dalloc(rnf);
      amgd_d2d(Dh, D, (size_t)rnf * 8);
      amgd_vunary(Dh, rnf, AMGD_V_SQRT);
      pmat *DAD = pm_copy(Af);
      pm_diag_op2(DAD, Dh, Dh, AMGD_SCALE2);
      double lambda[KMAX + 2];
      uint32_t k = p_lanczos(DAD, lambda);
      double a = lambda[0], bb = lambda[k - 1];
      amgd_vscale(D, rnf, 2. / (a + bb));
      L->rho = (bb - a) / (bb + a);
      double c;
      chebsim(&L->m, &c, L->rho, gamma2);
      amgd_free(Dh);
      pm_free(&DAD);
    } else {
      L->rho = 0;
      L->m = 1;
    }
    L->D = D;
    L->Af = Af;
    ph(PH_SMOOTH);
    add_time(&st->t_smoother_ms, &t0);
    pk_mark(level, PK_SMOOTH);
    pmat *Afc = pm_sub_mat(A, vf, vc, Pf, Pc), *Ac = pm_sub_mat(A, vc, vc, Pc, Pc);
    const uint32_t rnc = Pc->n;
    L->idc = (unsigned long *)amgd_alloc((size_t)rnc * 8 + 8);
    L->idf = (unsigned long *)amgd_alloc((size_t)rnf * 8 + 8);
    amgd_compact_ids(level == 0 ? h->id : h->lv[level - 1].idc, vc, n, L->idc, L->idf);
    g_pklvl = level;
    /* Af' for the transposed products (where Af's rows are long enough to pay, the one-GPU
       rule on the global counts) and A(C,F) = Afc' for the interpolation and the RAP */
    pmat *AfT = Af->rp->n && gnnz(Af) >= 64ull * Af->rp->n ? pm_transpose(Af) : NULL;
    pmat *Acf = pm_transpose(Afc);
    pmat *W = p_interpolation(Af, AfT, Ac, Afc, Acf, gamma2, itol);
    L->W = W;
    add_time(&st->t_interp_ms, &t0);
    pk_mark(level, PK_INTERP);
    /* Galerkin coarse operator: A = W'*AfP + A(C,F)*W + A(C,C) (amg_setup.c:339-372) */
    amgd_spgemm_set_timer(0);
    pmat *Wt = pm_transpose(W);
    pmat *AfW = p_spgemm_via_t(Af, AfT, W, Wt, NULL);
    pmat *AfP = pm_mpm(1., AfW, 1., Afc);
    pm_free(&AfW);
    L->AfP = AfP;
    pmat *WtAfP = pm_spgemm(Wt, AfP, 0);
    pmat *AcfW = p_spgemm_via_t(Acf, Afc, W, Wt, NULL);      /* Acf' = Afc exactly */
    pm_free(&AfT);
    amgd_spgemm_set_timer(-1);
    pmat *Atmp = pm_mpm(1., WtAfP, 1., AcfW);
    A = pm_mpm(1., Atmp, 1, Ac);
    st->rap_out_nnz += gnnz(A);
    pm_free(&Wt); pm_free(&WtAfP); pm_free(&Acf); pm_free(&AcfW); pm_free(&Atmp);
    pm_free(&Afc); pm_free(&Ac);
    amgd_free(vf);
    ph(PH_RAP);
    add_time(&st->t_rap_ms, &t0);
    pk_mark(level, PK_RAP);
    Pn = Pc;
    level++;
  }
  h->nlevels = level + 1;
  amgd_sync();
  st->t_total_ms = (amgd_wtime() - t_start) * 1e3;
  pk_report(h->nlevels);
  if (g_me == 0) amgd_ph_report(h->nlevels);
  amgd_comm_site_report();
  st->ub_events = (uint32_t)g_ub;
  st->nlevels = h->nlevels;
  if (verbose() && g_lmop_full)
    printf("partitioned setup: %lu interp_lmop calls on gathered data\n", (unsigned long)g_lmop_full);
  return 0;
}

/* the hierarchy gathered (every rank gets all of it) into the ABI struct */
static struct csr_mat *pcsr_to_host(const pmat *A) {
  dcsr *F = pm_gather_full(A);
  struct csr_mat *M = (struct csr_mat *)malloc(sizeof *M);
  M->rn = F->rn;
  M->cn = F->cn;
  M->row_off = (amg_uint *)malloc(((size_t)F->rn + 1) * sizeof(amg_uint));
  M->col = (amg_uint *)malloc((F->nnz ? F->nnz : 1) * sizeof(amg_uint));
  M->a = (double *)malloc((F->nnz ? F->nnz : 1) * sizeof(double));
  amgd_to_host_cols(F, M->row_off, M->col, M->a);
  dcsr_free(&F);
  return M;
}
__attribute__((visibility("hidden"))) int amgd_phier_export(const amgd_phier *h, struct amg_setup_data *data) {
  uint32_t nl = h->nlevels, cap = nl + 1;
  data->tolc = h->tolc;
  data->gamma = h->gamma;
  data->n = (double *)malloc(cap * 8); data->nnz = (double *)malloc(cap * 8);
  data->nnzf = (double *)malloc(cap * 8); data->nnzfp = (double *)malloc(cap * 8);
  data->m = (double *)malloc(cap * 8); data->rho = (double *)malloc(cap * 8);
  data->A = (struct csr_mat **)malloc(cap * sizeof(void *));
  data->Af = (struct csr_mat **)malloc(cap * sizeof(void *));
  data->W = (struct csr_mat **)malloc(cap * sizeof(void *));
  data->AfP = (struct csr_mat **)malloc(cap * sizeof(void *));
  data->idc = (amg_uint **)malloc(cap * sizeof(void *));
  data->idf = (amg_uint **)malloc(cap * sizeof(void *));
  data->C = (double **)malloc(cap * sizeof(void *));
  data->F = (double **)malloc(cap * sizeof(void *));
  data->D = (double **)malloc(cap * sizeof(void *));
  data->id = (amg_uint *)malloc((size_t)h->n0 * sizeof(amg_uint) + 8);
  amgd_d2h(data->id, h->id, (size_t)h->n0 * 8);
  for (uint32_t l = 0; l < nl; l++) {
    const plevel *L = &h->lv[l];
    data->n[l] = L->Pn->n;
    data->A[l] = pcsr_to_host(L->A);
    data->nnz[l] = (double)data->A[l]->row_off[data->A[l]->rn];
    if (l + 1 == nl) break;
    uint32_t rn = L->Pn->n, rnf = L->Pf->n, rnc = rn - rnf;
    uint8_t *vc = (uint8_t *)malloc(rn + 1);
    amgd_d2h(vc, L->vc, rn);
    data->C[l] = (double *)malloc((size_t)rn * 8 + 8);
    data->F[l] = (double *)malloc((size_t)rn * 8 + 8);
    for (uint32_t i = 0; i < rn; i++) { data->C[l][i] = vc[i] ? 1. : 0.; data->F[l][i] = vc[i] ? 0. : 1.; }
    free(vc);
    data->D[l] = (double *)malloc((size_t)rnf * 8 + 8);
    amgd_d2h(data->D[l], L->D, (size_t)rnf * 8);
    data->m[l] = L->m;
    data->rho[l] = L->rho;
    data->Af[l] = pcsr_to_host(L->Af);
    data->W[l] = pcsr_to_host(L->W);
    data->AfP[l] = pcsr_to_host(L->AfP);
    data->nnzf[l] = (double)data->Af[l]->row_off[data->Af[l]->rn];
    data->nnzfp[l] = (double)data->AfP[l]->row_off[data->AfP[l]->rn];
    data->idc[l] = (amg_uint *)malloc((size_t)rnc * 8 + 8);
    data->idf[l] = (amg_uint *)malloc((size_t)rnf * 8 + 8);
    amgd_d2h(data->idc[l], L->idc, (size_t)rnc * 8);
    amgd_d2h(data->idf[l], L->idf, (size_t)rnf * 8);
  }
  data->nlevels = nl;
  data->nullspace = (amg_uint)h->nullspace;
  return 0;
}
__attribute__((visibility("hidden"))) void amgd_phier_free(amgd_phier **hp) {
  amgd_phier *h = *hp;
  if (!h) return;
  for (uint32_t l = 0; l < h->nlevels || (l < h->cap && h->lv[l].A); l++) {
    plevel *L = &h->lv[l];
    pm_free(&L->A); pm_free(&L->Af); pm_free(&L->W); pm_free(&L->AfP);
    if (L->vc) amgd_free(L->vc);
    if (L->D) amgd_free(L->D);
    if (L->idc) amgd_free(L->idc);
    if (L->idf) amgd_free(L->idf);
    apart_free(&L->Pn);
    apart_free(&L->Pf);
  }
  if (h->id) amgd_free(h->id);
  free(h->lv);
  free(h);
  *hp = NULL;
}
/* after an unwound (out-of-HBM) setup: the host side of a partial hierarchy -- pmat and
   dcsr headers, partitions, the level array.  Its device blocks were released by the
   unwind already (amgd_try), so nothing here touches the device pool. */
static void pm_free_host(pmat **A) {
  if (!A || !*A) return;
  free((*A)->m);
  free(*A);
  *A = NULL;
}
__attribute__((visibility("hidden"))) void amgd_phier_free_host(amgd_phier **hp) {
  amgd_phier *h = *hp;
  if (!h) return;
  for (uint32_t l = 0; h->lv && l < h->cap; l++) {
    plevel *L = &h->lv[l];
    if (!L->A && !L->Pn) continue;
    pm_free_host(&L->A); pm_free_host(&L->Af); pm_free_host(&L->W); pm_free_host(&L->AfP);
    apart_free(&L->Pn);
    apart_free(&L->Pf);
  }
  free(h->lv);
  free(h);
  *hp = NULL;
}
/* the rows this rank holds (its partition of level 0) and the levels */
__attribute__((visibility("hidden"))) void amgd_phier_info(const amgd_phier *h, uint32_t *nlevels,
                                                           uint32_t *r0, uint32_t *r1) {
  *nlevels = h->nlevels;
  *r0 = h->lv[0].Pn->split[g_me];
  *r1 = h->lv[0].Pn->split[g_me + 1];
}
