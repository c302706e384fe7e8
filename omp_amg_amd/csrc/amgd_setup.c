/*
 * amgd_setup.c -- host driver (C) of the MI355X-native AMG setup.
 *
 * Follows the reference setup loop (nicooff/omp_amg amg_setup.c:60-400) level
 * by level; every array operation is a HIP kernel behind the thin C ABI of
 * amgd.h, all data stays in HBM, and the host only steers: it reads back the
 * scalars that decide control flow (coarsening norm bound, Lanczos alpha/beta,
 * PCG rho, skeleton-expansion counts) and runs the small tridiagonal
 * eigen-solve of Lanczos (tdeig, amg_setup.c:2712) on the CPU.
 *
 * Parity contract (DESIGN.md "Parity"): integer structure -- C/F sets, ids,
 * every CSR pattern -- is identical to the reference; values agree to the last
 * bit except where a global dot product feeds them (PCG / Lanczos use a
 * fixed-order tree reduction on the GPU, the reference sums left to right).
 *
 * Compiled with -ffp-contract=off so host arithmetic (chebsim, tdeig,
 * threshold expressions) rounds exactly like the reference's ISO-C build.
 */
#define _POSIX_C_SOURCE 200809L
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "amgd.h"
#include "amg_setup.h"
#include "crs.h"
#include "omp_amg_amd.h"
#include "amgd_psetup.h"

#define API __attribute__((visibility("default")))

static double *dalloc(uint64_t n) { return (double *)amgd_alloc_f64(n * 8 + 8); }
static double *dones(uint64_t n) { double *p = dalloc(n); amgd_vfill(p, n, 1.0); return p; }
static double *dzeros(uint64_t n) { double *p = dalloc(n); amgd_vfill(p, n, 0.0); return p; }
#define SWAPD(a, b) do { double *t_ = (a); (a) = (b); (b) = t_; } while (0)

static amgd_stats g_st;
static uint64_t g_ub;                  /* reference-undefined events (non-termination) */
/* where they fired (the first AMGD_UB_LOG of a setup): site 1 find_support theta -> 0, 2 a
   one-row R, 3 a sweep that removed nothing, 4 the selection count past nnz(R) + nc, 5 the
   interpolation loop's skeleton stalled (amg_setup.c:1316-1330, :700-860) */
static void ub_note(int site, int level) {
  if (g_ub < AMGD_UB_LOG) { g_st.ub_site[g_ub] = (uint8_t)site; g_st.ub_level[g_ub] = (uint8_t)level; }
  g_ub++;
}
#define UB(site) ub_note((site), g_lvl)
static int g_verbose = -1;
static int verbose(void) {
  if (g_verbose < 0) { const char *e = getenv("AMGD_VERBOSE"); g_verbose = e && *e && *e != '0'; }
  return g_verbose;
}

/* debug dumps of intermediates (AMGD_DUMP=<dir>), compared against the oracle's */
static int g_lvl = 0, g_it = 0;
static void dump_dev(const char *name, const void *d, size_t bytes) {
  const char *dir = getenv("AMGD_DUMP");
  if (!dir || !*dir) return;
  char fn[512];
  snprintf(fn, sizeof fn, "%s/L%d_it%d_%s.bin", dir, g_lvl, g_it, name);
  void *h = malloc(bytes + 8);
  amgd_d2h(h, d, bytes);
  FILE *f = fopen(fn, "wb");
  if (f) { fwrite(h, 1, bytes, f); fclose(f); }
  free(h);
}
static void dump_csr(const char *name, const dcsr *A) {
  char n2[256];
  snprintf(n2, sizeof n2, "%s_ro", name); dump_dev(n2, A->ro, ((size_t)A->rn + 1) * 8);
  snprintf(n2, sizeof n2, "%s_col", name); dump_dev(n2, A->col, A->nnz * 4);
  snprintf(n2, sizeof n2, "%s_a", name); dump_dev(n2, A->a, A->nnz * 8);
}

/* phase profile (AMGD_PHASES=1): device-synchronised time per (level, phase),
   printed at the end of the setup; costs one stream sync per mark.  Shared with the
   partitioned driver (amgd_psetup.c) through amgd_ph_mark / amgd_ph_report (amgd.h). */
static const char *ph_name[PH_N] = {"coarsen", "smoother", "interp0", "qfactor", "W0", "S_pat",
                                    "lmop", "pcg", "W", "AfW", "R", "fs_setup", "fs_spmv",
                                    "fs_max", "fs_sel", "expand", "exp_R0", "final", "rap"};
#define PH_MAXL 64
static double g_ph[PH_MAXL][PH_N], g_ph_t;
static double g_phpk[PH_MAXL][PH_N];      /* GB: pool peak inside the phase */
static int g_phases = -1;
static int phases_on(void) {
  if (g_phases < 0) { const char *e = getenv("AMGD_PHASES"); g_phases = e && *e && *e != '0'; }
  return g_phases;
}
__attribute__((visibility("hidden"))) void amgd_ph_mark(int lvl, int id) {
  if (!phases_on()) return;
  amgd_sync();
  double t = amgd_wtime();
  const double pk = amgd_pool_ipeak_take() / 1e9;
  if (id >= 0 && lvl >= 0 && lvl < PH_MAXL) {
    g_ph[lvl][id] += (t - g_ph_t) * 1e3;
    if (pk > g_phpk[lvl][id]) g_phpk[lvl][id] = pk;
  }
  g_ph_t = t;
}
static void ph(int id) { amgd_ph_mark(g_lvl, id); }
__attribute__((visibility("hidden"))) void amgd_ph_report(uint32_t nl) {
  if (!phases_on()) return;
  double tot[PH_N] = {0};
  fprintf(stderr, "phase ms per level:\nlvl");
  for (int p = 0; p < PH_N; p++) fprintf(stderr, " %9s", ph_name[p]);
  fprintf(stderr, "\n");
  for (uint32_t l = 0; l < nl && l < PH_MAXL; l++) {
    fprintf(stderr, "%3u", l);
    for (int p = 0; p < PH_N; p++) { fprintf(stderr, " %9.1f", g_ph[l][p]); tot[p] += g_ph[l][p]; }
    fprintf(stderr, "\n");
  }
  fprintf(stderr, "sum");
  for (int p = 0; p < PH_N; p++) fprintf(stderr, " %9.1f", tot[p]);
  fprintf(stderr, "\nphase peak GB (pool in use, max inside the phase):\nlvl");
  for (int p = 0; p < PH_N; p++) fprintf(stderr, " %9s", ph_name[p]);
  fprintf(stderr, "\n");
  for (uint32_t l = 0; l < nl && l < PH_MAXL; l++) {
    fprintf(stderr, "%3u", l);
    for (int p = 0; p < PH_N; p++) fprintf(stderr, " %9.2f", g_phpk[l][p]);
    fprintf(stderr, "\n");
  }
  uint64_t nm, nr;
  double gb, ms;
  amgd_pool_stats(&nm, &gb, &ms, &nr);
  fprintf(stderr, "pool: %lu driver allocations, %.1f GB, %.1f ms in hipMalloc, %lu cache flushes\n",
          (unsigned long)nm, gb, ms, (unsigned long)nr);
  memset(g_ph, 0, sizeof g_ph);
  memset(g_phpk, 0, sizeof g_phpk);
}

/* X = A*B, given At = A' and Bt = B'.  When A has long columns (mean row of At
   >= 64 and at least twice B's mean row), X' = Bt*At has the longer B-operand
   rows and runs better on the k-sequential SpGEMM kernels; it is the same Gustavson sum (k ascending over the
   shared index, products commute, same exact-zero drop), transposed back stably.
   Bit-identical to amgd_spgemm(A, B) either way. */
static dcsr *spgemm_via_t(const dcsr *A, const dcsr *At, const dcsr *B, const dcsr *Bt) {
  const uint64_t avg_at = At && At->rn ? At->nnz / At->rn : 0, avg_b = B->rn ? B->nnz / B->rn : 0;
  if (!At || !Bt || avg_at < 64 || avg_at < 2 * avg_b) return amgd_spgemm(A, B);
  dcsr *Xt = amgd_spgemm(Bt, At);
  dcsr *X = amgd_transpose(Xt, NULL);
  dcsr_free(&Xt);
  return X;
}
/* the same choice, but the transposed product is returned as it comes (*tr = 1) for a
   caller that can go on in transposed form */
static dcsr *spgemm_via_t_raw(const dcsr *A, const dcsr *At, const dcsr *B, const dcsr *Bt, int *tr) {
  const uint64_t avg_at = At && At->rn ? At->nnz / At->rn : 0, avg_b = B->rn ? B->nnz / B->rn : 0;
  *tr = !(!At || !Bt || avg_at < 64 || avg_at < 2 * avg_b);
  return *tr ? amgd_spgemm(Bt, At) : amgd_spgemm(A, B);
}

/* ------------------------------------------------------------------------ */
/* coarsen (amg_setup.c:2737)                                                */
/* ------------------------------------------------------------------------ */
static dcsr *strength(const dcsr *A) {
  /* D = 1/sqrt(diag(A)); S = |D A D|; S = S - diag(S)  (amg_setup.c:2741-2758) */
  double *D = dalloc(A->cn);
  amgd_diag(A, D);
  amgd_vunary(D, A->rn, AMGD_V_SQRT);
  amgd_vunary(D, A->rn, AMGD_V_INV);
  dcsr *S = dcsr_copy(A);
  amgd_diag_op2(S, D, D, AMGD_SCALE2_ABS);          /* |D*A*D| in one pass */
  amgd_diag(S, D);
  amgd_diag_op(S, D, AMGD_DMINUS);
  amgd_free(D);
  return S;
}

/* The sweep loop keeps one buffer per stage (g, w1, w2a, w2, w, mask1, x1, Amax,
   m1, mask2, x2, m2) so that, after the first sweep, each stage is recomputed
   only on the rows within its dependency radius of the previous sweep's new C
   points (amgd_coarsen.hip); the other rows already hold the values a full
   sweep would produce.  Large dirty sets, long-row graphs and small levels run
   the full kernels into the same buffers.  AMGD_CS_INC=0 forces full sweeps. */
static void coarsen(const dcsr *A, uint8_t *vc, double ctol) {
  uint32_t n = A->cn;
  dcsr *S = strength(A);
  dcsr *St = amgd_transpose(S, NULL);
  uint8_t *vf = (uint8_t *)amgd_alloc(n + 1), *ma = (uint8_t *)amgd_alloc(n + 1);
  uint8_t *mb = (uint8_t *)amgd_alloc(n + 1);
  double *vfd = dones(n), *g = dalloc(n), *w1 = dalloc(n), *w2a = dalloc(n), *w2 = dalloc(n);
  double *w = dalloc(n), *x1 = dalloc(n), *x2 = dalloc(n), *m1 = dalloc(n), *m2 = dalloc(n);
  double *amax = dalloc(n);
  uint32_t *anyvc = (uint32_t *)amgd_alloc(4);
  uint32_t *front[2], *cnt[2], *stamp = (uint32_t *)amgd_alloc(4ull * n + 4);
  for (int q = 0; q < 2; q++) {
    front[q] = (uint32_t *)amgd_alloc(4ull * n + 4);
    cnt[q] = (uint32_t *)amgd_alloc(64);
  }
  const char *e1 = getenv("AMGD_CS_INC"), *e2 = getenv("AMGD_CS_MIN_ROWS");
  const uint64_t min_rows = e2 && *e2 ? strtoull(e2, NULL, 10) : 65536;
  const int inc = !(e1 && *e1 && atoi(e1) == 0) && n >= min_rows &&
                  S->nnz + St->nnz <= 64ull * n;
  const uint32_t limit = n / 4;
  /* very short rows: one thread per listed row (list mode) beats the block filter */
  const char *e3 = getenv("AMGD_CS_LIST_NNZ");
  const int list_mode = S->nnz <= (uint64_t)(e3 && *e3 ? atoi(e3) : 12) * n;
  amgd_memset(vc, 0, n);
  amgd_memset(vf, 1, n);
  amgd_memset(anyvc, 0, 4);
  amgd_memset(stamp, 0, 4ull * n);
  amgd_memset(cnt[0], 0, 64);
  int it = 0, cur = 0;
  for (;;) {
    it++;
    /* rows within r hops of the last sweep's new C points */
    amgd_csrows rows_, *rows = NULL;
    if (inc && it > 1 &&
        amgd_cs_grow(S, St, front[cur], cnt[cur], stamp, 8u * it, limit, rows_.cum)) {
      rows_.list = list_mode ? front[cur] : NULL;
      rows_.fs = stamp;
      rows_.fb = 8u * it;
      rows = &rows_;
      amgd_route_hit(AMGD_R_CS_INC);
    }
    amgd_cs_spmv(S, vfd, g, vf, rows, 1);          /* g   = vf.*(S*vf)  */
    amgd_cs_spmv(S, g, w1, vf, rows, 2);           /* w1  = vf.*(S*g)   */
    amgd_cs_spmv(S, w1, w2a, vf, rows, 3);         /* w2a = vf.*(S*w1)  */
    amgd_cs_spmv(S, w2a, w2, vf, rows, 4);         /* w2  = vf.*(S*w2a) */
    /* w = (1./w1).*w2; mask1 = w > ctol^2; x1 = mask1.*g */
    amgd_cs_w_mask1(n, w1, w2, w, ctol * ctol, g, ma, x1, rows, 4);
    uint64_t mi = 0;
    double wm = 0;
    double w1m = amgd_max_first2(w1, w, n, &mi, &wm);    /* max(w1) (first index), max(w) */
    double b = (w1m < wm) ? sqrt(w1m) : sqrt(wm);
    if (b <= ctol) {
      uint32_t any = 0;
      amgd_d2h(&any, anyvc, 4);
      if (!any) { uint8_t one = 1; amgd_h2d(vc + mi, &one, 1); }
      if (verbose()) printf("  coarsen: %d sweeps, norm bound = %f\n", it, b);
      break;
    }
    amgd_cs_amax(S, vf, 0.1, amax, rows, 1);        /* Amax: same (S, vf) for both calls */
    amgd_cs_gather(St, vf, x1, amax, m1, rows, 5);  /* m1 = mat_max(S,vf,mask.*g)  */
    amgd_cs_mask2(n, g, m1, ma, mb, x2, rows, 5);   /* mask2 = mask1 & (g-m1>=0)   */
    amgd_cs_gather(St, vf, x2, amax, m2, rows, 6);  /* m2 = mat_max(S,vf,mask.*id) */
    const int nx = cur ^ 1;
    amgd_memset(cnt[nx], 0, 64);
    amgd_cs_mask3(n, m2, mb, vc, vf, vfd, anyvc, front[nx], cnt[nx], stamp, 8u * it + 8, rows, 6);
    cur = nx;
    if (getenv("AMGD_CLOG") && (it % 10 == 1))
      fprintf(stderr, "coarsen n %u sweep %d active %lu rows %u\n", n, it,
              (unsigned long)amgd_u8_count(vf, n), rows ? rows->cum[6] : n);
  }
  dcsr_free(&S); dcsr_free(&St);
  amgd_free(vf); amgd_free(ma); amgd_free(mb); amgd_free(vfd); amgd_free(g); amgd_free(w1);
  amgd_free(w2a); amgd_free(w2); amgd_free(w); amgd_free(x1); amgd_free(x2); amgd_free(m1);
  amgd_free(m2); amgd_free(amax); amgd_free(anyvc); amgd_free(stamp);
  for (int q = 0; q < 2; q++) { amgd_free(front[q]); amgd_free(cnt[q]); }
}

/* ------------------------------------------------------------------------ */
/* Lanczos + tdeig (amg_setup.c:2435-2726); tdeig runs on the host           */
/* ------------------------------------------------------------------------ */
#include "amgd_hostmath.h"

#define KMAX 299
static uint32_t lanczos(const dcsr *A, double *out) {
  uint32_t rn = A->rn;
  /* start vector: libc rand()/RAND_MAX, like the reference (amg_setup.c:2445-2448),
     so the process-wide rand() stream advances identically */
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
    double fr = amgd_fro_minus_eye(A), fro = sqrt(fr), fro2 = fro * fro;
    fro = sqrt(fro2);
    if (fro < 1e-11) { l[0] = 1; l[1] = 1; y[0] = 0; y[1] = 0; k = 2; change = 0.0; }
    else change = 1.0;
  }
  if (rn == 1) {
    double a00;
    amgd_d2h(&a00, A->a, 8);
    l[0] = a00; l[1] = a00; y[0] = 0; y[1] = 0; k = 2; change = 0.0;
  }
  double *qk = dzeros(A->cn), *qkm1 = dalloc(rn), *Aqk = dalloc(rn);
  while (k < KMAX && (change > 1e-5 || y[0] > 1e-3 || y[k - 1] > 1e-3)) {
    k++;
    amgd_lanczos_step(r, 1. / beta, qk, qkm1, rn);           /* qkm1 = qk; qk = r/beta */
    amgd_spmv(A, qk, Aqk, 0, NULL, 1, NULL);
    double alpha = amgd_dot(qk, Aqk, rn);
    amgd_lanczos_resid(r, Aqk, qk, alpha, qkm1, beta, rn);    /* r = Aqk - a qk - b qkm1 */
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

static double g_pcg_rho, g_pcg_stop;     /* last pcg's final rho and stop level (trace) */
/* PCG (amg_setup.c:2242): z = M.*r, at most min(n,100) iterations; r is overwritten */
static uint32_t pcg(double *x, const dcsr *A, double *r, const double *M, double tol, const double *b) {
  uint32_t rn = A->rn;
  amgd_vfill(x, rn, 0.0);
  if (rn == 0) return 0;
  double *p = dzeros(A->cn), *z = dalloc(rn), *w = dalloc(rn);
  amgd_vmul_dot_prep(z, M, r, rn);
  double rho = amgd_dot(r, z, rn);
  double rho_0 = amgd_dot3(M, b, rn);
  double rho_stop = tol * tol * rho_0, rho_old = 1, alpha, beta;
  uint32_t n = rn <= 100 ? rn : 100, k = 0;
  while (rho > rho_stop && k < n) {
    k++;
    beta = rho / rho_old;
    amgd_pcg_p(p, z, beta, rn);                  /* p = p*beta + z */
    amgd_spmv(A, p, w, 0, NULL, 1, NULL);
    alpha = amgd_dot(p, w, rn);
    alpha = rho / alpha;
    amgd_pcg_xrz(x, r, z, p, w, M, alpha, rn);   /* x += p*a; r -= w*a; z = M.*r */
    rho_old = rho;
    rho = amgd_dot(r, z, rn);
  }
  g_pcg_rho = rho;
  g_pcg_stop = rho_stop;
  amgd_free(p); amgd_free(z); amgd_free(w);
  return k;
}

/* ------------------------------------------------------------------------ */
/* interpolation (amg_setup.c:598-1493)                                      */
/* ------------------------------------------------------------------------ */
typedef struct {
  dcsr *Wt;          /* W_skel^T: coarse x fine pattern */
  uint32_t *kpos;    /* per W_skel entry: its position in the support (row of Wt) */
  double *Q;         /* packed Q factors per coarse column */
  uint64_t *qoff;
  dcsr *S;           /* constraint operator of this skeleton (solve_constraint), kept for
                        the final solve: same skeleton, alpha and u -> same S */
  dcsr *W0, *W0t;    /* W0 of this skeleton (lambda = 0) and its transpose, likewise reused */
} skel_factor;

static dcsr *g_prevS;
static void factor_free(skel_factor *f) {
  dcsr_free(&f->Wt);
  amgd_free(f->kpos);
  amgd_free(f->Q);
  amgd_free(f->qoff);
  if (f->S) {                          /* kept: the next iteration's S grows from its pattern */
    dcsr_free(&g_prevS);
    g_prevS = f->S;
    f->S = NULL;
  }
  if (f->W0) dcsr_free(&f->W0);
  if (f->W0t) dcsr_free(&f->W0t);
}

/* The constraint operator's pattern S = pattern(Wn Wn') (Wn: W_skel without its zero
   entries, every value > 0, so no sum cancels -- amgd_spgemm_pattern) across one level's
   interpolation loop.  expand_support only adds skeleton entries (late iterations +0.004 %
   to +1 %).  With dW = Wn \ Wn_prev:
     pattern(Wn Wn') = pattern(Wn_prev Wn_prev') U pattern(Wn dW') U pattern(Wn dW')'
   (S(i,j) needs a k with Wn(i,k) and Wn(j,k): both old -> the old S; Wn(j,k) new -> Wn dW';
   Wn(i,k) new -> (Wn dW')'), so the previous S is merged (mpm on positive values: a sorted
   union) with the small product instead of the whole product being formed again.  Taken
   only when Wn_prev is a subset of Wn (ones(Wn) - ones(Wn_prev) has no negative entry) and
   Wn's values are all > 0, and only when the new entries are at most 1/16 of Wn.  The same
   pattern, sorted, as the product; interp_lmop then
   writes every value.  AMGD_SPAT_INC=0 / amgd_spat_set_inc(0): the whole product each time. */
static dcsr *g_prevS = NULL, *g_prevWn = NULL;   /* the last iteration's S and Wn (values 1) */
static int g_spat_inc = -1;
static uint64_t g_spat_stats[3];                  /* incremental, whole, same pattern */
static int spat_inc_on(void) {
  if (g_spat_inc < 0) { const char *e = getenv("AMGD_SPAT_INC"); g_spat_inc = e && *e ? atoi(e) : 1; }
  return g_spat_inc;
}
void amgd_spat_set_inc(int on) { g_spat_inc = on; }
void amgd_spat_stats(uint64_t *out) { for (int q = 0; q < 3; q++) out[q] = g_spat_stats[q]; }
/* after an unwound setup the kept blocks were released by the rollback: forget them */
void amgd_spat_forget(void) { g_prevS = NULL; g_prevWn = NULL; }
static void spat_drop(void) { dcsr_free(&g_prevS); dcsr_free(&g_prevWn); }
static dcsr *s_pattern(const dcsr *W_skel, const dcsr *Wt) {
  dcsr *Wn = amgd_drop_zeros(W_skel);
  dcsr *S = NULL;
  const int pos = Wn->nnz == 0 || amgd_count_gt(Wn->a, Wn->nnz, 0.0, NULL) == Wn->nnz;
  if (spat_inc_on() && pos && g_prevS && g_prevWn && g_prevWn->rn == Wn->rn && g_prevWn->cn == Wn->cn &&
      g_prevS->rn == Wn->rn && Wn->nnz >= g_prevWn->nnz && Wn->nnz - g_prevWn->nnz <= Wn->nnz / 16) {
    dcsr *W1 = dcsr_empty_like_pattern(Wn);
    amgd_vfill(W1->a, W1->nnz, 1.0);
    dcsr *dW = amgd_mpm(1.0, W1, -1.0, g_prevWn);      /* new entries +1, lost entries -1 */
    dcsr_free(&W1);
    /* only for small growth: past 1/16 of the skeleton the product with the new entries, its
       transpose and the merge cost more than the whole product (256^3, level 1: the early
       iterations grow the skeleton 2-4x) */
    if (dW->nnz <= Wn->nnz / 16 && dW->nnz == Wn->nnz - g_prevWn->nnz &&
        (dW->nnz == 0 || amgd_count_gt(dW->a, dW->nnz, 0.0, NULL) == dW->nnz)) {
      if (dW->nnz == 0) {                                /* the same skeleton: the same pattern */
        S = g_prevS;
        g_prevS = NULL;
        g_spat_stats[2]++;
        amgd_route_hit(AMGD_R_SPAT_INC);
      } else {
        dcsr *dWt = amgd_transpose(dW, NULL);
        dcsr *P = amgd_spgemm_pattern(Wn, dWt);
        dcsr_free(&dWt);
        amgd_vfill(P->a, P->nnz, 1.0);
        dcsr *Pt = amgd_transpose(P, NULL);
        dcsr *PP = amgd_mpm(1.0, P, 1.0, Pt);
        dcsr_free(&P); dcsr_free(&Pt);
        amgd_vfill(g_prevS->a, g_prevS->nnz, 1.0);
        S = amgd_mpm(1.0, g_prevS, 1.0, PP);
        dcsr_free(&PP);
        g_spat_stats[0]++;
        amgd_route_hit(AMGD_R_SPAT_INC);
      }
    }
    dcsr_free(&dW);
  }
  if (!S) {
    dcsr *Wnt = amgd_drop_zeros(Wt);
    S = amgd_spgemm_pattern(Wn, Wnt);
    dcsr_free(&Wnt);
    g_spat_stats[1]++;
  }
  dcsr_free(&g_prevS);                                   /* the caller's S becomes the next one's */
  dcsr_free(&g_prevWn);
  if (spat_inc_on() && pos) {
    amgd_vfill(Wn->a, Wn->nnz, 1.0);
    g_prevWn = Wn;
  } else {
    dcsr_free(&Wn);
  }
  return S;
}

/* solve_constraint (amg_setup.c:1499) */
static void solve_constraint(double *lam, const dcsr *W_skel, skel_factor *fac, const dcsr *W0,
                             const double *alpha, const double *u, const double *v, double tol) {
  uint32_t nf = W_skel->rn, nc = W_skel->cn;
  double *au2 = dalloc(nc);
  amgd_vop(au2, u, u, nc, AMGD_V_MUL);
  amgd_vop(au2, au2, alpha, nc, AMGD_V_MUL);
  if (!fac->S) {
    /* W_skel * W_skel' (mxm iftrsp=1) with its exact zeros dropped.  The zero-valued
       skeleton entries (min_skel's orphans at column 0) contribute +0 products only,
       so the product of the operands without them is the same matrix, values and
       pattern -- without the orphans' dense all-zero block of products. */
    /* lmop overwrites every value of S (interp_lmop zeroes St first, amg_setup.c:1609): the
       pattern is all that is needed, and the skeleton values are all 1: no sum cancels */
    fac->S = s_pattern(W_skel, fac->Wt);
    ph(PH_SPAT);
    amgd_lmop(fac->S, W_skel, fac->kpos, fac->Wt, fac->Q, fac->qoff, au2);
    if (phases_on())
      fprintf(stderr, "L%u lmop: S %.3f GB, W_skel %.3f GB, supports %.3f GB, Q %.0f, QQ %.3f GB\n", g_lvl,
              fac->S->nnz * 12.0 / 1e9, W_skel->nnz * 12.0 / 1e9, fac->Wt->nnz * 12.0 / 1e9, 0.0,
              amgd_lmop_qq_bytes() / 1e9);
    ph(PH_LMOP);
  }
  dcsr *S = fac->S;
  dump_csr("S", S);
  double *resid = dalloc(nf), *d = dalloc(nf);
  amgd_spmv(W0, u, resid, 1.0, v, -1.0, NULL);        /* resid = v - W0*u */
  amgd_diag(S, d);
  uint8_t *dl = (uint8_t *)amgd_alloc(nf + 1);
  amgd_u8_nonzero(d, dl, nf);
  uint64_t ncond = amgd_u8_count(dl, nf);
  double *q = dalloc(ncond), *xx = dalloc(ncond);
  if (ncond != nf) {                                   /* S = S(i,i); lam(~i) = 0 */
    amgd_vzero_where(lam, dl, nf);
    S = amgd_sub_mat(S, dl, dl);
    double *rc = dalloc(nf), *dc = dalloc(nf), *lc = dalloc(nf);
    amgd_vcompact(rc, resid, dl, nf);
    amgd_vcompact(dc, d, dl, nf);
    amgd_vcompact(lc, lam, dl, nf);
    amgd_spmv(S, lc, q, 1., rc, -1., NULL);
    amgd_vunary(dc, ncond, AMGD_V_INV);
    const uint32_t its = pcg(xx, S, q, dc, tol, rc);
    if (verbose())
      printf("   constraint: %lu of %u rows, pcg %u its, rho %.9e stop %.9e\n", (unsigned long)ncond, nf,
             its, g_pcg_rho, g_pcg_stop), fflush(stdout);
    amgd_vexpand_add(lam, xx, dl, nf);
    amgd_free(rc); amgd_free(dc); amgd_free(lc);
  } else {
    amgd_spmv(S, lam, q, 1., resid, -1., NULL);       /* q = resid - S*lam */
    amgd_vunary(d, nf, AMGD_V_INV);
    const uint32_t its = pcg(xx, S, q, d, tol, resid);
    if (verbose())
      printf("   constraint: %u of %u rows, pcg %u its, rho %.9e stop %.9e\n", nf, nf, its, g_pcg_rho,
             g_pcg_stop), fflush(stdout);
    amgd_vop(lam, lam, xx, nf, AMGD_V_ADD);
  }
  if (S != fac->S) dcsr_free(&S);
  amgd_free(au2); amgd_free(resid); amgd_free(d); amgd_free(dl); amgd_free(q); amgd_free(xx);
  ph(PH_PCG);
}

/* solve_weights (amg_setup.c:1437): W0 (lambda = 0), constraint lam, W */
static void solve_weights(dcsr **W, dcsr **Wt_out, const dcsr **W0, double *lam,
                          const dcsr *W_skel, skel_factor *fac, const dcsr *Amt,
                          const double *alpha, const double *u, const double *v, double tol) {
  uint32_t nf = W_skel->rn, nc = W_skel->cn;
  double *au = dalloc(nc), *zeros = dzeros(nf);
  amgd_vop(au, alpha, u, nc, AMGD_V_MUL);
  if (!fac->W0) {
    dcsr *W0t = dcsr_empty_like_pattern(fac->Wt);
    amgd_qapply(fac->Wt, fac->Q, fac->qoff, Amt, au, zeros, W0t->a);
    fac->W0 = amgd_transpose(W0t, NULL);
    fac->W0t = W0t;
    ph(PH_W0);
  }
  *W0 = fac->W0;
  solve_constraint(lam, W_skel, fac, *W0, alpha, u, v, tol);
  dcsr *Wt = dcsr_empty_like_pattern(fac->Wt);
  amgd_qapply(fac->Wt, fac->Q, fac->qoff, Amt, au, lam, Wt->a);
  *W = amgd_transpose(Wt, NULL);
  if (Wt_out) *Wt_out = Wt;
  else dcsr_free(&Wt);
  amgd_free(au); amgd_free(zeros);
  ph(PH_W);
}



/* AMGD_FS_AMX=0 / amgd_fs_set_amx(0) (tests, A/B): find_support selects by its own pass
   over the bad columns (k_fs_select) even after a full sweep's fused product */
static int g_fs_amx = -1;
void amgd_fs_set_amx(int on) { g_fs_amx = on; }
static int fs_amx_on(void) {
  if (g_fs_amx < 0) {
    const char *e = getenv("AMGD_FS_AMX");
    return !(e && *e == '0');
  }
  return g_fs_amx;
}
/* the first sweep's products when the caller already formed them from the same R
   (interpolation's w1 / w2 test, amg_setup.c:870-880: rs = R*1, w = R'rs, tmp = R w,
   w2 = R' tmp -- the same ordered sums), else NULL */
typedef struct { const double *rs, *w, *tmp, *w2; } fs_first;
/* find_support (amg_setup.c:1260).  Rt / perm: R's transpose and its CSC -> CSR map
   when the caller already made them (taken over and freed here), else NULL. */
static dcsr *find_support(const dcsr *R, dcsr *Rt, uint64_t *perm, double goal, const fs_first *f1) {
  uint32_t nf = R->rn, nc = R->cn;
  dcsr *Rl = dcsr_copy(R);
  if (!Rt) Rt = amgd_transpose(R, &perm);
  double *onec = dones(nc), *rs = dalloc(nf), *w = dalloc(nc), *w2 = dalloc(nc), *tmp = dalloc(nf);
  double *vv = dalloc(nc), *sumR = dalloc(nc);
  uint64_t cap = R->nnz + nc + 16, ns = 0;
  uint32_t *si = (uint32_t *)amgd_alloc(cap * 4), *sj = (uint32_t *)amgd_alloc(cap * 4);
  double theta = 0.5;
  int it = 0;
  /* rs = R*1 and sumR = sum(R,1) change only where a sweep removed an entry:
     computed in full once, then re-summed for those rows / columns (amgd_fs_select) */
  if (f1) amgd_d2d(rs, f1->rs, (size_t)nf * 8);
  else amgd_spmv(Rl, onec, rs, 0., NULL, 1., NULL);       /* rs = R*1 */
  amgd_colsum(Rt, sumR);
  /* Incremental sweeps: a sweep that removed few entries changes rs only on their
     rows D; w = R'rs then changes on the columns C1 of D, tmp = R w on the rows D2
     of C1, w2 = R' tmp on the columns C3 of D2 (zeroed entries stay in the
     pattern).  Those lists are recomputed with the same ordered row sums; every
     other entry keeps its value.  Large dirty sets fall back to full products. */
  const char *e_inc = getenv("AMGD_FS_INC");          /* 0 off, 2 at every size (tests) */
  const int fs_mode = e_inc && *e_inc ? atoi(e_inc) : 1;
  const int fs_inc = fs_mode == 2 || (fs_mode == 1 && nf >= 4096);
  const uint32_t cap_c = nc / 4 + 1, cap_r = nf / 4 + 1;
  uint32_t *st_r = NULL, *st_c = NULL, *L1 = NULL, *L2 = NULL, *L3 = NULL, tag = 0;
  if (fs_inc) {
    st_r = (uint32_t *)amgd_alloc((size_t)nf * 4 + 4);
    st_c = (uint32_t *)amgd_alloc((size_t)nc * 4 + 4);
    amgd_memset(st_r, 0, (size_t)nf * 4);
    amgd_memset(st_c, 0, (size_t)nc * 4);
    L1 = (uint32_t *)amgd_alloc((size_t)cap_c * 4 + 4);
    L2 = (uint32_t *)amgd_alloc((size_t)cap_r * 4 + 4);
    L3 = (uint32_t *)amgd_alloc((size_t)cap_c * 4 + 4);
  }
  uint64_t prev_off = 0;
  uint32_t prev_nsel = 0;
  const int fslog = getenv("AMGD_FSLOG") != NULL;
  amgd_rowmax_pin(Rl);                 /* the sweeps zero values, never move entries */
  amgd_rowmax_pin(Rt);
  /* full sweeps: the selection's per-column first maximum comes out of w = R' rs */
  uint64_t *amx = fs_amx_on() ? (uint64_t *)amgd_alloc((size_t)nc * 8 + 8) : NULL;
  int amx_ok = 0;
  ph(PH_FS);
  for (;;) {
    it++;
    int done = 0;
    uint32_t n1 = 0, n2 = 0, n3 = 0;
    double t0 = 0, t1 = 0;
    if (fslog) { amgd_sync(); t0 = amgd_wtime(); }
    if (fs_inc && it > 1 && prev_nsel <= cap_c) {
      n1 = amgd_fs_expand(Rl, si + prev_off, prev_nsel, st_c, ++tag, L1, cap_c);
      if (n1 <= cap_c) {
        n2 = amgd_fs_expand(Rt, L1, n1, st_r, ++tag, L2, cap_r);
        if (n2 <= cap_r) {
          n3 = amgd_fs_expand(Rl, L2, n2, st_c, ++tag, L3, cap_c);
          if (n3 <= cap_c) {
            if (fslog) { amgd_sync(); t1 = amgd_wtime(); }
            amgd_spmv_rows(Rt, L1, n1, rs, w);          /* w  on C1 */
            amgd_spmv_rows(Rl, L2, n2, w, tmp);         /* tmp on D2 */
            amgd_spmv_rows(Rt, L3, n3, tmp, w2);        /* w2 on C3 */
            done = 1;
            amgd_route_hit(AMGD_R_FS_INC);
          }
        }
      }
    }
    if (!done && it == 1 && f1) {                         /* the caller's products */
      amgd_d2d(w, f1->w, (size_t)nc * 8);
      amgd_d2d(tmp, f1->tmp, (size_t)nf * 8);
      amgd_d2d(w2, f1->w2, (size_t)nc * 8);
      done = 1;
    }
    amx_ok = 0;
    if (!done) {
      if (amx) amx_ok = amgd_spmv_amax(Rt, rs, w, amx);  /* w = R'*rs (row order) */
      else amgd_spmvt(Rt, rs, w);
      amgd_spmv(Rl, w, tmp, 0., NULL, 1., NULL);
      amgd_spmvt(Rt, tmp, w2);                            /* w2 = R'*(R*w) */
    }
    ph(PH_FS_MV);
    amgd_vdiv_guard(vv, w2, w, nc);
    double mv = amgd_max_first(vv, nc, NULL), mw = mv;   /* max(v) twice, amg_setup.c:1316-1317 */
    ph(PH_FS_MAX);
    if (mv < goal || mw < goal) break;
    while (mw <= (1 + theta) * goal && theta > 0) theta = theta / 2.;
    if (theta == 0) { UB(1); break; }                   /* reference spins forever */
    if (nf <= 1) { UB(2); break; }                      /* maski = 1: never terminates */
    uint32_t nrem = 0;
    if (amx_ok) amgd_route_hit(AMGD_R_FS_AMX);
    uint32_t nsel = amx_ok ? amgd_fs_select_amx(Rl, Rt, perm, rs, w, sumR, (1 + theta) * goal, amx, si + ns,
                                                sj + ns, &nrem)
                           : amgd_fs_select(Rl, Rt, perm, rs, w, sumR, (1 + theta) * goal, si + ns, sj + ns, &nrem);
    prev_off = ns;
    prev_nsel = nsel;
    ns += nsel;
    if (fslog) {
      amgd_sync();
      fprintf(stderr, "fs L%d nf %u nc %u nnz %lu it %d sel %u rem %u theta %g | %s n %u/%u/%u expand %.3f ms, sweep+max+sel %.3f ms\n",
              g_lvl, nf, nc, (unsigned long)R->nnz, it, nsel, nrem, theta, done ? "inc" : "full",
              n1, n2, n3, done ? (t1 - t0) * 1e3 : 0., (amgd_wtime() - (done ? t1 : t0)) * 1e3);
    }
    ph(PH_FS_SEL);
    if (nrem == 0) { UB(3); break; }                    /* no progress: reference loops */
    if (ns + nc > cap) { UB(4); break; }
  }
  double *ones = dones(ns);
  dcsr *Sk = amgd_coo2csr(ns, si, sj, ones, nf, nc, 1);
  if (verbose()) printf("    find_support: %d sweeps, %lu entries (R %u x %u, nnz %lu)\n", it,
                       (unsigned long)ns, nf, nc, (unsigned long)R->nnz);
  amgd_free(ones);
  if (fs_inc) {
    amgd_free(st_r); amgd_free(st_c); amgd_free(L1); amgd_free(L2); amgd_free(L3);
  }
  amgd_rowmax_unpin(Rl);
  amgd_rowmax_unpin(Rt);
  if (amx) amgd_free(amx);
  dcsr_free(&Rl); dcsr_free(&Rt); amgd_free(perm);
  amgd_free(onec); amgd_free(rs); amgd_free(w); amgd_free(w2); amgd_free(tmp); amgd_free(vv);
  amgd_free(sumR); amgd_free(si); amgd_free(sj);
  return Sk;
}

/* R0 = |Dfsqrti*(Af*W0 + Ar)|*Dcs (amg_setup.c:870-895), needed only on the bad rows of
   expand_support: the product is formed for those rows alone (rows are independent, so
   they carry exactly the reference's values; the others are never read) */
typedef struct {
  const dcsr *Af, *AfT, *W0, *W0t, *Ar;
  const double *Dfsqrti, *Dcs;
} r0_ctx;
static dcsr *scale_abs_scale(const dcsr *X, const double *Dl, const double *Dr);
static dcsr *r0_rows(const r0_ctx *c, const uint8_t *bad) {
  dcsr *Afb = amgd_rows_masked(c->Af, bad);
  /* (Af restricted to the bad rows)' only where spgemm_via_t will use it (its mean row is
     nnz(Afb) / cols(Af)); from Af' by a column mask when the level keeps Af' (same
     entries in the same order as the transpose), else by a transpose */
  const uint64_t avg_at = c->Af->cn ? Afb->nnz / c->Af->cn : 0, avg_b = c->W0->rn ? c->W0->nnz / c->W0->rn : 0;
  dcsr *AfbT = NULL;
  if (avg_at >= 64 && avg_at >= 2 * avg_b)
    AfbT = c->AfT ? amgd_cols_masked(c->AfT, bad) : amgd_transpose(Afb, NULL);
  dcsr *AfW0 = spgemm_via_t(Afb, AfbT, c->W0, c->W0t);
  dcsr_free(&Afb);
  if (AfbT) dcsr_free(&AfbT);
  dcsr *Arb = amgd_rows_masked(c->Ar, bad);
  dcsr *Arhat0 = amgd_mpm(1., AfW0, 1., Arb);
  dcsr_free(&AfW0); dcsr_free(&Arb);
  dcsr *R0 = scale_abs_scale(Arhat0, c->Dfsqrti, c->Dcs);
  dcsr_free(&Arhat0);
  return R0;
}

/* expand_support (amg_setup.c:907) */
static dcsr *expand_support(const dcsr *W_skel, const dcsr *R, dcsr *Rt, uint64_t *perm,
                            const r0_ctx *r0c, double gamma, const fs_first *f1) {
  dcsr *M = find_support(R, Rt, perm, gamma, f1);
  ph(PH_FS);
  if (phases_on() && verbose())
    printf("    find_support: R %u x %u nnz %lu\n", R->rn, R->cn, (unsigned long)R->nnz);
  dcsr *ns = amgd_mpm(1., M, 1., W_skel);
  dcsr_free(&M);
  uint32_t nbad = 0;
  uint8_t *bad = amgd_bad_rows(ns, &nbad);
  if (nbad == 0) {
    amgd_skel_binarize(ns, 0);
    amgd_free(bad);
    ph(PH_EXP);
    return ns;
  }
  ph(PH_EXP);
  dcsr *R0 = r0_rows(r0c, bad);
  ph(PH_EXP_R0);
  if (verbose()) printf("    expand_support: %u bad rows of %u\n", nbad, W_skel->rn);
  dcsr *R0W = amgd_mxmpoint(R0, W_skel);
  dcsr *Xf = amgd_mpm(1., R0, -1., R0W);
  dcsr_free(&R0W); dcsr_free(&R0);
  uint32_t *pi = NULL, *pj = NULL;
  uint64_t np = amgd_expand_pick(Xf, bad, &pi, &pj);
  double *ones = dones(np);
  dcsr *N = amgd_coo2csr(np, pi, pj, ones, W_skel->rn, W_skel->cn, 1);
  dcsr *out = amgd_mpm(1., ns, 1., N);
  amgd_skel_binarize(out, 1);
  dcsr_free(&N); dcsr_free(&ns); dcsr_free(&Xf);
  amgd_free(ones); amgd_free(pi); amgd_free(pj); amgd_free(bad);
  ph(PH_EXP);
  return out;
}

static dcsr *scale_abs_scale(const dcsr *X, const double *Dl, const double *Dr) {
  dcsr *R = dcsr_copy(X);
  amgd_diag_op2(R, Dl, Dr, AMGD_SCALE_ABS);          /* |Dl*X|*Dr in one pass */
  return R;
}

/* diagnostics only (tools/oracle_trace.py on 27-point grids, where the interpolation
   loop does not settle): AMGD_TRACE_MAX_IT / AMGD_TRACE_MAX_S end the process cleanly
   after that many interpolation iterations on one level / seconds since the first */
static void trace_limit(int it) {
  static double t_first = -1;
  static long max_it = -2;
  static double max_s = -2;
  if (max_it == -2) {
    const char *a = getenv("AMGD_TRACE_MAX_IT"), *b = getenv("AMGD_TRACE_MAX_S");
    max_it = a && *a ? atol(a) : -1;
    max_s = b && *b ? atof(b) : -1;
  }
  if (max_it < 0 && max_s < 0) return;
  if (t_first < 0) t_first = amgd_wtime();
  if ((max_it >= 0 && it >= max_it) || (max_s >= 0 && amgd_wtime() - t_first >= max_s)) {
    printf("TRACE LIMIT: stopped at interpolation iteration %d after %.1f s\n", it,
           amgd_wtime() - t_first);
    fflush(stdout);
    amgd_sync();
    exit(3);
  }
}

static dcsr *interpolation(const dcsr *Af, const dcsr *AfT, const dcsr *Ac, const dcsr *Ar,
                           const dcsr *ArT, double gamma2, double tol) {
  uint32_t rnf = Af->rn, rnc = Ac->rn, cnc = Ac->cn, cnr = Ar->cn;
  double *Df = dalloc(rnf), *Dfinv = dalloc(rnf);
  amgd_diag(Af, Df);
  amgd_diag(Af, Dfinv);
  amgd_vunary(Dfinv, rnf, AMGD_V_INV);
  double *uc = dones(cnr), *tmp = dalloc(rnf), *v = dalloc(rnf), *b = dones(rnf);
  amgd_spmv(Ar, uc, tmp, 0, NULL, -1, NULL);          /* tmp = -Ar*uc */
  pcg(v, Af, tmp, Df, 1e-16, b);                     /* v = pcg(Af, -Ar*uc, diag(Af)) */
  g_it = 0;
  dump_dev("v", v, (size_t)rnf * 8);
  double *Dc = dalloc(cnc), *Dcinv = dalloc(cnc);
  amgd_diag(Ac, Dc);
  amgd_diag(Ac, Dcinv);
  amgd_vunary(Dcinv, rnc, AMGD_V_INV);
  dcsr *ArD = dcsr_copy(Ar);
  amgd_vals_sqr(ArD);
  amgd_diag_op2(ArD, Dfinv, Dcinv, AMGD_SCALE2);
  dcsr *W_skel = amgd_min_skel(ArD);                 /* one strongest C per F row */
  dcsr_free(&ArD);
  double *lam = dzeros(rnf), *alpha = dalloc(cnc);
  amgd_d2d(alpha, Dc, (size_t)cnc * 8);
  double *Dfsqrti = Dfinv;
  amgd_vunary(Dfsqrti, rnf, AMGD_V_SQRT);
  dcsr *Amt = amgd_transpose(Ar, NULL);              /* -Ar' */
  amgd_vals_scale(Amt, -1.0);
  double *Dcs = dalloc(cnc), *w1 = dalloc(cnc), *w2 = dalloc(cnc), *onesc = dones(cnc), *r = dalloc(cnc);
  double *rs1 = dalloc(rnf);
  dcsr *W = NULL;
  uint64_t prev_nnz = (uint64_t)-1;
  int it = 0;
  /* the previous iteration's supports and factors: supports the expansion left
     unchanged take their factor by copy (amgd_qfactor_reuse) */
  dcsr *prevWt = NULL;
  double *prevQ = NULL;
  uint64_t *prevQoff = NULL;
  ph(PH_IPRE);
  for (;;) {
    it++;
    skel_factor fac;
    memset(&fac, 0, sizeof fac);
    uint64_t *wperm = NULL;
    fac.Wt = amgd_transpose(W_skel, &wperm);
    fac.kpos = amgd_lmop_kpos(fac.Wt, wperm);
    amgd_free(wperm);
    fac.Q = amgd_qfactor_reuse(fac.Wt, Af, &fac.qoff, NULL, prevWt, prevQ, prevQoff);
    if (prevWt) { dcsr_free(&prevWt); amgd_free(prevQ); amgd_free(prevQoff); prevQ = NULL; prevQoff = NULL; }
    ph(PH_QF);
    dcsr *Wtmp;
    const dcsr *W0;
    g_it = it;
    dump_csr("Wskel", W_skel);
    dump_dev("alpha", alpha, (size_t)cnc * 8);
    dump_dev("lam_in", lam, (size_t)rnf * 8);
    dcsr *Wtmp_t = NULL;
    solve_weights(&Wtmp, &Wtmp_t, &W0, lam, W_skel, &fac, Amt, alpha, uc, v, tol);
    dump_csr("W0", W0);
    dump_csr("Wtmp", Wtmp);
    dump_dev("lam_out", lam, (size_t)rnf * 8);
    /* Arhat = Af*W + Ar, R = |Dfsqrti*Arhat|*Dcs and R' (with its CSC -> CSR map, for
       find_support).  Where Af*W runs as (W'*Af')' the product comes transposed: every
       step from Arhat to R is entry-wise (mpm, mxmpoint, the scaling) and the column sums
       of W.*(Arhat+Ar) are the row sums of its transpose, so the chain runs on the
       transposes as they come -- the same entries, values and orders -- and only R is
       transposed back, instead of AfW', W.*Arr and R each being transposed once. */
    int trp = 0;
    /* the final weights share this product's operand patterns (same skeleton): its
       symbolic phase is kept for the Galerkin Af*W (amgd_spgemm_sym_next) */
    if (amgd_nshards() == 1) amgd_spgemm_sym_next(1);
    dcsr *AfWx = spgemm_via_t_raw(Af, AfT, Wtmp, Wtmp_t, &trp);
    dcsr *R, *Rt;
    uint64_t *Rperm = NULL;
    if (!trp) {
      dcsr *Arhat = amgd_mpm(1., AfWx, 1., Ar);
      dcsr_free(&AfWx); dcsr_free(&Wtmp_t);
      ph(PH_AFW);
      dcsr *Arr = amgd_mpm(1.0, Arhat, 1.0, Ar);
      dcsr *ArW = amgd_mxmpoint(Wtmp, Arr);
      dcsr_free(&Arr);
      dcsr *ArWt = amgd_transpose(ArW, NULL);
      amgd_colsum(ArWt, Dcs);                        /* sum(W.*(Arhat+Ar), 1) */
      dcsr_free(&ArW); dcsr_free(&ArWt);
      amgd_vop(Dcs, Dcs, Dc, cnc, AMGD_V_ADD);
      amgd_vunary(Dcs, cnc, AMGD_V_INV);
      amgd_vunary(Dcs, cnc, AMGD_V_SQRT);
      R = scale_abs_scale(Arhat, Dfsqrti, Dcs);      /* |Dfsqrti*Arhat|*Dcsqrti */
      dcsr_free(&Arhat);
      /* R' with its CSC -> CSR map: find_support (expand_support) takes both over, so R
         is transposed once per iteration */
      Rt = amgd_transpose(R, &Rperm);
    } else {
      dcsr *ArhatT = amgd_mpm(1., AfWx, 1., ArT);   /* (Af*W + Ar)' */
      dcsr_free(&AfWx);
      ph(PH_AFW);
      dcsr *ArrT = amgd_mpm(1.0, ArhatT, 1.0, ArT);
      dcsr *ArWT = amgd_mxmpoint(Wtmp_t, ArrT);      /* (W.*Arr)' */
      dcsr_free(&ArrT); dcsr_free(&Wtmp_t);
      amgd_colsum(ArWT, Dcs);                        /* sum(W.*(Arhat+Ar), 1) */
      dcsr_free(&ArWT);
      amgd_vop(Dcs, Dcs, Dc, cnc, AMGD_V_ADD);
      amgd_vunary(Dcs, cnc, AMGD_V_INV);
      amgd_vunary(Dcs, cnc, AMGD_V_SQRT);
      Rt = ArhatT;                                   /* R' = |Dfsqrti*Arhat|*Dcsqrti, transposed */
      amgd_diag_op2(Rt, Dfsqrti, Dcs, AMGD_SCALE_ABS_T);
      uint64_t *p = NULL;
      R = amgd_transpose(Rt, &p);                    /* p: R position -> R' position */
      Rperm = amgd_perm_inverse(p, R->nnz);          /* R' position -> R position */
      amgd_free(p);
    }
    amgd_spmv(R, onesc, rs1, 0., NULL, 1., NULL);
    amgd_spmvt(Rt, rs1, w1);                         /* w1 = ((R*1)'*R)' */
    amgd_spmv(R, w1, tmp, 0., NULL, 1., NULL);
    amgd_spmvt(Rt, tmp, w2);                         /* w2 = ((R*w1)'*R)' */
    amgd_vdiv_guard(r, w2, w1, cnc);
    double maxr = 0;
    uint64_t n = amgd_count_gt(r, cnc, gamma2, &maxr);
    double w1m = amgd_max_first(w1, cnc, NULL);
    if (verbose())
      printf("   %lu nzs, %lu cols > %g, worst = %g\n", (unsigned long)W_skel->nnz,
             (unsigned long)n, sqrt(gamma2), sqrt(maxr)), fflush(stdout);
    trace_limit(it);
    int stalled = prev_nnz == W_skel->nnz;   /* reference would loop forever */
    if (stalled) UB(5);
    prev_nnz = W_skel->nnz;
    ph(PH_R);
    if (n == 0 || w1m <= gamma2 || stalled) {
      dcsr_free(&Rt);
      amgd_free(Rperm);
      /* same skeleton, alpha and u: the factor's S and W0 are reused */
      solve_weights(&W, NULL, &W0, lam, W_skel, &fac, Amt, alpha, uc, v, 1e-16);
      double *wuc = dalloc(rnf);
      amgd_spmv(W, uc, wuc, 0., NULL, 1., NULL);
      amgd_scale_diag_match(W, v, wuc);
      amgd_free(wuc);
      ph(PH_FINAL);
      dcsr_free(&Wtmp);
      dcsr_free(&R);
      factor_free(&fac);
      break;
    }
    amgd_alpha_update(alpha, Dc, w2, cnc);
    r0_ctx r0c = {Af, AfT, W0, fac.W0t, Ar, Dfsqrti, Dcs};
    const fs_first f1 = {rs1, w1, tmp, w2};          /* find_support's first sweep */
    dcsr *nsk = expand_support(W_skel, R, Rt, Rperm, &r0c, gamma2, &f1);
    dcsr_free(&W_skel);
    W_skel = nsk;
    dcsr_free(&Wtmp);
    dcsr_free(&R);
    prevWt = fac.Wt; prevQ = fac.Q; prevQoff = fac.qoff;   /* kept for the next factorization */
    fac.Wt = NULL; fac.Q = NULL; fac.qoff = NULL;
    factor_free(&fac);
  }
  dcsr_free(&W_skel); dcsr_free(&Amt);
  spat_drop();
  amgd_free(Df); amgd_free(Dfinv); amgd_free(uc); amgd_free(tmp); amgd_free(v); amgd_free(b);
  amgd_free(Dc); amgd_free(Dcinv); amgd_free(lam); amgd_free(alpha); amgd_free(Dcs);
  amgd_free(w1); amgd_free(w2); amgd_free(onesc); amgd_free(r); amgd_free(rs1);
  return W;
}

/* ------------------------------------------------------------------------ */
/* hierarchy                                                                 */
/* ------------------------------------------------------------------------ */
typedef struct {
  dcsr *A, *Af, *W, *AfP;
  uint8_t *vc;
  double *D;
  unsigned long *idc, *idf;
  double m, rho;
} level_t;

struct amgd_hier {
  amgd_phier *ph;         /* partitioned mode: the row blocks of this rank (amgd_psetup.c) */
  uint32_t nlevels, cap, n0;
  level_t *lv;
  unsigned long *id;      /* device, level-0 ids 1..n */
  int nullspace;
  double tolc, gamma;
};

static void add_time(double *acc, double *t0) {
  amgd_sync();
  double t = amgd_wtime();
  *acc += (t - *t0) * 1e3;
  *t0 = t;
}

API int amgd_init(int device) { return amgd_rt_init(device); }
API void amgd_shutdown(void) { amgd_rt_shutdown(); }
API void amgd_set_exact_dots(int on) { amgd_set_exact(on); }
API const char *amgd_error(void) { return amgd_last_error(); }
API void amgd_get_stats(amgd_stats *st) { *st = g_st; }
API void *amgd_dev_alloc(size_t bytes) { return amgd_alloc(bytes); }
API void amgd_dev_free(void *p) { amgd_free(p); }
API void amgd_dev_sync(void) { amgd_sync(); }
API void amgd_dev_upload(void *d, const void *h, size_t n) { amgd_h2d(d, h, n); }
API void amgd_dev_download(void *h, const void *d, size_t n) { amgd_d2h(h, d, n); }

extern uint64_t amgd_spmv_bytes(void);
extern uint64_t amgd_spmv_bytes_strict(void);
extern uint64_t amgd_spmv_launches(void);
extern uint64_t amgd_spgemm_launches(void);
extern void amgd_spmv_bytes_reset(void);
extern void amgd_spmv_rw_counts(uint64_t *bytes, uint64_t *launches);
static void rw_stats(void) {
  amgd_spmv_rw_counts(g_st.spmv_rw_bytes_strict, g_st.spmv_rw_launches);
  for (int i = 0; i < 3; i++) g_st.spmv_rw_ms[i] = amgd_timer_ms(2 + i);
}
extern void amgd_spgemm_set_timer(int slot);
extern void amgd_spgemm_bytes_reset(void);
extern uint64_t amgd_spgemm_bytes(void);

typedef struct {
  uint64_t nz;
  const uint32_t *dAi, *dAj;
  const double *dAv;
  amgd_hier *h;          /* the hierarchy under construction (host part freed on failure) */
} setup_args;
static int setup_body(void *arg);
/* partitioned mode: dAi / dAj / dAv are this rank's entries */
static int psetup_try(void *arg) {
  setup_args *sa = (setup_args *)arg;
  memset(&g_st, 0, sizeof g_st);
  amgd_reset_call_state();
  amgd_pool_peak_reset();
  amgd_timer_reset();
  amgd_spmv_bytes_reset();
  amgd_spgemm_bytes_reset();
  amgd_hier *h = (amgd_hier *)calloc(1, sizeof(amgd_hier));
  sa->h = h;
  const int rc = amgd_psetup_body(sa->nz, sa->dAi, sa->dAj, sa->dAv, &h->ph, &g_st);
  h->nlevels = g_st.nlevels;
  g_st.rap_kernel_ms = amgd_timer_ms(0);
  g_st.spmv_kernel_ms = amgd_timer_ms(1);
  g_st.spmv_bytes = amgd_spmv_bytes();
  g_st.spmv_bytes_strict = amgd_spmv_bytes_strict();
  g_st.spmv_launches = amgd_spmv_launches();
  g_st.rap_launches = amgd_spgemm_launches();
  g_st.rap_bytes = amgd_spgemm_bytes();
  rw_stats();
  amgd_spmv_bytes_reset();
  amgd_spgemm_bytes_reset();
  g_st.peak_bytes = amgd_pool_peak_bytes();
  return rc;
}

/* Out of HBM anywhere in the setup: amgd_try unwinds it, releases every device block
   the setup had allocated, and this returns -2 with the text in amgd_error() (the
   reference's allocator exits the process instead, fail.c); *out is left NULL. */
API int amgd_setup_device(uint64_t nz, const uint32_t *dAi, const uint32_t *dAj, const double *dAv,
                          amgd_hier **out, int flags) {
  (void)flags;
  *out = NULL;
  if (amgd_rt_init(0) != 0) {
    fprintf(stderr, "omp_amg_amd: %s\n", amgd_last_error());
    return -1;
  }
  setup_args a = {nz, dAi, dAj, dAv, NULL};
  int rc = amgd_try(amgd_comm_partitioned() ? psetup_try : setup_body, &a);
  if (rc != 0) {
    /* device blocks: released by the unwind; the host structs of a partial hierarchy here */
    if (a.h) {
      if (a.h->ph) amgd_phier_free_host(&a.h->ph);
      free(a.h->lv);
      free(a.h);
    }
    return rc;
  }
  *out = a.h;
  return 0;
}

static int setup_body(void *arg) {
  setup_args *sa = (setup_args *)arg;
  const uint64_t nz = sa->nz;
  const uint32_t *dAi = sa->dAi, *dAj = sa->dAj;
  const double *dAv = sa->dAv;
  memset(&g_st, 0, sizeof g_st);
  g_ub = 0;
  amgd_reset_call_state();
  amgd_pool_peak_reset();               /* amgd_stats.peak_bytes: this setup's peak */
  amgd_timer_reset();
  amgd_spmv_bytes_reset();
  amgd_sync();
  double t_start = amgd_wtime(), t0 = t_start;
  dcsr *A = amgd_build_csr(nz, dAi, dAj, dAv);
  add_time(&g_st.t_build_ms, &t0);

  const double tol = 0.5, ctol = 0.7, itol = 1e-4;
  const double gamma2 = 1. - sqrt(1. - tol), gamma = sqrt(gamma2);
  amgd_hier *h = (amgd_hier *)calloc(1, sizeof(amgd_hier));
  sa->h = h;
  h->cap = 64;
  h->lv = (level_t *)calloc(h->cap, sizeof(level_t));
  h->tolc = ctol;
  h->gamma = gamma;
  h->n0 = A->rn;
  h->id = (unsigned long *)amgd_alloc((size_t)A->rn * 8 + 8);
  amgd_ids_iota(h->id, A->rn);
  g_st.rows0 = A->rn;
  g_st.nnz0 = A->nnz;
  uint32_t level = 0;
  for (;;) {
    if (level + 1 >= h->cap) {
      h->cap *= 2;
      h->lv = (level_t *)realloc(h->lv, h->cap * sizeof(level_t));
      memset(h->lv + h->cap / 2, 0, (h->cap / 2) * sizeof(level_t));
    }
    level_t *L = &h->lv[level];
    uint32_t rn = A->rn, cn = A->cn;
    g_lvl = (int)level;
    L->A = A;
    ph(-1);
    if (verbose()) printf("Level %u, dim(A) = %u, nnz(A)/dim(A) = %f\n", level + 1, cn,
                          cn ? (double)A->nnz / cn : 0.0), fflush(stdout);
    if (cn <= 1) {
      double a0 = 0;
      if (A->nnz) amgd_d2h(&a0, A->a, 8);
      h->nullspace = a0 < 1e-9 ? 1 : 0;
      break;
    }
    /* --- coarsen --- */
    uint8_t *vc = (uint8_t *)amgd_alloc(rn + 1), *vf = (uint8_t *)amgd_alloc(rn + 1);
    coarsen(A, vc, ctol);
    amgd_u8_not(vc, vf, rn);
    L->vc = vc;
    ph(PH_COARSEN);
    add_time(&g_st.t_coarsen_ms, &t0);
    /* --- smoother --- */
    dcsr *Af = amgd_sub_mat(A, vf, vf);
    uint32_t rnf = Af->rn;
    double *s = dalloc(rnf), *D = dalloc(rnf);
    amgd_rowsum_sq_inv(Af, s);                      /* s = 1./sum(Af.*Af) */
    amgd_diag(Af, D);
    amgd_vop(D, D, s, rnf, AMGD_V_MUL);
    amgd_free(s);
    if (rnf >= 2) {
      double *Dh = dalloc(rnf);
      amgd_d2d(Dh, D, (size_t)rnf * 8);
      amgd_vunary(Dh, rnf, AMGD_V_SQRT);
      dcsr *DAD = dcsr_copy(Af);
      amgd_diag_op2(DAD, Dh, Dh, AMGD_SCALE2);
      double lambda[KMAX + 2];
      uint32_t k = lanczos(DAD, lambda);
      double a = lambda[0], b = lambda[k - 1];
      amgd_vscale(D, rnf, 2. / (a + b));
      L->rho = (b - a) / (b + a);
      double c;
      chebsim(&L->m, &c, L->rho, gamma2);
      amgd_free(Dh);
      dcsr_free(&DAD);
    } else {
      L->rho = 0;
      L->m = 1;
    }
    L->D = D;
    L->Af = Af;
    ph(PH_SMOOTH);
    add_time(&g_st.t_smoother_ms, &t0);
    /* --- interpolation --- */
    dcsr *Afc = amgd_sub_mat(A, vf, vc), *Ac = amgd_sub_mat(A, vc, vc);
    uint32_t rnc = Ac->rn;
    L->idc = (unsigned long *)amgd_alloc((size_t)rnc * 8 + 8);
    L->idf = (unsigned long *)amgd_alloc((size_t)rnf * 8 + 8);
    amgd_compact_ids(level == 0 ? h->id : h->lv[level - 1].idc, vc, rn, L->idc, L->idf);
    /* Af' for the transposed products (only where Af's rows are long enough to pay) */
    dcsr *AfT = Af->rn && Af->nnz >= 64ull * Af->rn ? amgd_transpose(Af, NULL) : NULL;
    dcsr *Acf = amgd_transpose(Afc, NULL);           /* Afc' = A(C,F): interpolation and RAP */
    dcsr *W = interpolation(Af, AfT, Ac, Afc, Acf, gamma2, itol);
    L->W = W;
    add_time(&g_st.t_interp_ms, &t0);
    /* --- Galerkin coarse operator: A = W'*AfP + A(C,F)*W + A(C,C) --- */
    amgd_spgemm_set_timer(0);
    dcsr *Wt = amgd_transpose(W, NULL);
    if (amgd_nshards() == 1) amgd_spgemm_sym_next(2);   /* the loop's last Af*W symbolic phase */
    dcsr *AfW = spgemm_via_t(Af, AfT, W, Wt);
    amgd_spgemm_sym_drop();
    dcsr *AfP = amgd_mpm(1., AfW, 1., Afc);
    dcsr_free(&AfW);
    L->AfP = AfP;
    dcsr *WtAfP = amgd_spgemm(Wt, AfP);
    dcsr *AcfW = spgemm_via_t(Acf, Afc, W, Wt);      /* Acf' = Afc exactly */
    if (AfT) dcsr_free(&AfT);
    amgd_spgemm_set_timer(-1);
    dcsr *Atmp = amgd_mpm(1., WtAfP, 1., AcfW);
    A = amgd_mpm(1., Atmp, 1, Ac);
    g_st.rap_out_nnz += A->nnz;
    dcsr_free(&Wt); dcsr_free(&WtAfP); dcsr_free(&Acf); dcsr_free(&AcfW); dcsr_free(&Atmp);
    dcsr_free(&Afc); dcsr_free(&Ac);
    amgd_free(vf);
    ph(PH_RAP);
    add_time(&g_st.t_rap_ms, &t0);
    level++;
  }
  h->nlevels = level + 1;
  amgd_ph_report(h->nlevels);
  amgd_sync();
  g_st.t_total_ms = (amgd_wtime() - t_start) * 1e3;
  g_st.rap_kernel_ms = amgd_timer_ms(0);
  g_st.spmv_kernel_ms = amgd_timer_ms(1);
  g_st.spmv_bytes = amgd_spmv_bytes();
  g_st.spmv_bytes_strict = amgd_spmv_bytes_strict();
  g_st.spmv_launches = amgd_spmv_launches();
  g_st.rap_launches = amgd_spgemm_launches();
  rw_stats();
  amgd_spmv_bytes_reset();
  g_st.rap_bytes = amgd_spgemm_bytes();
  amgd_spgemm_bytes_reset();
  g_st.nlevels = h->nlevels;
  g_st.ub_events = (uint32_t)g_ub;
  g_st.peak_bytes = amgd_pool_peak_bytes();
  return 0;
}

static struct csr_mat *csr_to_host(const dcsr *A) {
  struct csr_mat *M = (struct csr_mat *)malloc(sizeof *M);
  M->rn = A->rn;
  M->cn = A->cn;
  M->row_off = (amg_uint *)malloc(((size_t)A->rn + 1) * sizeof(amg_uint));
  M->col = (amg_uint *)malloc((A->nnz ? A->nnz : 1) * sizeof(amg_uint));
  M->a = (double *)malloc((A->nnz ? A->nnz : 1) * sizeof(double));
  amgd_to_host_cols(A, M->row_off, M->col, M->a);
  return M;
}

API int amgd_hier_export(const amgd_hier *h, struct amg_setup_data *data) {
  amgd_sync();
  double t0 = amgd_wtime();
  if (h->ph) {
    const int rc = amgd_phier_export(h->ph, data);
    g_st.t_copy_ms = (amgd_wtime() - t0) * 1e3;
    return rc;
  }
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
    const level_t *L = &h->lv[l];
    data->n[l] = L->A->cn;
    data->nnz[l] = (double)L->A->nnz;
    data->A[l] = csr_to_host(L->A);
    if (l + 1 == nl) break;
    uint32_t rn = L->A->rn, rnf = L->Af->rn, rnc = rn - rnf;
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
    data->nnzf[l] = (double)L->Af->nnz;
    data->nnzfp[l] = (double)L->AfP->nnz;
    data->Af[l] = csr_to_host(L->Af);
    data->W[l] = csr_to_host(L->W);
    data->AfP[l] = csr_to_host(L->AfP);
    data->idc[l] = (amg_uint *)malloc((size_t)rnc * 8 + 8);
    data->idf[l] = (amg_uint *)malloc((size_t)rnf * 8 + 8);
    amgd_d2h(data->idc[l], L->idc, (size_t)rnc * 8);
    amgd_d2h(data->idf[l], L->idf, (size_t)rnf * 8);
  }
  data->nlevels = nl;
  data->nullspace = (amg_uint)h->nullspace;
  g_st.t_copy_ms = (amgd_wtime() - t0) * 1e3;
  return 0;
}

API void amgd_hier_free(amgd_hier **hp) {
  amgd_hier *h = *hp;
  if (!h) return;
  if (h->ph) {
    amgd_phier_free(&h->ph);
    free(h);
    *hp = NULL;
    return;
  }
  for (uint32_t l = 0; l < h->nlevels; l++) {
    level_t *L = &h->lv[l];
    dcsr_free(&L->A); dcsr_free(&L->Af); dcsr_free(&L->W); dcsr_free(&L->AfP);
    if (L->vc) amgd_free(L->vc);
    if (L->D) amgd_free(L->D);
    if (L->idc) amgd_free(L->idc);
    if (L->idf) amgd_free(L->idf);
  }
  amgd_free(h->id);
  free(h->lv);
  free(h);
  *hp = NULL;
}

/* ------------------------------------------------------------------------ */
/* drop-in host ABI (amg_setup.h)                                            */
/* ------------------------------------------------------------------------ */
API void amg_setup(amg_uint n, const amg_uint *Ai, const amg_uint *Aj, const double *Av,
                   struct amg_setup_data *data) {
  /* amg_setup has no status (amg_setup.h:5): every failure leaves data with nlevels = 0
     and the reason in amgd_error() */
  if (amgd_rt_init(0) != 0) {
    fprintf(stderr, "omp_amg_amd: amg_setup needs a HIP device: %s\n", amgd_last_error());
    memset(data, 0, sizeof *data);
    return;
  }
  uint32_t *hi = (uint32_t *)malloc((size_t)n * 4 + 4), *hj = (uint32_t *)malloc((size_t)n * 4 + 4);
  for (amg_uint k = 0; k < n; k++) {
    if (Ai[k] > 0xfffffffeul || Aj[k] > 0xfffffffeul) {
      amgd_set_error("amg_setup: an index exceeds the 32-bit range of the device CSR");
      fprintf(stderr, "omp_amg_amd: entry %lu: index exceeds 32-bit range\n", (unsigned long)k);
      free(hi); free(hj);
      memset(data, 0, sizeof *data);
      return;
    }
    hi[k] = (uint32_t)Ai[k];
    hj[k] = (uint32_t)Aj[k];
  }
  uint32_t *di = (uint32_t *)amgd_alloc((size_t)n * 4 + 4), *dj = (uint32_t *)amgd_alloc((size_t)n * 4 + 4);
  double *dv = dalloc(n);
  amgd_h2d(di, hi, (size_t)n * 4);
  amgd_h2d(dj, hj, (size_t)n * 4);
  amgd_h2d(dv, Av, (size_t)n * 8);
  free(hi); free(hj);
  amgd_hier *h = NULL;
  /* amg_setup takes the WHOLE matrix on the calling process (amg_setup.h:5): with a
     multi-process communicator in partitioned mode (where amgd_setup_device takes this
     rank's share) it runs the one-GPU setup on this process alone -- no collective, so
     one rank calling it cannot hang in an exchange the others never enter */
  const int susp = amgd_comm_partitioned() && amgd_comm_procs() > 1;
  if (susp) amgd_comm_suspend_partition(1);
  const int rc = amgd_setup_device(n, di, dj, dv, &h, 0);
  if (susp) amgd_comm_suspend_partition(0);
  amgd_free(di); amgd_free(dj); amgd_free(dv);
  if (rc != 0) {
    /* no hierarchy: data is left with nlevels = 0 and amgd_error() says why */
    fprintf(stderr, "omp_amg_amd: amg_setup failed: %s\n", amgd_last_error());
    memset(data, 0, sizeof *data);
    return;
  }
  amgd_hier_export(h, data);
  amgd_hier_free(&h);
}

static void free_csr_host(struct csr_mat **M) {
  if (*M) { free((*M)->row_off); free((*M)->col); free((*M)->a); free(*M); *M = NULL; }
}

API void free_data(struct amg_setup_data **data) {
  struct amg_setup_data *d = *data;
  if (!d) return;
  free(d->n); free(d->nnz); free(d->nnzf); free(d->nnzfp); free(d->m); free(d->rho);
  for (amg_uint i = 0; i < d->nlevels; i++) free_csr_host(&d->A[i]);
  for (amg_uint i = 0; i + 1 < d->nlevels; i++) {
    free(d->C[i]); free(d->F[i]); free(d->D[i]); free(d->idc[i]); free(d->idf[i]);
    free_csr_host(&d->Af[i]); free_csr_host(&d->W[i]); free_csr_host(&d->AfP[i]);
  }
  free(d->id); free(d->idc); free(d->idf); free(d->C); free(d->F); free(d->D);
  free(d->A); free(d->Af); free(d->W); free(d->AfP);
  free(d);
  *data = NULL;
}

/* amg_export (amg_setup.c:405-595): the Nek5000 AMG file set */
static uint64_t max_row(const struct csr_mat *m) {
  uint64_t mx = 0;
  for (amg_uint i = 0; i < m->rn; i++) if (m->row_off[i + 1] - m->row_off[i] > mx) mx = m->row_off[i + 1] - m->row_off[i];
  return mx;
}
static void save_mats(amg_uint *len, amg_uint n, amg_uint nl, const amg_uint *lvl, amg_uint **id,
                      struct csr_mat **mat, const char *fn) {
  const double magic = 3.14159;
  FILE *f = fopen(fn, "w");
  if (!f) { perror(fn); return; }
  fwrite(&magic, sizeof(double), 1, f);
  uint64_t mx = 0;
  for (amg_uint i = 0; i < nl; i++) { uint64_t l = max_row(mat[i]); if (l > mx) mx = l; }
  double *buf = (double *)malloc((2 * mx + 1) * sizeof(double));
  amg_uint *row = (amg_uint *)calloc(nl + 1, sizeof(amg_uint));
  for (amg_uint i = 0; i < n; i++) {
    amg_uint l = lvl[i] - 1;
    if (l > nl) { printf("level out of bounds\n"); continue; }
    if (l == nl) { len[i] = 0; continue; }
    struct csr_mat *M = mat[l];
    amg_uint j = row[l]++;
    if (j >= M->rn) { printf("row out of bounds\n"); continue; }
    amg_uint kb = M->row_off[j], ke = M->row_off[j + 1];
    double *p = buf;
    for (amg_uint k = kb; k != ke; ++k) *p++ = (double)id[l][M->col[k]], *p++ = M->a[k];
    len[i] = ke - kb;
    fwrite(buf, sizeof(double), 2 * (ke - kb), f);
  }
  for (amg_uint i = 0; i < nl; i++) if (row[i] != mat[i]->rn) printf("matrices not exhausted\n");
  free(row); free(buf);
  fclose(f);
  printf("%d matrices written to %s\n", (int)nl, fn);
}
API void amg_export(struct amg_setup_data *data) {
  amg_uint nl = data->nlevels, n = (amg_uint)data->n[0];
  amg_uint *lvl = (amg_uint *)malloc(n * sizeof(amg_uint) + 8);
  for (amg_uint i = 0; i < n; i++) lvl[i] = 1;
  for (amg_uint i = 0; i + 1 < nl; i++)
    for (amg_uint j = 0; j < (amg_uint)data->n[i + 1]; j++) lvl[data->idc[i][j] - 1] += 1;
  double *dvec = (double *)malloc(n * sizeof(double) + 8);
  for (amg_uint i = 0; i + 1 < nl; i++) {
    amg_uint m = (amg_uint)(data->n[i] - data->n[i + 1]);
    for (amg_uint j = 0; j < m; j++) dvec[data->idf[i][j] - 1] = data->D[i][j];
  }
  amg_uint k = data->idc[nl - 2][0] - 1;
  dvec[k] = data->nullspace != 0 ? 0. : 1. / data->A[nl - 1]->a[0];
  amg_uint *Wl = (amg_uint *)malloc(n * sizeof(amg_uint) + 8);
  amg_uint *Pl = (amg_uint *)malloc(n * sizeof(amg_uint) + 8);
  amg_uint *Fl = (amg_uint *)malloc(n * sizeof(amg_uint) + 8);
  save_mats(Wl, n, nl - 1, lvl, data->idc, data->W, "amg_W.dat");
  save_mats(Pl, n, nl - 1, lvl, data->idc, data->AfP, "amg_AfP.dat");
  save_mats(Fl, n, nl - 1, lvl, data->idf, data->Af, "amg_Aff.dat");
  FILE *f = fopen("amg.dat", "w");
  if (f) {
    const double magic = 3.14159, stamp = 2.01;
    double t;
    fwrite(&magic, sizeof(double), 1, f);
    fwrite(&stamp, sizeof(double), 1, f);
    t = (double)nl; fwrite(&t, sizeof(double), 1, f);
    fwrite(data->m, sizeof(double), nl - 1, f);
    fwrite(data->rho, sizeof(double), nl - 1, f);
    t = (double)n; fwrite(&t, sizeof(double), 1, f);
    for (amg_uint i = 0; i < n; i++) {
      double rec[6] = {(double)data->id[i], (double)lvl[i], (double)Wl[i], (double)Pl[i], (double)Fl[i], dvec[i]};
      fwrite(rec, sizeof(double), 6, f);
    }
    fclose(f);
    printf("Vectors written to %s\n", "amg.dat");
  }
  free(Wl); free(Pl); free(Fl); free(dvec); free(lvl);
}

/* ------------------------------------------------------------------------ */
/* gslib crs.h (reference crs.h:8-21, amg.c:475)                             */
/* ------------------------------------------------------------------------ */
struct crs_data { amgd_hier *h; amg_uint un; amg_uint null_space; };

/* crs_setup (reference amg.c:475): rank comm->id of comm->np passes its local
   matrix -- n local dofs with global ids id[0..n), nz entries in local indices.  The
   reference hands the assembled matrix, keyed by global id (its amg_dump,
   amg.c:1048-1072, drops entries touching id 0 and exact zeros), to the setup.  Here
   every rank's entries are mapped to global ids on the host and uploaded; for np > 1
   (library communicator amgd_comm_init_rccl / _host, rank = comm->id, size = comm->np):
   * default, the partitioned setup: each rank's entries go to the
     owners of their rows (duplicates -- dofs shared between ranks -- summed in rank
     order), every rank keeps its row blocks of the hierarchy;
   * after amgd_comm_set_partitioned(0), the round-2 replicated mode: the entries are
     completed into one COO on every rank (allgatherv, rank order) and every rank keeps
     the whole hierarchy, its heavy kernels row-sharded (amgd_comm.hip).
   Global ids must be 1..N (row id-1 of the assembled matrix).  Returns NULL (message on
   stderr, amgd_error()) on a communicator that does not match comm, or when the setup
   runs out of HBM. */
API struct crs_data *crs_setup(amg_uint n, const unsigned long *id, amg_uint nz, const amg_uint *Ai,
                               const amg_uint *Aj, const double *A, amg_uint null_space,
                               const struct comm *comm) {
  const int np = comm ? (int)comm->np : 1, me = comm ? (int)comm->id : 0;
  if (amgd_rt_init(0) != 0) {
    fprintf(stderr, "omp_amg_amd: crs_setup needs a HIP device: %s\n", amgd_last_error());
    return NULL;
  }
  if (np > 1 && (amgd_comm_procs() != np || amgd_comm_rank() != me)) {
    fprintf(stderr, "omp_amg_amd: crs_setup with np = %d needs the library communicator of the same "
            "ranks (amgd_comm_init_rccl / amgd_comm_init_host; have %d processes, rank %d)\n", np,
            amgd_comm_procs(), amgd_comm_rank());
    return NULL;
  }
  /* local dof k is global id[k]; entries touching id 0 are dropped (amg.c:1065).  Local
     indices must be < n and ids < 2^32 (the device CSR keeps u32 columns): a violation on
     any rank makes every rank return NULL (the flag travels with the entry counts, so no
     rank is left waiting in a collective) */
  amg_uint *I = (amg_uint *)malloc(nz * sizeof(amg_uint) + 8), *J = (amg_uint *)malloc(nz * sizeof(amg_uint) + 8);
  double *V = (double *)malloc(nz * sizeof(double) + 8);
  amg_uint m = 0;
  const char *why = NULL;
  for (amg_uint k = 0; k < nz && !why; k++) {
    amg_uint i = Ai[k], j = Aj[k];
    if (i >= n || j >= n) { why = "local index >= n"; break; }
    if (id[i] == 0 || id[j] == 0 || A[k] == 0) continue;
    if (id[i] - 1 > 0xfffffffeul || id[j] - 1 > 0xfffffffeul) { why = "global id exceeds the 32-bit range"; break; }
    I[m] = id[i] - 1; J[m] = id[j] - 1; V[m] = A[k]; m++;
  }
  uint64_t *cnt = (uint64_t *)calloc((size_t)np + 1, 8), *pre = (uint64_t *)calloc((size_t)np + 1, 8);
  cnt[me] = why ? ~0ull : m;
  if (np > 1) amgd_allgather_u64(cnt);
  int bad_rank = -1;
  for (int r = 0; r < np; r++) if (cnt[r] == ~0ull && bad_rank < 0) bad_rank = r;
  if (bad_rank >= 0) {
    amgd_set_error(why ? why : "invalid input on another rank");
    fprintf(stderr, "omp_amg_amd: crs_setup: rank %d: %s\n", bad_rank, why ? why : "(see that rank)");
    free(cnt); free(pre); free(I); free(J); free(V);
    return NULL;
  }
  struct crs_data *d = (struct crs_data *)calloc(1, sizeof *d);
  /* entries of every rank: counts (above), then one allgatherv of (i, j, v) -- or, in
     partitioned mode, each rank hands its own entries to the partitioned setup, which
     routes them to the owners of their rows (the same rank order for duplicates) */
  const int part = np > 1 && amgd_comm_part_default();
  const int part_was = amgd_comm_part_get();
  if (part) amgd_comm_set_partitioned(1);
  for (int r = 0; r < np; r++) pre[r + 1] = pre[r] + (part && r != me ? 0 : cnt[r]);
  const uint64_t M = pre[np];
  uint32_t *di = (uint32_t *)amgd_alloc(M * 4 + 4), *dj = (uint32_t *)amgd_alloc(M * 4 + 4);
  double *dv = dalloc(M);
  uint32_t *hi = (uint32_t *)malloc(m * 4 + 4), *hj = (uint32_t *)malloc(m * 4 + 4);
  for (amg_uint k = 0; k < m; k++) { hi[k] = (uint32_t)I[k]; hj[k] = (uint32_t)J[k]; }
  amgd_h2d(di + pre[me], hi, m * 4); amgd_h2d(dj + pre[me], hj, m * 4); amgd_h2d(dv + pre[me], V, m * 8);
  free(hi); free(hj); free(I); free(J); free(V);
  if (np > 1 && !part) {
    uint64_t *off = (uint64_t *)malloc(3 * ((size_t)np + 1) * 8);
    void *bufs[3] = {di, dj, dv};
    for (int r = 0; r <= np; r++) {
      off[r] = 4 * pre[r];
      off[(np + 1) + r] = 4 * pre[r];
      off[2 * (np + 1) + r] = 8 * pre[r];
    }
    amgd_allgatherv(3, bufs, off);
    free(off);
  }
  free(cnt); free(pre);
  /* np == 1: the whole matrix is this process's, the one-GPU setup */
  const int susp = np <= 1 && amgd_comm_partitioned() && amgd_comm_procs() > 1;
  if (susp) amgd_comm_suspend_partition(1);
  const int rc = amgd_setup_device(M, di, dj, dv, &d->h, 0);
  if (susp) amgd_comm_suspend_partition(0);
  if (part) amgd_comm_part_set(part_was);
  amgd_free(di); amgd_free(dj); amgd_free(dv);
  if (rc != 0) {
    fprintf(stderr, "omp_amg_amd: crs_setup failed: %s\n", amgd_last_error());
    free(d);
    return NULL;
  }
  d->un = n;
  d->null_space = null_space;
  return d;
}
API void crs_solve(double *x, struct crs_data *data, double *b) {
  (void)x; (void)data; (void)b;
  fprintf(stderr, "omp_amg_amd: crs_solve (AMG V-cycle) is not implemented; setup only\n");
  abort();
}
API void crs_stats(struct crs_data *data) {
  printf("AMG stats: %u levels (setup %.3f ms)\n", data && data->h ? data->h->nlevels : 0, g_st.t_total_ms);
}
API int amgd_crs_export(const struct crs_data *data, struct amg_setup_data *out) {
  if (!data || !data->h) return -1;
  return amgd_hier_export(data->h, out);
}
API void crs_free(struct crs_data *data) {
  if (!data) return;
  amgd_hier_free(&data->h);
  free(data);
}
