/*
 * oracle/amg_oracle.c -- TEST INFRASTRUCTURE, NOT THE PRODUCT.
 *
 * A CPU restatement of the reference serial AMG setup (nicooff/omp_amg,
 * amg_setup.c + amg_tools.c).  Every floating-point operation is performed in
 * the same order and with the same operands as the reference so results are
 * bit-identical; the *algorithms* are restated with sparse-efficient data
 * structures (the reference's mxm is O(rows^2), amg_setup.c:1920-1938; its
 * expand_support materialises dense w x nbad matrices, amg_setup.c:1034-1093).
 *
 * Pinned against the compiled reference (oracle/_ref/libref_amg.so) by
 * tests/golden/make_golden.py (fixtures written from the reference only where the oracle
 * matches it bit for bit) and tests/test_oracle_golden.py (every fixture and the
 * reference-made digests of tests/golden/digests.json).
 *
 * Deviations are confined to inputs on which the reference is undefined
 * (documented in DESIGN.md "Reference UB"):
 *   - sp_add whose x-support is not a subset of y (amg_setup.c:1665-1677)
 *     overruns the row in the reference; here missing entries are skipped.
 *   - transpose/coo2csr of an empty matrix leave row_off uninitialised in the
 *     reference (amg_setup.c:2017, 3693); here they are all zero.
 */
#define _POSIX_C_SOURCE 200809L
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "amg_oracle.h"

#define API __attribute__((visibility("default")))

typedef uint32_t u32;
typedef uint64_t u64;

/* internal CSR: 64-bit row offsets, 32-bit columns */
typedef struct { u32 rn, cn; u64 *ro; u32 *col; double *a; } ocsr;

/* events where the reference is undefined:
 *   oracle_ub_events     -- the reference would not terminate (we stop instead)
 *   oracle_overflow_events -- sp_add walks off the end of St (reference reads /
 *                           writes past the heap block; in-bounds values are
 *                           unaffected, so results still agree when it survives) */
static u64 oracle_ub_events = 0, oracle_overflow_events = 0;

static void *xmalloc(size_t n) {
  void *p = malloc(n ? n : 1);
  if (!p) { fprintf(stderr, "oracle: out of memory (%zu bytes)\n", n); abort(); }
  return p;
}
#define NEW(T, n) ((T *)xmalloc(sizeof(T) * (size_t)(n)))

static ocsr *csr_new(u32 rn, u32 cn, u64 nz) {
  ocsr *A = NEW(ocsr, 1);
  A->rn = rn; A->cn = cn;
  A->ro = NEW(u64, (size_t)rn + 1);
  A->col = NEW(u32, nz);
  A->a = NEW(double, nz);
  A->ro[0] = 0;
  return A;
}
static void csr_free(ocsr **A) {
  if (*A) { free((*A)->ro); free((*A)->col); free((*A)->a); free(*A); *A = NULL; }
}
static u64 nnz(const ocsr *A) { return A->ro[A->rn]; }
static ocsr *csr_copy(const ocsr *A) {
  ocsr *B = csr_new(A->rn, A->cn, nnz(A));
  memcpy(B->ro, A->ro, ((size_t)A->rn + 1) * sizeof(u64));
  memcpy(B->col, A->col, nnz(A) * sizeof(u32));
  memcpy(B->a, A->a, nnz(A) * sizeof(double));
  return B;
}
static void csr_shrink(ocsr *A) {
  u64 z = nnz(A);
  A->col = realloc(A->col, (z ? z : 1) * sizeof(u32));
  A->a = realloc(A->a, (z ? z : 1) * sizeof(double));
}

static int o_lvl = 0, o_it = 0;
static void dump_raw(const char *name, const void *p, size_t bytes) {
  const char *dir = getenv("ORACLE_DUMP");
  if (!dir || !*dir) return;
  char fn[512];
  snprintf(fn, sizeof fn, "%s/L%d_it%d_%s.bin", dir, o_lvl, o_it, name);
  FILE *f = fopen(fn, "wb");
  if (f) { fwrite(p, 1, bytes, f); fclose(f); }
}
static void dump_ocsr(const char *name, const ocsr *A) {
  char n2[256];
  snprintf(n2, sizeof n2, "%s_ro", name); dump_raw(n2, A->ro, ((size_t)A->rn + 1) * 8);
  snprintf(n2, sizeof n2, "%s_col", name); dump_raw(n2, A->col, A->ro[A->rn] * 4);
  snprintf(n2, sizeof n2, "%s_a", name); dump_raw(n2, A->a, A->ro[A->rn] * 8);
}

/* ------------------------------------------------------------------------
 * COO -> CSR, stable by (i, j): coo2csr (amg_setup.c:3684) sorts with
 * sarray_sort_2(i, j), a stable radix sort; duplicates are kept in input order.
 * Two stable counting passes (by j, then by i) give the same permutation.
 * ---------------------------------------------------------------------- */
static ocsr *coo2csr(u64 nz, const u32 *I, const u32 *J, const double *V, u32 rn, u32 cn) {
  u64 *cnt = NEW(u64, (size_t)(cn > rn ? cn : rn) + 1);
  u64 *p1 = NEW(u64, nz);
  u64 k;
  memset(cnt, 0, ((size_t)cn + 1) * sizeof(u64));
  for (k = 0; k < nz; k++) cnt[J[k] + 1]++;
  for (u32 c = 0; c < cn; c++) cnt[c + 1] += cnt[c];
  for (k = 0; k < nz; k++) p1[cnt[J[k]]++] = k;        /* stable by j */
  ocsr *A = csr_new(rn, cn, nz);
  memset(A->ro, 0, ((size_t)rn + 1) * sizeof(u64));
  for (k = 0; k < nz; k++) A->ro[I[k] + 1]++;
  for (u32 r = 0; r < rn; r++) A->ro[r + 1] += A->ro[r];
  memcpy(cnt, A->ro, (size_t)rn * sizeof(u64));
  for (k = 0; k < nz; k++) {                           /* stable by i */
    u64 src = p1[k];
    u64 dst = cnt[I[src]]++;
    A->col[dst] = J[src];
    A->a[dst] = V[src];
  }
  free(cnt); free(p1);
  return A;
}

/* build_csr_dim (amg_setup.c:3656): drops entries whose value is exactly 0 */
static ocsr *build_csr_dim(u64 n, const u32 *I, const u32 *J, const double *V, u32 rn, u32 cn) {
  u32 *I2 = NEW(u32, n), *J2 = NEW(u32, n);
  double *V2 = NEW(double, n);
  u64 k = 0;
  for (u64 i = 0; i < n; i++)
    if (V[i] != 0.) { I2[k] = I[i]; J2[k] = J[i]; V2[k] = V[i]; k++; }
  ocsr *A = coo2csr(k, I2, J2, V2, rn, cn);
  free(I2); free(J2); free(V2);
  return A;
}

/* sub_mat (amg_setup.c:3058): subA = A(vr~=0, vc~=0) with column renumbering */
static ocsr *sub_mat(const ocsr *A, const double *vr, const double *vc) {
  u32 *g2l = NEW(u32, A->cn);
  u32 subcn = 0, subrn = 0;
  u64 subnz = 0;
  for (u32 c = 0; c < A->cn; c++) g2l[c] = (vc[c] != 0) ? subcn++ : (u32)-1;
  for (u32 i = 0; i < A->rn; i++)
    if (vr[i] != 0) {
      subrn++;
      for (u64 j = A->ro[i]; j < A->ro[i + 1]; j++) subnz += (vc[A->col[j]] != 0);
    }
  ocsr *S = csr_new(subrn, subcn, subnz);
  u32 r = 0; u64 o = 0;
  for (u32 i = 0; i < A->rn; i++) {
    if (vr[i] == 0) continue;
    for (u64 j = A->ro[i]; j < A->ro[i + 1]; j++)
      if (vc[A->col[j]] != 0) { S->col[o] = g2l[A->col[j]]; S->a[o] = A->a[j]; o++; }
    S->ro[++r] = o;
  }
  free(g2l);
  return S;
}

/* build_csr (amg_setup.c:3612): drop zero values, sort, drop empty rows/cols.
 * Dimensions: max index + 1 over the entries (the reference reads coo_A[i]
 * with the unfiltered index, amg_setup.c:3632, which is the same for inputs
 * without explicit zeros). */
static ocsr *build_csr(u64 n, const amg_uint *Ai, const amg_uint *Aj, const double *Av) {
  u32 *I = NEW(u32, n), *J = NEW(u32, n);
  double *V = NEW(double, n);
  u64 k = 0; u32 rn = 0, cn = 0;
  for (u64 i = 0; i < n; i++) {
    if (Av[i] != 0.) { I[k] = (u32)Ai[i]; J[k] = (u32)Aj[i]; V[k] = Av[i]; k++; }
    if ((u32)Ai[i] + 1 > rn) rn = (u32)Ai[i] + 1;
    if ((u32)Aj[i] + 1 > cn) cn = (u32)Aj[i] + 1;
  }
  ocsr *T = coo2csr(k, I, J, V, rn, cn);
  free(I); free(J); free(V);
  double *zr = NEW(double, cn > rn ? cn : rn);
  for (u32 i = 0; i < (cn > rn ? cn : rn); i++) zr[i] = (i < rn && T->ro[i + 1] != T->ro[i]) ? 1. : 0.;
  ocsr *A = sub_mat(T, zr, zr);
  free(zr); csr_free(&T);
  return A;
}

/* transpose (amg_setup.c:2000): sort by (j, i) -- a stable counting sort */
static ocsr *transpose(const ocsr *A) {
  u64 z = nnz(A);
  ocsr *T = csr_new(A->cn, A->rn, z);
  memset(T->ro, 0, ((size_t)A->cn + 1) * sizeof(u64));
  for (u64 k = 0; k < z; k++) T->ro[A->col[k] + 1]++;
  for (u32 c = 0; c < A->cn; c++) T->ro[c + 1] += T->ro[c];
  u64 *pos = NEW(u64, (size_t)A->cn + 1);
  memcpy(pos, T->ro, ((size_t)A->cn + 1) * sizeof(u64));
  for (u32 i = 0; i < A->rn; i++)
    for (u64 k = A->ro[i]; k < A->ro[i + 1]; k++) {
      u64 d = pos[A->col[k]]++;
      T->col[d] = i; T->a[d] = A->a[k];
    }
  free(pos);
  return T;
}

static int cmp_u32(const void *a, const void *b) {
  u32 x = *(const u32 *)a, y = *(const u32 *)b;
  return x < y ? -1 : x > y;
}

/* X = A*B with the reference's arithmetic (mxm, amg_setup.c:1894):
 *   X[i][j] = sum over k ascending of B[k][j]*A[i][k], started at +0.0,
 *   entries whose sum is exactly 0 are dropped, columns ascending.
 * The reference scatters A's row into a dense x (x[col]=a, so for duplicate
 * columns the LAST value wins) and dots it with every row of B^T; a
 * Gustavson row-merge over k ascending performs the identical additions. */
static ocsr *spgemm(const ocsr *A, const ocsr *B) {
  u32 rn = A->rn, cn = B->cn;
  u64 cap = 1024, z = 0;
  u32 *col = NEW(u32, cap);
  double *val = NEW(double, cap);
  ocsr *X = NEW(ocsr, 1);
  X->rn = rn; X->cn = cn; X->ro = NEW(u64, (size_t)rn + 1); X->ro[0] = 0;
  double *acc = NEW(double, cn ? cn : 1);
  u32 *mark = NEW(u32, cn ? cn : 1), *list = NEW(u32, cn ? cn : 1);
  for (u32 j = 0; j < cn; j++) mark[j] = (u32)-1;
  for (u32 i = 0; i < rn; i++) {
    u32 nl = 0;
    for (u64 ka = A->ro[i]; ka < A->ro[i + 1]; ka++) {
      if (ka + 1 < A->ro[i + 1] && A->col[ka + 1] == A->col[ka]) continue; /* last wins */
      u32 k = A->col[ka]; double av = A->a[ka];
      for (u64 kb = B->ro[k]; kb < B->ro[k + 1]; kb++) {
        u32 j = B->col[kb];
        if (mark[j] != i) { mark[j] = i; acc[j] = 0.0; list[nl++] = j; }
        acc[j] += B->a[kb] * av;
      }
    }
    qsort(list, nl, sizeof(u32), cmp_u32);
    for (u32 t = 0; t < nl; t++) {
      double v = acc[list[t]];
      if (v != 0.0) {
        if (z == cap) { cap *= 2; col = realloc(col, cap * sizeof(u32)); val = realloc(val, cap * sizeof(double)); }
        col[z] = list[t]; val[z] = v; z++;
      }
    }
    X->ro[i + 1] = z;
  }
  free(acc); free(mark); free(list);
  X->col = col; X->a = val;
  csr_shrink(X);
  return X;
}

/* mpm (amg_setup.c:1684): X = alpha*A + beta*B; a both-present exact zero is dropped */
static ocsr *mpm(double alpha, const ocsr *A, double beta, const ocsr *B) {
  if (A->rn != B->rn || A->cn != B->cn) { fprintf(stderr, "oracle mpm: dims\n"); abort(); }
  u64 cap = nnz(A) + nnz(B);
  ocsr *X = csr_new(A->rn, A->cn, cap);
  u64 o = 0;
  for (u32 i = 0; i < A->rn; i++) {
    u64 ja = A->ro[i], ea = A->ro[i + 1], jb = B->ro[i], eb = B->ro[i + 1];
    while (ja < ea || jb < eb) {
      if (ja < ea && jb < eb) {
        if (A->col[ja] == B->col[jb]) {
          double s = alpha * A->a[ja] + beta * B->a[jb];
          if (s != 0.) { X->col[o] = A->col[ja]; X->a[o] = s; o++; }
          ja++; jb++;
        } else if (A->col[ja] < B->col[jb]) {
          X->col[o] = A->col[ja]; X->a[o] = alpha * A->a[ja]; o++; ja++;
        } else {
          X->col[o] = B->col[jb]; X->a[o] = beta * B->a[jb]; o++; jb++;
        }
      } else if (ja == ea) {
        X->col[o] = B->col[jb]; X->a[o] = beta * B->a[jb]; o++; jb++;
      } else {
        X->col[o] = A->col[ja]; X->a[o] = alpha * A->a[ja]; o++; ja++;
      }
    }
    X->ro[i + 1] = o;
  }
  csr_shrink(X);
  return X;
}

/* mxmpoint (amg_setup.c:1807): X = A.*B on the intersection; zeros kept */
static ocsr *mxmpoint(const ocsr *A, const ocsr *B) {
  if (A->rn != B->rn || A->cn != B->cn) { fprintf(stderr, "oracle mxmpoint: dims\n"); abort(); }
  u64 cap = nnz(A) < nnz(B) ? nnz(A) : nnz(B);
  ocsr *X = csr_new(A->rn, A->cn, cap);
  u64 o = 0;
  for (u32 i = 0; i < A->rn; i++) {
    u64 ja = A->ro[i], ea = A->ro[i + 1], jb = B->ro[i], eb = B->ro[i + 1];
    while (ja < ea && jb < eb) {
      if (A->col[ja] == B->col[jb]) { X->col[o] = A->col[ja]; X->a[o] = A->a[ja] * B->a[jb]; o++; ja++; jb++; }
      else if (A->col[ja] < B->col[jb]) ja++;
      else jb++;
    }
    X->ro[i + 1] = o;
  }
  csr_shrink(X);
  return X;
}

/* apply_M (amg_tools.c:76): z = alpha*y + beta*(M x), or beta*(M x) when alpha==0||!y */
static void apply_M(double *z, double alpha, const double *y, double beta, const ocsr *M, const double *x) {
  for (u32 i = 0; i < M->rn; i++) {
    double t = 0;
    for (u64 j = M->ro[i]; j < M->ro[i + 1]; j++) t += M->a[j] * x[M->col[j]];
    z[i] = (alpha == 0. || y == NULL) ? beta * t : alpha * y[i] + beta * t;
  }
}
/* apply_Mt (amg_tools.c:102): z = M^T x, scattered in row order */
static void apply_Mt(double *z, const ocsr *M, const double *x) {
  for (u32 i = 0; i < M->cn; i++) z[i] = 0;
  for (u32 i = 0; i < M->rn; i++) {
    double xi = x[i];
    for (u64 j = M->ro[i]; j < M->ro[i + 1]; j++) z[M->col[j]] += M->a[j] * xi;
  }
}

/* diag (amg_setup.c:3363): first stored (i,i), else 0 */
static void diag(double *D, const ocsr *A) {
  for (u32 i = 0; i < A->rn; i++) {
    double d = 0.;
    for (u64 j = A->ro[i]; j < A->ro[i + 1]; j++) if (A->col[j] == i) { d = A->a[j]; break; }
    D[i] = d;
  }
}
enum { DPLUS, DMINUS, DMULT, MULTD };
/* diagcsr_op (amg_setup.c:3389) */
static void diagcsr_op(ocsr *A, const double *D, int op) {
  for (u32 i = 0; i < A->rn; i++)
    for (u64 j = A->ro[i]; j < A->ro[i + 1]; j++) {
      if (op == DPLUS) { if (A->col[j] == i) { A->a[j] = A->a[j] + D[i]; break; } }
      else if (op == DMINUS) { if (A->col[j] == i) { A->a[j] = A->a[j] - D[i]; break; } }
      else if (op == DMULT) A->a[j] = A->a[j] * D[i];
      else A->a[j] = A->a[j] * D[A->col[j]];
    }
}

/* vv_dot (amg_setup.c:3193) and array_op norm2 (amg_setup.c:3309) */
static double vv_dot(const double *a, const double *b, u64 n) {
  double r = 0;
  for (u64 i = 0; i < n; i++) r += a[i] * b[i];
  return r;
}
static double norm2(const double *a, u64 n) {
  double r = 0;
  for (u64 i = 0; i < n; i++) r += a[i] * a[i];
  return sqrt(r);
}
/* extr_op max (amg_setup.c:3281): first index of the maximum */
static double vmax(const double *a, u64 n, u64 *idx) {
  double e = a[0]; u64 k = 0;
  for (u64 i = 1; i < n; i++) if (a[i] > e) { e = a[i]; k = i; }
  if (idx) *idx = k;
  return e;
}

/* mat_max (amg_setup.c:3535) */
static void mat_max(double *y, const ocsr *A, const double *f, const double *x, double tol) {
  for (u32 i = 0; i < A->cn; i++) y[i] = -DBL_MAX;
  for (u32 i = 0; i < A->rn; i++) {
    double xj = x[i], Amax = 0;
    for (u64 j = A->ro[i]; j < A->ro[i + 1]; j++)
      if (f[A->col[j]] != 0 && fabs(A->a[j]) > Amax) Amax = fabs(A->a[j]);
    Amax *= tol;
    for (u64 j = A->ro[i]; j < A->ro[i + 1]; j++) {
      u32 k = A->col[j];
      if (f[k] == 0 || fabs(A->a[j]) < Amax) continue;
      if (xj > y[k]) y[k] = xj;
    }
  }
}

/* coarsen (amg_setup.c:2737): strength S = |D^-1/2 A D^-1/2| - diag, then
 * repeated independent-set C marking until the norm bound <= ctol */
static void coarsen(double *vc, const ocsr *A, double ctol) {
  u32 n = A->cn;
  double *D = NEW(double, n);
  diag(D, A);
  for (u32 i = 0; i < n; i++) D[i] = sqrt(D[i]);
  for (u32 i = 0; i < n; i++) D[i] = 1. / D[i];
  ocsr *S = csr_copy(A);
  diagcsr_op(S, D, DMULT);
  diagcsr_op(S, D, MULTD);
  for (u64 k = 0; k < nnz(S); k++) S->a[k] = fabs(S->a[k]);
  diag(D, S);
  diagcsr_op(S, D, DMINUS);
  free(D);
  for (u32 i = 0; i < n; i++) vc[i] = 0.;
  int anyvc = 0;
  double *vf = NEW(double, n), *g = NEW(double, n), *w1 = NEW(double, n), *w2 = NEW(double, n);
  double *tmp = NEW(double, n), *w = NEW(double, n), *mask = NEW(double, n), *m = NEW(double, n);
  for (u32 i = 0; i < n; i++) vf[i] = 1.;
  for (;;) {
    apply_M(g, 0, vf, 1., S, vf);
    for (u32 i = 0; i < n; i++) g[i] = g[i] * vf[i];
    apply_M(w1, 0, g, 1., S, g);
    for (u32 i = 0; i < n; i++) w1[i] = w1[i] * vf[i];
    apply_M(w2, 0, w1, 1., S, w1);
    for (u32 i = 0; i < n; i++) w2[i] = w2[i] * vf[i];
    apply_M(tmp, 0, w2, 1., S, w2);
    for (u32 i = 0; i < n; i++) w2[i] = tmp[i] * vf[i];
    for (u32 i = 0; i < n; i++) { w[i] = 1. / w1[i]; w[i] = w[i] * w2[i]; if (w1[i] == 0) w[i] = 0.; }
    u64 mi;
    double w1m = vmax(w1, n, &mi), wm = vmax(w, n, NULL);
    double b = (w1m < wm) ? sqrt(w1m) : sqrt(wm);
    if (b <= ctol) { if (anyvc == 0) vc[mi] = 1.; break; }
    for (u32 i = 0; i < n; i++) mask[i] = (w[i] > ctol * ctol) ? 1. : 0.;
    for (u32 i = 0; i < n; i++) tmp[i] = g[i] * mask[i];
    mat_max(m, S, vf, tmp, 0.1);
    for (u32 i = 0; i < n; i++) { g[i] = g[i] - m[i]; tmp[i] = (g[i] >= 0.) ? 1. : 0.;
                                  mask[i] = (mask[i] != 0. && tmp[i] != 0.) ? 1. : 0.; }
    for (u32 i = 0; i < n; i++) { g[i] = (double)i + 1.0; tmp[i] = mask[i] * g[i]; }
    mat_max(m, S, vf, tmp, 0.1);
    for (u32 i = 0; i < n; i++) { g[i] = g[i] - m[i]; tmp[i] = (g[i] > 0.) ? 1. : 0.;
                                  mask[i] = (mask[i] != 0. && tmp[i] != 0.) ? 1. : 0.; }
    for (u32 i = 0; i < n; i++) vc[i] = (vc[i] == 0. && mask[i] == 0.) ? 0. : 1.;
    if (!anyvc) for (u32 i = 0; i < n; i++) if (vc[i] == 1.) { anyvc = 1; break; }
    for (u32 i = 0; i < n; i++)
      vf[i] = ((vf[i] == 0. && mask[i] != 0.) || (vf[i] != 0. && mask[i] == 0.)) ? 1. : 0.;
  }
  csr_free(&S);
  free(vf); free(g); free(w1); free(w2); free(tmp); free(w); free(mask); free(m);
}

/* ---- tdeig & helpers (amg_setup.c:2613-2726) ---- */
#define EPS (128 * DBL_EPSILON)
static double sum_3(double a, double b, double c) {
  if ((a >= 0 && b >= 0) || (a <= 0 && b <= 0)) return (a + b) + c;
  else if ((a >= 0 && c >= 0) || (a <= 0 && c <= 0)) return (a + c) + b;
  else return a + (b + c);
}
static double rat_root(double a, double b, double c, double sign) {
  double bh = (fabs(b) + sqrt(b * b + 4 * a * c)) / 2;
  return sign * (b * sign <= 0 ? bh / a : c / bh);
}
static double sec_root(double *y, const double *d, const double *v, int ri, int n) {
  double dl = d[ri], dr = d[ri + 1], L = dr - dl;
  double x0l = L / 2, x0r = -L / 2;
  double al, ar, bln, blp, brn, brp, cl, cr, fn, fp, lambda0, lambda;
  double tol = L;
  if (fabs(dl) > tol) tol = fabs(dl);
  if (fabs(dr) > tol) tol = fabs(dr);
  tol *= EPS;
  for (;;) {
    if (fabs(x0l) == 0 || x0l < 0) { *y = 0; return dl; }
    if (fabs(x0r) == 0 || x0r > 0) { *y = 0; return dr; }
    lambda0 = fabs(x0l) < fabs(x0r) ? dl + x0l : dr + x0r;
    al = ar = cl = cr = bln = blp = brn = brp = 0;
    fn = fp = 0;
    for (int i = 1; i <= ri; ++i) {
      double den = (d[i] - dl) - x0l, fac = v[i] / den, num = sum_3(d[i], -dr, -2 * x0r);
      fn += v[i] * fac; fac *= fac; ar += fac;
      if (num > 0) brp += fac * num; else brn += fac * num;
      bln += fac * (d[i] - dl);
      cl += fac * x0l * x0l;
    }
    for (int i = ri + 1; i <= n; ++i) {
      double den = (d[i] - dr) - x0r, fac = v[i] / den, num = sum_3(d[i], -dl, -2 * x0l);
      fp += v[i] * fac; fac *= fac; al += fac;
      if (num > 0) blp += fac * num; else bln += fac * num;
      brp += fac * (d[i] - dr);
      cr += fac * x0r * x0r;
    }
    if (lambda0 > 0) fp += lambda0; else fn += lambda0;
    if (v[0] < 0) fp -= v[0], blp -= v[0], brp -= v[0];
    else fn -= v[0], bln -= v[0], brn -= v[0];
    if (fp + fn > 0) {
      x0l = rat_root(1 + al, sum_3(dl, blp, bln), cl, 1);
      lambda = dl + x0l; x0r = x0l - L;
    } else {
      x0r = rat_root(1 + ar, sum_3(dr, brp, brn), cr, -1);
      lambda = dr + x0r; x0l = x0r + L;
    }
    if (fabs(lambda - lambda0) < tol) {
      double ty = 0, fac;
      for (int i = 1; i <= ri; ++i) fac = v[i] / ((d[i] - dl) - x0l), ty += fac * fac;
      for (int i = ri + 1; i <= n; ++i) fac = v[i] / ((d[i] - dr) - x0r), ty += fac * fac;
      *y = 1 / sqrt(1 + ty);
      return lambda;
    }
  }
}
static void tdeig(double *lambda, double *y, double *d, const double *v, int n) {
  double v1norm = 0, mn = v[0], mx = v[0];
  for (int i = 1; i <= n; ++i) {
    double vi = fabs(v[i]), a = d[i] - vi, b = d[i] + vi;
    v1norm += vi;
    if (a < mn) mn = a;
    if (b > mx) mx = b;
  }
  d[0] = v[0] - v1norm < mn ? v[0] - v1norm : mn;
  d[n + 1] = v[0] + v1norm > mx ? v[0] + v1norm : mx;
  for (int i = 0; i <= n; ++i) lambda[i] = sec_root(&y[i], d, v, i, n);
}

/* lanczos (amg_setup.c:2435); start vector from libc rand() like the reference */
static u32 lanczos(double **lambda, const ocsr *A) {
  u32 rn = A->rn;
  double *r = NEW(double, rn);
  for (u32 i = 0; i < rn; i++) r[i] = (double)rand() / (double)RAND_MAX;
  const u32 kmax = 299;
  double *l = *lambda = NEW(double, kmax);
  double *y = NEW(double, kmax), *d = NEW(double, kmax + 1), *v = NEW(double, kmax);
  double beta = norm2(r, rn), beta2 = beta * beta;
  beta = sqrt(beta2);
  u32 k = 0;
  double change;
  /* norm(A - I, 'fro') over the stored values (dminus on the first diagonal) */
  {
    double fr = 0;
    for (u32 i = 0; i < rn; i++) {
      int done = 0;
      for (u64 j = A->ro[i]; j < A->ro[i + 1]; j++) {
        double a = A->a[j];
        if (!done && A->col[j] == i) { a = a - 1.; done = 1; }
        fr += a * a;
      }
    }
    double fronorm = sqrt(fr), fronorm2 = fronorm * fronorm;
    fronorm = sqrt(fronorm2);
    if (fronorm < 1e-11) { l[0] = 1; l[1] = 1; y[0] = 0; y[1] = 0; k = 2; change = 0.0; }
    else change = 1.0;
  }
  if (rn == 1) { double a00 = A->a[0]; l[0] = a00; l[1] = a00; y[0] = 0; y[1] = 0; k = 2; change = 0.0; }
  double *qk = NEW(double, A->cn), *qkm1 = NEW(double, rn), *aq = NEW(double, rn), *Aqk = NEW(double, rn);
  for (u32 i = 0; i < A->cn; i++) qk[i] = 0.;
  while (k < kmax && (change > 1e-5 || y[0] > 1e-3 || y[k - 1] > 1e-3)) {
    k++;
    memcpy(qkm1, qk, rn * sizeof(double));
    double sc = 1. / beta;
    for (u32 i = 0; i < rn; i++) qk[i] = r[i] * sc;
    apply_M(Aqk, 0, NULL, 1, A, qk);
    double alpha = vv_dot(qk, Aqk, rn);
    for (u32 i = 0; i < rn; i++) {
      aq[i] = qk[i] * alpha;
      qkm1[i] = qkm1[i] * beta;
      r[i] = Aqk[i];
      r[i] = r[i] - aq[i];
      r[i] = r[i] - qkm1[i];
    }
    if (k == 1) { l[0] = alpha; y[0] = 1; }
    else {
      double l0 = l[0], lkm2 = l[k - 2];
      d[0] = 0;
      for (u32 i = 1; i < k; i++) d[i] = l[i - 1];
      d[k] = 0;
      v[0] = alpha;
      for (u32 i = 1; i < k; i++) v[i] = beta * y[i - 1];
      tdeig(l, y, d, v, (int)k - 1);
      change = fabs(l0 - l[0]) + fabs(lkm2 - l[k - 1]);
    }
    beta = norm2(r, rn); beta2 = beta * beta; beta = sqrt(beta2);
    if (beta == 0) break;
  }
  u32 nl = 0;
  for (u32 i = 0; i < k; i++) if (y[i] < 0.01) (*lambda)[nl++] = l[i];
  free(r); free(qk); free(qkm1); free(aq); free(Aqk); free(y); free(d); free(v);
  return nl;
}

/* chebsim (amg_setup.c:2412) */
static void chebsim(double *m, double *c, double rho, double tol) {
  double alpha = 0.25 * rho * rho, cp = 1, gamma = 1, d, cn;
  *m = 1; *c = rho;
  while (*c > tol) {
    *m += 1;
    d = alpha * (1 + gamma);
    gamma = d / (1 - d);
    cn = (1 + gamma) * rho * (*c) - gamma * cp;
    cp = *c; *c = cn;
  }
}

/* pcg (amg_setup.c:2242); M multiplies (z = M.*r), r is overwritten */
static double g_pcg_rho, g_pcg_stop;     /* last pcg's final rho and stop level (trace) */
static u64 g_offrow;                     /* sp_add landings past row j's end (trace) */
static u32 pcg(double *x, const ocsr *A, double *r, const double *M, double tol, const double *b) {
  u32 rn = A->rn;
  for (u32 i = 0; i < rn; i++) x[i] = 0.;
  double *p = NEW(double, A->cn), *z = NEW(double, rn), *w = NEW(double, rn);
  for (u32 i = 0; i < A->cn; i++) p[i] = 0.;
  for (u32 i = 0; i < rn; i++) z[i] = M[i] * r[i];
  double rho = vv_dot(r, z, rn), rho_0 = 0;
  for (u32 i = 0; i < rn; i++) rho_0 += (M[i] * b[i]) * b[i];
  double rho_stop = tol * tol * rho_0;
  u32 n = rn <= 100 ? rn : 100, k = 0;
  if (n == 0) { free(p); free(z); free(w); return 0; }
  double rho_old = 1, alpha, beta;
  while (rho > rho_stop && k < n) {
    k++;
    beta = rho / rho_old;
    for (u32 i = 0; i < rn; i++) { p[i] = p[i] * beta; p[i] = p[i] + z[i]; }
    apply_M(w, 0, NULL, 1, A, p);
    alpha = vv_dot(p, w, rn);
    alpha = rho / alpha;
    for (u32 i = 0; i < rn; i++) {
      x[i] = x[i] + p[i] * alpha;
      r[i] = r[i] - w[i] * alpha;
      z[i] = M[i] * r[i];
    }
    rho_old = rho;
    rho = vv_dot(r, z, rn);
  }
  g_pcg_rho = rho;
  g_pcg_stop = rho_stop;
  free(p); free(z); free(w);
  return k;
}

/* min_skel (amg_setup.c:2198): one entry per row at the first max, value 1 if max>0 */
static ocsr *min_skel(const ocsr *R) {
  ocsr *W = csr_new(R->rn, R->cn, R->rn);
  for (u32 i = 0; i < R->rn; i++) {
    double ym = -DBL_MAX; u32 j = 0;
    for (u64 k = R->ro[i]; k < R->ro[i + 1]; k++) if (R->a[k] > ym) { ym = R->a[k]; j = R->col[k]; }
    W->a[i] = ym > 0.0 ? 1.0 : 0.0;
    W->col[i] = j;
    W->ro[i + 1] = i + 1;
  }
  return W;
}

/* ---- interp (amg_setup.c:2053) / interp_lmop (amg_setup.c:1589) ----
 * Per row i of Wt (a coarse point), Q is the packed upper-triangular
 * A-orthonormalisation of A restricted to the support Qj (sorted). */

/* sp_restrict_sorted (amg_setup.c:2180): y[m] = x at index Ri[m] (first match) or 0 */
static void sp_restrict_sorted(double *y, u32 Rn, const u32 *Ri, u64 xn, const u32 *xi, const double *x) {
  u32 m = 0; u64 t = 0;
  if (Rn == 0) return;
  while (t < xn && m < Rn) {
    if (Ri[m] < xi[t]) { y[m++] = 0; continue; }
    if (Ri[m] == xi[t]) { y[m++] = x[t]; }
    t++;
  }
  while (m < Rn) y[m++] = 0;
}
/* mv_utt (amg_setup.c:2122): y[i] = sum_{j<=i} U[tri(i)+j] x[j], i<n */
static void mv_utt(double *y, u32 n, const double *U, const double *x) {
  for (u32 i = 0; i < n; i++) {
    double v = 0;
    for (u32 j = 0; j <= i; j++) v += (*U++) * x[j];
    y[i] = v;
  }
}
/* mv_ut (amg_setup.c:2138) */
static void mv_ut(double *y, u32 n, const double *U, const double *x) {
  for (u32 j = 0; j < n; ++j) {
    y[j] = 0;
    for (u32 i = 0; i <= j; ++i) y[i] += (*U++) * x[j];
  }
}
/* build Q for one support; Q has nz(nz+1)/2 entries, sqv1/sqv2 scratch nz */
static void build_Q(double *Q, const u32 *Qj, u32 nz, const ocsr *At, double *sqv1, double *sqv2) {
  double *qk = Q;
  for (u32 k = 0; k < nz; ++k, qk += k) {
    u32 s = Qj[k];
    sp_restrict_sorted(sqv1, k + 1, Qj, At->ro[s + 1] - At->ro[s], &At->col[At->ro[s]], &At->a[At->ro[s]]);
    mv_utt(sqv2, k, Q, sqv1);
    mv_ut(qk, k, Q, sqv2);
    double alpha = sqv1[k];
    for (u32 m = 0; m < k; ++m) alpha -= sqv1[m] * qk[m];
    alpha = -1.0 / sqrt(alpha);
    for (u32 m = 0; m < k; ++m) qk[m] *= alpha;
    qk[k] = -alpha;
  }
}
/* kernel-level checker (tests/test_gpu_kernels.py): Q factors of every row of
 * Wt (supports) against At, packed one after another in row order */
API void oracle_qfactor(u32 wrn, const u64 *wro, const u32 *wcol, u32 arn, const u64 *aro,
                        const u32 *acol, const double *aa, double *Q) {
  ocsr At = {arn, arn, (u64 *)aro, (u32 *)acol, (double *)aa};
  u64 off = 0;
  for (u32 c = 0; c < wrn; c++) {
    u32 nz = (u32)(wro[c + 1] - wro[c]);
    double *s1 = NEW(double, nz + 1), *s2 = NEW(double, nz + 1);
    build_Q(Q + off, wcol + wro[c], nz, &At, s1, s2);
    free(s1); free(s2);
    off += (u64)nz * (nz + 1) / 2;
  }
}
static u32 max_row(const ocsr *A) {
  u32 mx = 0;
  for (u32 i = 0; i < A->rn; i++) { u64 l = A->ro[i + 1] - A->ro[i]; if (l > mx) mx = (u32)l; }
  return mx;
}
static void interp(ocsr *Wt, const ocsr *At, const ocsr *Bt, const double *u, const double *lambda) {
  u32 mz = max_row(Wt);
  double *sqv1 = NEW(double, mz + 1), *sqv2 = NEW(double, mz + 1), *Q = NEW(double, (u64)mz * (mz + 1) / 2 + 1);
  for (u32 i = 0; i < Wt->rn; i++) {
    u64 wir = Wt->ro[i];
    const u32 *Qj = &Wt->col[wir];
    u32 nz = (u32)(Wt->ro[i + 1] - wir);
    build_Q(Q, Qj, nz, At, sqv1, sqv2);
    sp_restrict_sorted(sqv1, nz, Qj, Bt->ro[i + 1] - Bt->ro[i], &Bt->col[Bt->ro[i]], &Bt->a[Bt->ro[i]]);
    for (u32 k = 0; k < nz; ++k) sqv1[k] += u[i] * lambda[Qj[k]];
    mv_utt(sqv2, nz, Q, sqv1);
    mv_ut(&Wt->a[wir], nz, Q, sqv2);
  }
  free(sqv1); free(sqv2); free(Q);
}
/* sp_add (amg_setup.c:1665): y += alpha*x, walking y's column list forward.
 * The reference never checks the row end: an x index absent from row j lands
 * on the next stored entry whose column is >= it, possibly in a following row
 * of St (this happens whenever the skeleton holds a zero-valued entry from
 * min_skel, i.e. an F row without C neighbours).  We reproduce that walk on
 * the global arrays; only running off the end of St is undefined (counted). */
static void sp_add_ref(ocsr *St, u32 j, double alpha, u32 xn, const u32 *xi, const double *x) {
  u64 t = St->ro[j], end = nnz(St);
  if (St->ro[j + 1] == t) return;
  for (u32 m = 0; m < xn; m++) {
    while (t < end && St->col[t] < xi[m]) t++;
    if (t >= end) { oracle_overflow_events++; return; }
    if (t >= St->ro[j + 1]) g_offrow++;
    St->a[t] += alpha * x[m];
    t++;
  }
}
static void interp_lmop(ocsr *St, const ocsr *At, const double *u, const ocsr *W_skelt) {
  u32 mz = max_row(W_skelt);
  double *sqv1 = NEW(double, mz + 1), *sqv2 = NEW(double, mz + 1);
  double *Q = NEW(double, (u64)mz * (mz + 1) / 2 + 1), *QQt = NEW(double, (u64)mz * mz + 1);
  for (u64 k = 0; k < nnz(St); k++) St->a[k] = 0.0;
  for (u32 i = 0; i < W_skelt->rn; i++) {
    const u32 *Qj = &W_skelt->col[W_skelt->ro[i]];
    u32 nz = (u32)(W_skelt->ro[i + 1] - W_skelt->ro[i]);
    double ui = u[i];
    for (u64 k = 0; k < (u64)nz * nz; k++) QQt[k] = 0;
    double *qk = Q;
    for (u32 k = 0; k < nz; ++k, qk += k) {
      u32 s = Qj[k];
      sp_restrict_sorted(sqv1, k + 1, Qj, At->ro[s + 1] - At->ro[s], &At->col[At->ro[s]], &At->a[At->ro[s]]);
      mv_utt(sqv2, k, Q, sqv1);
      mv_ut(qk, k, Q, sqv2);
      double alpha = sqv1[k];
      for (u32 m = 0; m < k; ++m) alpha -= sqv1[m] * qk[m];
      alpha = -1.0 / sqrt(alpha);
      for (u32 m = 0; m < k; ++m) qk[m] *= alpha;
      qk[k] = -alpha;
      for (u32 m = 0; m <= k; ++m) {
        u64 mnz = (u64)m * nz; double qkm = qk[m];
        for (u32 j = 0; j <= k; ++j) QQt[mnz + j] += qkm * qk[j];
      }
    }
    qk = QQt;
    for (u32 k = 0; k < nz; ++k, qk += nz) {
      sp_add_ref(St, Qj[k], ui, nz, Qj, qk);
    }
  }
  free(sqv1); free(sqv2); free(Q); free(QQt);
}

/* solve_constraint (amg_setup.c:1499) */
static void solve_constraint(double *lam, const ocsr *W_skel, const ocsr *W_skelt, const ocsr *Af,
                             const ocsr *W0, const double *alpha, const double *u, const double *v, double tol) {
  u32 nf = W_skel->rn, nc = W_skel->cn;
  double *au2 = NEW(double, nc);
  for (u32 i = 0; i < nc; i++) { au2[i] = u[i] * u[i]; au2[i] = au2[i] * alpha[i]; }
  ocsr *Wsk_t = transpose(W_skel);         /* mxm(S, W_skel, W_skel, 1.) = W_skel * W_skel^T */
  ocsr *S = spgemm(W_skel, Wsk_t);
  csr_free(&Wsk_t);
  g_offrow = 0;
  const u64 ovf0 = oracle_overflow_events;
  interp_lmop(S, Af, au2, W_skelt);
  const u64 offrow = g_offrow, ovf = oracle_overflow_events - ovf0;
  dump_ocsr("S", S);
  double *resid = NEW(double, nf), *d = NEW(double, nf), *dl = NEW(double, nf);
  apply_M(resid, 1.0, v, -1.0, W0, u);
  diag(d, S);
  int ifall = 0;
  for (u32 i = 0; i < nf; i++) { dl[i] = (d[i] != 0.) ? 1. : 0.; if (dl[i] == 0.) { ifall = 1; lam[i] = 0.; } }
  if (ifall) { ocsr *sub = sub_mat(S, dl, dl); csr_free(&S); S = sub; }
  u32 nco = 0;
  double *lc = NEW(double, nf);
  for (u32 i = 0; i < nf; i++) if (dl[i] != 0.) { resid[nco] = resid[i]; d[nco] = d[i]; lc[nco] = lam[i]; nco++; }
  double *q = NEW(double, nco ? nco : 1), *x = NEW(double, nco ? nco : 1);
  apply_M(q, 1., resid, -1., S, lc);
  for (u32 i = 0; i < nco; i++) d[i] = 1. / d[i];
  const u32 its = pcg(x, S, q, d, tol, resid);
  if (getenv("ORACLE_VERBOSE"))
    printf("   constraint: %u of %u rows, pcg %u its, rho %.9e stop %.9e, sp_add off-row %lu past-end %lu\n",
           nco, nf, its, g_pcg_rho, g_pcg_stop, (unsigned long)offrow, (unsigned long)ovf), fflush(stdout);
  u32 t = 0;
  for (u32 i = 0; i < nf; i++) if (dl[i] != 0.) lam[i] += x[t++];
  csr_free(&S);
  free(au2); free(resid); free(d); free(dl); free(lc); free(q); free(x);
}

/* solve_weights (amg_setup.c:1437) */
static void solve_weights(ocsr **W, ocsr **W0, double *lam, const ocsr *W_skel, const ocsr *Af,
                          const ocsr *Ar, u32 rnc, const double *alpha, const double *u,
                          const double *v, double tol) {
  u32 rnf = Af->rn;
  double *au = NEW(double, rnc), *zeros = NEW(double, rnf);
  for (u32 i = 0; i < rnc; i++) au[i] = alpha[i] * u[i];
  for (u32 i = 0; i < rnf; i++) zeros[i] = 0.0;
  ocsr *W0t = transpose(W_skel);
  ocsr *Amt = transpose(Ar);
  for (u64 k = 0; k < nnz(Amt); k++) Amt->a[k] = Amt->a[k] * -1.0;
  interp(W0t, Af, Amt, au, zeros);
  *W0 = transpose(W0t);
  csr_free(&W0t);
  ocsr *Wt = transpose(W_skel);
  solve_constraint(lam, W_skel, Wt, Af, *W0, alpha, u, v, tol);
  interp(Wt, Af, Amt, au, lam);
  csr_free(&Amt);
  *W = transpose(Wt);
  csr_free(&Wt);
  free(au); free(zeros);
}

/* stable descending sort of (col, val) by val -- glibc qsort is a merge sort
 * here (msort.c), stable, with cmp_coo_v_revert (amg_setup.c:1252) */
typedef struct { u32 j; double v; } cv;
static void msort_desc(cv *a, u32 n, cv *tmp) {
  if (n < 2) return;
  u32 h = n / 2;
  msort_desc(a, h, tmp); msort_desc(a + h, n - h, tmp);
  u32 i = 0, j = h, o = 0;
  while (i < h && j < n) tmp[o++] = (a[j].v > a[i].v) ? a[j++] : a[i++];
  while (i < h) tmp[o++] = a[i++];
  while (j < n) tmp[o++] = a[j++];
  memcpy(a, tmp, n * sizeof(cv));
}

/* find_support (amg_setup.c:1260) -- entries are removed by zeroing their value,
 * which is equivalent for every later use (find_support). */
static ocsr *find_support(const ocsr *R, double goal) {
  u32 nf = R->rn, nc = R->cn;
  u64 nzR = nnz(R);
  ocsr *Rl = csr_copy(R);
  ocsr *Rt = transpose(R);          /* pattern + map CSC position -> CSR position */
  u64 *pos = NEW(u64, nzR ? nzR : 1);
  {
    u64 *cur = NEW(u64, (size_t)nc + 1);
    memcpy(cur, Rt->ro, ((size_t)nc + 1) * sizeof(u64));
    for (u32 i = 0; i < nf; i++) for (u64 k = R->ro[i]; k < R->ro[i + 1]; k++) pos[cur[R->col[k]]++] = k;
    free(cur);
  }
  u64 cap = 1024, ns = 0;
  u32 *si = NEW(u32, cap), *sj = NEW(u32, cap);
  double *rs = NEW(double, nf), *w = NEW(double, nc), *w2 = NEW(double, nc), *tmp = NEW(double, nf);
  double *vv = NEW(double, nc), *sumR = NEW(double, nc), *onec = NEW(double, nc);
  for (u32 i = 0; i < nc; i++) onec[i] = 1.;
  double theta = 0.5;
  for (;;) {
    u64 removed = 0;
    apply_M(rs, 0., NULL, 1., Rl, onec);
    apply_Mt(w, Rl, rs);
    apply_M(tmp, 0., NULL, 1., Rl, w);
    apply_Mt(w2, Rl, tmp);
    for (u32 i = 0; i < nc; i++) { vv[i] = w2[i] / w[i]; if (w[i] == 0.) vv[i] = 0.; }
    double mv = vmax(vv, nc, NULL), mw = mv;      /* reference takes max(v) twice (amg_setup.c:1316-1317) */
    if (mv < goal || mw < goal) break;
    if (getenv("ORACLE_VERBOSE")) printf("  find_support: max v = %g theta=%g\n", mv, theta), fflush(stdout);
    while (mw <= (1 + theta) * goal && theta > 0) theta = theta / 2.;
    if (theta == 0) { oracle_ub_events++; break; }   /* reference spins forever */
    for (u32 c = 0; c < nc; c++) sumR[c] = 0.0;
    for (u64 k = 0; k < nzR; k++) sumR[Rl->col[k]] += Rl->a[k];
    for (u32 c = 0; c < nc; c++) {
      if (!(w[c] > (1 + theta) * goal && sumR[c] != 0.)) continue;
      u32 mi = 0;
      if (nf > 1) {
        double mx = -DBL_MAX;
        for (u64 t = Rt->ro[c]; t < Rt->ro[c + 1]; t++) {
          u64 p = pos[t];
          u32 i = Rt->col[t];
          double x = Rl->a[p] * rs[i];
          if (x > mx) { mx = x; mi = i; }
        }
      } else break;   /* reference: maski = 1 (amg_setup.c:1369), a row outside the
                         1-row matrix, so nothing is ever removed and it loops forever */
      if (ns == cap) { cap *= 2; si = realloc(si, cap * sizeof(u32)); sj = realloc(sj, cap * sizeof(u32)); }
      si[ns] = mi; sj[ns] = c; ns++;
      /* R = R - R.*M: the chosen entry becomes an exact zero and is dropped */
      if (nf > 1)
        for (u64 t = Rt->ro[c]; t < Rt->ro[c + 1]; t++) if (Rt->col[t] == mi) { Rl->a[pos[t]] = 0.0; removed++; break; }
    }
    /* no entry removed: the reference repeats this iteration forever */
    if (removed == 0) { oracle_ub_events++; break; }
  }
  double *ones = NEW(double, ns ? ns : 1);
  for (u64 k = 0; k < ns; k++) ones[k] = 1.;
  ocsr *Sk = build_csr_dim(ns, si, sj, ones, nf, nc);
  csr_free(&Rl); csr_free(&Rt);
  free(pos); free(si); free(sj); free(rs); free(w); free(w2); free(tmp); free(vv); free(sumR); free(onec); free(ones);
  return Sk;
}

/* expand_support (amg_setup.c:907), the dense w x nbad algebra restated per bad row */
static ocsr *expand_support(const ocsr *W_skel, const ocsr *R, const ocsr *R0, double gamma) {
  ocsr *M = find_support(R, gamma);
  u32 nf = W_skel->rn, nc = W_skel->cn;
  ocsr *ns = mpm(1., M, 1., W_skel);
  csr_free(&M);
  double *bad = NEW(double, nf);
  u32 nbad = 0;
  for (u32 i = 0; i < nf; i++) {
    bad[i] = 0.;
    for (u64 j = ns->ro[i]; j < ns->ro[i + 1]; j++) if (ns->a[j] == 2.) { bad[i] = 1.; nbad++; break; }
  }
  if (nbad == 0) {
    for (u64 k = 0; k < nnz(ns); k++) if (ns->a[k] == 2.) ns->a[k] = 1.;
    free(bad);
    return ns;
  }
  ocsr *R0W = mxmpoint(R0, W_skel);
  ocsr *Xf = mpm(1., R0, -1, R0W);
  csr_free(&R0W);
  u32 *ni = NULL, *nj = NULL;
  u64 nn = 0, ncap = 0;
  u32 mrow = max_row(Xf);
  cv *row = NEW(cv, mrow + 1), *tmp = NEW(cv, mrow + 1);
  for (u32 i = 0; i < nf; i++) {
    if (bad[i] == 0.) continue;
    u32 len = 0;
    for (u64 j = Xf->ro[i]; j < Xf->ro[i + 1]; j++) { row[len].j = Xf->col[j]; row[len].v = fabs(Xf->a[j]); len++; }
    msort_desc(row, len, tmp);
    /* S = cumsum over ranks (amg_setup.c:1220), V = sum/2, N = 1 + #{S - V < 0} */
    double tot = 0.0;
    for (u32 p = 0; p < len; p++) if (row[p].v != 0.) tot += row[p].v;
    double V = tot * 0.5;
    u32 cnt = 0;
    if (V != 0.) {
      double s = 0.0;
      for (u32 p = 0; p < len; p++) { if (row[p].v != 0.) s += row[p].v; if (s - V < 0) cnt++; }
    }
    u32 N = cnt + 1;
    for (u32 p = 0; p < len && p < N; p++) {
      if (nn == ncap) { ncap = ncap ? 2 * ncap : 1024; ni = realloc(ni, ncap * sizeof(u32)); nj = realloc(nj, ncap * sizeof(u32)); }
      ni[nn] = i; nj[nn] = row[p].j; nn++;
    }
  }
  free(row); free(tmp); csr_free(&Xf); free(bad);
  double *ones = NEW(double, nn ? nn : 1);
  for (u64 k = 0; k < nn; k++) ones[k] = 1.;
  ocsr *Nm = build_csr_dim(nn, ni, nj, ones, nf, nc);
  free(ni); free(nj); free(ones);
  ocsr *out = mpm(1., ns, 1., Nm);
  csr_free(&Nm); csr_free(&ns);
  for (u64 k = 0; k < nnz(out); k++) if (out->a[k] != 0.) out->a[k] = 1.;
  return out;
}

/* interpolation (amg_setup.c:598) */
static ocsr *interpolation(const ocsr *Af, const ocsr *Ac, const ocsr *Ar, double gamma2, double tol) {
  u32 rnf = Af->rn, rnc = Ac->rn, cnc = Ac->cn, cnr = Ar->cn;
  double *Df = NEW(double, rnf), *Dfinv = NEW(double, rnf);
  diag(Df, Af); diag(Dfinv, Af);
  for (u32 i = 0; i < rnf; i++) Dfinv[i] = 1. / Dfinv[i];
  double *uc = NEW(double, cnr);
  for (u32 i = 0; i < cnr; i++) uc[i] = 1.;
  double *tmp = NEW(double, rnf), *v = NEW(double, rnf), *b = NEW(double, rnf);
  apply_M(tmp, 0, NULL, -1, Ar, uc);
  for (u32 i = 0; i < rnf; i++) b[i] = 1.0;
  pcg(v, Af, tmp, Df, 1e-16, b);
  o_it = 0;
  dump_raw("v", v, rnf * 8);
  double *Dc = NEW(double, cnc), *Dcinv = NEW(double, cnc);
  diag(Dc, Ac); diag(Dcinv, Ac);
  for (u32 i = 0; i < rnc; i++) Dcinv[i] = 1. / Dcinv[i];
  ocsr *ArD = csr_copy(Ar);
  for (u64 k = 0; k < nnz(ArD); k++) ArD->a[k] = ArD->a[k] * ArD->a[k];
  diagcsr_op(ArD, Dfinv, DMULT);
  diagcsr_op(ArD, Dcinv, MULTD);
  ocsr *W_skel = min_skel(ArD);
  csr_free(&ArD);
  if (getenv("ORACLE_VERBOSE")) {
    u32 z = 0, e = 0;
    for (u32 i = 0; i < W_skel->rn; i++) { z += W_skel->a[i] == 0.0; e += Ar->ro[i+1] == Ar->ro[i]; }
    printf("min_skel: %u zero-valued entries, %u empty Ar rows of %u\n", z, e, W_skel->rn);
  }
  double *lam = NEW(double, rnf), *alpha = NEW(double, cnc);
  for (u32 i = 0; i < rnf; i++) lam[i] = 0.;
  memcpy(alpha, Dc, cnc * sizeof(double));
  double *Dfsqrti = Dfinv;
  for (u32 i = 0; i < rnf; i++) Dfsqrti[i] = sqrt(Dfsqrti[i]);
  double *Dcs = NEW(double, cnc), *w1 = NEW(double, cnc), *w2 = NEW(double, cnc), *ones = NEW(double, cnc), *r = NEW(double, cnc);
  for (u32 i = 0; i < cnc; i++) ones[i] = 1.0;
  ocsr *W = NULL;
  u64 prev_nnz = (u64)-1;
  int it = 0;
  for (;;) {
    ocsr *Wtmp, *W0;
    o_it = ++it;
    dump_ocsr("Wskel", W_skel);
    dump_raw("alpha", alpha, cnc * 8);
    dump_raw("lam_in", lam, rnf * 8);
    solve_weights(&Wtmp, &W0, lam, W_skel, Af, Ar, rnc, alpha, uc, v, tol);
    dump_ocsr("W0", W0);
    dump_ocsr("Wtmp", Wtmp);
    dump_raw("lam_out", lam, rnf * 8);
    ocsr *AfW = spgemm(Af, W0);
    ocsr *Arhat0 = mpm(1., AfW, 1., Ar);
    csr_free(&AfW);
    AfW = spgemm(Af, Wtmp);
    ocsr *Arhat = mpm(1., AfW, 1., Ar);
    csr_free(&AfW);
    ocsr *Arr = mpm(1.0, Arhat, 1.0, Ar);
    ocsr *ArW = mxmpoint(Wtmp, Arr);
    csr_free(&Arr);
    for (u32 c = 0; c < cnc; c++) Dcs[c] = 0.0;
    for (u64 k = 0; k < nnz(ArW); k++) Dcs[ArW->col[k]] += ArW->a[k];
    csr_free(&ArW);
    for (u32 c = 0; c < cnc; c++) { Dcs[c] = Dcs[c] + Dc[c]; Dcs[c] = 1. / Dcs[c]; Dcs[c] = sqrt(Dcs[c]); }
    ocsr *R = csr_copy(Arhat);
    diagcsr_op(R, Dfsqrti, DMULT);
    for (u64 k = 0; k < nnz(R); k++) R->a[k] = fabs(R->a[k]);
    diagcsr_op(R, Dcs, MULTD);
    ocsr *R0 = csr_copy(Arhat0);
    diagcsr_op(R0, Dfsqrti, DMULT);
    for (u64 k = 0; k < nnz(R0); k++) R0->a[k] = fabs(R0->a[k]);
    diagcsr_op(R0, Dcs, MULTD);
    apply_M(tmp, 0., NULL, 1., R, ones);
    apply_Mt(w1, R, tmp);
    apply_M(tmp, 0., NULL, 1., R, w1);
    apply_Mt(w2, R, tmp);
    for (u32 c = 0; c < cnc; c++) { r[c] = w2[c] / w1[c]; if (w1[c] == 0) r[c] = 0.; }
    u32 n = 0;
    double maxr = 0.;
    for (u32 c = 0; c < cnc; c++) { if (r[c] > gamma2) n++; if (r[c] > maxr) maxr = r[c]; }
    if (getenv("ORACLE_VERBOSE"))
      printf(" %d nzs, %d cols > %g, worst = %g\n", (int)nnz(W_skel), (int)n, sqrt(gamma2), sqrt(maxr)), fflush(stdout);
    double w1m = vmax(w1, cnc, NULL);
    /* The reference loops forever once expand_support stops adding entries
     * (it only terminates through n==0 || max(w1)<=gamma2).  Stop instead and
     * count the event: such inputs are outside the reference's defined domain. */
    int stalled = prev_nnz == nnz(W_skel);
    if (stalled) oracle_ub_events++;
    prev_nnz = nnz(W_skel);
    if (n == 0 || w1m <= gamma2 || stalled) {
      csr_free(&W0);
      ocsr *Wf;
      solve_weights(&Wf, &W0, lam, W_skel, Af, Ar, rnc, alpha, uc, v, 1e-16);
      double *wuc = NEW(double, rnf);
      apply_M(wuc, 0., NULL, 1., Wf, uc);
      for (u32 i = 0; i < rnf; i++)
        if (wuc[i] != 0.)
          for (u64 j = Wf->ro[i]; j < Wf->ro[i + 1]; j++)
            if (i == Wf->col[j]) { double vw = v[i] / wuc[i]; Wf->a[j] = vw * Wf->a[j]; }
      free(wuc);
      W = Wf;
      csr_free(&Wtmp); csr_free(&W0); csr_free(&Arhat0); csr_free(&Arhat); csr_free(&R0); csr_free(&R);
      break;
    }
    for (u32 c = 0; c < cnc; c++) { double x = w2[c] > 1e-6 ? w2[c] : 1e-6; alpha[c] = Dc[c] / x; }
    ocsr *nsk = expand_support(W_skel, R, R0, gamma2);
    csr_free(&W_skel);
    W_skel = nsk;
    csr_free(&Wtmp); csr_free(&W0); csr_free(&Arhat0); csr_free(&Arhat); csr_free(&R0); csr_free(&R);
  }
  csr_free(&W_skel);
  free(Df); free(Dfinv); free(uc); free(tmp); free(v); free(b); free(Dc); free(Dcinv);
  free(lam); free(alpha); free(Dcs); free(w1); free(w2); free(ones); free(r);
  return W;
}

/* ---- ABI conversion ---- */
static struct csr_mat *to_abi(const ocsr *A) {
  struct csr_mat *M = NEW(struct csr_mat, 1);
  u64 z = nnz(A);
  M->rn = A->rn; M->cn = A->cn;
  M->row_off = NEW(amg_uint, (size_t)A->rn + 1);
  M->col = NEW(amg_uint, z);
  M->a = NEW(double, z);
  for (u32 i = 0; i <= A->rn; i++) M->row_off[i] = A->ro[i];
  for (u64 k = 0; k < z; k++) { M->col[k] = A->col[k]; M->a[k] = A->a[k]; }
  return M;
}
static void free_abi(struct csr_mat **M) {
  if (*M) { free((*M)->row_off); free((*M)->col); free((*M)->a); free(*M); *M = NULL; }
}

/* amg_setup (amg_setup.c:60) */
API void amg_setup(amg_uint n, const amg_uint *Ai, const amg_uint *Aj, const double *Av,
                   struct amg_setup_data *data) {
  ocsr *A = build_csr(n, Ai, Aj, Av);
  double tol = 0.5, ctol = 0.7, itol = 1e-4;
  double gamma2 = 1. - sqrt(1. - tol), gamma = sqrt(gamma2);
  data->tolc = ctol; data->gamma = gamma;
  u32 cap = 100;
  data->n = NEW(double, cap); data->nnz = NEW(double, cap);
  data->nnzf = NEW(double, cap); data->nnzfp = NEW(double, cap);
  data->m = NEW(double, cap); data->rho = NEW(double, cap);
  data->id = NEW(amg_uint, A->rn);
  data->idc = NEW(amg_uint *, cap); data->idf = NEW(amg_uint *, cap);
  data->C = NEW(double *, cap); data->F = NEW(double *, cap); data->D = NEW(double *, cap);
  data->A = NEW(struct csr_mat *, cap); data->Af = NEW(struct csr_mat *, cap);
  data->W = NEW(struct csr_mat *, cap); data->AfP = NEW(struct csr_mat *, cap);
  for (u32 k = 0; k < A->rn; k++) data->id[k] = k + 1;
  u32 level = 0;
  for (;;) {
    if (level + 1 >= cap) {
      cap *= 2;
#define GROW(p, T) p = realloc(p, sizeof(T) * cap)
      GROW(data->n, double); GROW(data->nnz, double); GROW(data->nnzf, double); GROW(data->nnzfp, double);
      GROW(data->m, double); GROW(data->rho, double); GROW(data->idc, amg_uint *); GROW(data->idf, amg_uint *);
      GROW(data->C, double *); GROW(data->F, double *); GROW(data->D, double *);
      GROW(data->A, struct csr_mat *); GROW(data->Af, struct csr_mat *);
      GROW(data->W, struct csr_mat *); GROW(data->AfP, struct csr_mat *);
#undef GROW
    }
    u32 rn = A->rn, cn = A->cn;
    data->n[level] = cn;
    data->nnz[level] = (double)nnz(A);
    data->A[level] = to_abi(A);
    o_lvl = (int)level;
    if (getenv("ORACLE_VERBOSE")) printf("Level %u, dim(A) = %u, nnz = %lu\n", level + 1, cn, (unsigned long)nnz(A)), fflush(stdout);
    if (cn <= 1) {
      data->nullspace = 0;
      if (A->a[0] < 1e-9) data->nullspace = 1;
      break;
    }
    double *vc = NEW(double, rn), *vf = NEW(double, rn);
    coarsen(vc, A, ctol);
    if (getenv("ORACLE_VERBOSE")) printf("coarsened\n"), fflush(stdout);
    for (u32 i = 0; i < cn; i++) vf[i] = (vc[i] == 0.) ? 1. : 0.;
    data->C[level] = NEW(double, rn); memcpy(data->C[level], vc, rn * sizeof(double));
    data->F[level] = NEW(double, rn); memcpy(data->F[level], vf, rn * sizeof(double));
    ocsr *Af = sub_mat(A, vf, vf);
    u32 rnf = Af->rn;
    double *s = NEW(double, rnf), *D = NEW(double, rnf);
    for (u32 i = 0; i < rnf; i++) {
      double t = 0;
      for (u64 j = Af->ro[i]; j < Af->ro[i + 1]; j++) t += Af->a[j] * Af->a[j];
      s[i] = 1. / t;
    }
    diag(D, Af);
    for (u32 i = 0; i < rnf; i++) D[i] = D[i] * s[i];
    if (rnf >= 2) {
      double *Dh = NEW(double, rnf);
      for (u32 i = 0; i < rnf; i++) Dh[i] = sqrt(D[i]);
      ocsr *DAD = csr_copy(Af);
      diagcsr_op(DAD, Dh, DMULT);
      diagcsr_op(DAD, Dh, MULTD);
      double *lambda;
      u32 k = lanczos(&lambda, DAD);
      double a = lambda[0], b = lambda[k - 1];
      double sc = 2. / (a + b);
      for (u32 i = 0; i < rnf; i++) D[i] = D[i] * sc;
      data->D[level] = NEW(double, rnf); memcpy(data->D[level], D, rnf * sizeof(double));
      double rho = (b - a) / (b + a), m, c;
      data->rho[level] = rho;
      chebsim(&m, &c, rho, gamma2);
      data->m[level] = m;
      data->Af[level] = to_abi(Af);
      free(Dh); free(lambda); csr_free(&DAD);
    } else {
      data->D[level] = NEW(double, rnf); memcpy(data->D[level], D, rnf * sizeof(double));
      data->rho[level] = 0; data->m[level] = 1;
      data->Af[level] = to_abi(Af);
    }
    data->nnzf[level] = (double)nnz(Af);
    ocsr *Afc = sub_mat(A, vf, vc), *Ac = sub_mat(A, vc, vc);
    u32 rnc = Ac->rn;
    data->idc[level] = NEW(amg_uint, rnc);
    data->idf[level] = NEW(amg_uint, rnf);
    amg_uint *idl = level == 0 ? data->id : data->idc[level - 1];
    u32 cc = 0, cf = 0;
    for (u32 i = 0; i < rn; i++) { if (vc[i] == 1.) data->idc[level][cc++] = idl[i]; else data->idf[level][cf++] = idl[i]; }
    ocsr *W = interpolation(Af, Ac, Afc, gamma2, itol);
    data->W[level] = to_abi(W);
    ocsr *AfW = spgemm(Af, W);                 /* mxm(AfW, Af, Wt, 1.) */
    ocsr *AfP = mpm(1., AfW, 1., Afc);
    csr_free(&AfW);
    data->AfP[level] = to_abi(AfP);
    data->nnzfp[level] = (double)nnz(AfP);
    ocsr *Wt = transpose(W);
    ocsr *WtAfP = spgemm(Wt, AfP);             /* mxm(WtAfP, Wt, AfP, 0.) */
    ocsr *Acf = transpose(Afc);
    ocsr *AcfW = spgemm(Acf, W);               /* mxm(AcfW, Acf, Wt, 1.) */
    ocsr *Atmp = mpm(1., WtAfP, 1., AcfW);
    csr_free(&A);
    A = mpm(1., Atmp, 1, Ac);
    level++;
    free(vf); free(vc); free(s); free(D);
    csr_free(&Af); csr_free(&Afc); csr_free(&Ac); csr_free(&W); csr_free(&Wt);
    csr_free(&Atmp); csr_free(&Acf); csr_free(&AcfW); csr_free(&AfP); csr_free(&WtAfP);
  }
  data->nlevels = level + 1;
  csr_free(&A);
}

/* ---- amg_export (amg_setup.c:405) and its file writers ---- */
static u32 max_row_nnz(const struct csr_mat *m) {
  u32 mx = 0;
  for (amg_uint i = 0; i < m->rn; i++) { amg_uint l = m->row_off[i + 1] - m->row_off[i]; if (l > mx) mx = (u32)l; }
  return mx;
}
static void savemats(amg_uint *len, amg_uint n, amg_uint nl, const amg_uint *lvl, amg_uint **id,
                     struct csr_mat **mat, const char *fn) {
  const double magic = 3.14159;
  FILE *f = fopen(fn, "w");
  if (!f) { perror(fn); return; }
  fwrite(&magic, sizeof(double), 1, f);
  u32 mx = 0;
  for (amg_uint i = 0; i < nl; i++) { u32 l = max_row_nnz(mat[i]); if (l > mx) mx = l; }
  double *buf = NEW(double, 2 * (size_t)mx + 1);
  amg_uint *row = NEW(amg_uint, nl + 1);
  for (amg_uint i = 0; i < nl; i++) row[i] = 0;
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
  free(row); free(buf);
  fclose(f);
}
API void amg_export(struct amg_setup_data *data) {
  amg_uint nl = data->nlevels, n = (amg_uint)data->n[0];
  amg_uint *lvl = NEW(amg_uint, n);
  for (amg_uint i = 0; i < n; i++) lvl[i] = 1;
  for (amg_uint i = 0; i + 1 < nl; i++) {
    amg_uint m = (amg_uint)data->n[i + 1];
    for (amg_uint j = 0; j < m; j++) lvl[data->idc[i][j] - 1] += 1;
  }
  double *dvec = NEW(double, n);
  for (amg_uint i = 0; i + 1 < nl; i++) {
    amg_uint m = (amg_uint)(data->n[i] - data->n[i + 1]);
    for (amg_uint j = 0; j < m; j++) dvec[data->idf[i][j] - 1] = data->D[i][j];
  }
  amg_uint k = data->idc[nl - 2][0] - 1;
  if (data->nullspace != 0) dvec[k] = 0.;
  else dvec[k] = 1. / data->A[nl - 1]->a[0];
  amg_uint *Wl = NEW(amg_uint, n), *Pl = NEW(amg_uint, n), *Fl = NEW(amg_uint, n);
  savemats(Wl, n, nl - 1, lvl, data->idc, data->W, "amg_W.dat");
  savemats(Pl, n, nl - 1, lvl, data->idc, data->AfP, "amg_AfP.dat");
  savemats(Fl, n, nl - 1, lvl, data->idf, data->Af, "amg_Aff.dat");
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
  }
  free(Wl); free(Pl); free(Fl); free(dvec); free(lvl);
}

API unsigned long oracle_ub_count(void) { return oracle_ub_events; }
API unsigned long oracle_overflow_count(void) { return oracle_overflow_events; }

API void free_data(struct amg_setup_data **data) {
  if (!*data) return;
  struct amg_setup_data *d = *data;
  free(d->n); free(d->nnz); free(d->nnzf); free(d->nnzfp); free(d->m); free(d->rho);
  for (amg_uint i = 0; i < d->nlevels; i++) free_abi(&d->A[i]);
  for (amg_uint i = 0; i + 1 < d->nlevels; i++) {
    free(d->C[i]); free(d->F[i]); free(d->D[i]); free(d->idc[i]); free(d->idf[i]);
    free_abi(&d->Af[i]); free_abi(&d->W[i]); free_abi(&d->AfP[i]);
  }
  free(d->id); free(d->idc); free(d->idf); free(d->C); free(d->F); free(d->D);
  free(d->A); free(d->Af); free(d->W); free(d->AfP);
  free(d);
  *data = NULL;
}
