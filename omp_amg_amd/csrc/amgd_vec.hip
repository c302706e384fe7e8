// amgd_vec.hip -- element-wise kernels (coarsening, Lanczos, PCG, id bookkeeping).
// Each kernel performs the same IEEE operations, in the same order, as the
// reference's vector helpers (amg_setup.c:3164-3342) at the call sites noted.
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cstdio>
#include <algorithm>

#include "amgd.h"
#include "amgd_dev.h"

__global__ void k_vfill(double *a, uint64_t n, double v) { GRID_STRIDE(i, n) a[i] = v; }
extern "C" void amgd_vfill(double *a, uint64_t n, double v) {
  if (n) k_vfill<<<grid_for(n), 256, 0, amgd_s()>>>(a, n, v);
}

__global__ void k_vop(double *c, const double *a, const double *b, uint64_t n, int op) {
  GRID_STRIDE(i, n) {
    double x = a[i], y = b[i], r;
    switch (op) {
      case AMGD_V_MUL: r = x * y; break;
      case AMGD_V_ADD: r = x + y; break;
      case AMGD_V_SUB: r = x - y; break;
      default: r = x / y; break;
    }
    c[i] = r;
  }
}
extern "C" void amgd_vop(double *c, const double *a, const double *b, uint64_t n, int op) {
  if (n) k_vop<<<grid_for(n), 256, 0, amgd_s()>>>(c, a, b, n, op);
}
__global__ void k_vunary(double *a, uint64_t n, int op) {
  GRID_STRIDE(i, n) a[i] = op == AMGD_V_INV ? 1. / a[i] : sqrt(a[i]);
}
extern "C" void amgd_vunary(double *a, uint64_t n, int op) {
  if (n) k_vunary<<<grid_for(n), 256, 0, amgd_s()>>>(a, n, op);
}
__global__ void k_vscale(double *a, uint64_t n, double s) { GRID_STRIDE(i, n) a[i] = a[i] * s; }
extern "C" void amgd_vscale(double *a, uint64_t n, double s) {
  if (n) k_vscale<<<grid_for(n), 256, 0, amgd_s()>>>(a, n, s);
}
__global__ void k_u8f(const uint8_t *m, double *d, uint64_t n) { GRID_STRIDE(i, n) d[i] = m[i] ? 1. : 0.; }
extern "C" void amgd_u8_to_f64(const uint8_t *m, double *d, uint64_t n) {
  if (n) k_u8f<<<grid_for(n), 256, 0, amgd_s()>>>(m, d, n);
}

// idc/idf split (amg_setup.c:321-326): stable partition by the C mask
__global__ void k_mask_u32(const uint8_t *m, uint32_t n, uint32_t *o) { GRID_STRIDE(i, n) o[i] = m[i] ? 1u : 0u; }
__global__ void k_split_ids(const unsigned long *id, const uint8_t *vc, const uint32_t *pre,
                            uint32_t n, unsigned long *idc, unsigned long *idf) {
  GRID_STRIDE(i, n) {
    uint32_t p = pre[i];
    if (vc[i]) idc[p] = id[i];
    else idf[i - p] = id[i];
  }
}
extern "C" void amgd_compact_ids(const unsigned long *id, const uint8_t *vc, uint32_t n,
                                 unsigned long *idc, unsigned long *idf) {
  uint32_t *pre = (uint32_t *)amgd_alloc(((size_t)n + 1) * 4);
  k_mask_u32<<<grid_for(n), 256, 0, amgd_s()>>>(vc, n, pre);
  amgd_scan_u32(pre, n);
  k_split_ids<<<grid_for(n), 256, 0, amgd_s()>>>(id, vc, pre, n, idc, idf);
  amgd_free(pre);
}

// ---------------- Lanczos (amg_setup.c:2522-2582) ----------------
// qkm1 = qk; qk = r * (1/beta)
__global__ void k_lz_step(const double *r, double sc, double *qk, double *qkm1, uint64_t n) {
  GRID_STRIDE(i, n) {
    qkm1[i] = qk[i];
    qk[i] = r[i] * sc;
  }
}
// r = ((Aqk - qk*alpha) - qkm1*beta); qkm1 := qkm1*beta
__global__ void k_lz_resid(double *r, const double *Aqk, const double *qk, double alpha,
                           double *qkm1, double beta, uint64_t n) {
  GRID_STRIDE(i, n) {
    double aq = qk[i] * alpha;
    double q1 = qkm1[i] * beta;
    qkm1[i] = q1;
    double t = Aqk[i];
    t = t - aq;
    r[i] = t - q1;
  }
}
extern "C" void amgd_lanczos_step(const double *r, double sc, double *qk, double *qkm1,
                                  uint64_t n) {
  if (n) k_lz_step<<<grid_for(n), 256, 0, amgd_s()>>>(r, sc, qk, qkm1, n);
}
extern "C" void amgd_lanczos_resid(double *r, const double *Aqk, const double *qk, double alpha,
                                   double *qkm1, double beta, uint64_t n) {
  if (n) k_lz_resid<<<grid_for(n), 256, 0, amgd_s()>>>(r, Aqk, qk, alpha, qkm1, beta, n);
}

// ---------------- PCG (amg_setup.c:2293-2329) ----------------
__global__ void k_pcg_p(double *p, const double *z, double beta, uint64_t n) {
  GRID_STRIDE(i, n) {
    double t = p[i] * beta;
    p[i] = t + z[i];
  }
}
extern "C" void amgd_pcg_p(double *p, const double *z, double beta, uint64_t n) {
  if (n) k_pcg_p<<<grid_for(n), 256, 0, amgd_s()>>>(p, z, beta, n);
}
__global__ void k_pcg_xrz(double *x, double *r, double *z, const double *p, const double *w,
                          const double *M, double alpha, uint64_t n) {
  GRID_STRIDE(i, n) {
    x[i] = x[i] + p[i] * alpha;
    double ri = r[i] - w[i] * alpha;
    r[i] = ri;
    z[i] = M[i] * ri;
  }
}
extern "C" void amgd_pcg_xrz(double *x, double *r, double *z, const double *p, const double *w,
                             const double *M, double alpha, uint64_t n) {
  if (n) k_pcg_xrz<<<grid_for(n), 256, 0, amgd_s()>>>(x, r, z, p, w, M, alpha, n);
}
__global__ void k_vmul(double *z, const double *M, const double *r, uint64_t n) {
  GRID_STRIDE(i, n) z[i] = M[i] * r[i];
}
extern "C" void amgd_vmul_dot_prep(double *z, const double *M, const double *r, uint64_t n) {
  if (n) k_vmul<<<grid_for(n), 256, 0, amgd_s()>>>(z, M, r, n);
}

// ---------------- coarsening (amg_setup.c:2787-2874) ----------------
// w = (1./w1) .* w2; w(w1==0) = 0
__global__ void k_coarsen_w(const double *w1, const double *w2, double *w, uint32_t n) {
  GRID_STRIDE(i, n) {
    double t = 1. / w1[i];
    t = t * w2[i];
    w[i] = w1[i] == 0 ? 0. : t;
  }
}
extern "C" void amgd_coarsen_w(const double *w1, const double *w2, double *w, uint32_t n) {
  if (n) k_coarsen_w<<<grid_for(n), 256, 0, amgd_s()>>>(w1, w2, w, n);
}
// mask = w > ctol^2; x = g .* mask
__global__ void k_mask1(const double *w, double ctol2, const double *g, uint8_t *mask, double *x,
                        uint32_t n) {
  GRID_STRIDE(i, n) {
    uint8_t m = w[i] > ctol2 ? 1 : 0;
    mask[i] = m;
    x[i] = g[i] * (m ? 1. : 0.);
  }
}
extern "C" void amgd_coarsen_mask1(const double *w, double ctol2, const double *g, uint8_t *mask,
                                   double *x, uint32_t n) {
  if (n) k_mask1<<<grid_for(n), 256, 0, amgd_s()>>>(w, ctol2, g, mask, x, n);
}
// mat_max (amg_setup.c:3535) as a gather over S^T, split in two launches:
//   Amax_i = tol * max_{j in row i, f[col]!=0} |a_ij|        (amgd_mat_amax)
//   y_k = max over rows i of column k with f[k]!=0 && |a_ik| >= Amax_i of x_i
//                                                             (amgd_mat_max_gather)
// Both are max-reductions (order-free, exact), so G lanes share a row: G is the
// power of two nearest the mean row length (4..64), each group reduces with
// xor-shuffles inside the wavefront.  Amax depends only on (S, f), so the
// coarsening sweep computes it once for both of its mat_max calls.
template <int G>
__global__ __launch_bounds__(256) void k_amax_g(const uint64_t *ro, const uint32_t *col,
                                                const double *a, uint32_t rn, const uint8_t *f,
                                                double tol, double *amax,
                                                const uint32_t *fs, uint32_t fb, uint32_t fr) {
  const uint32_t sub = threadIdx.x & (G - 1);
  const uint64_t g0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) / G;
  const uint64_t gs = (uint64_t)gridDim.x * (256 / G);
  for (uint64_t i = g0; i < rn; i += gs) {
    if (fs && fs[i] - fb > fr) continue;        // row filter (group-uniform)
    double m = 0;
    for (uint64_t k = ro[i] + sub; k < ro[i + 1]; k += G) {
      double v = fabs(a[k]);
      if (f[col[k]] != 0 && v > m) m = v;
    }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) { double u = __shfl_xor(m, o, 64); m = u > m ? u : m; }
    if (sub == 0) amax[i] = m * tol;
  }
}
template <int G>
__global__ __launch_bounds__(256) void k_matmax_gather_g(const uint64_t *tro, const uint32_t *tcol,
                                                         const double *ta, uint32_t n,
                                                         const uint8_t *f, const double *x,
                                                         const double *amax, double *y,
                                                         const uint32_t *fs, uint32_t fb,
                                                         uint32_t fr) {
  const uint32_t sub = threadIdx.x & (G - 1);
  const uint64_t g0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) / G;
  const uint64_t gs = (uint64_t)gridDim.x * (256 / G);
  for (uint64_t k = g0; k < n; k += gs) {
    if (fs && fs[k] - fb > fr) continue;        // row filter (group-uniform)
    double m = -DBL_MAX;
    if (f[k] != 0)
      for (uint64_t t = tro[k] + sub; t < tro[k + 1]; t += G) {
        uint32_t i = tcol[t];
        if (fabs(ta[t]) < amax[i]) continue;
        double xi = x[i];
        if (xi > m) m = xi;
      }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) { double u = __shfl_xor(m, o, 64); m = u > m ? u : m; }
    if (sub == 0) y[k] = m;
  }
}
static int lanes_for(uint64_t nnz, uint64_t rn) {
  uint64_t avg = rn ? (nnz + rn - 1) / rn : 1;
  int G = 4;
  while (G < 64 && (uint64_t)G * 2 <= avg) G <<= 1;
  return G;
}
#define MM_LAUNCH(KER, G, n, ...)                                                              \
  do {                                                                                         \
    int gb_ = grid_for((uint64_t)(n) * (G), 256, 65536);                                       \
    KER<G><<<gb_, 256, 0, amgd_s()>>>(__VA_ARGS__);                                            \
  } while (0)
#define MM_DISPATCH(KER, G, n, ...)                                                            \
  switch (G) {                                                                                 \
    case 4: MM_LAUNCH(KER, 4, n, __VA_ARGS__); break;                                          \
    case 8: MM_LAUNCH(KER, 8, n, __VA_ARGS__); break;                                          \
    case 16: MM_LAUNCH(KER, 16, n, __VA_ARGS__); break;                                        \
    case 32: MM_LAUNCH(KER, 32, n, __VA_ARGS__); break;                                        \
    default: MM_LAUNCH(KER, 64, n, __VA_ARGS__); break;                                        \
  }
extern "C" void amgd_mat_amax(const dcsr *S, const uint8_t *f, double tol, double *amax) {
  if (!S->rn) return;
  int G = lanes_for(S->nnz, S->rn);
  MM_DISPATCH(k_amax_g, G, S->rn, S->ro, S->col, S->a, S->rn, f, tol, amax, nullptr, 0u, 0u);
  KCHECK();
}
// the same two launches restricted to rows i with fs[i] - fb <= fr
extern "C" void amgd_mat_amax_filt(const dcsr *S, const uint8_t *f, double tol, double *amax,
                                   const uint32_t *fs, uint32_t fb, uint32_t fr) {
  if (!S->rn) return;
  int G = lanes_for(S->nnz, S->rn);
  MM_DISPATCH(k_amax_g, G, S->rn, S->ro, S->col, S->a, S->rn, f, tol, amax, fs, fb, fr);
  KCHECK();
}
extern "C" void amgd_mat_max_gather_filt(const dcsr *St, const uint8_t *f, const double *x,
                                         const double *amax, double *y, const uint32_t *fs,
                                         uint32_t fb, uint32_t fr) {
  if (!St->rn) return;
  int G = lanes_for(St->nnz, St->rn);
  MM_DISPATCH(k_matmax_gather_g, G, St->rn, St->ro, St->col, St->a, St->rn, f, x, amax, y, fs, fb,
              fr);
  KCHECK();
}
extern "C" void amgd_mat_max_gather(const dcsr *St, const uint8_t *f, const double *x,
                                    const double *amax, double *y) {
  if (!St->rn) return;
  int G = lanes_for(St->nnz, St->rn);
  MM_DISPATCH(k_matmax_gather_g, G, St->rn, St->ro, St->col, St->a, St->rn, f, x, amax, y,
              nullptr, 0u, 0u);
  KCHECK();
}
extern "C" void amgd_mat_max(const dcsr *S, const dcsr *St, const uint8_t *f, const double *x,
                             double tol, double *amax, double *y) {
  amgd_mat_amax(S, f, tol, amax);
  amgd_mat_max_gather(St, f, x, amax, y);
}
// g = g - m; mask = mask & (g >= 0); g = id; x = mask .* id
__global__ void k_mask2(double *g, const double *m, uint8_t *mask, double *x, uint32_t n) {
  GRID_STRIDE(i, n) {
    double gi = g[i] - m[i];
    uint8_t mk = (mask[i] && gi >= 0.) ? 1 : 0;
    mask[i] = mk;
    double id = (double)i + 1.0;
    g[i] = id;
    x[i] = (mk ? 1. : 0.) * id;
  }
}
extern "C" void amgd_coarsen_mask2(double *g, const double *m, uint8_t *mask, double *x,
                                   uint32_t n) {
  if (n) k_mask2<<<grid_for(n), 256, 0, amgd_s()>>>(g, m, mask, x, n);
}
// mask = mask & (id - m > 0); vc |= mask; vf ^= mask; anyvc
__global__ void k_mask3(const double *m, uint8_t *mask, uint8_t *vc, uint8_t *vf, double *vfd,
                        uint32_t n, uint32_t *anyvc) {
  GRID_STRIDE(i, n) {
    double gi = ((double)i + 1.0) - m[i];
    uint8_t mk = (mask[i] && gi > 0.) ? 1 : 0;
    mask[i] = mk;
    uint8_t c = (vc[i] || mk) ? 1 : 0;
    vc[i] = c;
    if (c) *anyvc = 1;
    uint8_t f = (vf[i] != mk) ? 1 : 0;
    vf[i] = f;
    vfd[i] = f ? 1. : 0.;
  }
}
extern "C" void amgd_coarsen_mask3(const double *m, uint8_t *mask, uint8_t *vc, uint8_t *vf,
                                   double *vfd, uint32_t n, uint32_t *anyvc) {
  if (n) k_mask3<<<grid_for(n), 256, 0, amgd_s()>>>(m, mask, vc, vf, vfd, n, anyvc);
}

// ---------------- misc ----------------
__global__ void k_vdiv_guard(double *r, const double *num, const double *den, uint64_t n) {
  GRID_STRIDE(i, n) {
    double t = num[i] / den[i];
    r[i] = den[i] == 0 ? 0. : t;
  }
}
extern "C" void amgd_vdiv_guard(double *r, const double *num, const double *den, uint64_t n) {
  if (n) k_vdiv_guard<<<grid_for(n), 256, 0, amgd_s()>>>(r, num, den, n);
}
// alpha = dc ./ max(w2, 1e-6)   (amg_setup.c:860-865)
__global__ void k_alpha_update(double *alpha, const double *Dc, const double *w2, uint64_t n) {
  GRID_STRIDE(i, n) {
    double x = w2[i] > 1e-6 ? w2[i] : 1e-6;
    alpha[i] = Dc[i] / x;
  }
}
extern "C" void amgd_alpha_update(double *alpha, const double *Dc, const double *w2, uint64_t n) {
  if (n) k_alpha_update<<<grid_for(n), 256, 0, amgd_s()>>>(alpha, Dc, w2, n);
}
__global__ void k_u8_not(const uint8_t *a, uint8_t *b, uint64_t n) { GRID_STRIDE(i, n) b[i] = a[i] ? 0 : 1; }
extern "C" void amgd_u8_not(const uint8_t *a, uint8_t *b, uint64_t n) {
  if (n) k_u8_not<<<grid_for(n), 256, 0, amgd_s()>>>(a, b, n);
}
__global__ void k_u8_nonzero(const double *a, uint8_t *m, uint64_t n) { GRID_STRIDE(i, n) m[i] = a[i] != 0. ? 1 : 0; }
extern "C" void amgd_u8_nonzero(const double *a, uint8_t *m, uint64_t n) {
  if (n) k_u8_nonzero<<<grid_for(n), 256, 0, amgd_s()>>>(a, m, n);
}
extern "C" uint64_t amgd_u8_count(const uint8_t *m, uint64_t n) {
  if (!n) return 0;
  uint32_t *map = (uint32_t *)amgd_alloc((n + 1) * 4);
  uint32_t c = amgd_mask_rank(m, (uint32_t)n, map);
  amgd_free(map);
  return c;
}
__global__ void k_vcompact(double *dst, const double *src, const uint8_t *mask, const uint32_t *map,
                           uint64_t n) {
  GRID_STRIDE(i, n) if (mask[i]) dst[map[i]] = src[i];
}
__global__ void k_vexpand_add(double *dst, const double *src, const uint8_t *mask,
                              const uint32_t *map, uint64_t n) {
  GRID_STRIDE(i, n) if (mask[i]) dst[i] = dst[i] + src[map[i]];
}
extern "C" void amgd_vcompact(double *dst, const double *src, const uint8_t *mask, uint64_t n) {
  if (!n) return;
  uint32_t *map = (uint32_t *)amgd_alloc((n + 1) * 4);
  amgd_mask_rank(mask, (uint32_t)n, map);
  k_vcompact<<<grid_for(n), 256, 0, amgd_s()>>>(dst, src, mask, map, n);
  amgd_free(map);
}
extern "C" void amgd_vexpand_add(double *dst, const double *src, const uint8_t *mask, uint64_t n) {
  if (!n) return;
  uint32_t *map = (uint32_t *)amgd_alloc((n + 1) * 4);
  amgd_mask_rank(mask, (uint32_t)n, map);
  k_vexpand_add<<<grid_for(n), 256, 0, amgd_s()>>>(dst, src, mask, map, n);
  amgd_free(map);
}
__global__ void k_vzero_where(double *a, const uint8_t *keep, uint64_t n) { GRID_STRIDE(i, n) if (!keep[i]) a[i] = 0.; }
extern "C" void amgd_vzero_where(double *a, const uint8_t *keep, uint64_t n) {
  if (n) k_vzero_where<<<grid_for(n), 256, 0, amgd_s()>>>(a, keep, n);
}
__global__ void k_ids_iota(unsigned long *id, uint64_t n) { GRID_STRIDE(i, n) id[i] = i + 1; }
extern "C" void amgd_ids_iota(unsigned long *id, uint64_t n) {
  if (n) k_ids_iota<<<grid_for(n), 256, 0, amgd_s()>>>(id, n);
}
