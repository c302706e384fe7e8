// amgd_coarsen.hip -- incremental coarsening sweeps (amg_setup.c:2737-2874).
//
// Every quantity of a coarsening sweep is local: row i of g, w1, w2, w, the
// strength masks and both mat_max results depends only on vf within a fixed
// number of hops of i in S's graph (g 1, w1 2, w2 4, w/mask1 4, Amax 1, m1 and
// mask2 5, m2 and mask3 6).  vf changes only at the points a sweep turns into C
// points (D0), so the next sweep's values differ from the last sweep's only
// within 6 hops of D0; everywhere else the persistent per-stage buffers already
// hold exactly what a full recomputation would produce.  A sweep therefore
//   1. grows D0 hop by hop (S and S^T neighbours; the first visit claims a row
//      with a CAS of its stamp to 8*sweep + hop; LDS-aggregated appends),
//   2. recomputes each stage on the rows within its radius, either
//      * list mode (very short rows, level 0 of a 7-point grid): the BFS list is
//        in hop order, so the rows within r hops are its prefix; one thread per
//        row, or
//      * filter mode: each stage's usual kernel with the row filter
//        "stamp - 8*sweep <= radius" -- the SpMV skips 256-row blocks without
//        such a row and recomputes the others whole (same kernel, same
//        arithmetic), the mat_max and elementwise kernels skip rows;
//      the per-row arithmetic is the full kernels' either way (left-to-right
//      sums from +0.0, order-free maxima), and
//   3. writes the new C points (stamp 8*(sweep+1)) as the next sweep's D0 list.
// When the 6-hop set is large the sweep runs the full kernels instead (same
// buffers, same values), so the C/F sets are bit-identical either way.
#include <float.h>
#include "amgd.h"
#include "amgd_dev.h"

#define CS_HOPS 6
#define DIRTY(i) (fs == nullptr || fs[i] - fb <= fr)
// stage rows: LIST -> list[r] for r < n; else every row i < n passing the filter
#define CS_ROWS(i, n)                                                                           \
  for (uint64_t r_ = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r_ < (uint64_t)(n);       \
       r_ += (uint64_t)gridDim.x * blockDim.x)                                                  \
    for (uint32_t i = LIST ? list[r_] : (uint32_t)r_, once_ = 1; once_; once_ = 0)              \
      if (LIST || DIRTY(i))

// one BFS hop: frontier = front[cum(r-2) .. cum(r-1)), new rows appended at cum(r-1)+.
// A thread walks one frontier row's S and S^T neighbours; claimed rows are
// gathered in LDS and appended with one global atomic per block and chunk.
#define HOP_CAP 4096
__device__ __forceinline__ void cs_claim(uint32_t i, uint32_t *stamp, uint32_t key,
                                         uint32_t base8, uint32_t *buf, uint32_t *nb,
                                         uint32_t *front, uint32_t hi, uint32_t *cntr) {
  const uint32_t old = stamp[i];
  if (old >= base8 || atomicCAS(&stamp[i], old, key) != old) return;
  const uint32_t p = atomicAdd(nb, 1u);
  if (p < HOP_CAP) buf[p] = i;
  else front[hi + atomicAdd(cntr, 1u)] = i;      // LDS buffer full: direct append
}
__global__ __launch_bounds__(256) void k_cs_hop(const uint64_t *sro, const uint32_t *scol,
                                                const uint64_t *tro, const uint32_t *tcol,
                                                uint32_t *front, uint32_t *cnt, int r,
                                                uint32_t *stamp, uint32_t base8, uint32_t limit) {
  __shared__ uint32_t buf[HOP_CAP];
  __shared__ uint32_t nb, gbase;
  uint32_t lo = 0;
  for (int q = 0; q < r - 1; q++) lo += cnt[q];
  const uint32_t hi = lo + cnt[r - 1];
  if (hi > limit) return;                      // the host falls back to a full sweep
  const uint32_t key = base8 + (uint32_t)r;
  for (uint64_t c = lo + (uint64_t)blockIdx.x * 256; c < hi; c += (uint64_t)gridDim.x * 256) {
    if (threadIdx.x == 0) nb = 0;
    __syncthreads();
    const uint64_t idx = c + threadIdx.x;
    if (idx < hi) {
      const uint32_t j = front[idx];
      for (uint64_t k = sro[j]; k < sro[j + 1]; k++)
        cs_claim(scol[k], stamp, key, base8, buf, &nb, front, hi, &cnt[r]);
      for (uint64_t k = tro[j]; k < tro[j + 1]; k++)
        cs_claim(tcol[k], stamp, key, base8, buf, &nb, front, hi, &cnt[r]);
    }
    __syncthreads();
    const uint32_t m = nb < HOP_CAP ? nb : HOP_CAP;
    if (threadIdx.x == 0) gbase = m ? atomicAdd(&cnt[r], m) : 0u;
    __syncthreads();
    for (uint32_t t = threadIdx.x; t < m; t += 256) front[hi + gbase + t] = buf[t];
    __syncthreads();
  }
}

extern "C" int amgd_cs_grow(const dcsr *S, const dcsr *St, uint32_t *front, uint32_t *cnt_d,
                            uint32_t *stamp, uint32_t base8, uint32_t limit, uint32_t *cum) {
  hipStream_t s = amgd_s();
  const int g = grid_for((uint64_t)S->rn, 256, 4096);
  for (int r = 1; r <= CS_HOPS; r++)
    k_cs_hop<<<g, 256, 0, s>>>(S->ro, S->col, St->ro, St->col, front, cnt_d, r, stamp, base8,
                               limit);
  KCHECK();
  uint32_t c[8];
  amgd_d2h(c, cnt_d, sizeof(c));
  uint32_t t = 0, cu[CS_HOPS + 1];
  for (int r = 0; r <= CS_HOPS; r++) {
    t += c[r];
    cu[r] = t;
    if (t > limit) return 0;                   // cum untouched
  }
  for (int r = 0; r <= CS_HOPS; r++) cum[r] = cu[r];
  return 1;
}

// z_i = (S x)_i * vf_i over listed rows, left-to-right from +0.0: the
// arithmetic of k_spmv with alpha = 0, beta = 1 and a row mask
__global__ void k_cs_spmv_list(const uint64_t *ro, const uint32_t *col, const double *a,
                               const uint32_t *list, uint32_t n, const double *x, double *z,
                               const uint8_t *f) {
  GRID_STRIDE(r, n) {
    const uint32_t i = list[r];
    double t = 0;
    for (uint64_t k = ro[i]; k < ro[i + 1]; k++) {
      const double p = a[k] * x[col[k]];
      t += p;
    }
    double v = 1.0 * t;
    v = v * (f[i] ? 1.0 : 0.0);
    z[i] = v;
  }
}
__global__ void k_cs_amax_list(const uint64_t *ro, const uint32_t *col, const double *a,
                               const uint32_t *list, uint32_t n, const uint8_t *f, double tol,
                               double *amax) {
  GRID_STRIDE(r, n) {
    const uint32_t i = list[r];
    double m = 0;
    for (uint64_t k = ro[i]; k < ro[i + 1]; k++) {
      const double v = fabs(a[k]);
      if (f[col[k]] != 0 && v > m) m = v;
    }
    amax[i] = m * tol;
  }
}
__global__ void k_cs_gather_list(const uint64_t *tro, const uint32_t *tcol, const double *ta,
                                 const uint32_t *list, uint32_t n, const uint8_t *f,
                                 const double *x, const double *amax, double *y) {
  GRID_STRIDE(r, n) {
    const uint32_t k = list[r];
    double m = -DBL_MAX;
    if (f[k] != 0)
      for (uint64_t t = tro[k]; t < tro[k + 1]; t++) {
        const uint32_t i = tcol[t];
        if (fabs(ta[t]) < amax[i]) continue;
        const double xi = x[i];
        if (xi > m) m = xi;
      }
    y[k] = m;
  }
}
// w = (1./w1).*w2, w(w1==0) = 0; mask1 = w > ctol^2; x1 = g.*mask1  (k_coarsen_w + k_mask1)
template <bool LIST>
__global__ void k_cs_w_mask1(const uint32_t *list, uint32_t n, const double *w1, const double *w2,
                             double *w, double ctol2, const double *g, uint8_t *ma, double *x1,
                             const uint32_t *fs, uint32_t fb, uint32_t fr) {
  CS_ROWS(i, n) {
    double t = 1. / w1[i];
    t = t * w2[i];
    const double wi = w1[i] == 0 ? 0. : t;
    w[i] = wi;
    const uint8_t m = wi > ctol2 ? 1 : 0;
    ma[i] = m;
    x1[i] = g[i] * (m ? 1. : 0.);
  }
}
// mask2 = mask1 & (g - m1 >= 0); x2 = mask2 .* id   (k_mask2 without overwriting g)
template <bool LIST>
__global__ void k_cs_mask2(const uint32_t *list, uint32_t n, const double *g, const double *m1,
                           const uint8_t *ma, uint8_t *mb, double *x2, const uint32_t *fs,
                           uint32_t fb, uint32_t fr) {
  CS_ROWS(i, n) {
    const double gi = g[i] - m1[i];
    const uint8_t mk = (ma[i] && gi >= 0.) ? 1 : 0;
    mb[i] = mk;
    x2[i] = (mk ? 1. : 0.) * ((double)i + 1.0);
  }
}
// mask3 = mask2 & (id - m2 > 0); vc |= mask3; vf ^= mask3; new C points -> next D0
template <bool LIST>
__global__ void k_cs_mask3(const uint32_t *list, uint32_t n, const double *m2, const uint8_t *mb,
                           uint8_t *vc, uint8_t *vf, double *vfd, uint32_t *anyvc, uint32_t *d0,
                           uint32_t *d0cnt, uint32_t *stamp, uint32_t next_base8,
                           const uint32_t *fs, uint32_t fb, uint32_t fr) {
  // wave-uniform trip count (wave_append needs every lane)
  for (uint64_t rb = (uint64_t)blockIdx.x * blockDim.x; rb < (uint64_t)n;
       rb += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = rb + threadIdx.x;
    bool mk = false;
    uint32_t i = 0;
    if (r < n) {
      i = LIST ? list[r] : (uint32_t)r;
      if (LIST || DIRTY(i)) {
        const double gi = ((double)i + 1.0) - m2[i];
        mk = mb[i] && gi > 0.;
        if (mk) {
          vc[i] = 1;
          *anyvc = 1;
          const uint8_t fv = vf[i] ? 0 : 1;
          vf[i] = fv;
          vfd[i] = fv ? 1. : 0.;
          stamp[i] = next_base8;
        }
      }
    }
    const unsigned pos = wave_append(d0cnt, mk);
    if (mk) d0[pos] = i;
  }
}

// launch helpers: rows == NULL -> all rows; rows->list -> its prefix of radius R;
// else the stamp filter of radius R
#define CS_FS(rows) ((rows) ? (rows)->fs : nullptr), ((rows) ? (rows)->fb : 0u)
static inline uint32_t cs_n(const amgd_csrows *rows, uint32_t n, uint32_t R) {
  return rows && rows->list ? rows->cum[R] : n;
}
#define CS_LAUNCH(KER, rows, n, R, ...)                                                         \
  do {                                                                                          \
    const uint32_t nn_ = cs_n(rows, n, R);                                                      \
    if (!nn_) break;                                                                            \
    if (rows && rows->list)                                                                     \
      KER<true><<<grid_for(nn_), 256, 0, amgd_s()>>>(rows->list, nn_, __VA_ARGS__, nullptr,     \
                                                     0u, R);                                    \
    else                                                                                        \
      KER<false><<<grid_for(nn_), 256, 0, amgd_s()>>>(nullptr, nn_, __VA_ARGS__, CS_FS(rows),   \
                                                      R);                                       \
    KCHECK();                                                                                   \
  } while (0)

extern "C" void amgd_cs_spmv(const dcsr *S, const double *x, double *z, const uint8_t *f,
                             const amgd_csrows *rows, uint32_t R) {
  if (!rows) { amgd_spmv(S, x, z, 0.0, NULL, 1.0, f); return; }
  if (rows->list) {
    const uint32_t n = rows->cum[R];
    if (n) k_cs_spmv_list<<<grid_for(n), 256, 0, amgd_s()>>>(S->ro, S->col, S->a, rows->list, n,
                                                             x, z, f);
    KCHECK();
    return;
  }
  amgd_spmv_filt(S, x, z, f, rows->fs, rows->fb, R);
}
extern "C" void amgd_cs_amax(const dcsr *S, const uint8_t *f, double tol, double *amax,
                             const amgd_csrows *rows, uint32_t R) {
  if (!rows) { amgd_mat_amax(S, f, tol, amax); return; }
  if (rows->list) {
    const uint32_t n = rows->cum[R];
    if (n) k_cs_amax_list<<<grid_for(n), 256, 0, amgd_s()>>>(S->ro, S->col, S->a, rows->list, n,
                                                             f, tol, amax);
    KCHECK();
    return;
  }
  amgd_mat_amax_filt(S, f, tol, amax, rows->fs, rows->fb, R);
}
extern "C" void amgd_cs_gather(const dcsr *St, const uint8_t *f, const double *x,
                               const double *amax, double *y, const amgd_csrows *rows,
                               uint32_t R) {
  if (!rows) { amgd_mat_max_gather(St, f, x, amax, y); return; }
  if (rows->list) {
    const uint32_t n = rows->cum[R];
    if (n) k_cs_gather_list<<<grid_for(n), 256, 0, amgd_s()>>>(St->ro, St->col, St->a,
                                                               rows->list, n, f, x, amax, y);
    KCHECK();
    return;
  }
  amgd_mat_max_gather_filt(St, f, x, amax, y, rows->fs, rows->fb, R);
}
extern "C" void amgd_cs_w_mask1(uint32_t n, const double *w1, const double *w2, double *w,
                                double ctol2, const double *g, uint8_t *ma, double *x1,
                                const amgd_csrows *rows, uint32_t R) {
  CS_LAUNCH(k_cs_w_mask1, rows, n, R, w1, w2, w, ctol2, g, ma, x1);
}
extern "C" void amgd_cs_mask2(uint32_t n, const double *g, const double *m1, const uint8_t *ma,
                              uint8_t *mb, double *x2, const amgd_csrows *rows, uint32_t R) {
  CS_LAUNCH(k_cs_mask2, rows, n, R, g, m1, ma, mb, x2);
}
extern "C" void amgd_cs_mask3(uint32_t n, const double *m2, const uint8_t *mb, uint8_t *vc,
                              uint8_t *vf, double *vfd, uint32_t *anyvc, uint32_t *d0,
                              uint32_t *d0cnt, uint32_t *stamp, uint32_t next_base8,
                              const amgd_csrows *rows, uint32_t R) {
  CS_LAUNCH(k_cs_mask3, rows, n, R, m2, mb, vc, vf, vfd, anyvc, d0, d0cnt, stamp, next_base8);
}

// ---------------------------------------------------------------------------
// Partitioned mode (amgd_psetup.c): the BFS runs on global-row views of S and S^T in
// which only the rank's own rows hold entries, so each rank expands its own frontier
// rows; after every hop the ranks' new rows are exchanged and claimed here, so every
// rank ends each hop with the same set of rows (stamped with the same hop).
// ---------------------------------------------------------------------------
extern "C" void amgd_cs_hop1(const dcsr *S, const dcsr *St, uint32_t *front, uint32_t *cnt_d, int r,
                             uint32_t *stamp, uint32_t base8, uint32_t limit) {
  const int g = grid_for((uint64_t)S->rn, 256, 4096);
  k_cs_hop<<<g, 256, 0, amgd_s()>>>(S->ro, S->col, St->ro, St->col, front, cnt_d, r, stamp, base8, limit);
  KCHECK();
}
__global__ void k_cs_claim_ext(const uint32_t *ids, uint64_t n, uint32_t *stamp, uint32_t key, uint32_t base8,
                               uint32_t *front, uint32_t hi0, uint32_t *cntr) {
  GRID_STRIDE(t, n) {
    const uint32_t i = ids[t];
    const uint32_t old = stamp[i];
    if (old >= base8 || atomicCAS(&stamp[i], old, key) != old) continue;
    front[hi0 + atomicAdd(cntr, 1u)] = i;
  }
}
// rows ids[0..n) of another rank's hop r: claimed and appended to hop r's segment of
// front (hi0 = the segment's start, cntr = its count)
extern "C" void amgd_cs_claim_ext(const uint32_t *ids, uint64_t n, uint32_t *stamp, uint32_t base8, int r,
                                  uint32_t *front, uint32_t hi0, uint32_t *cntr) {
  if (n) k_cs_claim_ext<<<grid_for(n), 256, 0, amgd_s()>>>(ids, n, stamp, base8 + (uint32_t)r, base8, front, hi0,
                                                          cntr);
  KCHECK();
}
