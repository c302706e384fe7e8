// amgd_lmop.hip -- the constraint operator S of interp_lmop (amg_setup.c:1589-1648),
// row-pull formulation.
//
// Reference: S starts at zero; for every coarse point c (ascending) with support
// Qj (row c of W_skel^T, nz points) and Q factor q_0..q_{nz-1}:
//   QQt[k][m] = sum_{t >= max(k,m)} q_t[k] * q_t[m]     (t ascending, from +0)
//   for k: sp_add walks row Qj[k] of S and adds u_c * QQt[k][m] where it meets
//          column Qj[m]                               (amg_setup.c:1665)
// S is W_skel * W_skel^T with exact zeros dropped (mxm, amg_setup.c:1894).  When
// every W_skel value in column c is nonzero ("clean" c; W_skel values are 0/1),
// every pair (Qj[k], Qj[m]) is a stored entry of S and the walk lands exactly on
// it.  Then
//   S(i, j) = sum over c in row i of W_skel (ascending) of u_c * QQt_c[k_ic][m_jc]
// -- a sparse product of W_skel (values u_c) with per-(i, c) rows of QQt_c,
// accumulated in ascending c: one work-group per row of S pulls its
// contributions in exactly the reference's order, no keys, no sort.
//
// Coarse points whose column holds a zero ("dirty": min_skel puts the F points
// without a C neighbour at column 0 with value 0, amg_setup.c:2198) may land
// off-pattern; they go through the general walk (amgd_lmop_general) first.
// That is order-exact as long as every dirty c precedes every clean c (the
// dirty contributions then open every sum); otherwise, or if any clean
// contribution misses its column, the whole operator takes the general path.
//
// QQt_c (nz x nz, row-major) is formed by a batched lower-triangular
// U^T U kernel: a product term with t < max(k, m) is an exact zero added to
// +0, so summing t from the tile start instead of max(k, m) keeps every bit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "amgd.h"
#include "amgd_dev.h"

__device__ __forceinline__ uint64_t tri2(uint64_t i) { return i * (i + 1) / 2; }

// ---------------------------------------------------------------------------
// classification: dirty[c] = column c of W_skel holds a zero value
// ---------------------------------------------------------------------------
__global__ void k_lmop_classify(const uint64_t *tro, const double *ta, uint32_t nc,
                                uint8_t *dirty, unsigned *st) {
  // st[0] = max dirty c + 1 (0: none), st[1] = min clean nonempty c (~0: none)
  GRID_STRIDE(c, nc) {
    uint64_t a = tro[c], b = tro[c + 1];
    uint8_t d = 0;
    for (uint64_t q = a; q < b; q++)
      if (ta[q] == 0.0) { d = 1; break; }
    dirty[c] = d;
    if (d) atomicMax(&st[0], (unsigned)c + 1u);
    else if (b > a) atomicMin(&st[1], (unsigned)c);
  }
}

// QQt sizes: nz^2 for clean c in [ca, cb), else 0; small/large lists
__global__ void k_qq_size(const uint64_t *tro, const uint8_t *dirty, uint32_t nc, uint32_t ca,
                          uint32_t cb, uint64_t *sz) {
  GRID_STRIDE(c, nc) {
    uint64_t nz = tro[c + 1] - tro[c];
    sz[c] = (c >= ca && c < cb && !dirty[c]) ? nz * nz : 0;
  }
}

#define QQ_SMALL 64
#define QQ_TS 32
// small supports (nz <= 64): one wavefront per coarse point, U in LDS,
// one lane per QQt entry
__global__ __launch_bounds__(64) void k_qq_small(const uint64_t *tro, const uint8_t *dirty,
                                                 uint32_t ca, uint32_t cb, const double *Q,
                                                 const uint64_t *qoff, const uint64_t *qqoff,
                                                 double *QQ) {
  __shared__ double U[QQ_SMALL * (QQ_SMALL + 1) / 2];
  const int lane = threadIdx.x;
  for (uint32_t c = ca + blockIdx.x; c < cb; c += gridDim.x) {
    const uint32_t nz = (uint32_t)(tro[c + 1] - tro[c]);
    if (nz == 0 || nz > QQ_SMALL || dirty[c]) continue;
    const double *Qc = Q + qoff[c];
    const uint32_t tn = nz * (nz + 1) / 2;
    for (uint32_t e = lane; e < tn; e += 64) U[e] = Qc[e];
    __syncthreads();
    double *out = QQ + qqoff[c];
    const uint32_t n2 = nz * nz;
    for (uint32_t idx = lane; idx < n2; idx += 64) {
      const uint32_t k = idx / nz, m = idx - k * nz;
      double acc = 0.0;
      for (uint32_t t = k > m ? k : m; t < nz; t++) {
        const double *ut = U + tri2(t);
        acc += ut[k] * ut[m];
      }
      out[idx] = acc;
    }
    __syncthreads();
  }
}

// large supports: 32x32 tiles of the upper triangle (kt <= mt), 64 lanes, 4x4 per lane;
// the tile list is a prefix over the large coarse points (tp[i] = first tile of lc[i])
__global__ __launch_bounds__(64) void k_qq_tile(const uint32_t *lc, uint32_t nl, const uint64_t *tp,
                                                uint64_t ntiles, const uint64_t *tro,
                                                const double *Q, const uint64_t *qoff,
                                                const uint64_t *qqoff, double *QQ) {
  const int lane = threadIdx.x, tx = lane & 7, ty = lane >> 3;
  for (uint64_t g = blockIdx.x; g < ntiles; g += gridDim.x) {
    uint32_t lo = 0, hi = nl;                      // last i with tp[i] <= g
    while (hi - lo > 1) {
      uint32_t mid = (lo + hi) >> 1;
      if (tp[mid] <= g) lo = mid; else hi = mid;
    }
    const uint32_t c = lc[lo];
    const uint32_t nz = (uint32_t)(tro[c + 1] - tro[c]);
    const uint32_t T = (nz + QQ_TS - 1) / QQ_TS;
    uint64_t r = g - tp[lo];
    uint32_t kt = 0;
    while (r >= T - kt) { r -= T - kt; kt++; }
    const uint32_t mt = kt + (uint32_t)r;
    const double *Qc = Q + qoff[c];
    const uint32_t k0 = kt * QQ_TS + ty * 4, m0 = mt * QQ_TS + tx * 4;
    double acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
      for (int b = 0; b < 4; b++) acc[a][b] = 0.0;
    for (uint32_t t = mt * QQ_TS; t < nz; t++) {
      const double *ut = Qc + tri2(t);
      double av[4], bv[4];
#pragma unroll
      for (int a = 0; a < 4; a++) av[a] = (k0 + a <= t) ? ut[k0 + a] : 0.0;
#pragma unroll
      for (int b = 0; b < 4; b++) bv[b] = (m0 + b <= t) ? ut[m0 + b] : 0.0;
#pragma unroll
      for (int a = 0; a < 4; a++)
#pragma unroll
        for (int b = 0; b < 4; b++) acc[a][b] += av[a] * bv[b];
    }
    double *out = QQ + qqoff[c];
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
      for (int b = 0; b < 4; b++) {
        const uint32_t k = k0 + a, m = m0 + b;
        if (k < nz && m < nz) {
          out[(uint64_t)k * nz + m] = acc[a][b];
          if (kt != mt) out[(uint64_t)m * nz + k] = acc[a][b];
        }
      }
  }
}
__global__ void k_qq_tilecount(const uint32_t *lc, uint32_t nl, const uint64_t *tro, uint64_t *tp) {
  GRID_STRIDE(i, nl) {
    uint32_t c = lc[i];
    uint64_t T = (tro[c + 1] - tro[c] + QQ_TS - 1) / QQ_TS;
    tp[i] = T * (T + 1) / 2;
  }
}
__global__ void k_qq_large_list(const uint64_t *tro, const uint8_t *dirty, uint32_t ca,
                                uint32_t cb, uint32_t *lc, unsigned *cnt) {
  uint64_t n = cb - ca;
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t iters = (n + stride - 1) / stride;
  for (uint64_t it = 0; it < iters; it++) {      // uniform trip count (wave_append)
    uint64_t i = i0 + it * stride;
    bool take = false;
    uint32_t c = ca + (uint32_t)i;
    if (i < n) take = !dirty[c] && tro[c + 1] - tro[c] > QQ_SMALL;
    unsigned p = wave_append(cnt, take);
    if (take) lc[p] = c;
  }
}

// ---------------------------------------------------------------------------
// row pull: S(i, :) in LDS windows of W positions; the contributions of row i
// are enumerated flat over (entry e of W_skel row i, m): a window of NT entries
// is set up (one lane each: c, k, m-range inside the position window),
// prefix-summed, and every lane takes one contribution; contributions of
// different entries (= different c) are added layer by layer in ascending c.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lb_u32(const uint32_t *a, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__device__ __forceinline__ uint32_t ub_u32(const uint32_t *a, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    uint32_t mid = (lo + hi) >> 1;
    if (a[mid] <= x) lo = mid + 1; else hi = mid;
  }
  return lo;
}
template <int NT>
__device__ __forceinline__ void layer_sync() {
  if (NT == 64) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}

template <int NT, int W>
__global__ __launch_bounds__(NT) void k_lmop_pull(
    const uint32_t *rows, uint32_t nrows, const uint64_t *sro, const uint32_t *scol, double *sa,
    const uint64_t *wro, const uint32_t *wcol, const uint32_t *kpos, const uint64_t *tro,
    const uint32_t *tcol, const uint8_t *dirty, uint32_t ca, uint32_t cb, const double *u,
    const double *QQ, const uint64_t *qqoff, unsigned *miss) {
  __shared__ uint32_t cols[W];
  __shared__ double vals[W];
  __shared__ uint32_t wend[NT];
  __shared__ uint64_t wtc[NT], wqq[NT];
  __shared__ double wu[NT];
  __shared__ uint32_t wtot[NT / 64];
  const int t = threadIdx.x;
  for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    const uint32_t i = rows[r];
    const uint64_t s0 = sro[i], s1 = sro[i + 1];
    const uint64_t e0 = wro[i], e1 = wro[i + 1];
    for (uint64_t p0 = s0; p0 < s1; p0 += W) {
      const uint32_t wn = (uint32_t)min((uint64_t)W, s1 - p0);
      const bool whole = (p0 == s0) && (p0 + wn == s1);
      for (uint32_t q = t; q < wn; q += NT) { cols[q] = scol[p0 + q]; vals[q] = sa[p0 + q]; }
      __syncthreads();
      const uint32_t clo = cols[0], chi = cols[wn - 1];
      for (uint64_t eb = e0; eb < e1; eb += NT) {
        const uint64_t e = eb + t;
        uint32_t len = 0;
        uint64_t tc = 0, qq = 0;
        double uc = 0.0;
        if (e < e1) {
          const uint32_t c = wcol[e];
          if (c >= ca && c < cb && !dirty[c]) {
            const uint64_t t0 = tro[c];
            const uint32_t nz = (uint32_t)(tro[c + 1] - t0);
            uint32_t mlo = 0, mhi = nz;
            if (!whole) {
              mlo = lb_u32(tcol + t0, nz, clo);
              mhi = ub_u32(tcol + t0, nz, chi);
            }
            if (mhi > mlo) {
              len = mhi - mlo;
              tc = t0 + mlo;
              qq = qqoff[c] + (uint64_t)kpos[e] * nz + mlo;
              uc = u[c];
            }
          }
        }
        const uint32_t inc = block_incl_scan<NT>(len, wtot);
        wend[t] = inc;
        wtc[t] = tc;
        wqq[t] = qq;
        wu[t] = uc;
        __syncthreads();
        const uint32_t T = wend[NT - 1];
        for (uint32_t q0 = 0; q0 < T; q0 += NT) {
          const uint32_t q = q0 + t;
          const bool v = q < T;
          int l = 0;
          uint32_t p = 0;
          double x = 0.0;
          if (v) {
            int lo = 0, hi = NT - 1;
            while (lo < hi) {
              int mid = (lo + hi) >> 1;
              if (wend[mid] > q) hi = mid; else lo = mid + 1;
            }
            l = lo;
            const uint32_t off = q - (l ? wend[l - 1] : 0u);
            const uint32_t j = tcol[wtc[l] + off];
            x = wu[l] * QQ[wqq[l] + off];
            p = lb_u32(cols, wn, j);
            if (p >= wn || cols[p] != j) { atomicAdd(miss, 1u); p = 0xffffffffu; }
          }
          // layers of this chunk: entries [lf, ll]
          const uint32_t qb = min(q0 + NT, T) - 1;
          int lf, ll;
          {
            int lo = 0, hi = NT - 1;
            while (lo < hi) { int mid = (lo + hi) >> 1; if (wend[mid] > q0) hi = mid; else lo = mid + 1; }
            lf = lo;
            lo = lf; hi = NT - 1;
            while (lo < hi) { int mid = (lo + hi) >> 1; if (wend[mid] > qb) hi = mid; else lo = mid + 1; }
            ll = lo;
          }
          if (lf == ll) {
            if (v && p != 0xffffffffu) vals[p] = vals[p] + x;
          } else {
            for (int lay = lf; lay <= ll; lay++) {
              if (v && l == lay && p != 0xffffffffu) vals[p] = vals[p] + x;
              layer_sync<NT>();
            }
          }
          layer_sync<NT>();
        }
        __syncthreads();
      }
      for (uint32_t q = t; q < wn; q += NT) sa[p0 + q] = vals[q];
      __syncthreads();
    }
  }
}

// S rows [r0, r0 + n) by length: (0, small] -> ls (thread per row), (small, lim] -> l0
// (wave), > lim -> l1
__global__ void k_srow_bins(const uint64_t *sro, uint32_t r0, uint32_t n, uint32_t lim, uint32_t *l0,
                            uint32_t *l1, unsigned *cnt, uint32_t small, uint32_t *ls) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t iters = (n + stride - 1) / stride;
  for (uint64_t it = 0; it < iters; it++) {
    uint64_t i = r0 + i0 + it * stride;
    uint64_t L = i < (uint64_t)r0 + n ? sro[i + 1] - sro[i] : 0;
    bool s = L > 0 && L <= small, a = L > small && L <= lim, b = L > lim;
    unsigned pa = wave_append(&cnt[0], a);
    unsigned pb = wave_append(&cnt[1], b);
    unsigned ps = wave_append(&cnt[2], s);
    if (a) l0[pa] = (uint32_t)i;
    if (b) l1[pb] = (uint32_t)i;
    if (s) ls[ps] = (uint32_t)i;
  }
}
// Row pull for short S rows (<= SC entries: the fine levels, 10^6 - 10^7 rows of a few
// dozen): one THREAD per row instead of a wavefront.  The row's columns and values sit
// in this thread's LDS column slice; its W_skel entries are taken in ascending c (the
// layers of k_lmop_pull), and each support's columns, ascending, are matched to the
// row's ascending columns by one forward merge pointer.  Every S entry receives its
// contributions u_c * QQ in ascending c on top of its current value -- k_lmop_pull's
// sums; a column missing from the row counts a miss (the caller then redoes S exactly).
template <int SC>
__global__ __launch_bounds__(128) void k_lmop_pull_small(
    const uint32_t *rows, uint32_t nrows, const uint64_t *sro, const uint32_t *scol, double *sa,
    const uint64_t *wro, const uint32_t *wcol, const uint32_t *kpos, const uint64_t *tro,
    const uint32_t *tcol, const uint8_t *dirty, uint32_t ca, uint32_t cb, const double *u,
    const double *QQ, const uint64_t *qqoff, unsigned *miss) {
  __shared__ uint32_t cs[SC][128];
  __shared__ double vs[SC][128];
  const int t = threadIdx.x;
  GRID_STRIDE(r, nrows) {
    const uint32_t i = rows[r];
    const uint64_t s0 = sro[i];
    const uint32_t n = (uint32_t)(sro[i + 1] - s0);
    for (uint32_t q = 0; q < n; q++) { cs[q][t] = scol[s0 + q]; vs[q][t] = sa[s0 + q]; }
    unsigned nmiss = 0;
    const uint64_t e1 = wro[i + 1];
    for (uint64_t e = wro[i]; e < e1; e++) {
      const uint32_t c = wcol[e];
      if (c < ca || c >= cb || dirty[c]) continue;
      const uint64_t t0 = tro[c];
      const uint32_t nz = (uint32_t)(tro[c + 1] - t0);
      const uint64_t qq = qqoff[c] + (uint64_t)kpos[e] * nz;
      const double uc = u[c];
      uint32_t p = 0;
      for (uint32_t m = 0; m < nz; m++) {
        const uint32_t j = tcol[t0 + m];
        while (p < n && cs[p][t] < j) p++;
        if (p < n && cs[p][t] == j) {
          vs[p][t] = vs[p][t] + uc * QQ[qq + m];
          p++;
        } else {
          nmiss++;
        }
      }
    }
    if (nmiss) atomicAdd(miss, nmiss);
    for (uint32_t q = 0; q < n; q++) sa[s0 + q] = vs[q][t];
  }
}
// AMGD_LMOP_SMALL (default 1; 0: off): S rows of at most 32 entries take
// k_lmop_pull_small -- 256^3 setup -0.1 to -0.2 s in interleaved A/Bs
// (profiles/r03/ab256_r03s2_*, ab256_r03t_*)
static int g_lmop_small = -1;
extern "C" void amgd_lmop_set_small(int n) { g_lmop_small = n; }
static uint32_t lmop_small() {
  if (g_lmop_small < 0) { const char *e = getenv("AMGD_LMOP_SMALL"); g_lmop_small = e && *e ? atoi(e) : 1; }
  return g_lmop_small > 0 ? 32u : 0u;
}

// kpos[e] = position of the row of W_skel entry e inside its column's support
// (row c of Wt); perm (from amgd_transpose) maps Wt entries to W_skel entries
__global__ void k_kpos(const uint64_t *tro, uint32_t nc, const uint64_t *perm, uint32_t *kpos) {
  GRID_STRIDE(c, nc) {
    for (uint64_t q = tro[c]; q < tro[c + 1]; q++) kpos[perm[q]] = (uint32_t)(q - tro[c]);
  }
}
extern "C" uint32_t *amgd_lmop_kpos(const dcsr *Wt, const uint64_t *perm) {
  uint32_t *kp = (uint32_t *)amgd_alloc(Wt->nnz * 4 + 4);
  if (Wt->rn && Wt->nnz) k_kpos<<<grid_for(Wt->rn), 256, 0, amgd_s()>>>(Wt->ro, Wt->rn, perm, kp);
  KCHECK();
  return kp;
}

extern "C" void amgd_lmop_general(dcsr *S, const dcsr *Wt, const double *Q, const uint64_t *qoff,
                                  const double *u, uint32_t cb, uint32_t ce);

#define LMOP_SHARD_MIN (1ull << 24)   // S entries below which every rank pulls all rows
static uint64_t qq_budget() {
  static uint64_t b = 0;
  if (!b) {
    const char *e = getenv("AMGD_QQ_BUDGET_MB");
    b = (e && *e) ? (uint64_t)atoll(e) << 20 : (16ull << 30);
    if (b < (1u << 20)) b = 1u << 20;
  }
  return b;
}
static int g_lmop_mode = -1;   // 1: force the key/sort path (AMGD_LMOP=general, tests)
static int lmop_mode() {
  if (g_lmop_mode < 0) {
    const char *e = getenv("AMGD_LMOP");
    g_lmop_mode = (e && e[0] == 'g') ? 1 : 0;
  }
  return g_lmop_mode;
}
extern "C" void amgd_lmop_set_mode(int m) { g_lmop_mode = m; }

static uint64_t g_lmop_stats[5];   // fast calls, general calls, dirty-prefix calls, misses, pruned supports
extern "C" void amgd_lmop_stats(uint64_t *out) { for (int i = 0; i < 5; i++) out[i] = g_lmop_stats[i]; }
extern "C" void amgd_lmop_stats_reset(void) { for (int i = 0; i < 5; i++) g_lmop_stats[i] = 0; }
extern "C" void amgd_lmop_note_pruned(void) { g_lmop_stats[4]++; }

// Partitioned mode (amgd_psetup.c p_lmop): S and Wskel are global-row views of a rank's
// rows, Wt / Q / qoff the supports those rows reference; every path below then computes
// exactly this rank's rows (walks starting in other ranks' rows find them empty), and a walk
// that would run into the next rank's rows is flagged (amgd_lmop_spill_detect).  With a
// prefix set (amgd_lmop_set_prefix(D)), the contributions of the coarse points [0, D) --
// every dirty one -- are already in S (p_lmop walks them on the whole S pattern): S is not
// cleared and only [D, nc) is added, all clean.  Returns 0.
static uint32_t g_lmop_prefix = 0;
static int g_lmop_missed = 0;
static uint64_t g_lmop_qq_bytes = 0;   // QQ^t bytes of the last call (all chunks)
extern "C" uint64_t amgd_lmop_qq_bytes(void) { return g_lmop_qq_bytes; }
extern "C" int amgd_lmop_missed(void) { const int m = g_lmop_missed; g_lmop_missed = 0; return m; }
extern "C" void amgd_lmop_set_prefix(uint32_t d) { g_lmop_prefix = d; }
extern "C" void amgd_lmop_classify_view(const dcsr *Wt, uint32_t *dend, uint32_t *cmin) {
  const uint32_t nc = Wt->rn;
  unsigned hst[4] = {0u, 0xffffffffu, 0u, 0u};
  if (nc && Wt->nnz) {
    uint8_t *dirty = (uint8_t *)amgd_alloc((size_t)nc + 1);
    unsigned *st = (unsigned *)amgd_alloc(16);
    amgd_h2d(st, hst, 16);
    k_lmop_classify<<<grid_for(nc), 256, 0, amgd_s()>>>(Wt->ro, Wt->a, nc, dirty, st);
    KCHECK();
    amgd_d2h(hst, st, 8);
    amgd_free(dirty); amgd_free(st);
  }
  *dend = hst[0];
  *cmin = hst[1];
}
extern "C" int amgd_lmop(dcsr *S, const dcsr *Wskel, const uint32_t *kpos, const dcsr *Wt,
                         const double *Q, const uint64_t *qoff, const double *u) {
  hipStream_t s = amgd_s();
  const uint32_t pre = g_lmop_prefix;
  if (!pre) amgd_memset(S->a, 0, S->nnz * 8);
  const uint32_t nc = Wt->rn;
  if (nc == 0 || Wt->nnz == 0 || S->nnz == 0 || pre >= nc) return 0;
  if (lmop_mode() == 1 || kpos == nullptr) {
    g_lmop_stats[1]++;
    amgd_lmop_general(S, Wt, Q, qoff, u, pre, nc);
    return 0;
  }
  uint8_t *dirty = (uint8_t *)amgd_alloc((size_t)nc + 1);
  unsigned *st = (unsigned *)amgd_alloc(16);
  unsigned hst[4] = {0u, 0xffffffffu, 0u, 0u};
  amgd_h2d(st, hst, 16);
  k_lmop_classify<<<grid_for(nc), 256, 0, s>>>(Wt->ro, Wt->a, nc, dirty, st);
  KCHECK();
  amgd_d2h(hst, st, 8);
  uint32_t dend = hst[0];
  const uint32_t cmin = hst[1];
  if (pre) {
    dend = pre;                       // [0, pre) done; every dirty point lies below pre
  } else if (cmin == 0xffffffffu || (dend > 0 && dend - 1 > cmin)) {
    // no clean point, or a dirty point after a clean one: order needs the general walk
    g_lmop_stats[1]++;
    amgd_lmop_general(S, Wt, Q, qoff, u, 0, nc);
    amgd_free(dirty); amgd_free(st);
    return 0;
  } else if (dend > 0) {              // dirty prefix [0, dend): opens every sum it touches
    g_lmop_stats[2]++;
    // the walk on the supports of [0, dend) only: a row-prefix view of Wt, so the general
    // walk's per-support set-up (offsets, row of entry, host copies) is O(dend), not O(nc)
    // -- the partitioned driver's form (p_lmop_prefix), 0.3-0.4 s faster at 256^3
    dcsr wv = *Wt;
    wv.rn = dend;
    amgd_d2h(&wv.nnz, Wt->ro + dend, 8);
    amgd_lmop_general(S, &wv, Q, qoff, u, 0, dend);
  }
  // S rows binned by length: thread / wave with a 1024-wide window / 256 threads with
  // 4096-wide windows.  Multi-GPU: S rows are independent, so each rank pulls the rows of
  // its shards (contiguous ranges of equal S nnz) and one allgatherv of the values
  // completes S everywhere (the dirty prefix above ran on every rank, over all rows)
  const uint32_t nf = S->rn;
  const int N = amgd_nshards();
  const bool sharded = N > 1 && nf >= (uint32_t)N && amgd_shard_worth(S->nnz, LMOP_SHARD_MIN);
  std::vector<uint32_t> split(N + 1, 0);
  int sf = 0, sl = 1;
  uint32_t r0 = 0, r1 = nf;
  if (sharded) {
    amgd_shard_split(S->ro, nf, split.data());
    amgd_my_shards(&sf, &sl);
    r0 = split[sf];
    r1 = split[sl];
  }
  uint32_t *rl = (uint32_t *)amgd_alloc(3 * ((size_t)nf + 1) * 4);
  uint32_t *rl1 = rl + nf + 1, *rls = rl1 + nf + 1;
  unsigned *rc = (unsigned *)amgd_alloc(16);
  amgd_memset(rc, 0, 12);
  const uint32_t small = lmop_small();
  if (r1 > r0)
    k_srow_bins<<<grid_for(r1 - r0), 256, 0, s>>>(S->ro, r0, r1 - r0, 1024, rl, rl1, rc, small, rls);
  unsigned hrc[3];
  amgd_d2h(hrc, rc, 12);
  // QQt chunks by coarse range within the memory budget
  uint64_t *sz = (uint64_t *)amgd_alloc(((size_t)nc + 1) * 8);
  k_qq_size<<<grid_for(nc), 256, 0, s>>>(Wt->ro, dirty, nc, 0, nc, sz);
  amgd_scan_u64(sz, nc);
  std::vector<uint64_t> hsz(nc + 1);
  amgd_d2h(hsz.data(), sz, ((size_t)nc + 1) * 8);
  g_lmop_qq_bytes = hsz[nc] * 8;
  const uint64_t budget = qq_budget() / 8;
  uint32_t *lc = (uint32_t *)amgd_alloc(((size_t)nc + 1) * 4);
  uint64_t *tp = (uint64_t *)amgd_alloc(((size_t)nc + 1) * 8);
  unsigned *lcnt = (unsigned *)amgd_alloc(8);
  unsigned *miss = (unsigned *)amgd_alloc(8);
  amgd_memset(miss, 0, 4);
  uint32_t ca = dend;
  while (ca < nc) {
    uint32_t cb = ca + 1;
    while (cb < nc && hsz[cb + 1] - hsz[ca] <= budget) cb++;
    const uint64_t need = hsz[cb] - hsz[ca];
    if (need == 0) { ca = cb; continue; }
    double *QQ = (double *)amgd_alloc_f64(need * 8 + 8);
    const double *QQb = QQ - hsz[ca];     // qqoff (= sz prefix) is global: rebase
    // small supports
    k_qq_small<<<(int)std::min<uint32_t>(cb - ca, 65536u), 64, 0, s>>>(Wt->ro, dirty, ca, cb, Q,
                                                                       qoff, sz, (double *)QQb);
    // large supports, tiled
    amgd_memset(lcnt, 0, 4);
    k_qq_large_list<<<grid_for(cb - ca), 256, 0, s>>>(Wt->ro, dirty, ca, cb, lc, lcnt);
    unsigned nl = 0;
    amgd_d2h(&nl, lcnt, 4);
    if (nl) {
      k_qq_tilecount<<<grid_for(nl), 256, 0, s>>>(lc, nl, Wt->ro, tp);
      uint64_t ntiles = amgd_scan_u64(tp, nl);
      k_qq_tile<<<(int)std::min<uint64_t>(ntiles, 1u << 20), 64, 0, s>>>(
          lc, nl, tp, ntiles, Wt->ro, Q, qoff, sz, (double *)QQb);
    }
    KCHECK();
    if (hrc[2])
      k_lmop_pull_small<32><<<grid_for(hrc[2], 128, 16384), 128, 0, s>>>(
          rls, hrc[2], S->ro, S->col, S->a, Wskel->ro, Wskel->col, kpos, Wt->ro, Wt->col, dirty, ca,
          cb, u, QQb, sz, miss);
    if (hrc[0])
      k_lmop_pull<64, 1024><<<(int)std::min<unsigned>(hrc[0], 1u << 20), 64, 0, s>>>(
          rl, hrc[0], S->ro, S->col, S->a, Wskel->ro, Wskel->col, kpos, Wt->ro, Wt->col, dirty, ca,
          cb, u, QQb, sz, miss);
    if (hrc[1])
      k_lmop_pull<256, 4096><<<(int)std::min<unsigned>(hrc[1], 1u << 16), 256, 0, s>>>(
          rl1, hrc[1], S->ro, S->col, S->a, Wskel->ro, Wskel->col, kpos, Wt->ro, Wt->col, dirty,
          ca, cb, u, QQb, sz, miss);
    KCHECK();
    amgd_free(QQ);
    ca = cb;
  }
  unsigned hm = 0;
  amgd_d2h(&hm, miss, 4);
  if (sharded) {
    // every rank holds its rows' values; a miss on any rank sends all of them to the
    // exact walk (the counts are summed over the ranks first)
    std::vector<uint64_t> mv(N, 0);
    for (int q = sf; q < sl; q++) mv[q] = q == sf ? hm : 0;
    amgd_allgather_u64(mv.data());
    uint64_t tot = 0;
    for (int q = 0; q < N; q++) tot += mv[q];
    hm = (unsigned)std::min<uint64_t>(tot, 0xffffffffu);
    if (!hm) {
      std::vector<uint64_t> pre(N + 1), off(N + 1);
      amgd_gather_u64_at(S->ro, split.data(), N + 1, pre.data());
      for (int q = 0; q <= N; q++) off[q] = 8 * pre[q];
      void *b = S->a;
      amgd_allgatherv(1, &b, off.data());
    }
  }
  if (hm && pre) {
    // partitioned, prefix done: the caller redoes the operator (amgd_lmop_missed)
    g_lmop_stats[3] += hm;
    g_lmop_missed = 1;
  } else if (hm) {
    // a clean contribution missed its column: S is not W_skel*W_skel' -- redo exactly
    g_lmop_stats[3] += hm;
    g_lmop_stats[1]++;
    amgd_memset(S->a, 0, S->nnz * 8);
    amgd_lmop_general(S, Wt, Q, qoff, u, 0, nc);
  } else {
    g_lmop_stats[0]++;
  }
  amgd_free(rl); amgd_free(rc); amgd_free(sz); amgd_free(lc); amgd_free(tp); amgd_free(lcnt);
  amgd_free(miss); amgd_free(dirty); amgd_free(st);
  return 0;
}
