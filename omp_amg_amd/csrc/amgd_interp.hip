// amgd_interp.hip -- energy-minimising interpolation kernels (amg_setup.c:598-1493).
//
// Per coarse point c (row c of Wt = W_skel^T) the reference builds an
// A-orthonormal packed upper-triangular Q of A restricted to the support
// Qj = Wt(c,:) (interp / interp_lmop, amg_setup.c:2053, 1589).  Q depends only
// on (A, support), so it is factored once per skeleton here (amgd_qfactor) and
// re-applied for W0, the constraint operator S and W.  Within a column the
// k-steps are sequential; the 64..256 threads of a block take distinct output
// entries of mv_utt / mv_ut (amg_setup.c:2122/2138), each summed in the
// reference's order, so every Q entry is bit-identical to the reference.
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#include "amgd.h"
#include "amgd_dev.h"

__device__ __forceinline__ uint64_t tri(uint64_t i) { return i * (i + 1) / 2; }

// value of row [a0,a1) at column j (first match), or 0  -- sp_restrict_sorted
__device__ __forceinline__ double row_lookup(const uint32_t *col, const double *a, uint64_t a0,
                                             uint64_t a1, uint32_t j) {
  uint64_t lo = a0, hi = a1;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (col[mid] < j) lo = mid + 1;
    else hi = mid;
  }
  return (lo < a1 && col[lo] == j) ? a[lo] : 0.0;
}

// ---------------------------------------------------------------------------
// min_skel (amg_setup.c:2198)
// ---------------------------------------------------------------------------
__global__ void k_min_skel(const uint64_t *ro, const uint32_t *col, const double *a, uint32_t rn,
                           uint64_t *wro, uint32_t *wcol, double *wa) {
  GRID_STRIDE(i, rn) {
    double ym = -DBL_MAX;
    uint32_t j = 0;
    for (uint64_t k = ro[i]; k < ro[i + 1]; k++)
      if (a[k] > ym) { ym = a[k]; j = col[k]; }
    wa[i] = ym > 0.0 ? 1.0 : 0.0;
    wcol[i] = j;
    wro[i + 1] = i + 1;
    if (i == 0) wro[0] = 0;
  }
}
extern "C" dcsr *amgd_min_skel(const dcsr *R) {
  dcsr *W = dcsr_new(R->rn, R->cn, R->rn);
  if (R->rn)
    k_min_skel<<<grid_for(R->rn), 256, 0, amgd_s()>>>(R->ro, R->col, R->a, R->rn, W->ro, W->col, W->a);
  else
    amgd_memset(W->ro, 0, 8);
  KCHECK();
  return W;
}

// ---------------------------------------------------------------------------
// Q factor (interp, amg_setup.c:2053-2099).  Per support of nz points, for
// k = 0..nz-1:
//   s1[m] = A(Qj[k], Qj[m])  (m <= k)
//   s2[i] = sum_{j<=i} U[i][j] s1[j]          (mv_utt, i < k)
//   qk[i] = sum_{j=i}^{k-1} U[j][i] s2[j]     (mv_ut)
//   al = -1/sqrt(s1[k] - sum_m s1[m] qk[m]);  U[k][i] = qk[i] al, U[k][k] = -al
// U is the packed row-major triangle (row i at tri(i)).  Every sum keeps the
// reference's order, one lane per output.  Three tiers by nz:
//   nz <=  64 / <= 128 : the whole triangle in LDS, one wavefront per support
//   nz <= 1024         : 256 threads, U in HBM; loads are issued QB at a time
//                        ahead of the ordered adds (the sums are latency-bound
//                        chains), mv_ut walks j in lock-step so every load
//                        instruction of a wave is one coalesced row segment
//   nz  > 1024         : (the orphan support gathered at coarse point 0) all
//                        lanes of a cooperative grid, three grid barriers per k
// ---------------------------------------------------------------------------
#define QF_LDS_NZ 512

// s1[m] = A(sk, Qj[m]) for m <= k (row_lookup's first match), by one coalesced pass over
// row sk with each column located in the support by bisection in the LDS copy Qs of Qj
// (k+1 bisections of the A row would be chains of dependent HBM loads).  Callers sync.
template <int NT>
__device__ __forceinline__ void gather_s1(double *s1, const uint32_t *Qs, uint32_t k,
                                          const uint32_t *acol, const double *aa, uint64_t a0,
                                          uint64_t a1) {
  const uint32_t t = threadIdx.x;
  // cost model in LDS-latency units (an HBM load ~ 4): scan = rounds over the row x
  // (load + bisection in Qs), lookup = rounds over m x a bisection of dependent loads
  const uint32_t len = (uint32_t)(a1 - a0);
  const uint32_t lg_len = 32 - __clz(len | 1), lg_k = 32 - __clz(k + 1);
  const uint32_t scan = ((len + NT - 1) / NT) * (4 + lg_k);
  const uint32_t look = ((k + NT) / NT) * lg_len * 4;
  if (look < scan) {
    for (uint32_t m = t; m <= k; m += NT) s1[m] = row_lookup(acol, aa, a0, a1, Qs[m]);
    return;
  }
  for (uint32_t m = t; m <= k; m += NT) s1[m] = 0.0;
  __syncthreads();
  for (uint64_t e = a0 + t; e < a1; e += NT) {
    const uint32_t j = acol[e];
    if (e > a0 && acol[e - 1] == j) continue;
    uint32_t lo = 0, hi = k + 1;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (Qs[mid] < j) lo = mid + 1;
      else hi = mid;
    }
    if (lo <= k && Qs[lo] == j) s1[lo] = aa[e];
  }
}

// LDS-resident triangle.  Every dot is one ordered chain; the LDS reads of a chain
// are issued LB at a time ahead of its adds (a read -> mul -> add chain per element
// would pay the LDS latency on every term).  Reads past a chain's end stay inside
// the padded arrays and their terms are not added.
#define LB 8
template <int NZMAX, int NT>
__global__ __launch_bounds__(NT) void k_qfactor_lds(const uint32_t *rows, uint32_t nrows,
                                                    const uint64_t *wro, const uint32_t *wcol,
                                                    const uint64_t *aro, const uint32_t *acol,
                                                    const double *aa, const uint64_t *qoff,
                                                    double *Q) {
  constexpr uint32_t TN = NZMAX * (NZMAX + 1) / 2;
  __shared__ double U[TN + NZMAX + LB];
  __shared__ double s1[NZMAX + LB], s2[NZMAX + LB], qk[NZMAX + LB];
  __shared__ uint32_t Qs[NZMAX];
  __shared__ double sh_al;
  const int t = threadIdx.x;
  for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    const uint32_t c = rows[r];
    const uint64_t w0 = wro[c];
    const uint32_t nz = (uint32_t)(wro[c + 1] - w0);
    for (uint32_t m = t; m < nz; m += NT) Qs[m] = wcol[w0 + m];
    __syncthreads();
    for (uint32_t k = 0; k < nz; k++) {
      const uint32_t sk = Qs[k];
      gather_s1<NT>(s1, Qs, k, acol, aa, aro[sk], aro[sk + 1]);
      __syncthreads();
      for (uint32_t i = t; i < k; i += NT) {          // s2[i] = sum_{j<=i} U[i][j] s1[j]
        const double *Ui = U + tri(i);
        double v = 0;
        for (uint32_t j0 = 0; j0 <= i; j0 += LB) {
          double u[LB], x[LB];
#pragma unroll
          for (int q = 0; q < LB; q++) { u[q] = Ui[j0 + q]; x[q] = s1[j0 + q]; }
#pragma unroll
          for (int q = 0; q < LB; q++)
            if (j0 + q <= i) v += u[q] * x[q];
        }
        s2[i] = v;
      }
      __syncthreads();
      for (uint32_t i = t; i < k; i += NT) {          // qk[i] = sum_{j=i}^{k-1} U[j][i] s2[j]
        double y = 0;
        uint32_t off = (uint32_t)tri(i) + i;          // U[i][i]
        for (uint32_t j0 = i; j0 < k; j0 += LB) {
          double u[LB], x[LB];
          uint32_t o = off;
#pragma unroll
          for (int q = 0; q < LB; q++) {
            const uint32_t j = j0 + q;
            u[q] = U[j < k ? o : 0];
            x[q] = s2[j];
            o += j + 1;
          }
#pragma unroll
          for (int q = 0; q < LB; q++)
            if (j0 + q < k) y += u[q] * x[q];
          off = o;
        }
        qk[i] = y;
      }
      __syncthreads();
      if (t == 0) {
        double al = s1[k];
        for (uint32_t m0 = 0; m0 < k; m0 += LB) {
          double x[LB], y[LB];
#pragma unroll
          for (int q = 0; q < LB; q++) { x[q] = s1[m0 + q]; y[q] = qk[m0 + q]; }
#pragma unroll
          for (int q = 0; q < LB; q++)
            if (m0 + q < k) al -= x[q] * y[q];
        }
        sh_al = -1.0 / sqrt(al);
      }
      __syncthreads();
      const double al = sh_al;
      double *out = U + tri(k);
      for (uint32_t i = t; i < k; i += NT) out[i] = qk[i] * al;
      if (t == 0) out[k] = -al;
      __syncthreads();
    }
    double *Qc = Q + qoff[c];
    const uint32_t tn = nz * (nz + 1) / 2;
    for (uint32_t e = t; e < tn; e += NT) Qc[e] = U[e];
    __syncthreads();
  }
}

// sum_{j<n} u[j]*x[j] in order, loads issued QB at a time (latency hiding)
#define QB 32
__device__ __forceinline__ double seq_dot_batched(const double *u, const double *x, uint32_t n) {
  double v = 0;
  for (uint32_t j0 = 0; j0 < n; j0 += QB) {
    double r[QB];
#pragma unroll
    for (int q = 0; q < QB; q++) r[q] = (j0 + q < n) ? u[j0 + q] : 0.0;
#pragma unroll
    for (int q = 0; q < QB; q++)
      if (j0 + q < n) v += r[q] * x[j0 + q];
  }
  return v;
}
// qk[i] = sum_{j=i}^{k-1} U[tri(j)+i] s2[j]; the lanes of a wave (i = ib+lane) walk j in
// lock-step from ib so each load instruction reads 64 consecutive doubles of row j
__device__ __forceinline__ double mv_ut_lane(const double *U, const double *s2, uint32_t ib,
                                            uint32_t i, uint32_t k) {
  double y = 0;
  for (uint32_t j0 = ib; j0 < k; j0 += QB) {
    double r[QB];
#pragma unroll
    for (int q = 0; q < QB; q++) {
      uint32_t j = j0 + q;
      r[q] = (j < k && j >= i) ? U[tri(j) + i] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < QB; q++) {
      uint32_t j = j0 + q;
      if (j < k && j >= i) y += r[q] * s2[j];
    }
  }
  return y;
}

// mid supports: one 256-thread block each, U in HBM (the output), s1/s2/qk in LDS
__global__ __launch_bounds__(256) void k_qfactor_mid(const uint32_t *rows, uint32_t nrows,
                                                     const uint64_t *wro, const uint32_t *wcol,
                                                     const uint64_t *aro, const uint32_t *acol,
                                                     const double *aa, const uint64_t *qoff,
                                                     double *Q) {
  __shared__ double s1[1024], s2[1024], qk[1024];
  __shared__ uint32_t Qs[1024];
  __shared__ double sh_al;
  const int t = threadIdx.x, lane = t & 63;
  for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    const uint32_t c = rows[r];
    const uint64_t w0 = wro[c];
    const uint32_t nz = (uint32_t)(wro[c + 1] - w0);
    for (uint32_t m = t; m < nz; m += 256) Qs[m] = wcol[w0 + m];
    double *U = Q + qoff[c];
    __syncthreads();
    for (uint32_t k = 0; k < nz; k++) {
      const uint32_t sk = Qs[k];
      gather_s1<256>(s1, Qs, k, acol, aa, aro[sk], aro[sk + 1]);
      __syncthreads();
      for (uint32_t i = t; i < k; i += 256) s2[i] = seq_dot_batched(U + tri(i), s1, i + 1);
      __syncthreads();
      for (uint32_t ib = t - lane; ib < k; ib += 256) {
        const uint32_t i = ib + lane;
        double y = mv_ut_lane(U, s2, ib, i, k);
        if (i < k) qk[i] = y;
      }
      __syncthreads();
      if (t == 0) {
        double al = s1[k];
        for (uint32_t m = 0; m < k; m++) al -= s1[m] * qk[m];
        sh_al = -1.0 / sqrt(al);
      }
      __syncthreads();
      const double al = sh_al;
      double *out = U + tri(k);
      for (uint32_t i = t; i < k; i += 256) out[i] = qk[i] * al;
      if (t == 0) out[k] = -al;
      __syncthreads();
    }
  }
}

// mid supports, blocked over B consecutive k-steps.  The rows s1_k (k in [k0, k0+B))
// are rows of A, known in advance, so one pass over the finished rows i < k0 yields
// s2_k[i] for all B steps (B ordered chains per lane, each U element read once for
// B terms), and one pass over their columns yields the prefix j < k0 of every
// qk_k[i] chain; each chain is then continued in order over j in [k0, k) as the
// block's rows are produced.  The row produced at step k (U[k][j] = qk[j] al) feeds
// s2_{k'}[k] of the later steps of the block on lanes of wave 0.  U is read twice per
// B steps instead of twice per step; every sum keeps the reference's order.
#define QB2 16
template <int NZMAX, int B, int NTT = 256>
__global__ __launch_bounds__(NTT) void k_qfactor_blk(const uint32_t *rows, uint32_t nrows,
                                                     const uint64_t *wro, const uint32_t *wcol,
                                                     const uint64_t *aro, const uint32_t *acol,
                                                     const double *aa, const uint64_t *qoff,
                                                     double *Q) {
  constexpr uint32_t NT = NTT, RPT = (NZMAX + NT - 1) / NT, PAD = NZMAX + 16;
  __shared__ uint32_t Qs[NZMAX];
  __shared__ double S1[B * PAD], S2[B * PAD], qk[PAD];
  __shared__ double sh_al;
  const uint32_t t = threadIdx.x, lane = t & 63;
  for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    const uint32_t c = rows[r];
    const uint64_t w0 = wro[c];
    const uint32_t nz = (uint32_t)(wro[c + 1] - w0);
    for (uint32_t m = t; m < nz; m += NT) Qs[m] = wcol[w0 + m];
    double *U = Q + qoff[c];
    __syncthreads();
    for (uint32_t k0 = 0; k0 < nz; k0 += B) {
      const uint32_t bn = min((uint32_t)B, nz - k0);
      // s1 rows of the block (zero, then scatter or look up).  All bn rows are
      // gathered in one flat pass over (row, entry) or (row, m) pairs, so the loads
      // of the whole block are in flight together instead of row after row.
      for (uint32_t b = 0; b < bn; b++)
        for (uint32_t m = t; m <= k0 + b; m += NT) S1[b * PAD + m] = 0.0;
      uint64_t ra0[B];
      uint32_t rlen[B], spre[B + 1], lpre[B + 1];
      uint32_t look_cost = 0, scan_cost = 0;
      spre[0] = lpre[0] = 0;
#pragma unroll
      for (int b = 0; b < B; b++) {
        ra0[b] = 0;
        rlen[b] = 0;
        if ((uint32_t)b < bn) {
          const uint32_t k = k0 + b, sk = Qs[k];
          ra0[b] = aro[sk];
          rlen[b] = (uint32_t)(aro[sk + 1] - ra0[b]);
          const uint32_t lg_len = 32 - __clz(rlen[b] | 1), lg_k = 32 - __clz(k + 1);
          look_cost += (k + 1) * lg_len * 4;
          scan_cost += rlen[b] * (4 + lg_k);
        }
        spre[b + 1] = spre[b] + rlen[b];
        lpre[b + 1] = lpre[b] + ((uint32_t)b < bn ? k0 + b + 1 : 0u);
      }
      __syncthreads();
      if (look_cost < scan_cost) {
        for (uint32_t fl = t; fl < lpre[B]; fl += NT) {
          uint32_t b = 0;
#pragma unroll
          for (int q = 1; q < B; q++) b += fl >= lpre[q] ? 1u : 0u;
          const uint32_t m = fl - lpre[b];
          S1[b * PAD + m] = row_lookup(acol, aa, ra0[b], ra0[b] + rlen[b], Qs[m]);
        }
      } else {
        for (uint32_t fl = t; fl < spre[B]; fl += NT) {
          uint32_t b = 0;
#pragma unroll
          for (int q = 1; q < B; q++) b += fl >= spre[q] ? 1u : 0u;
          const uint64_t a0 = ra0[b], e = a0 + (fl - spre[b]);
          const uint32_t k = k0 + b;
          const uint32_t j = acol[e];
          if (e > a0 && acol[e - 1] == j) continue;
          uint32_t lo = 0, hi = k + 1;
          while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (Qs[mid] < j) lo = mid + 1;
            else hi = mid;
          }
          if (lo <= k && Qs[lo] == j) S1[b * PAD + lo] = aa[e];
        }
      }
      __syncthreads();
      // s2_k[i], i < k0, for every step of the block: one pass over rows i
      for (uint32_t i = t; i < k0; i += NT) {
        double acc[B];
#pragma unroll
        for (int b = 0; b < B; b++) acc[b] = 0.0;
        const double *Ui = U + tri(i);
        for (uint32_t j0 = 0; j0 <= i; j0 += QB2) {
          double u[QB2];
#pragma unroll
          for (int q = 0; q < QB2; q++) u[q] = (j0 + q <= i) ? Ui[j0 + q] : 0.0;
#pragma unroll
          for (int q = 0; q < QB2; q++)
            if (j0 + q <= i) {
#pragma unroll
              for (int b = 0; b < B; b++) acc[b] += u[q] * S1[b * PAD + j0 + q];
            }
        }
#pragma unroll
        for (int b = 0; b < B; b++)
          if ((uint32_t)b < bn) S2[b * PAD + i] = acc[b];
      }
      __syncthreads();
      // prefix j < k0 of qk_k[i] for every step: one pass over columns i < k0, the
      // lanes of a wave walking j in lock-step (each load one row segment)
      double part[RPT][B];
#pragma unroll
      for (uint32_t rr = 0; rr < RPT; rr++) {
        const uint32_t ib = (t - lane) + rr * NT, i = ib + lane;
#pragma unroll
        for (int b = 0; b < B; b++) part[rr][b] = 0.0;
        for (uint32_t j0 = ib; j0 < k0; j0 += QB2) {
          double u[QB2];
#pragma unroll
          for (int q = 0; q < QB2; q++) {
            const uint32_t j = j0 + q;
            u[q] = (j < k0 && j >= i) ? U[tri(j) + i] : 0.0;
          }
#pragma unroll
          for (int q = 0; q < QB2; q++) {
            const uint32_t j = j0 + q;
            if (j < k0 && j >= i) {
#pragma unroll
              for (int b = 0; b < B; b++) part[rr][b] += u[q] * S2[b * PAD + j];
            }
          }
        }
      }
      // the steps of the block
#pragma unroll
      for (int b = 0; b < B; b++) {
        if ((uint32_t)b < bn) {
          const uint32_t k = k0 + b;
#pragma unroll
          for (uint32_t rr = 0; rr < RPT; rr++) {
            const uint32_t i = t + rr * NT;
            if (i < k) {
              double y = i < k0 ? part[rr][b] : 0.0;
              for (uint32_t j = max(i, k0); j < k; j++) y += U[tri(j) + i] * S2[b * PAD + j];
              qk[i] = y;
            }
          }
          __syncthreads();
          if (t == 0) {
            const double *s1 = S1 + b * PAD;
            double al = s1[k];
            for (uint32_t m0 = 0; m0 < k; m0 += LB) {
              double x[LB], y[LB];
#pragma unroll
              for (int q = 0; q < LB; q++) { x[q] = s1[m0 + q]; y[q] = qk[m0 + q]; }
#pragma unroll
              for (int q = 0; q < LB; q++)
                if (m0 + q < k) al -= x[q] * y[q];
            }
            sh_al = -1.0 / sqrt(al);
          }
          __syncthreads();
          const double al = sh_al;
          double *out = U + tri(k);
          for (uint32_t i = t; i < k; i += NT) out[i] = qk[i] * al;
          if (t == 0) out[k] = -al;
          // s2_{k'}[k] for the later steps k' of the block, one chain per lane of wave 0
          if (t < bn - 1 - b) {
            const double *s1 = S1 + (b + 1 + t) * PAD;
            double v = 0;
            for (uint32_t j0 = 0; j0 < k; j0 += LB) {
              double x[LB], y[LB];
#pragma unroll
              for (int q = 0; q < LB; q++) { x[q] = qk[j0 + q]; y[q] = s1[j0 + q]; }
#pragma unroll
              for (int q = 0; q < LB; q++)
                if (j0 + q < k) v += (x[q] * al) * y[q];
            }
            v += (-al) * s1[k];
            S2[(b + 1 + t) * PAD + k] = v;
          }
          __syncthreads();
        }
      }
    }
  }
}

// grid barrier for the cooperative kernel (all blocks resident)
__device__ __forceinline__ void grid_sync(unsigned *bar, unsigned nblocks, unsigned &gen) {
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned a = atomicAdd(&bar[0], 1u);
    if (a == nblocks - 1) {
      atomicExch(&bar[0], 0u);
      __threadfence();
      atomicAdd(&bar[1], 1u);
    } else {
      while (__hip_atomic_load(&bar[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == gen)
        __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  __threadfence();
  gen++;
}

// huge supports (nz <= QF_COOP_MAX): one support at a time over a cooperative
// grid of 64-lane blocks; s1/s2/qk are global (shared by the blocks) and staged
// through LDS where a block reads them serially
// (LDS = false, supports past QF_COOP_MAX: the blocks read s1 / s2 / qk straight
// from global memory instead of LDS copies -- same values, same order)
#define QF_COOP_MAX 8192
template <bool LDS>
__global__ __launch_bounds__(64) void k_qfactor_coop(uint32_t c, const uint64_t *wro,
                                                     const uint32_t *wcol, const uint64_t *aro,
                                                     const uint32_t *acol, const double *aa,
                                                     const uint64_t *qoff, double *Q,
                                                     double *s1b, double *s2, double *qk,
                                                     unsigned *bar) {
  extern __shared__ double xs[];      // 2 * nz doubles (LDS)
  __shared__ double sh_al;
  const uint32_t lane = threadIdx.x, G = gridDim.x;
  const uint32_t gt = blockIdx.x * 64 + lane, GT = G * 64;
  const uint64_t w0 = wro[c];
  const uint32_t nz = (uint32_t)(wro[c + 1] - w0);
  const uint32_t *Qj = wcol + w0;
  double *U = Q + qoff[c];
  double *xa = xs, *xb = xs + nz;
  unsigned gen = 0;
  for (uint32_t k = 0; k <= nz; k++) {
    if (k > 0) {                                   // finish row k-1 (every block computes al)
      const uint32_t kp = k - 1;
      const double *s1p = s1b + (uint64_t)(kp & 1) * nz;
      if (LDS) {
        for (uint32_t m = lane; m <= kp; m += 64) { xa[m] = s1p[m]; xb[m] = qk[m]; }
      } else {
        xa = (double *)s1p;
        xb = qk;
      }
      __syncthreads();
      if (lane == 0) {
        double al = xa[kp];
        for (uint32_t m = 0; m < kp; m++) al -= xa[m] * xb[m];
        sh_al = -1.0 / sqrt(al);
      }
      __syncthreads();
      const double al = sh_al;
      for (uint32_t i = gt; i < kp; i += GT) U[tri(kp) + i] = xb[i] * al;
      if (gt == 0) U[tri(kp) + kp] = -al;
    }
    if (k == nz) break;
    double *s1 = s1b + (uint64_t)(k & 1) * nz;
    const uint32_t sk = Qj[k];
    const uint64_t a0 = aro[sk], a1 = aro[sk + 1];
    for (uint32_t m = gt; m <= k; m += GT) s1[m] = row_lookup(acol, aa, a0, a1, Qj[m]);
    grid_sync(bar, G, gen);
    if (LDS) for (uint32_t m = lane; m <= k; m += 64) xa[m] = s1[m];
    else xa = s1;
    __syncthreads();
    for (uint32_t i = gt; i < k; i += GT) s2[i] = seq_dot_batched(U + tri(i), xa, i + 1);
    grid_sync(bar, G, gen);
    if (LDS) for (uint32_t m = lane; m < k; m += 64) xa[m] = s2[m];
    else xa = s2;
    __syncthreads();
    for (uint32_t ib = gt - lane; ib < k; ib += GT) {
      const uint32_t i = ib + lane;
      double y = mv_ut_lane(U, xa, ib, i, k);
      if (i < k) qk[i] = y;
    }
    grid_sync(bar, G, gen);
  }
}

// huge supports, sparse form.  The orphan support's Gram matrix A(Qj,Qj) is nearly
// diagonal (orphans are isolated points), so its factor is ~0.5% dense.  A product
// term that is exactly zero cannot change a sum that starts at +0 (the sum never
// becomes -0), so each sum of the dense loop equals the sum over its structurally
// nonzero terms taken in the same order.  One block walks k; U is kept as rows
// (ascending columns) plus per-column linked lists (ascending rows):
//   s1 = A(sk, Qj[0..k]) nonzeros                (row of A, positions by bisection)
//   s2[i], i in rows of U reached from s1's columns   (row dot, ascending j)
//   qk[i'], i' in columns of the rows with s2 != 0    (column walk, ascending j)
//   al = s1[k] - sum_m s1[m] qk[m]   (m ascending over s1's nonzeros)
// The unstored entries of row k are qk*al = +0 * (negative) = -0; the triangle is
// prefilled with -0.  Any non-finite value, al <= 0 or a capacity overflow sets the
// status and the support is factored by the dense cooperative kernel instead.
#define QS_NONE 0xffffffffu
#define QS_SORT 2048
struct QsBuf {
  double *s1, *s2, *qk, *uval;
  uint32_t *m2, *m3, *L2, *chead, *ctail, *ucol, *urow, *nxt, *rowptr;
  uint32_t cap;
  unsigned *status;
};
template <int NT>
__device__ __forceinline__ void lds_sort_u32(uint32_t *x, uint32_t n) {
  uint32_t P = 1;
  while (P < n) P <<= 1;
  for (uint32_t i = n + threadIdx.x; i < P; i += NT) x[i] = QS_NONE;
  __syncthreads();
  for (uint32_t kk = 2; kk <= P; kk <<= 1)
    for (uint32_t j = kk >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < P; i += NT) {
        uint32_t l = i ^ j;
        if (l > i) {
          uint32_t a = x[i], b = x[l];
          if ((a > b) == ((i & kk) == 0)) { x[i] = b; x[l] = a; }
        }
      }
      __syncthreads();
    }
}
__global__ void k_fill_negzero(double *q, uint64_t n) {
  GRID_STRIDE(i, n) q[i] = -0.0;
}
template <int NT>
__global__ __launch_bounds__(NT) void k_qfactor_sparse(uint32_t c, const uint64_t *wro,
                                                       const uint32_t *wcol, const uint64_t *aro,
                                                       const uint32_t *acol, const double *aa,
                                                       const uint64_t *qoff, double *Q, QsBuf b) {
  __shared__ uint32_t L1[QS_SORT], L3[QS_SORT];
  __shared__ unsigned n1, n2, n3, fail;
  __shared__ double sh_al;
  const uint32_t t = threadIdx.x;
  const uint64_t w0 = wro[c];
  const uint32_t nz = (uint32_t)(wro[c + 1] - w0);
  const uint32_t *Qj = wcol + w0;
  double *U = Q + qoff[c];
  if (t == 0) { fail = 0; b.rowptr[0] = 0; }
  for (uint32_t k = 0; k < nz; k++) {
    if (t == 0) { n1 = 0; n2 = 0; n3 = 0; }
    __syncthreads();
    // s1: the first match of each support column in row sk (row_lookup), m <= k
    const uint32_t sk = Qj[k];
    const uint64_t a0 = aro[sk], a1 = aro[sk + 1];
    for (uint64_t e = a0 + t; e < a1; e += NT) {
      const uint32_t j = acol[e];
      if (e > a0 && acol[e - 1] == j) continue;
      uint32_t lo = 0, hi = k + 1;
      while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (Qj[mid] < j) lo = mid + 1;
        else hi = mid;
      }
      if (lo <= k && Qj[lo] == j) {
        const double v = aa[e];
        if (v != 0.0) {
          if (!isfinite(v)) fail = 1;
          b.s1[lo] = v;
          unsigned p = atomicAdd(&n1, 1u);
          if (p < QS_SORT) L1[p] = lo;
          else fail = 1;
        }
      }
    }
    __syncthreads();
    if (fail) break;
    const uint32_t N1 = n1;
    lds_sort_u32<NT>(L1, N1);
    // rows i < k with a stored U[i][j], j in s1's columns
    for (uint32_t q = t; q < N1; q += NT) {
      const uint32_t j = L1[q];
      if (j >= k) continue;
      for (uint32_t e = b.chead[j]; e != QS_NONE; e = b.nxt[e]) {
        const uint32_t i = b.urow[e];
        if (atomicExch(&b.m2[i], 1u) == 0u) b.L2[atomicAdd(&n2, 1u)] = i;
      }
    }
    __syncthreads();
    const uint32_t N2 = n2;
    for (uint32_t q = t; q < N2; q += NT) {         // s2[i] = sum_j U[i][j] s1[j]
      const uint32_t i = b.L2[q];
      double v = 0;
      for (uint32_t e = b.rowptr[i]; e < b.rowptr[i + 1]; e++) v += b.uval[e] * b.s1[b.ucol[e]];
      b.s2[i] = v;
    }
    __syncthreads();
    for (uint32_t q = t; q < N2; q += NT) {         // qk's candidate columns
      const uint32_t i = b.L2[q];
      if (b.s2[i] == 0.0) continue;
      for (uint32_t e = b.rowptr[i]; e < b.rowptr[i + 1]; e++) {
        const uint32_t i2 = b.ucol[e];
        if (atomicExch(&b.m3[i2], 1u) == 0u) {
          unsigned p = atomicAdd(&n3, 1u);
          if (p < QS_SORT) L3[p] = i2;
          else fail = 1;
        }
      }
    }
    __syncthreads();
    if (fail) break;
    const uint32_t N3 = n3;
    lds_sort_u32<NT>(L3, N3);
    for (uint32_t q = t; q < N3; q += NT) {         // qk[i'] = sum_j U[j][i'] s2[j]
      const uint32_t i2 = L3[q];
      double y = 0;
      for (uint32_t e = b.chead[i2]; e != QS_NONE; e = b.nxt[e]) y += b.uval[e] * b.s2[b.urow[e]];
      b.qk[i2] = y;
    }
    __syncthreads();
    if (t == 0) {
      double al = b.s1[k];
      for (uint32_t q = 0; q < N1; q++) {
        const uint32_t m = L1[q];
        if (m < k) al -= b.s1[m] * b.qk[m];
      }
      if (!(al > 0.0) || !isfinite(al)) fail = 1;
      sh_al = -1.0 / sqrt(al);
      if (b.rowptr[k] + N3 + 1 > b.cap) fail = 1;
    }
    __syncthreads();
    if (fail) break;
    const double al = sh_al;
    const uint32_t base = b.rowptr[k];
    double *out = U + tri(k);
    for (uint32_t q = t; q < N3; q += NT) {         // row k, ascending columns
      const uint32_t i2 = L3[q], e = base + q;
      const double v = b.qk[i2] * al;
      if (!isfinite(v)) fail = 1;
      out[i2] = v;
      b.ucol[e] = i2;
      b.urow[e] = k;
      b.uval[e] = v;
      b.nxt[e] = QS_NONE;
      const uint32_t tl = b.ctail[i2];
      if (tl == QS_NONE) b.chead[i2] = e;
      else b.nxt[tl] = e;
      b.ctail[i2] = e;
      b.m3[i2] = 0;
      b.qk[i2] = 0.0;
    }
    if (t == 0) {
      const uint32_t e = base + N3;
      out[k] = -al;
      b.ucol[e] = k;
      b.urow[e] = k;
      b.uval[e] = -al;
      b.nxt[e] = QS_NONE;
      b.chead[k] = e;
      b.ctail[k] = e;
      b.rowptr[k + 1] = e + 1;
    }
    for (uint32_t q = t; q < N1; q += NT) b.s1[L1[q]] = 0.0;
    for (uint32_t q = t; q < N2; q += NT) {
      const uint32_t i = b.L2[q];
      b.m2[i] = 0;
      b.s2[i] = 0.0;
    }
    __syncthreads();
  }
  __syncthreads();
  if (t == 0) *b.status = fail;
}

__global__ void k_qsize(const uint64_t *wro, uint32_t rn, uint64_t *sz) {
  GRID_STRIDE(c, rn) {
    uint64_t nz = wro[c + 1] - wro[c];
    sz[c] = nz * (nz + 1) / 2;
  }
}
// columns binned by support size nz (empty supports skipped) against lim[0..nb-2]
struct BinLim {
  uint32_t l[7];
};
// (columns cb <= c < ce only: a shard's range)
__global__ void k_bin_nz(const uint64_t *wro, uint32_t cb, uint32_t ce, BinLim lim, int nb,
                         uint32_t *lists, unsigned *cnt, uint64_t lstride,
                         const uint8_t *skip = nullptr) {
  const uint64_t n = ce - cb;
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t c0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t iters = (n + stride - 1) / stride;
  for (uint64_t it = 0; it < iters; it++) {   // uniform trip count (wave_append)
    uint64_t c = cb + c0 + it * stride;
    uint64_t nz = c < ce ? wro[c + 1] - wro[c] : 0;
    int bin = nb - 1;
    for (int q = nb - 2; q >= 0; q--)
      if (nz <= lim.l[q]) bin = q;
    for (int q = 0; q < nb; q++) {
      bool take = nz != 0 && bin == q && !(skip && c < ce && skip[c]);
      unsigned p = wave_append(&cnt[q], take);
      if (take) lists[(uint64_t)q * lstride + p] = (uint32_t)c;
    }
  }
}
__global__ void k_max_nz(const uint64_t *wro, uint32_t rn, unsigned long long *mx) {
  unsigned long long m = 0;
  GRID_STRIDE(c, rn) m = max(m, (unsigned long long)(wro[c + 1] - wro[c]));
  atomicMax(mx, m);
}

struct RowSplit {
  uint32_t *sl, *bl;
  unsigned ns, nb;
  uint64_t maxnz;
};
static RowSplit split_rows(const dcsr *Wt, uint32_t cap, uint32_t cb, uint32_t ce) {
  RowSplit rs;
  const uint64_t L = (uint64_t)Wt->rn + 1;
  rs.sl = (uint32_t *)amgd_alloc(2 * L * 4);
  rs.bl = rs.sl + L;
  unsigned *cnt = (unsigned *)amgd_alloc(32);
  amgd_memset(cnt, 0, 32);
  if (ce > cb) {
    k_bin_nz<<<grid_for(ce - cb), 256, 0, amgd_s()>>>(Wt->ro, cb, ce, BinLim{{cap}}, 2, rs.sl, cnt, L);
    k_max_nz<<<grid_for(Wt->rn), 256, 0, amgd_s()>>>(Wt->ro, Wt->rn, (unsigned long long *)(cnt + 4));
  }
  unsigned h[8];
  amgd_d2h(h, cnt, 32);
  amgd_free(cnt);
  rs.ns = h[0];
  rs.nb = h[1];
  uint64_t mx;
  memcpy(&mx, &h[4], 8);
  rs.maxnz = mx;
  return rs;
}
static void free_split(RowSplit &rs) { amgd_free(rs.sl); }

static int g_qf_sparse = -1;   // 0: dense cooperative only, 1: sparse first, 2: tiny capacity
static bool g_qf_sparse_forced = false;   // set by the environment or a test
static int qf_sparse_mode() {
  if (g_qf_sparse < 0) {
    const char *e = getenv("AMGD_QF_SPARSE");
    g_qf_sparse = e ? atoi(e) : 1;
    g_qf_sparse_forced = e != nullptr;
  }
  return g_qf_sparse;
}
static int qf_blocked() {
  static int b = -1;
  if (b < 0) {
    const char *e = getenv("AMGD_QF_BLOCKED");
    b = e ? atoi(e) : 1;
  }
  return b;
}
static uint32_t g_coop_lds_max = QF_COOP_MAX;   // tests: smaller forces the global-memory variant
extern "C" void amgd_qfactor_set_coop_lds(int m) { g_coop_lds_max = m < 0 ? QF_COOP_MAX : (uint32_t)m; }
static unsigned long g_qf_stats[3];   // huge supports factored sparse / sent to the dense kernel / split
extern "C" void amgd_qfactor_set_sparse(int m) {
  g_qf_sparse = m;
  g_qf_sparse_forced = m >= 0 && m != 1;   // 1 (the default) restores the automatic choice
}
extern "C" void amgd_qfactor_stats(unsigned long *st) {
  st[0] = g_qf_stats[0];
  st[1] = g_qf_stats[1];
  st[2] = g_qf_stats[2];
  g_qf_stats[0] = g_qf_stats[1] = g_qf_stats[2] = 0;
}
#define QF_T0 32
#define QF_T1 64
#define QF_T2 128
#define QF_T3 1024
// ---------------------------------------------------------------------------
// Huge supports split by connected components.  The Gram matrix A(Qj, Qj) of the
// orphan support (min_skel's column 0) is block-diagonal over the connected
// components of A restricted to Qj.  In the reference's factor every term that
// couples two components has an exact zero factor, so each sum it adds to starts
// at +0 and ends with the same bits over its own component only, and every
// cross-component entry of U is qk * al = +0 * (negative) = -0.  The support is
// therefore factored as independent sub-supports (one per component, members in
// ascending order, through the usual tiers) and scattered into the -0-filled
// triangle: bit-identical to factoring the whole support, in parallel instead of
// one sequential k-loop over tens of thousands of points.
// ---------------------------------------------------------------------------
__global__ void k_cc_init(const uint32_t *Qj, uint32_t nz, uint32_t *pos, uint32_t *lab) {
  GRID_STRIDE(k, nz) {
    pos[Qj[k]] = (uint32_t)k;
    lab[k] = (uint32_t)k;
  }
}
__global__ void k_cc_reset(const uint32_t *Qj, uint32_t nz, uint32_t *pos) {
  GRID_STRIDE(k, nz) pos[Qj[k]] = 0xffffffffu;
}
// min-label hooking over the edges of A inside the support, then pointer jumping
__global__ void k_cc_hook(const uint32_t *Qj, uint32_t nz, const uint64_t *aro,
                          const uint32_t *acol, const uint32_t *pos, uint32_t *lab,
                          unsigned *changed) {
  GRID_STRIDE(k, nz) {
    const uint32_t r = Qj[k];
    uint32_t m = lab[k];
    for (uint64_t e = aro[r]; e < aro[r + 1]; e++) {
      const uint32_t p = pos[acol[e]];
      if (p != 0xffffffffu) m = min(m, lab[p]);
    }
    bool ch = false;
    for (uint64_t e = aro[r]; e < aro[r + 1]; e++) {   // both ends of each edge (any pattern)
      const uint32_t p = pos[acol[e]];
      if (p == 0xffffffffu) continue;
      const uint32_t lp = lab[p];
      if (m < lp) { atomicMin(&lab[lp], m); atomicMin(&lab[p], m); ch = true; }
    }
    const uint32_t lk = lab[k];
    if (m < lk) { atomicMin(&lab[lk], m); atomicMin(&lab[k], m); ch = true; }
    if (ch) *changed = 1u;
  }
}
__global__ void k_cc_init_iota(uint32_t nz, uint32_t *lab) { GRID_STRIDE(k, nz) lab[k] = (uint32_t)k; }
__global__ void k_cc_jump(uint32_t nz, uint32_t *lab) {
  GRID_STRIDE(k, nz) {
    uint32_t l = lab[k];
    while (lab[l] != l) l = lab[l];
    lab[k] = l;
  }
}
__global__ void k_cc_keys(uint32_t nz, const uint32_t *lab, uint64_t *key) {
  GRID_STRIDE(k, nz) key[k] = ((uint64_t)lab[k] << 32) | k;
}
// component heads in the (label, k) order -> per-member component start flags
__global__ void k_cc_heads(uint32_t nz, const uint64_t *skey, uint64_t *head) {
  GRID_STRIDE(t, nz) head[t] = (t == 0 || (skey[t] >> 32) != (skey[t - 1] >> 32)) ? 1 : 0;
}
__global__ void k_cc_sub(uint32_t nz, const uint64_t *skey, const uint64_t *hscan,
                         const uint32_t *Qj, uint64_t *sro, uint32_t *scol, uint32_t *member) {
  GRID_STRIDE(t, nz) {
    const uint32_t k = (uint32_t)(skey[t] & 0xffffffffu);
    scol[t] = Qj[k];
    member[t] = k;
    if (t == 0 || (skey[t] >> 32) != (skey[t - 1] >> 32)) sro[hscan[t]] = t;
  }
}
// U[tri(gi) + gj] = Qs[qoff_s[comp] + tri(li) + lj], one thread per member row
__global__ void k_cc_scatter(uint32_t nz, const uint64_t *sro, uint32_t ncomp,
                             const uint32_t *member, const uint64_t *qoff_s, const double *Qs,
                             double *U) {
  GRID_STRIDE(t, nz) {
    uint32_t lo = 0, hi = ncomp;                 // component of member t
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (sro[mid] <= t) lo = mid; else hi = mid;
    }
    const uint64_t m0 = sro[lo];
    const uint64_t li = t - m0, gi = member[t];
    const double *src = Qs + qoff_s[lo] + tri(li);
    double *dst = U + tri(gi);
    for (uint64_t lj = 0; lj <= li; lj++) dst[member[m0 + lj]] = src[lj];
  }
}
static int g_qf_split = -1;     // AMGD_QF_SPLIT=0: no component split of huge supports
static int g_qf_split_depth = 0;
extern "C" void amgd_qfactor_set_split(int on) { g_qf_split = on < 0 ? -1 : on; }
static void qfactor_range(const dcsr *Wt, const dcsr *A, const uint64_t *qoff, double *Q,
                          uint32_t cb, uint32_t ce, uint64_t tot);
// Factor support c by components if it has more than one; returns false (nothing
// done) when it is one component.
static bool qfactor_split(uint32_t c, const dcsr *Wt, const dcsr *A, uint64_t w0, uint32_t nz,
                          double *U) {
  if (g_qf_split < 0) { const char *e = getenv("AMGD_QF_SPLIT"); g_qf_split = e ? atoi(e) : 1; }
  if (!g_qf_split || g_qf_split_depth > 0) return false;
  hipStream_t s = amgd_s();
  const uint32_t *Qj = Wt->col + w0;
  uint32_t *pos = (uint32_t *)amgd_alloc((size_t)A->cn * 4 + 4);
  HIPCK(hipMemsetAsync(pos, 0xff, (size_t)A->cn * 4, s));
  uint32_t *lab = (uint32_t *)amgd_alloc((size_t)nz * 4 + 4);
  unsigned *chg = (unsigned *)amgd_alloc(16);
  k_cc_init<<<grid_for(nz), 256, 0, s>>>(Qj, nz, pos, lab);
  for (int round = 0; round < 1000000; round++) {
    HIPCK(hipMemsetAsync(chg, 0, 4, s));
    k_cc_hook<<<grid_for(nz), 256, 0, s>>>(Qj, nz, A->ro, A->col, pos, lab, chg);
    k_cc_jump<<<grid_for(nz), 256, 0, s>>>(nz, lab);
    unsigned h = 0;
    amgd_d2h(&h, chg, 4);
    if (!h) break;
  }
  amgd_free(pos);
  amgd_free(chg);
  uint64_t *key = (uint64_t *)amgd_alloc((size_t)nz * 8 + 8), *skey = (uint64_t *)amgd_alloc((size_t)nz * 8 + 8);
  k_cc_keys<<<grid_for(nz), 256, 0, s>>>(nz, lab, key);
  size_t tb = 0;
  HIPCK(rocprim::radix_sort_keys(nullptr, tb, key, skey, (size_t)nz, 0, 64, s));
  void *tmp = amgd_alloc(tb + 16);
  HIPCK(rocprim::radix_sort_keys(tmp, tb, key, skey, (size_t)nz, 0, 64, s));
  amgd_free(tmp); amgd_free(key); amgd_free(lab);
  uint64_t *hs = (uint64_t *)amgd_alloc((size_t)nz * 8 + 16);
  k_cc_heads<<<grid_for(nz), 256, 0, s>>>(nz, skey, hs);
  const uint32_t ncomp = (uint32_t)amgd_scan_u64(hs, nz);
  bool done = false;
  if (ncomp > 1) {
    dcsr sub;
    sub.rn = ncomp;
    sub.cn = Wt->cn;
    sub.nnz = nz;
    sub.ro = (uint64_t *)amgd_alloc(((size_t)ncomp + 1) * 8);
    sub.col = (uint32_t *)amgd_alloc((size_t)nz * 4 + 4);
    sub.a = nullptr;
    uint32_t *member = (uint32_t *)amgd_alloc((size_t)nz * 4 + 4);
    k_cc_sub<<<grid_for(nz), 256, 0, s>>>(nz, skey, hs, Qj, sub.ro, sub.col, member);
    const uint64_t endv = nz;
    amgd_h2d(sub.ro + ncomp, &endv, 8);
    uint64_t *qoff_s = (uint64_t *)amgd_alloc(((size_t)ncomp + 1) * 8);
    k_qsize<<<grid_for(ncomp), 256, 0, s>>>(sub.ro, ncomp, qoff_s);
    const uint64_t tot_s = amgd_scan_u64(qoff_s, ncomp);
    double *Qs = (double *)amgd_alloc_f64(tot_s * 8 + 8);
    g_qf_split_depth++;
    qfactor_range(&sub, A, qoff_s, Qs, 0, ncomp, tot_s);
    g_qf_split_depth--;
    const uint64_t tn = (uint64_t)nz * (nz + 1) / 2;
    k_fill_negzero<<<grid_for(tn, 256, 65536), 256, 0, s>>>(U, tn);
    k_cc_scatter<<<grid_for(nz), 256, 0, s>>>(nz, sub.ro, ncomp, member, qoff_s, Qs, U);
    KCHECK();
    amgd_free(Qs); amgd_free(qoff_s); amgd_free(member); amgd_free(sub.col);
    g_qf_stats[2]++;
    if (getenv("AMGD_SGLOG")) {
      std::vector<uint64_t> hro(ncomp + 1);
      amgd_d2h(hro.data(), sub.ro, (ncomp + 1) * 8);
      uint64_t mx = 0, big = 0;
      for (uint32_t q = 0; q < ncomp; q++) {
        mx = std::max(mx, hro[q + 1] - hro[q]);
        big += hro[q + 1] - hro[q] > 1024;
      }
      fprintf(stderr, "qfactor split: support %u of %u points -> %u components (largest %lu, %lu past 1024)\n",
              c, nz, ncomp, (unsigned long)mx, (unsigned long)big);
    }
    amgd_free(sub.ro);
    done = true;
  }
  amgd_free(hs); amgd_free(skey);
  return done;
}

// Reuse of the previous skeleton's factors (amgd_qfactor_reuse): a coarse point's Q
// depends only on its support (row of Wt) and on A, fixed over a level's interpolation
// loop; expand_support adds entries to a minority of the supports per iteration
// (256^3: +0.004 % to +2 % entries in the late iterations that cost most), so every
// support identical to the previous iteration's takes its packed triangle by copy --
// the same bits the factor kernels would write again.
static uint8_t *g_qskip = nullptr;          // per coarse point: 1 = copy (current call)
static const double *g_qp_q = nullptr;      // the previous call's factors
static const uint64_t *g_qp_off = nullptr;
// after an unwound setup g_qskip points into a block the rollback already released:
// forget it (never free it again)
extern "C" void amgd_interp_reset_state(void) {
  g_qskip = nullptr;
  g_qp_q = nullptr;
  g_qp_off = nullptr;
  g_qf_split_depth = 0;
}
static uint64_t g_qf_reused = 0, g_qf_factored = 0;
// 1 where row c of Wt equals row c of Wp (same length, same columns): one wavefront per row
__global__ void k_supp_same(const uint64_t *ro, const uint32_t *col, const uint64_t *pro,
                            const uint32_t *pcol, uint32_t rn, uint8_t *same, unsigned *nsame) {
  const int lane = threadIdx.x & 63;
  unsigned cnt = 0;
  for (uint64_t c = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; c < rn;
       c += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
    const uint64_t k0 = ro[c], n = ro[c + 1] - k0, p0 = pro[c];
    bool eq = n == pro[c + 1] - p0 && n != 0;
    for (uint64_t k = lane; eq && k < n; k += 64) {
      const bool d = col[k0 + k] != pcol[p0 + k];
      if (__ballot(d)) eq = false;
    }
    if (lane == 0) same[c] = eq ? 1 : 0;
    cnt += eq;
  }
  // one atomic per work-group (one per row serialised on a single address: ~11 ms a call)
  __shared__ unsigned part[4];
  if (lane == 0) part[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = part[0] + part[1] + part[2] + part[3];
    if (t) atomicAdd(nsame, t);
  }
}
// copy the packed triangles of the skipped supports cb <= c < ce (one block per support);
// triangles past QCOPY_BIG doubles (the orphan support: 10^4 - 10^5 points, up to GBs) are
// listed instead and copied by the whole grid (k_qcopy_big): one block per such support
// took 88 ms per call on the anisotropic 256^3 setup (1.9 s of its 33.7 s,
// profiles/r06/aniso256_kernel_stats_r06d.csv)
#define QCOPY_BIG (1ull << 18)
__global__ void k_qcopy(const uint8_t *skip, const uint64_t *wro, uint32_t cb, uint32_t ce,
                        const uint64_t *poff, const double *Qp, const uint64_t *qoff, double *Q,
                        uint32_t *big, unsigned *nbig) {
  for (uint64_t c = cb + blockIdx.x; c < ce; c += gridDim.x) {
    if (!skip[c]) continue;
    const uint64_t nz = wro[c + 1] - wro[c], tn = nz * (nz + 1) / 2;
    if (tn > QCOPY_BIG) {
      if (threadIdx.x == 0) big[atomicAdd(nbig, 1u)] = (uint32_t)c;
      continue;
    }
    const double *src = Qp + poff[c];
    double *dst = Q + qoff[c];
    for (uint64_t t = threadIdx.x; t < tn; t += blockDim.x) dst[t] = src[t];
  }
}
__global__ void k_qcopy_big(const uint32_t *big, const unsigned *nbig, const uint64_t *wro, const uint64_t *poff,
                            const double *Qp, const uint64_t *qoff, double *Q) {
  const unsigned n = *nbig;
  for (unsigned b = 0; b < n; b++) {
    const uint32_t c = big[b];
    const uint64_t nz = wro[c + 1] - wro[c], tn = nz * (nz + 1) / 2;
    const double *src = Qp + poff[c];
    double *dst = Q + qoff[c];
    GRID_STRIDE(t, tn) dst[t] = src[t];
  }
}

// the factors of the coarse points cb <= c < ce (all tiers), into Q at qoff
static void qfactor_range(const dcsr *Wt, const dcsr *A, const uint64_t *qoff, double *Q,
                          uint32_t cb, uint32_t ce, uint64_t tot) {
  hipStream_t s = amgd_s();
  static int sglog = -1;
  if (sglog < 0) sglog = getenv("AMGD_SGLOG") != nullptr;
  double t_start = 0;
  if (sglog) { amgd_sync(); t_start = amgd_wtime(); }
  const uint32_t rn = Wt->rn;
  const uint64_t L = (uint64_t)rn + 1;
  // bins: LDS 32 / 64 / 128, blocked 256 / 512 / 1024, huge
  constexpr int NB = 7, HUGE = 6;
  // (a component split of a huge support factors a sub-matrix: no reuse in there)
  const uint8_t *skip = g_qf_split_depth == 0 ? g_qskip : nullptr;
  uint32_t *lists = (uint32_t *)amgd_alloc(NB * L * 4);
  unsigned *cnt = (unsigned *)amgd_alloc(32);
  amgd_memset(cnt, 0, 32);
  unsigned hn[NB] = {0, 0, 0, 0, 0, 0, 0};
  if (ce > cb) {
    k_bin_nz<<<grid_for(ce - cb), 256, 0, s>>>(Wt->ro, cb, ce,
                                              BinLim{{QF_T0, QF_T1, QF_T2, 256, 512, QF_T3}}, NB,
                                              lists, cnt, L, skip);
    uint32_t *bigc = nullptr;
    if (skip) {
      bigc = (uint32_t *)amgd_alloc(4ull * (ce - cb) + 4);
      k_qcopy<<<(int)std::min<uint32_t>(ce - cb, 16384u), 256, 0, s>>>(skip, Wt->ro, cb, ce, g_qp_off,
                                                                        g_qp_q, qoff, Q, bigc, cnt + NB);
      k_qcopy_big<<<2048, 256, 0, s>>>(bigc, cnt + NB, Wt->ro, g_qp_off, g_qp_q, qoff, Q);
    }
    KCHECK();
    amgd_d2h(hn, cnt, NB * 4);
    if (bigc) amgd_free(bigc);
  }
  // Huge supports (the orphan support gathered at coarse point 0): one cooperative
  // launch each on a side stream, issued before the other tiers so that its
  // latency-bound k-loop runs beside them instead of after them.  The stream is
  // idle here (the tier counts were just read back), so no event is needed before.
  static hipStream_t s2 = nullptr;
  static hipEvent_t ev2 = nullptr;
  std::vector<void *> coop_bufs;
  std::vector<uint32_t> big, bignz;
  std::vector<unsigned *> bigstat;
  auto launch_coop = [&](uint32_t c, uint32_t nz) {
    double *s1b = (double *)amgd_alloc_f64((size_t)nz * 8 * 4 + 8);
    double *s2v = s1b + 2 * (size_t)nz, *qk = s1b + 3 * (size_t)nz;
    unsigned *bar = (unsigned *)amgd_alloc(16);
    HIPCK(hipMemsetAsync(bar, 0, 16, s2));
    coop_bufs.push_back(s1b);
    coop_bufs.push_back(bar);
    int G = (int)std::min<uint32_t>((nz + 63) / 64, 256u);
    const uint64_t *pwro = Wt->ro, *paro = A->ro, *pqoff = qoff;
    const uint32_t *pwcol = Wt->col, *pacol = A->col;
    const double *paa = A->a;
    void *args[] = {&c, &pwro, &pwcol, &paro, &pacol, &paa, &pqoff, &Q, &s1b, &s2v, &qk, &bar};
    static bool attr = false;
    if (!attr) {
      HIPCK(hipFuncSetAttribute((const void *)k_qfactor_coop<true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 2 * QF_COOP_MAX * 8));
      attr = true;
    }
    if (nz <= g_coop_lds_max)
      HIPCK(hipLaunchCooperativeKernel((const void *)k_qfactor_coop<true>, dim3(G), dim3(64), args,
                                       (unsigned)(2 * (size_t)nz * 8), s2));
    else
      HIPCK(hipLaunchCooperativeKernel((const void *)k_qfactor_coop<false>, dim3(G), dim3(64), args,
                                       0u, s2));
    KCHECK();
  };
  if (hn[HUGE]) {
    if (!s2) {
      HIPCK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
      HIPCK(hipEventCreateWithFlags(&ev2, hipEventDisableTiming));
    }
    big.resize(hn[HUGE]);
    amgd_d2h(big.data(), lists + HUGE * L, (size_t)hn[HUGE] * 4);
    std::vector<uint64_t> ro(rn + 1), qo(rn + 1);
    amgd_d2h(ro.data(), Wt->ro, (size_t)(rn + 1) * 8);
    amgd_d2h(qo.data(), qoff, (size_t)(rn + 1) * 8);
    // components of a split support (connected clusters, heavy fill) up to 8192 points
    // factor dense unless a mode is forced: 1537 points at aniso 256^3 level 0, sparse
    // 3.0 s -> dense 0.21 s
    const int sp0 = qf_sparse_mode();
    auto sp_of = [&](uint32_t nz) {
      return g_qf_split_depth > 0 && nz <= 8192 && !g_qf_sparse_forced ? 0 : sp0;
    };
    std::vector<uint32_t> bigs;
    for (uint32_t c : big) {
      const uint32_t nz = (uint32_t)(ro[c + 1] - ro[c]);
      if (!qfactor_split(c, Wt, A, ro[c], nz, Q + qo[c])) bigs.push_back(c);
    }
    big.swap(bigs);
    if (!big.empty()) amgd_sync();          // the side stream must see the split's writes ordered
    for (uint32_t c : big) {
      uint32_t nz = (uint32_t)(ro[c + 1] - ro[c]);
      bignz.push_back(nz);
      const int sp = sp_of(nz);
      if (!sp) {
        bigstat.push_back(nullptr);
        launch_coop(c, nz);
        continue;
      }
      // sparse attempt; the dense kernel runs after the tiers if it reports failure
      const uint64_t tn = (uint64_t)nz * (nz + 1) / 2;
      const uint32_t cap = sp == 2 ? nz + 8 : (uint32_t)std::min<uint64_t>(tn, 1u << 24);
      const size_t nd = (size_t)nz * 3 + cap, nu = (size_t)nz * 6 + (size_t)cap * 3 + 2;
      char *mem = (char *)amgd_alloc(nd * 8 + nu * 4 + 64);
      coop_bufs.push_back(mem);
      QsBuf qb;
      qb.s1 = (double *)mem;
      qb.s2 = qb.s1 + nz;
      qb.qk = qb.s2 + nz;
      qb.uval = qb.qk + nz;
      uint32_t *u = (uint32_t *)(qb.uval + cap);
      qb.m2 = u;
      qb.m3 = u + nz;
      qb.L2 = u + 2 * (size_t)nz;
      qb.chead = u + 3 * (size_t)nz;
      qb.ctail = u + 4 * (size_t)nz;
      qb.rowptr = u + 5 * (size_t)nz;               // nz + 1
      qb.ucol = u + 6 * (size_t)nz + 1;
      qb.urow = qb.ucol + cap;
      qb.nxt = qb.urow + cap;
      qb.status = qb.nxt + cap;
      qb.cap = cap;
      HIPCK(hipMemsetAsync(mem, 0, (size_t)nz * 3 * 8, s2));
      HIPCK(hipMemsetAsync(qb.m2, 0, (size_t)nz * 3 * 4, s2));
      HIPCK(hipMemsetAsync(qb.chead, 0xff, (size_t)nz * 2 * 4, s2));
      k_fill_negzero<<<grid_for(tn), 256, 0, s2>>>(Q + qo[c], tn);
      k_qfactor_sparse<256><<<1, 256, 0, s2>>>(c, Wt->ro, Wt->col, A->ro, A->col, A->a, qoff, Q, qb);
      KCHECK();
      bigstat.push_back(qb.status);
    }
    HIPCK(hipEventRecord(ev2, s2));
  }
  // tiers by support size: the LDS triangle sized to the tier keeps small supports at
  // high occupancy (nz <= 32: 4 KB per wavefront)
  // <= 32 points: the LDS triangle; 33-64 / 65-128: the blocked kernel, 4 k-steps per pass
  // (round 5 A/Bs: 8 steps per pass or the LDS kernel on these tiers measured slower)
  if (hn[0])
    k_qfactor_lds<QF_T0, 64><<<(int)std::min<unsigned>(hn[0], 65536u), 64, 0, s>>>(
        lists, hn[0], Wt->ro, Wt->col, A->ro, A->col, A->a, qoff, Q);
  if (hn[1])
    k_qfactor_blk<QF_T1, 4, 64><<<(int)std::min<unsigned>(hn[1], 65536u), 64, 0, s>>>(
        lists + L, hn[1], Wt->ro, Wt->col, A->ro, A->col, A->a, qoff, Q);
  if (hn[2])
    k_qfactor_blk<QF_T2, 4, 128><<<(int)std::min<unsigned>(hn[2], 65536u), 128, 0, s>>>(
        lists + 2 * L, hn[2], Wt->ro, Wt->col, A->ro, A->col, A->a, qoff, Q);
  if (qf_blocked()) {
    // B = 4 k-steps per pass for the 256- and 512-point tiers: the waves mostly wait
    // (SQ_WAIT_ANY ~80 %), and the smaller S1/S2 tiles let 4 blocks share a CU
    // (512 tier, 47782-column call at 256^3: B 8 -> 4: 419 -> 318 ms)
    if (hn[3])
      k_qfactor_blk<256, 4><<<(int)std::min<unsigned>(hn[3], 8192u), 256, 0, s>>>(
          lists + 3 * L, hn[3], Wt->ro, Wt->col, A->ro, A->col, A->a, qoff, Q);
    if (hn[4]) amgd_route_hit(AMGD_R_QF_T512);
    if (hn[5]) amgd_route_hit(AMGD_R_QF_T1024);
    if (hn[4])
      k_qfactor_blk<512, 4><<<(int)std::min<unsigned>(hn[4], 8192u), 256, 0, s>>>(
          lists + 4 * L, hn[4], Wt->ro, Wt->col, A->ro, A->col, A->a, qoff, Q);
    if (hn[5])
      k_qfactor_blk<QF_T3, 4><<<(int)std::min<unsigned>(hn[5], 8192u), 256, 0, s>>>(
          lists + 5 * L, hn[5], Wt->ro, Wt->col, A->ro, A->col, A->a, qoff, Q);
  } else {
    for (int q = 3; q < 6; q++)
      if (hn[q])
        k_qfactor_mid<<<(int)std::min<unsigned>(hn[q], 8192u), 256, 0, s>>>(
            lists + q * L, hn[q], Wt->ro, Wt->col, A->ro, A->col, A->a, qoff, Q);
  }
  KCHECK();
  if (hn[HUGE]) {                 // the library stream waits for the side stream
    bool redo = false;
    for (size_t q = 0; q < big.size(); q++) {
      if (!bigstat[q]) continue;
      unsigned st = 0;
      HIPCK(hipMemcpyAsync(&st, bigstat[q], 4, hipMemcpyDeviceToHost, s2));
      HIPCK(hipStreamSynchronize(s2));
      if (st) {                     // dense cooperative factor (overwrites the triangle)
        amgd_sync();                // scratch reuse is ordered after the library stream
        launch_coop(big[q], bignz[q]);
        redo = true;
      }
      g_qf_stats[st ? 1 : 0]++;
    }
    if (redo) HIPCK(hipEventRecord(ev2, s2));
    HIPCK(hipStreamWaitEvent(s, ev2, 0));
    for (void *p : coop_bufs) amgd_free(p);   // reuse is ordered after the wait
  }
  if (sglog) {
    amgd_sync();
    fprintf(stderr, "qfactor cols %u nnz %lu tiers %u/%u/%u/%u/%u/%u/%u (huge nz %u) Q %lu  %.2f ms\n",
            rn, (unsigned long)Wt->nnz, hn[0], hn[1], hn[2], hn[3], hn[4], hn[5], hn[6],
            bignz.empty() ? 0u : bignz[0], (unsigned long)tot, (amgd_wtime() - t_start) * 1e3);
  }
  amgd_free(lists); amgd_free(cnt);
}

// Q factors of every coarse point.  Sharded (amgd_comm.hip): coarse points split
// into contiguous ranges of equal factor work (nz^3), each rank factors its
// ranges into the global Q, one allgatherv of the Q segments completes it.
// Supports past the blocked tiers (> 1024 points: the orphan supports) are factored
// per connected component (qfactor_split) or by the sparse kernel, far below nz^3: their
// cost is capped at nz^2 * 1024, so one huge support no longer takes a rank's whole share.
__global__ void k_qcost(const uint64_t *wro, uint32_t rn, uint64_t *cost, const uint8_t *skip) {
  GRID_STRIDE(c, rn) {
    uint64_t nz = wro[c + 1] - wro[c];
    cost[c] = (skip && skip[c] ? nz * nz / 8 : nz <= 1024 ? nz * nz * nz : nz * nz * 1024) + 1;
  }
}
#define QF_SHARD_MIN (1ull << 30)   // factor work (sum nz^3) below which one GPU does all
static int g_qf_reuse = -1;     // AMGD_QF_REUSE=0 / amgd_qfactor_set_reuse(0): refactor every support
static int qf_reuse_on() {
  if (g_qf_reuse < 0) { const char *e = getenv("AMGD_QF_REUSE"); g_qf_reuse = e && *e ? atoi(e) : 1; }
  return g_qf_reuse;
}
extern "C" void amgd_qfactor_set_reuse(int on) { g_qf_reuse = on < 0 ? -1 : on; }
extern "C" void amgd_qfactor_reuse_stats(uint64_t *reused, uint64_t *factored) {
  *reused = g_qf_reused; *factored = g_qf_factored;
}
extern "C" double *amgd_qfactor(const dcsr *Wt, const dcsr *A, uint64_t **qoff_out,
                                uint64_t *qtotal) {
  return amgd_qfactor_reuse(Wt, A, qoff_out, qtotal, nullptr, nullptr, nullptr);
}
extern "C" double *amgd_qfactor_reuse(const dcsr *Wt, const dcsr *A, uint64_t **qoff_out,
                                      uint64_t *qtotal, const dcsr *Wp, const double *Qp,
                                      const uint64_t *qpoff) {
  hipStream_t s = amgd_s();
  const uint32_t rn = Wt->rn;
  const uint64_t L = (uint64_t)rn + 1;
  uint64_t *qoff = (uint64_t *)amgd_alloc(L * 8);
  if (rn) k_qsize<<<grid_for(rn), 256, 0, s>>>(Wt->ro, rn, qoff);
  uint64_t tot = amgd_scan_u64(qoff, rn);
  double *Q = (double *)amgd_alloc_f64(tot * 8 + 8);
  if (Wp && Qp && qpoff && Wp->rn == rn && rn && qf_reuse_on()) {
    g_qskip = (uint8_t *)amgd_alloc((size_t)rn + 1);
    unsigned *ns = (unsigned *)amgd_alloc(16);
    amgd_memset(ns, 0, 4);
    k_supp_same<<<grid_for((uint64_t)rn * 64, 256, 16384), 256, 0, s>>>(Wt->ro, Wt->col, Wp->ro, Wp->col,
                                                                       rn, g_qskip, ns);
    KCHECK();
    unsigned hs = 0;
    amgd_d2h(&hs, ns, 4);
    amgd_free(ns);
    g_qf_reused += hs;
    if (hs) amgd_route_hit(AMGD_R_QF_REUSE);
    g_qf_factored += rn - hs;
    if (hs == 0) { amgd_free(g_qskip); g_qskip = nullptr; }
    g_qp_q = Qp;
    g_qp_off = qpoff;
  } else {
    g_qf_factored += rn;
  }
  const int N = amgd_nshards();
  uint64_t work = 0;
  uint64_t *cost = nullptr;
  if (N > 1 && rn >= (uint32_t)N) {
    cost = (uint64_t *)amgd_alloc(L * 8);
    k_qcost<<<grid_for(rn), 256, 0, s>>>(Wt->ro, rn, cost, g_qskip);
    KCHECK();
    work = amgd_scan_u64(cost, rn);
  }
  if (!cost || !amgd_shard_worth(work, QF_SHARD_MIN)) {
    qfactor_range(Wt, A, qoff, Q, 0, rn, tot);
  } else {
    std::vector<uint32_t> split(N + 1);
    amgd_shard_split(cost, rn, split.data());
    std::vector<uint64_t> qo(N + 1);
    amgd_gather_u64_at(qoff, split.data(), N + 1, qo.data());
    int f, l;
    amgd_my_shards(&f, &l);
    for (int q = f; q < l; q++) qfactor_range(Wt, A, qoff, Q, split[q], split[q + 1], tot);
    for (auto &v : qo) v *= 8;
    void *b = Q;
    amgd_allgatherv(1, &b, qo.data());
  }
  if (cost) amgd_free(cost);
  if (g_qskip) { amgd_free(g_qskip); g_qskip = nullptr; }
  g_qp_q = nullptr;
  g_qp_off = nullptr;
  *qoff_out = qoff;
  if (qtotal) *qtotal = tot;
  return Q;
}


// ---------------------------------------------------------------------------
// Q application (the tail of interp, amg_setup.c:2100-2108):
//   out(c, :) = Q Q^t ( Bt(c, Qj) + u_c * lambda(Qj) )
// ---------------------------------------------------------------------------
template <int NT, bool GSCR>
__global__ __launch_bounds__(NT) void k_qapply(const uint32_t *rows, uint32_t nrows,
                                               const uint64_t *wro, const uint32_t *wcol,
                                               const double *Q, const uint64_t *qoff,
                                               const uint64_t *bro, const uint32_t *bcol,
                                               const double *ba, const double *u,
                                               const double *lambda, double *out, double *gscr,
                                               uint64_t gstride) {
  __shared__ double lds[GSCR ? 1 : 2 * QF_LDS_NZ];
  const int tid = threadIdx.x;
  for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    uint32_t c = rows[r];
    uint64_t w0 = wro[c];
    uint32_t nz = (uint32_t)(wro[c + 1] - w0);
    const uint32_t *Qj = wcol + w0;
    const double *Qc = Q + qoff[c];
    double *sqv1 = GSCR ? gscr + (uint64_t)blockIdx.x * gstride : lds;
    double *sqv2 = GSCR ? sqv1 + nz : lds + QF_LDS_NZ;
    uint64_t b0 = bro[c], b1 = bro[c + 1];
    double uc = u[c];
    for (uint32_t m = tid; m < nz; m += NT) {
      double v = row_lookup(bcol, ba, b0, b1, Qj[m]);
      sqv1[m] = v + uc * lambda[Qj[m]];
    }
    __syncthreads();
    for (uint32_t i = tid; i < nz; i += NT) {
      const double *U = Qc + tri(i);
      double v = 0;
      for (uint32_t j = 0; j <= i; j++) v += U[j] * sqv1[j];
      sqv2[i] = v;
    }
    __syncthreads();
    for (uint32_t i = tid; i < nz; i += NT) {
      double y = 0;
      for (uint32_t j = i; j < nz; j++) y += Qc[tri(j) + i] * sqv2[j];
      out[w0 + i] = y;
    }
    __syncthreads();
  }
}
// k_qapply's first triangular product with U staged through LDS in tiles of 64 rows x T
// columns (round 5).  Lane i walks row i of U left to right: in k_qapply every lane reads
// its own row, so one load instruction touches 64 cache lines (texture-address work per
// line, as in the long-row SpMV); a tile load covers 64 / T rows x T consecutive entries.
// Each lane then continues its chain over the tile in order: the same products, the
// same left-to-right sums.  The second product (lanes across i at fixed j) is coalesced
// already and unchanged.
template <int T>
__global__ __launch_bounds__(64) void k_qapply_t(const uint32_t *rows, uint32_t nrows,
                                                 const uint64_t *wro, const uint32_t *wcol,
                                                 const double *Q, const uint64_t *qoff,
                                                 const uint64_t *bro, const uint32_t *bcol,
                                                 const double *ba, const double *u,
                                                 const double *lambda, double *out) {
  __shared__ double sq1[QF_LDS_NZ], sq2[QF_LDS_NZ];
  __shared__ double tile[64][T + 1];
  const uint32_t lane = threadIdx.x;
  for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    const uint32_t c = rows[r];
    const uint64_t w0 = wro[c];
    const uint32_t nz = (uint32_t)(wro[c + 1] - w0);
    const uint32_t *Qj = wcol + w0;
    const double *Qc = Q + qoff[c];
    const uint64_t b0 = bro[c], b1 = bro[c + 1];
    const double uc = u[c];
    for (uint32_t m = lane; m < nz; m += 64) {
      const double v = row_lookup(bcol, ba, b0, b1, Qj[m]);
      sq1[m] = v + uc * lambda[Qj[m]];
    }
    __syncthreads();
    for (uint32_t i0 = 0; i0 < nz; i0 += 64) {
      const uint32_t i = i0 + lane, nr = min(64u, nz - i0), jend = i0 + nr;
      double v = 0;
      for (uint32_t j0 = 0; j0 < jend; j0 += T) {
#pragma unroll
        for (int q = 0; q < T; q++) {
          const uint32_t fl = (uint32_t)q * 64 + lane, rr = fl / T, jj = fl % T;
          const uint32_t ii = i0 + rr, j = j0 + jj;
          tile[rr][jj] = rr < nr && j <= ii ? Qc[tri(ii) + j] : 0.0;
        }
        __syncthreads();
        if (i < nz && i >= j0) {
          const uint32_t jn = min((uint32_t)T, i + 1 - j0);
          for (uint32_t jj = 0; jj < jn; jj++) v += tile[lane][jj] * sq1[j0 + jj];
        }
        __syncthreads();
      }
      if (i < nz) sq2[i] = v;
    }
    __syncthreads();
    for (uint32_t i = lane; i < nz; i += 64) {
      double y = 0;
      for (uint32_t j = i; j < nz; j++) y += Qc[tri(j) + i] * sq2[j];
      out[w0 + i] = y;
    }
    __syncthreads();
  }
}
// AMGD_QA_TILE / amgd_qa_set_tile (tests, A/B): 16 (default: 256^3 24.94 -> 24.84 s,
// profiles/r05/abq_qapply_tiles.txt), 32 (25.08 s), 0 the row-per-lane k_qapply<64>
static int g_qa_tile = -1;
extern "C" void amgd_qa_set_tile(int t) { g_qa_tile = t; }
// Small supports (nz <= SEG: most coarse points of the fine levels) take SEG lanes each,
// 256 / SEG supports per work-group, synchronised per wavefront: a 64-lane group per
// support left most lanes idle and paid three block barriers per support.  Same sums in
// the same order as k_qapply.
template <int SEG>
__global__ __launch_bounds__(256) void k_qapply_small(const uint32_t *rows, uint32_t nrows,
                                                      const uint64_t *wro, const uint32_t *wcol,
                                                      const double *Q, const uint64_t *qoff,
                                                      const uint64_t *bro, const uint32_t *bcol,
                                                      const double *ba, const double *u,
                                                      const double *lambda, double *out) {
  constexpr int G = 256 / SEG;
  __shared__ double s1[G][SEG], s2[G][SEG];
  const int g = threadIdx.x / SEG, m = threadIdx.x % SEG;
  for (uint64_t rb = (uint64_t)blockIdx.x * G; rb < nrows; rb += (uint64_t)gridDim.x * G) {
    const uint64_t r = rb + g;
    uint32_t c = 0, nz = 0;
    uint64_t w0 = 0;
    if (r < nrows) {
      c = rows[r];
      w0 = wro[c];
      nz = (uint32_t)(wro[c + 1] - w0);
    }
    const bool act = (uint32_t)m < nz;
    const double *Qc = act ? Q + qoff[c] : Q;
    if (act) {
      const uint32_t j = wcol[w0 + m];
      s1[g][m] = row_lookup(bcol, ba, bro[c], bro[c + 1], j) + u[c] * lambda[j];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (act) {
      const double *U = Qc + tri(m);
      double v = 0;
      for (int j = 0; j <= m; j++) v += U[j] * s1[g][j];
      s2[g][m] = v;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (act) {
      double y = 0;
      for (uint32_t j = m; j < nz; j++) y += Qc[tri(j) + m] * s2[g][j];
      out[w0 + m] = y;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}
// supports of a list with nz <= lim appended to small, the rest to rest (cnt[0], cnt[1])
// (nd: the list's length on the device, read instead of n)
__global__ void k_split_small(const uint32_t *list, unsigned n, const unsigned *nd,
                              const uint64_t *wro, uint32_t lim, uint32_t *small, uint32_t *rest,
                              unsigned *cnt) {
  if (nd) n = *nd;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t c0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t iters = (n + stride - 1) / stride;
  for (uint64_t it = 0; it < iters; it++) {   // uniform trip count (wave_append)
    const uint64_t r = c0 + it * stride;
    const bool v = r < n;
    const uint32_t c = v ? list[r] : 0;
    const bool sm = v && wro[c + 1] - wro[c] <= lim;
    const unsigned p = wave_append(&cnt[0], sm);
    if (sm) small[p] = c;
    const unsigned q = wave_append(&cnt[1], v && !sm);
    if (v && !sm) rest[q] = c;
  }
}
static int g_qa_small = -1;     // AMGD_QA_SMALL=0: every support <= 512 points on k_qapply<64>
// Huge supports (> QA_HUGE points: the orphan support of min_skel's zero column) are
// applied by three grid-wide kernels instead of one work-group: the same sums in the
// same order, spread over the chip (one lane per row of U for sqv2, one lane per
// column for out, lanes of a wave in lock-step over 32-element batches).
#define QA_HUGE 8192
static uint32_t g_qa_huge = QA_HUGE;      // tests: smaller sends more supports to the grid path
extern "C" void amgd_qapply_set_huge(int n) { g_qa_huge = n < 0 ? QA_HUGE : (uint32_t)n; }
__global__ void k_qa_big_s1(uint32_t c, const uint64_t *wro, const uint32_t *wcol,
                            const uint64_t *bro, const uint32_t *bcol, const double *ba,
                            const double *u, const double *lambda, double *sqv1) {
  const uint64_t w0 = wro[c];
  const uint32_t nz = (uint32_t)(wro[c + 1] - w0);
  const uint64_t b0 = bro[c], b1 = bro[c + 1];
  const double uc = u[c];
  GRID_STRIDE(m, nz) {
    const uint32_t j = wcol[w0 + m];
    sqv1[m] = row_lookup(bcol, ba, b0, b1, j) + uc * lambda[j];
  }
}
__global__ void k_qa_big_rows(uint32_t nz, const double *U, const double *sqv1, double *sqv2) {
  GRID_STRIDE(i, nz) sqv2[i] = seq_dot_batched(U + tri(i), sqv1, (uint32_t)i + 1);
}
__global__ void k_qa_big_cols(uint32_t nz, const double *U, const double *sqv2, double *out) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t ib = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) - lane; ib < nz;
       ib += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t i = (uint32_t)ib + lane;
    const double y = mv_ut_lane(U, sqv2, (uint32_t)ib, i, nz);
    if (i < nz) out[i] = y;
  }
}
static void qapply_range(const dcsr *Wt, const double *Q, const uint64_t *qoff, const dcsr *Bt,
                         const double *u, const double *lambda, double *out, uint32_t cb,
                         uint32_t ce) {
  hipStream_t s = amgd_s();
  RowSplit rs = split_rows(Wt, QF_LDS_NZ, cb, ce);
  if (rs.nb && rs.maxnz > g_qa_huge) {          // the huge supports: grid-wide kernels
    std::vector<uint32_t> bl(rs.nb);
    amgd_d2h(bl.data(), rs.bl, (size_t)rs.nb * 4);
    std::vector<uint64_t> ro(Wt->rn + 1ull), qo(Wt->rn + 1ull);
    amgd_d2h(ro.data(), Wt->ro, ((size_t)Wt->rn + 1) * 8);
    amgd_d2h(qo.data(), qoff, ((size_t)Wt->rn + 1) * 8);
    std::vector<uint32_t> keep;
    double *scr = (double *)amgd_alloc_f64(2 * rs.maxnz * 8 + 16);
    for (uint32_t c : bl) {
      const uint32_t nz = (uint32_t)(ro[c + 1] - ro[c]);
      if (nz <= g_qa_huge) { keep.push_back(c); continue; }
      double *sqv1 = scr, *sqv2 = scr + rs.maxnz + 1;
      k_qa_big_s1<<<grid_for(nz), 256, 0, s>>>(c, Wt->ro, Wt->col, Bt->ro, Bt->col, Bt->a, u,
                                              lambda, sqv1);
      k_qa_big_rows<<<grid_for(nz), 256, 0, s>>>(nz, Q + qo[c], sqv1, sqv2);
      k_qa_big_cols<<<grid_for(nz), 256, 0, s>>>(nz, Q + qo[c], sqv2, out + ro[c]);
      KCHECK();
    }
    amgd_free(scr);
    rs.nb = (unsigned)keep.size();
    if (rs.nb) amgd_h2d(rs.bl, keep.data(), (size_t)rs.nb * 4);
  }
  if (g_qa_small < 0) {
    const char *e = getenv("AMGD_QA_SMALL");
    g_qa_small = e && *e ? atoi(e) : 1;
  }
  if (rs.ns && g_qa_small) {        // <= 16 and 17..32 points: lane groups; the rest below
    uint32_t *l16 = (uint32_t *)amgd_alloc(3ull * rs.ns * 4 + 16);
    uint32_t *l32 = l16 + rs.ns, *lrest = l32 + rs.ns, *tmp = lrest;
    unsigned *cnt = (unsigned *)amgd_alloc(32);
    amgd_memset(cnt, 0, 32);
    k_split_small<<<grid_for(rs.ns), 256, 0, s>>>(rs.sl, rs.ns, nullptr, Wt->ro, 16, l16, tmp, cnt);
    k_split_small<<<grid_for(rs.ns), 256, 0, s>>>(tmp, rs.ns, cnt + 1, Wt->ro, 32, l32, rs.sl,
                                                 cnt + 2);
    unsigned h[4];
    KCHECK();
    amgd_d2h(h, cnt, 16);
    if (h[0])
      k_qapply_small<16><<<(int)std::min<uint64_t>((h[0] + 15) / 16, 65536), 256, 0, s>>>(
          l16, h[0], Wt->ro, Wt->col, Q, qoff, Bt->ro, Bt->col, Bt->a, u, lambda, out);
    if (h[2])
      k_qapply_small<32><<<(int)std::min<uint64_t>((h[2] + 7) / 8, 65536), 256, 0, s>>>(
          l32, h[2], Wt->ro, Wt->col, Q, qoff, Bt->ro, Bt->col, Bt->a, u, lambda, out);
    rs.ns = h[3];
    amgd_free(cnt);
    amgd_free(l16);
  }
  if (rs.ns) {
    int g = (int)std::min<unsigned>(rs.ns, 65536u);
    if (g_qa_tile == -1) {
      const char *e = getenv("AMGD_QA_TILE");
      g_qa_tile = e && *e ? atoi(e) : 16;
    }
    if (g_qa_tile == 16)
      k_qapply_t<16><<<g, 64, 0, s>>>(rs.sl, rs.ns, Wt->ro, Wt->col, Q, qoff, Bt->ro, Bt->col,
                                      Bt->a, u, lambda, out);
    else if (g_qa_tile == 32)
      k_qapply_t<32><<<g, 64, 0, s>>>(rs.sl, rs.ns, Wt->ro, Wt->col, Q, qoff, Bt->ro, Bt->col,
                                      Bt->a, u, lambda, out);
    else
      k_qapply<64, false><<<g, 64, 0, s>>>(rs.sl, rs.ns, Wt->ro, Wt->col, Q, qoff, Bt->ro, Bt->col,
                                           Bt->a, u, lambda, out, nullptr, 0);
  }
  if (rs.nb) {
    int g = (int)std::min<unsigned>(rs.nb, 1024u);
    uint64_t stride = 2 * rs.maxnz + 8;
    double *scr = (double *)amgd_alloc_f64((size_t)g * stride * 8);
    k_qapply<256, true><<<g, 256, 0, s>>>(rs.bl, rs.nb, Wt->ro, Wt->col, Q, qoff, Bt->ro, Bt->col,
                                          Bt->a, u, lambda, out, scr, stride);
    amgd_free(scr);
  }
  KCHECK();
  free_split(rs);
}
// sharded like the factor: ranges of equal work (nz^2), allgatherv of the out segments
__global__ void k_qacost(const uint64_t *wro, uint32_t rn, uint64_t *cost) {
  GRID_STRIDE(c, rn) {
    uint64_t nz = wro[c + 1] - wro[c];
    cost[c] = nz * nz + 1;
  }
}
#define QA_SHARD_MIN (1ull << 27)
extern "C" void amgd_qapply(const dcsr *Wt, const double *Q, const uint64_t *qoff, const dcsr *Bt,
                            const double *u, const double *lambda, double *out) {
  const int N = amgd_nshards();
  const uint32_t rn = Wt->rn;
  if (N <= 1 || rn < (uint32_t)N) {
    qapply_range(Wt, Q, qoff, Bt, u, lambda, out, 0, rn);
    return;
  }
  uint64_t *cost = (uint64_t *)amgd_alloc(((size_t)rn + 1) * 8);
  k_qacost<<<grid_for(rn), 256, 0, amgd_s()>>>(Wt->ro, rn, cost);
  KCHECK();
  const uint64_t work = amgd_scan_u64(cost, rn);
  if (!amgd_shard_worth(work, QA_SHARD_MIN)) {
    amgd_free(cost);
    qapply_range(Wt, Q, qoff, Bt, u, lambda, out, 0, rn);
    return;
  }
  std::vector<uint32_t> split(N + 1);
  amgd_shard_split(cost, rn, split.data());
  amgd_free(cost);
  std::vector<uint64_t> wo(N + 1);
  amgd_gather_u64_at(Wt->ro, split.data(), N + 1, wo.data());
  int f, l;
  amgd_my_shards(&f, &l);
  for (int q = f; q < l; q++) qapply_range(Wt, Q, qoff, Bt, u, lambda, out, split[q], split[q + 1]);
  for (auto &v : wo) v *= 8;
  void *b = out;
  amgd_allgatherv(1, &b, wo.data());
}

// ---------------------------------------------------------------------------
// interp_lmop (amg_setup.c:1589): S := sum over coarse c (ascending) of
// u_c * QQt_c scattered with sp_add's forward walk (amg_setup.c:1665).
// Contribution (c, k, m) = u_c * sum_{t>=max(k,m)} q_t[k]*q_t[m] lands where
// the walk over row Qj[k] of S meets column Qj[m] (or, if absent, the next
// stored entry -- the reference's behaviour).  Contributions are generated in
// (c, k, m) order, stably radix-sorted by landing position and added to S in
// that order: bit-identical to the reference's sequential accumulation.
// ---------------------------------------------------------------------------
// (1) landing positions: one thread per (c, k) replays sp_add's forward walk
// over S starting at row Qj[k].  The reference steps one stored entry at a
// time (and keeps going into the following rows when a column is absent);
// here each step is a lower_bound inside the current row plus, when the row
// is exhausted, a skip over whole rows using per-row / per-64-row /
// per-4096-row column maxima -- the same landing, O(log) instead of O(nnz).
// Partitioned mode (amgd_psetup.c p_lmop): S is a rank's global-row view (other ranks' rows
// empty).  A walk that starts in another rank's row finds it empty and lands nowhere -- its
// owner lands it -- but a walk that runs past this rank's last row would, in the whole S,
// go on into the next rank's rows: it is flagged here (d_lmop_spill) and the caller redoes
// the operator on gathered data.  Off on one GPU and on the last rank (the end of S is the
// end of S there: the reference's UB, skipped as before).
__device__ int d_lmop_spill_on = 0, d_lmop_spill = 0;
extern "C" void amgd_lmop_spill_detect(int on) {
  int z = 0;
  HIPCK(hipMemcpyToSymbolAsync(HIP_SYMBOL(d_lmop_spill_on), &on, sizeof(int), 0, hipMemcpyHostToDevice, amgd_s()));
  HIPCK(hipMemcpyToSymbolAsync(HIP_SYMBOL(d_lmop_spill), &z, sizeof(int), 0, hipMemcpyHostToDevice, amgd_s()));
  HIPCK(hipStreamSynchronize(amgd_s()));
}
extern "C" int amgd_lmop_spilled(void) {
  int v = 0;
  HIPCK(hipMemcpyFromSymbolAsync(&v, HIP_SYMBOL(d_lmop_spill), sizeof(int), 0, hipMemcpyDeviceToHost, amgd_s()));
  HIPCK(hipStreamSynchronize(amgd_s()));
  return v;
}
__device__ __forceinline__ uint64_t lower_bound_u32(const uint32_t *a, uint64_t lo, uint64_t hi,
                                                    uint32_t x) {
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (a[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
// first row r2 > r with rowmax[r2] >= x, or nrows
__device__ uint32_t next_row_ge(const int64_t *rmax, const int64_t *b64, const int64_t *b4k,
                                uint32_t nrows, uint32_t r, int64_t x) {
  uint32_t r2 = r + 1;
  while (r2 < nrows && (r2 & 63)) { if (rmax[r2] >= x) return r2; r2++; }
  while (r2 < nrows && (r2 & 4095)) {
    if (b64[r2 >> 6] >= x) {
      for (uint32_t q = r2; q < r2 + 64 && q < nrows; q++) if (rmax[q] >= x) return q;
    }
    r2 += 64;
  }
  while (r2 < nrows) {
    if (b4k[r2 >> 12] >= x) {
      for (uint32_t q = r2; q < r2 + 4096 && q < nrows; q += 64)
        if (b64[q >> 6] >= x)
          for (uint32_t p = q; p < q + 64 && p < nrows; p++) if (rmax[p] >= x) return p;
    }
    r2 += 4096;
  }
  return nrows;
}
__global__ void k_rowmax(const uint64_t *ro, const uint32_t *col, uint32_t n, int64_t *rmax) {
  GRID_STRIDE(r, n) rmax[r] = ro[r + 1] > ro[r] ? (int64_t)col[ro[r + 1] - 1] : -1;
}
// 2^shift-row maxima, one wavefront per block of rows (coalesced)
__global__ void k_blockmax_wave(const int64_t *in, uint64_t n, int shift, int64_t *out,
                                uint64_t nout) {
  const int lane = threadIdx.x & 63;
  for (uint64_t b = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; b < nout;
       b += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
    int64_t m = -1;
    const uint64_t s0 = b << shift, s1 = min(n, (b + 1) << shift);
    for (uint64_t q = s0 + lane; q < s1; q += 64) m = in[q] > m ? in[q] : m;
    for (int o = 32; o; o >>= 1) { const int64_t y = __shfl_xor(m, o, 64); m = y > m ? y : m; }
    if (lane == 0) out[b] = m;
  }
}
__global__ void k_lmop_land(const uint32_t *erow, uint64_t e0, uint64_t e1, const uint64_t *wro,
                            const uint32_t *wcol, const uint64_t *sro, const uint32_t *scol,
                            uint32_t srn, uint64_t snnz, const int64_t *rmax, const int64_t *b64,
                            const int64_t *b4k, const uint64_t *coff, uint64_t cbase,
                            uint64_t *key) {
  for (uint64_t e = e0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < e1;
       e += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t c = erow[e];
    uint64_t w0 = wro[c];
    uint32_t nz = (uint32_t)(wro[c + 1] - w0);
    uint32_t k = (uint32_t)(e - w0);
    const uint32_t *Qj = wcol + w0;
    uint64_t o = coff[c] - cbase + (uint64_t)k * nz;
    uint32_t r = Qj[k];                      // walk starts in row Qj[k]
    uint64_t t = sro[r];
    bool live = sro[r + 1] != t;             // sp_add returns at once on an empty row
    for (uint32_t m = 0; m < nz; m++) {
      uint64_t land = snnz;                  // "no landing" sorts after every real position
      if (live) {
        uint32_t xm = Qj[m];
        uint64_t end = sro[r + 1];
        if (t < end && rmax[r] >= (int64_t)xm) {
          land = lower_bound_u32(scol, t, end, xm);
        } else {
          uint32_t r2 = next_row_ge(rmax, b64, b4k, srn, r, (int64_t)xm);
          if (r2 >= srn) {                   // reference runs off the end of St (UB)
            live = false;
            if (d_lmop_spill_on) d_lmop_spill = 1;
          }
          else { r = r2; land = lower_bound_u32(scol, sro[r2], sro[r2 + 1], xm); }
        }
        // next step starts after the landing; if that is the end of row r, the
        // "current row" test fails and the skip starts at row r+1 = position t
        if (live) t = land + 1;
      }
      key[o + m] = land;
    }
  }
}
// The same walk, one wavefront per (c, k), for long supports (the orphan support of
// a few thousand points: a thread's walk was a chain of nz binary searches).  The 64
// lanes search the next 64 columns Qj[m..m+63] from the current position t at once.
// Along a run of exact matches in the current row that IS the sequential walk: the
// columns increase, so each earlier landing lies before the next column's position
// and a search from t finds it.  The prefix of exact lanes is taken, then the first
// non-exact step: its search from t equals the one from its predecessor's landing + 1
// (everything in between is below its column) when it still lands in the row; a step
// that leaves the row (column past the row's last) runs the row skip as before.
__global__ __launch_bounds__(256) void k_lmop_land_wave(
    const uint32_t *erow, uint64_t e0, uint64_t e1, const uint64_t *wro, const uint32_t *wcol,
    const uint64_t *sro, const uint32_t *scol, uint32_t srn, uint64_t snnz, const int64_t *rmax,
    const int64_t *b64, const int64_t *b4k, const uint64_t *coff, uint64_t cbase, uint64_t *key) {
  const int lane = threadIdx.x & 63;
  for (uint64_t e = e0 + (((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6); e < e1;
       e += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
    const uint32_t c = erow[e];
    const uint64_t w0 = wro[c];
    const uint32_t nz = (uint32_t)(wro[c + 1] - w0);
    const uint32_t k = (uint32_t)(e - w0);
    const uint32_t *Qj = wcol + w0;
    const uint64_t o = coff[c] - cbase + (uint64_t)k * nz;
    uint32_t r = Qj[k];
    uint64_t t = sro[r];
    bool live = sro[r + 1] != t;
    uint32_t m = 0;
    while (m < nz) {
      if (!live) {
        for (uint32_t q = m + lane; q < nz; q += 64) key[o + q] = snnz;
        break;
      }
      const uint64_t end = sro[r + 1];
      const uint32_t nv = min(64u, nz - m);
      const bool valid = (uint32_t)lane < nv;
      const uint32_t xm = valid ? Qj[m + lane] : 0u;
      uint64_t L = end;
      bool inrow = false, exact = false;
      if (valid && t < end) {
        L = lower_bound_u32(scol, t, end, xm);
        inrow = L < end;                              // = rmax[r] >= xm
        exact = inrow && scol[L] == xm;
      }
      const uint64_t vmask = nv == 64 ? ~0ull : ((1ull << nv) - 1);
      const uint64_t nonex = ~(uint64_t)__ballot(exact) & vmask;
      const uint32_t f = nonex ? (uint32_t)(__ffsll((long long)nonex) - 1) : nv;
      const bool finrow = f < nv && __shfl((int)inrow, (int)f, 64) != 0;
      const uint32_t acc = f + (finrow ? 1u : 0u);
      if ((uint32_t)lane < acc) key[o + m + lane] = L;
      if (acc) {
        t = __shfl((unsigned long long)L, (int)acc - 1, 64) + 1;
        m += acc;
      }
      if (f < nv && !finrow) {                        // step m leaves row r (uniform)
        const uint32_t xf = Qj[m];
        const uint32_t r2 = next_row_ge(rmax, b64, b4k, srn, r, (int64_t)xf);
        uint64_t land = snnz;
        if (r2 >= srn) {
          if (d_lmop_spill_on) d_lmop_spill = 1;
          live = false;                               // reference runs off the end of St (UB)
        } else {
          r = r2;
          land = lower_bound_u32(scol, sro[r2], sro[r2 + 1], xf);
          t = land + 1;
        }
        if (lane == 0) key[o + m] = land;
        m++;
      }
    }
  }
}
static int g_lmop_wave = -1;          // test hook: -1 environment / default
extern "C" void amgd_lmop_set_wave(int n) { g_lmop_wave = n; }
static int lmop_land_wave_forced() {   // the pruned walk: per wavefront only when forced
  if (g_lmop_wave >= 0) return g_lmop_wave;
  const char *e = getenv("AMGD_LMOP_WAVE");
  return e && *e ? atoi(e) : 0;
}
static int lmop_land_wave_min() {     // support size from which the walk runs per wavefront
  if (g_lmop_wave >= 0) return g_lmop_wave;
  static int v = -2;
  if (v == -2) {
    const char *e = getenv("AMGD_LMOP_WAVE");
    v = e && *e ? atoi(e) : 64;       // 0: never
  }
  return v;
}
// (2) values: one thread per contribution (c, k, m):
//     u_c * sum_{t >= max(k,m)} q_t[k] * q_t[m], t ascending (QQt, amg_setup.c:1638-1642)
__global__ void k_lmop_val(uint64_t n, uint32_t c0, uint32_t c1, const uint64_t *coff,
                           uint64_t cbase, const uint64_t *wro, const double *Q,
                           const uint64_t *qoff, const double *u, const uint64_t *key,
                           uint64_t snnz, double *val) {
  GRID_STRIDE(o, n) {
    if (key[o] >= snnz) { val[o] = 0.0; continue; }
    uint64_t g = o + cbase;
    uint32_t lo = c0, hi = c1;            // last c with coff[c] <= g
    while (hi - lo > 1) {
      uint32_t mid = (lo + hi) >> 1;
      if (coff[mid] <= g) lo = mid; else hi = mid;
    }
    uint32_t c = lo;
    uint32_t nz = (uint32_t)(wro[c + 1] - wro[c]);
    uint64_t r = g - coff[c];
    uint32_t k = (uint32_t)(r / nz), m = (uint32_t)(r % nz);
    const double *Qc = Q + qoff[c];
    double q = 0.0;
    for (uint32_t tt = k > m ? k : m; tt < nz; tt++) {
      const double *qt = Qc + tri(tt);
      q += qt[k] * qt[m];
    }
    val[o] = u[c] * q;
  }
}
// sa holds the positions [lo, hi) of S (sa[0] = position lo); keys outside are dropped
__global__ void k_seg_accum(const uint64_t *key, const double *val, uint64_t n, uint64_t lo,
                            uint64_t hi, double *sa) {
  GRID_STRIDE(i, n) {
    uint64_t kk = key[i];
    if (kk < lo || kk >= hi) continue;
    if (i > 0 && key[i - 1] == kk) continue;     // not the head of its run
    double acc = sa[kk - lo];
    for (uint64_t t = i; t < n && key[t] == kk; t++) acc = acc + val[t];
    sa[kk - lo] = acc;
  }
}
// Partitioned mode: the walks run on the whole S pattern, the values of positions [lo, hi)
// only (a rank's rows) are kept, in `a` (amgd_lmop_set_window; off: S->a, all of S)
static double *g_win_a = nullptr;
static uint64_t g_win_lo = 0, g_win_hi = 0;
extern "C" void amgd_lmop_set_window(double *a, uint64_t lo, uint64_t hi) {
  g_win_a = a; g_win_lo = lo; g_win_hi = hi;
}
static void seg_accum(const uint64_t *key, const double *val, uint64_t n, const dcsr *S) {
  if (g_win_a)
    k_seg_accum<<<grid_for(n), 256, 0, amgd_s()>>>(key, val, n, g_win_lo, g_win_hi, g_win_a);
  else
    k_seg_accum<<<grid_for(n), 256, 0, amgd_s()>>>(key, val, n, 0, S->nnz, S->a);
}
__global__ void k_csq(const uint64_t *wro, uint32_t rn, uint64_t *sz) {
  GRID_STRIDE(c, rn) {
    uint64_t nz = wro[c + 1] - wro[c];
    sz[c] = nz * nz;
  }
}
extern void amgd_row_of_entry_launch(const uint64_t *ro, uint32_t rn, uint32_t *row);

// ---------------------------------------------------------------------------
// Huge supports, pruned.  Let G be the graph on the support with an edge k - t
// wherever the factor entry q_t[k] (k < t) is nonzero.  If k and m lie in different
// components of G, every product q_t[k] * q_t[m] has a zero factor, so the QQt entry
// sums only signed zeros from +0 and is +0, and u_c * (+0) is a signed zero: adding
// it to S (whose entries start at +0 and so never hold -0) changes no bit.  Such
// contributions are dropped; the walk still steps over them (each landing depends on
// the previous one), but only same-component keys are written, and each value sums
// over the component's members only (the other t contribute signed zeros too).  The
// kept contributions keep their (k, m) order, so the stable sort and the ordered
// accumulation are those of the full path.  For the orphan support of an anisotropic
// level 1 (10^4 - 3.4*10^4 points in ~100 components) this replaces nz^2 keys and
// nz^3 value work by sum(size^2) and sum(size^3).
// ---------------------------------------------------------------------------
__global__ void k_qnz_count(const double *U, uint32_t nz, uint64_t *cnt) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t t = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; t < nz;
       t += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
    const double *row = U + tri(t);
    uint32_t c = 0;
    for (uint64_t k = lane; k < t; k += 64) c += row[k] != 0.0;
    for (int o = 32; o; o >>= 1) c += __shfl_xor(c, o, 64);
    if (lane == 0) cnt[t] = c;
  }
}
__global__ void k_qnz_fill(const double *U, uint32_t nz, const uint64_t *eoff, uint32_t *ea,
                           uint32_t *eb) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t t = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; t < nz;
       t += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
    const double *row = U + tri(t);
    uint64_t o = eoff[t];
    for (uint64_t k0 = 0; k0 < t; k0 += 64) {
      const uint64_t k = k0 + lane;
      const bool p = k < t && row[k] != 0.0;
      const unsigned long long b = __ballot(p);
      if (p) {
        const uint64_t w = o + __popcll(b & ((1ull << lane) - 1));
        ea[w] = (uint32_t)t;
        eb[w] = (uint32_t)k;
      }
      o += __popcll(b);
    }
  }
}
__global__ void k_edge_hook(const uint32_t *ea, const uint32_t *eb, uint64_t ne, uint32_t *lab,
                            unsigned *changed) {
  GRID_STRIDE(e, ne) {
    const uint32_t a = lab[ea[e]], b = lab[eb[e]];
    if (a != b) {
      atomicMin(&lab[a > b ? a : b], a > b ? b : a);
      *changed = 1u;
    }
  }
}
// per member (sorted by (label, index)): component index and component offsets;
// hscan = exclusive scan of the head flags, so a head's component is hscan[t]
__global__ void k_comp_meta_x(uint32_t nz, const uint64_t *skey, const uint64_t *hscan,
                              uint32_t *compid, uint32_t *members, uint64_t *cro) {
  GRID_STRIDE(t, nz) {
    const uint32_t k = (uint32_t)(skey[t] & 0xffffffffu);
    const bool head = t == 0 || (skey[t] >> 32) != (skey[t - 1] >> 32);
    const uint32_t cid = (uint32_t)hscan[t] - (head ? 0u : 1u);
    members[t] = k;
    compid[k] = cid;
    if (head) cro[cid] = t;
  }
}
__global__ void k_comp_rank(uint32_t nz, const uint32_t *members, const uint32_t *compid,
                            const uint64_t *cro, uint32_t *rank, uint64_t *kcnt) {
  GRID_STRIDE(t, nz) {
    const uint32_t k = members[t];
    const uint32_t cid = compid[k];
    rank[k] = (uint32_t)(t - cro[cid]);
    kcnt[k] = cro[cid + 1] - cro[cid];
  }
}
// sp_add's walk for row k of the support (k_lmop_land), keys written for same-component m
__global__ void k_lmop_land_pr(const uint32_t *Qj, uint32_t nz, const uint64_t *sro,
                               const uint32_t *scol, uint32_t srn, uint64_t snnz,
                               const int64_t *rmax, const int64_t *b64, const int64_t *b4k,
                               const uint32_t *compid, const uint32_t *rank, const uint64_t *koff,
                               uint64_t *key) {
  GRID_STRIDE(k, nz) {
    const uint32_t ck = compid[k];
    const uint64_t o = koff[k];
    uint32_t r = Qj[k];
    uint64_t t = sro[r];
    bool live = sro[r + 1] != t;
    for (uint32_t m = 0; m < nz; m++) {
      uint64_t land = snnz;
      if (live) {
        const uint32_t xm = Qj[m];
        const uint64_t end = sro[r + 1];
        if (t < end && rmax[r] >= (int64_t)xm) {
          land = lower_bound_u32(scol, t, end, xm);
        } else {
          const uint32_t r2 = next_row_ge(rmax, b64, b4k, srn, r, (int64_t)xm);
          if (r2 >= srn) {
            live = false;
            if (d_lmop_spill_on) d_lmop_spill = 1;
          }
          else { r = r2; land = lower_bound_u32(scol, sro[r2], sro[r2 + 1], xm); }
        }
        if (live) t = land + 1;
      }
      if (compid[m] == ck) key[o + rank[m]] = land;
    }
  }
}
// k_lmop_land_pr with one wavefront per walk k (k_lmop_land_wave's steps: the next 64
// columns searched from the current position at once, the prefix of exact matches taken,
// then the first non-exact step or the row skip), keys written for the same-component m.
// The thread-per-walk form walked 10^4 - 3*10^4 steps per thread on the anisotropic
// level-1 orphan support: 186 ms per call, 1.5 s of the anisotropic 256^3 setup
// (profiles/r06/aniso256_kernel_stats_r06d.csv)
__global__ __launch_bounds__(256) void k_lmop_land_wave_pr(
    const uint32_t *Qj, uint32_t nz, const uint64_t *sro, const uint32_t *scol, uint32_t srn, uint64_t snnz,
    const int64_t *rmax, const int64_t *b64, const int64_t *b4k, const uint32_t *compid, const uint32_t *rank,
    const uint64_t *koff, uint64_t *key) {
  const int lane = threadIdx.x & 63;
  for (uint64_t k = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; k < nz;
       k += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
    const uint32_t ck = compid[k];
    const uint64_t o = koff[k];
    uint32_t r = Qj[k];
    uint64_t t = sro[r];
    bool live = sro[r + 1] != t;
    uint32_t m = 0;
    while (m < nz) {
      if (!live) {
        for (uint32_t q = m + lane; q < nz; q += 64)
          if (compid[q] == ck) key[o + rank[q]] = snnz;
        break;
      }
      const uint64_t end = sro[r + 1];
      const uint32_t nv = min(64u, nz - m);
      const bool valid = (uint32_t)lane < nv;
      const uint32_t xm = valid ? Qj[m + lane] : 0u;
      uint64_t L = end;
      bool inrow = false, exact = false;
      if (valid && t < end) {
        L = lower_bound_u32(scol, t, end, xm);
        inrow = L < end;
        exact = inrow && scol[L] == xm;
      }
      const uint64_t vmask = nv == 64 ? ~0ull : ((1ull << nv) - 1);
      const uint64_t nonex = ~(uint64_t)__ballot(exact) & vmask;
      const uint32_t f = nonex ? (uint32_t)(__ffsll((long long)nonex) - 1) : nv;
      const bool finrow = f < nv && __shfl((int)inrow, (int)f, 64) != 0;
      const uint32_t acc = f + (finrow ? 1u : 0u);
      if ((uint32_t)lane < acc && compid[m + lane] == ck) key[o + rank[m + lane]] = L;
      if (acc) {
        t = __shfl((unsigned long long)L, (int)acc - 1, 64) + 1;
        m += acc;
      }
      if (f < nv && !finrow) {                        // step m leaves row r (uniform)
        const uint32_t xf = Qj[m];
        const uint32_t r2 = next_row_ge(rmax, b64, b4k, srn, r, (int64_t)xf);
        uint64_t land = snnz;
        if (r2 >= srn) {
          if (d_lmop_spill_on) d_lmop_spill = 1;
          live = false;                               // reference runs off the end of St (UB)
        } else {
          r = r2;
          land = lower_bound_u32(scol, sro[r2], sro[r2 + 1], xf);
          t = land + 1;
        }
        if (lane == 0 && compid[m] == ck) key[o + rank[m]] = land;
        m++;
      }
    }
  }
}
__global__ void k_lmop_val_pr(uint64_t n, uint32_t nz, const uint64_t *koff, const uint32_t *compid,
                              const uint32_t *rank, const uint32_t *members, const uint64_t *cro,
                              const double *Qc, double uc, const uint64_t *key, uint64_t snnz,
                              double *val) {
  GRID_STRIDE(o, n) {
    if (key[o] >= snnz) { val[o] = 0.0; continue; }
    uint32_t lo = 0, hi = nz;                  // last k with koff[k] <= o
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (koff[mid] <= o) lo = mid; else hi = mid;
    }
    const uint32_t k = lo, j = (uint32_t)(o - koff[k]);
    const uint64_t c0 = cro[compid[k]], c1 = cro[compid[k] + 1];
    const uint32_t m = members[c0 + j];
    const uint32_t rk = rank[k];
    double q = 0.0;
    for (uint64_t p = c0 + (rk > j ? rk : j); p < c1; p++) {
      const double *qt = Qc + tri(members[p]);
      q += qt[k] * qt[m];
    }
    val[o] = uc * q;
  }
}
static int g_lmop_prune = -1;   // supports of at least this many points are pruned (0: never)
extern "C" void amgd_lmop_set_prune(int n) { g_lmop_prune = n; }
static uint32_t lmop_prune_min() {
  if (g_lmop_prune < 0) {
    const char *e = getenv("AMGD_LMOP_PRUNE");
    g_lmop_prune = e ? atoi(e) : 4096;
  }
  return (uint32_t)g_lmop_prune;
}
extern "C" void amgd_lmop_note_pruned(void);
// contributions of the single support c, pruned; false (nothing done) if its factor
// graph is connected
static bool lmop_pruned(dcsr *S, const dcsr *Wt, const double *Q, uint64_t qo, uint64_t w0,
                        uint32_t nz, double uc, const int64_t *rmax, const int64_t *b64,
                        const int64_t *b4k, int eb) {
  hipStream_t s = amgd_s();
  const double *U = Q + qo;
  uint64_t *cnt = (uint64_t *)amgd_alloc(((size_t)nz + 1) * 8);
  k_qnz_count<<<grid_for((uint64_t)nz * 64, 256, 16384), 256, 0, s>>>(U, nz, cnt);
  const uint64_t ne = amgd_scan_u64(cnt, nz);
  uint32_t *ea = (uint32_t *)amgd_alloc(ne * 4 + 4), *eb_ = (uint32_t *)amgd_alloc(ne * 4 + 4);
  k_qnz_fill<<<grid_for((uint64_t)nz * 64, 256, 16384), 256, 0, s>>>(U, nz, cnt, ea, eb_);
  amgd_free(cnt);
  uint32_t *lab = (uint32_t *)amgd_alloc((size_t)nz * 4 + 4);
  unsigned *chg = (unsigned *)amgd_alloc(16);
  k_cc_init_iota<<<grid_for(nz), 256, 0, s>>>(nz, lab);
  for (int it = 0; it < 100000 && ne; it++) {
    HIPCK(hipMemsetAsync(chg, 0, 4, s));
    k_edge_hook<<<grid_for(ne), 256, 0, s>>>(ea, eb_, ne, lab, chg);
    k_cc_jump<<<grid_for(nz), 256, 0, s>>>(nz, lab);
    unsigned h = 0;
    amgd_d2h(&h, chg, 4);
    if (!h) break;
  }
  amgd_free(chg); amgd_free(ea); amgd_free(eb_);
  uint64_t *key = (uint64_t *)amgd_alloc((size_t)nz * 8 + 8), *skey = (uint64_t *)amgd_alloc((size_t)nz * 8 + 8);
  k_cc_keys<<<grid_for(nz), 256, 0, s>>>(nz, lab, key);
  size_t tb = 0;
  HIPCK(rocprim::radix_sort_keys(nullptr, tb, key, skey, (size_t)nz, 0, 64, s));
  void *tmp = amgd_alloc(tb + 16);
  HIPCK(rocprim::radix_sort_keys(tmp, tb, key, skey, (size_t)nz, 0, 64, s));
  amgd_free(tmp); amgd_free(key); amgd_free(lab);
  uint64_t *hs = (uint64_t *)amgd_alloc((size_t)nz * 8 + 16);
  k_cc_heads<<<grid_for(nz), 256, 0, s>>>(nz, skey, hs);
  const uint32_t ncomp = (uint32_t)amgd_scan_u64(hs, nz);
  if (ncomp <= 1) { amgd_free(hs); amgd_free(skey); return false; }
  uint32_t *compid = (uint32_t *)amgd_alloc((size_t)nz * 4 + 4), *rank = (uint32_t *)amgd_alloc((size_t)nz * 4 + 4);
  uint32_t *members = (uint32_t *)amgd_alloc((size_t)nz * 4 + 4);
  uint64_t *cro = (uint64_t *)amgd_alloc(((size_t)ncomp + 1) * 8);
  k_comp_meta_x<<<grid_for(nz), 256, 0, s>>>(nz, skey, hs, compid, members, cro);
  const uint64_t endv = nz;
  amgd_h2d(cro + ncomp, &endv, 8);
  uint64_t *koff = (uint64_t *)amgd_alloc(((size_t)nz + 1) * 8);
  k_comp_rank<<<grid_for(nz), 256, 0, s>>>(nz, members, compid, cro, rank, koff);
  const uint64_t n = amgd_scan_u64(koff, nz);
  amgd_free(hs); amgd_free(skey);
  uint64_t *k1 = (uint64_t *)amgd_alloc(n * 8 + 8), *k2 = (uint64_t *)amgd_alloc(n * 8 + 8);
  double *v1 = (double *)amgd_alloc_f64(n * 8 + 8), *v2 = (double *)amgd_alloc_f64(n * 8 + 8);
  // the wavefront walk only when forced (amgd_lmop_set_wave / AMGD_LMOP_WAVE > 0): on the
  // anisotropic orphan support it measured slower than one thread per walk (222 vs 186 ms
  // per call: 64 searches per step against one; profiles/r06/aniso256_kernel_stats_r06l.csv)
  const int wmin = lmop_land_wave_forced();
  if (wmin > 0 && nz >= (uint32_t)wmin) {
    amgd_route_hit(AMGD_R_LMOP_WAVE);
    k_lmop_land_wave_pr<<<grid_for((uint64_t)nz * 64, 256, 65536), 256, 0, s>>>(Wt->col + w0, nz, S->ro, S->col,
                                                                               S->rn, S->nnz, rmax, b64, b4k,
                                                                               compid, rank, koff, k1);
  } else {
    k_lmop_land_pr<<<grid_for(nz, 64, 65536), 64, 0, s>>>(Wt->col + w0, nz, S->ro, S->col, S->rn,
                                                         S->nnz, rmax, b64, b4k, compid, rank,
                                                         koff, k1);
  }
  k_lmop_val_pr<<<grid_for(n, 256, 65536), 256, 0, s>>>(n, nz, koff, compid, rank, members, cro, U,
                                                       uc, k1, S->nnz, v1);
  KCHECK();
  tb = 0;
  HIPCK(rocprim::radix_sort_pairs(nullptr, tb, k1, k2, v1, v2, (size_t)n, 0, eb, s));
  tmp = amgd_alloc(tb + 16);
  HIPCK(rocprim::radix_sort_pairs(tmp, tb, k1, k2, v1, v2, (size_t)n, 0, eb, s));
  seg_accum(k2, v2, n, S);
  KCHECK();
  amgd_free(tmp); amgd_free(k1); amgd_free(k2); amgd_free(v1); amgd_free(v2);
  amgd_free(compid); amgd_free(rank); amgd_free(members); amgd_free(cro); amgd_free(koff);
  amgd_lmop_note_pruned();
  if (getenv("AMGD_SGLOG"))
    fprintf(stderr, "lmop pruned: support of %u points, %u components, %lu of %lu contributions\n",
            nz, ncomp, (unsigned long)n, (unsigned long)nz * nz);
  return true;
}

// General path: adds the contributions of coarse points c in [cb, ce) to S->a
// (which the caller has zeroed or already holds the contributions of c < cb).
extern "C" void amgd_lmop_general(dcsr *S, const dcsr *Wt, const double *Q, const uint64_t *qoff,
                                  const double *u, uint32_t cb, uint32_t ce) {
  hipStream_t s = amgd_s();
  uint32_t rn = Wt->rn;
  if (ce > rn) ce = rn;
  if (cb >= ce || Wt->nnz == 0) return;
  uint64_t *coff = (uint64_t *)amgd_alloc(((size_t)rn + 1) * 8);
  k_csq<<<grid_for(rn), 256, 0, s>>>(Wt->ro, rn, coff);
  amgd_scan_u64(coff, rn);
  std::vector<uint64_t> hcoff(rn + 1), hro(rn + 1);
  amgd_d2h(hcoff.data(), coff, (rn + 1) * 8);
  amgd_d2h(hro.data(), Wt->ro, (rn + 1) * 8);
  uint32_t *erow = (uint32_t *)amgd_alloc(Wt->nnz * 4 + 4);
  amgd_row_of_entry_launch(Wt->ro, rn, erow);
  uint32_t srn = S->rn;
  uint64_t n64 = ((uint64_t)srn + 63) >> 6, n4k = ((uint64_t)srn + 4095) >> 12;
  int64_t *rmax = (int64_t *)amgd_alloc(((size_t)srn + 1) * 8);
  int64_t *b64 = (int64_t *)amgd_alloc((n64 + 1) * 8), *b4k = (int64_t *)amgd_alloc((n4k + 1) * 8);
  if (srn) {
    k_rowmax<<<grid_for(srn), 256, 0, s>>>(S->ro, S->col, srn, rmax);
    k_blockmax_wave<<<grid_for(n64 * 64, 256, 16384), 256, 0, s>>>(rmax, srn, 6, b64, n64);
    k_blockmax_wave<<<grid_for(n4k * 64, 256, 16384), 256, 0, s>>>(rmax, srn, 12, b4k, n4k);
  }
  const uint64_t CH = std::max<uint64_t>(1, std::min<uint64_t>(hcoff[ce] - hcoff[cb], 1ull << 26));
  uint64_t *key = (uint64_t *)amgd_alloc(CH * 8 + 8), *key2 = (uint64_t *)amgd_alloc(CH * 8 + 8);
  double *val = (double *)amgd_alloc_f64(CH * 8 + 8), *val2 = (double *)amgd_alloc_f64(CH * 8 + 8);
  size_t tb = 0;
  int eb = 1;
  while (eb < 64 && (S->nnz >> eb) != 0) eb++;   // keys are 0..S->nnz
  HIPCK(rocprim::radix_sort_pairs(nullptr, tb, key, key2, val, val2, (size_t)CH, 0, eb, s));
  void *tmp = amgd_alloc(tb + 16);
  const uint32_t pmin = lmop_prune_min();
  std::vector<uint64_t> hqo;
  std::vector<double> hu;
  auto huge = [&](uint32_t c) { return pmin && hro[c + 1] - hro[c] >= pmin; };
  uint32_t c0 = cb;
  while (c0 < ce) {
    if (huge(c0)) {                        // a support of >= pmin points: pruned if it splits
      if (hqo.empty()) {
        hqo.resize(rn + 1);
        amgd_d2h(hqo.data(), qoff, (rn + 1) * 8);
        hu.resize(rn);
        amgd_d2h(hu.data(), u, (size_t)rn * 8);
      }
      if (lmop_pruned(S, Wt, Q, hqo[c0], hro[c0], (uint32_t)(hro[c0 + 1] - hro[c0]), hu[c0], rmax,
                      b64, b4k, eb)) {
        c0++;
        continue;
      }
    }
    uint32_t c1 = c0;
    // take whole coarse rows while they fit (a single oversized row gets its own chunk;
    // a support to prune starts a chunk of its own)
    while (c1 < ce && (hcoff[c1 + 1] - hcoff[c0] <= CH || c1 == c0) && (c1 == c0 || !huge(c1))) c1++;
    uint64_t n = hcoff[c1] - hcoff[c0];
    if (n > CH) {   // one huge support: grow buffers for it
      amgd_free(key); amgd_free(key2); amgd_free(val); amgd_free(val2); amgd_free(tmp);
      key = (uint64_t *)amgd_alloc(n * 8); key2 = (uint64_t *)amgd_alloc(n * 8);
      val = (double *)amgd_alloc_f64(n * 8); val2 = (double *)amgd_alloc_f64(n * 8);
      tb = 0;
      HIPCK(rocprim::radix_sort_pairs(nullptr, tb, key, key2, val, val2, (size_t)n, 0, eb, s));
      tmp = amgd_alloc(tb + 16);
    }
    uint64_t e0 = hro[c0], e1 = hro[c1];
    if (n && e1 > e0) {
      uint64_t maxnz = 0;
      for (uint32_t c = c0; c < c1; c++) maxnz = std::max<uint64_t>(maxnz, hro[c + 1] - hro[c]);
      const int wmin = lmop_land_wave_min();
      if (wmin > 0 && maxnz >= (uint64_t)wmin) {
        amgd_route_hit(AMGD_R_LMOP_WAVE);
        k_lmop_land_wave<<<grid_for((e1 - e0) * 64, 256, 65536), 256, 0, s>>>(
            erow, e0, e1, Wt->ro, Wt->col, S->ro, S->col, srn, S->nnz, rmax, b64, b4k, coff,
            hcoff[c0], key);
      } else {
        k_lmop_land<<<grid_for(e1 - e0, 256, 65536), 256, 0, s>>>(
            erow, e0, e1, Wt->ro, Wt->col, S->ro, S->col, srn, S->nnz, rmax, b64, b4k, coff,
            hcoff[c0], key);
      }
      k_lmop_val<<<grid_for(n, 256, 65536), 256, 0, s>>>(n, c0, c1, coff, hcoff[c0], Wt->ro, Q,
                                                          qoff, u, key, S->nnz, val);
      KCHECK();
      size_t tb2 = 0;
      HIPCK(rocprim::radix_sort_pairs(nullptr, tb2, key, key2, val, val2, (size_t)n, 0, eb, s));
      if (tb2 > tb) { amgd_free(tmp); tmp = amgd_alloc(tb2 + 16); tb = tb2; }
      HIPCK(rocprim::radix_sort_pairs(tmp, tb2, key, key2, val, val2, (size_t)n, 0, eb, s));
      seg_accum(key2, val2, n, S);
      KCHECK();
    }
    c0 = c1;
  }
  amgd_free(tmp); amgd_free(key); amgd_free(key2); amgd_free(val); amgd_free(val2);
  amgd_free(erow); amgd_free(coff); amgd_free(rmax); amgd_free(b64); amgd_free(b4k);
}

// ---------------------------------------------------------------------------
// find_support pieces (amg_setup.c:1260).  Removed entries are zeroed in place
// (equivalent for every later use: DESIGN.md "find_support").
// ---------------------------------------------------------------------------
// Outlier rows / columns of R (the orphan coarse point's: 10^4 - 10^5 entries among
// rows of ~10) take grid-wide kernels.  By default an outlier is longer than
// max(4096, 16 x M's mean row): where every row is long (coarse levels of a 3D Poisson
// hierarchy) the per-row kernels already fill the chip.  AMGD_FS_LONG /
// amgd_fs_set_long (tests) force an absolute threshold (0: never).
static int64_t g_fs_long = -1;        // -1: environment or automatic, -2: automatic
extern "C" void amgd_fs_set_long(int64_t n) { g_fs_long = n; }
static uint32_t fs_long(const dcsr *M) {
  if (g_fs_long == -1) {
    const char *e = getenv("AMGD_FS_LONG");
    g_fs_long = e && *e ? atoll(e) : -2;
  }
  if (g_fs_long == 0) return 0xffffffffu;
  if (g_fs_long > 0) return (uint32_t)g_fs_long;
  const uint64_t mean = M->rn ? M->nnz / M->rn : 0;
  return (uint32_t)std::min<uint64_t>(0xfffffffeu, std::max<uint64_t>(4096, 16 * mean));
}
__global__ void k_csc_gemv(const uint64_t *tro, const uint32_t *trow, const uint64_t *perm,
                           const double *a, const double *x, uint32_t n, double *z) {
  GRID_STRIDE(c, n) {
    double t = 0.0;
    for (uint64_t q = tro[c]; q < tro[c + 1]; q++) {
      double v = a[perm[q]];
      t += x ? v * x[trow[q]] : v;
    }
    z[c] = t;
  }
}
extern "C" void amgd_csc_gemv(const dcsr *Rt, const uint64_t *perm, const double *a,
                              const double *x, double *z) {
  if (Rt->rn)
    k_csc_gemv<<<grid_for(Rt->rn), 256, 0, amgd_s()>>>(Rt->ro, Rt->col, perm, a, x, Rt->rn, z);
  KCHECK();
}
// Per bad column c (w_c > (1+theta)*goal && sumR_c != 0): first row of the max of
// R(i,c)*rs_i (amg_setup.c:1343-1364), removed from R (both CSR and CSC copies).
// The bad columns are listed first (one thread per column), then one wavefront
// per listed column does the (value, position) max, first position on ties.
__global__ void k_fs_badlist(const double *w, const double *sumR, double thr, uint32_t n,
                             uint32_t *list, unsigned *cnt) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t iters = (n + stride - 1) / stride;
  for (uint64_t it = 0; it < iters; it++) {      // uniform trip count (wave_append)
    uint64_t c = i0 + it * stride;
    bool take = c < n && w[c] > thr && sumR[c] != 0.;
    unsigned p = wave_append(cnt, take);
    if (take) list[p] = (uint32_t)c;
  }
}
// G lanes per listed column (G = the power of two nearest the mean column length)
template <int G>
__global__ __launch_bounds__(256) void k_fs_select(const uint64_t *tro, const uint32_t *trow,
                                                   const uint64_t *perm, double *ta, double *a,
                                                   const double *rs, const uint32_t *list,
                                                   const unsigned *nlist, uint32_t *si,
                                                   uint32_t *sj, unsigned *removed,
                                                   uint32_t maxlen) {
  const uint32_t sub = threadIdx.x & (G - 1);
  const uint32_t n = *nlist;
  const uint64_t g0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) / G;
  const uint64_t gs = (uint64_t)gridDim.x * (256 / G);
  for (uint64_t r = g0; r < n; r += gs) {
    const uint32_t c = list[r];
    if (tro[c + 1] - tro[c] > maxlen) continue;      // long columns: k_fsl_part / k_fsl_fin
    double mx = -DBL_MAX;
    uint64_t best = ~0ull;
    // U entries per lane per step: their (row, value) loads, then their rs gathers, are in
    // flight together (round 4 walked one dependent row -> rs chain at a time); a position
    // past the column's end loads the last entry and is left out of the compare.  The
    // lane's positions are compared in ascending order, so the first maximum still wins.
    constexpr int U = 8;
    const uint64_t qb = tro[c], qe = tro[c + 1];
    for (uint64_t q0 = qb + sub; q0 < qe; q0 += (uint64_t)G * U) {
      uint32_t tr[U];
      double tv[U], rv[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t q = min(q0 + (uint64_t)u * G, qe - 1);
        tr[u] = trow[q];
        tv[u] = ta[q];
      }
#pragma unroll
      for (int u = 0; u < U; u++) rv[u] = rs[tr[u]];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t q = q0 + (uint64_t)u * G;
        const double x = tv[u] * rv[u];
        if (q < qe && x > mx) { mx = x; best = q; }
      }
    }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) {
      double om = __shfl_xor(mx, o, 64);
      unsigned long long ob = __shfl_xor((unsigned long long)best, o, 64);
      if (om > mx || (om == mx && ob < best)) { mx = om; best = ob; }
    }
    if (sub == 0) {              // slot r of the list: no contended counter
      si[r] = best != ~0ull ? trow[best] : 0u;
      sj[r] = c;
      if (best != ~0ull) { ta[best] = 0.0; if (perm) a[perm[best]] = 0.0; *removed = 1u; }
    }
  }
}
// Bad columns past fs_long() entries (k_fs_select skips them; llist holds their slots in
// the bad list): the same selection spread over the grid -- chunks of FSL_CH entries
// of every long column (offsets from a one-block scan of the device-side count), a
// (value, first position) maximum per chunk, then per column the chunks in order -- the
// first largest product of the column.  One 1024-thread block per column (round 5) took
// 142 us per call on the orphan column of anisotropic levels (1.9 s
// of the anisotropic 256^3 setup, profiles/r06/aniso256_kernel_stats_r06d.csv).
#define FSL_CH 2048
__global__ __launch_bounds__(256) void k_fsl_prep(const uint64_t *tro, const uint32_t *list, const uint32_t *llist,
                                                  const unsigned *nl, uint64_t *choff) {
  __shared__ uint32_t wt[4];
  __shared__ uint64_t carry;
  const unsigned n = *nl;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (unsigned b = 0; b < n; b += 256) {
    const unsigned t = b + threadIdx.x;
    uint32_t c = 0;
    if (t < n) {
      const uint32_t col = list[llist[t]];
      c = (uint32_t)((tro[col + 1] - tro[col] + FSL_CH - 1) / FSL_CH);
    }
    const uint32_t incl = block_incl_scan<256>(c, wt);
    const uint64_t base = carry;
    if (t < n) choff[t] = base + incl - c;
    __syncthreads();
    if (threadIdx.x == 255) carry = base + incl;     // the batch's total (past n: zeros)
    __syncthreads();
  }
  if (threadIdx.x == 0) choff[n] = carry;
}
__device__ __forceinline__ unsigned fsl_row_of(const uint64_t *choff, unsigned n, uint64_t g) {
  unsigned lo = 0, hi = n;                       // last t with choff[t] <= g
  while (hi - lo > 1) {
    const unsigned mid = (lo + hi) >> 1;
    if (choff[mid] <= g) lo = mid; else hi = mid;
  }
  return lo;
}
__global__ __launch_bounds__(256) void k_fsl_part(const uint64_t *tro, const uint32_t *trow, const double *ta,
                                                  const double *rs, const uint32_t *list, const uint32_t *llist,
                                                  const unsigned *nl, const uint64_t *choff, double *pv,
                                                  uint64_t *pp) {
  __shared__ double smx[4];
  __shared__ unsigned long long sbest[4];
  const unsigned n = *nl;
  if (!n) return;
  const uint64_t G = choff[n];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint64_t g = blockIdx.x; g < G; g += gridDim.x) {
    const unsigned t = fsl_row_of(choff, n, g);
    const uint32_t c = list[llist[t]];
    const uint64_t q0 = tro[c] + (g - choff[t]) * FSL_CH, q1 = min(tro[c + 1], q0 + FSL_CH);
    double mx = -DBL_MAX;
    uint64_t best = ~0ull;
    for (uint64_t q = q0 + threadIdx.x; q < q1; q += 256) {
      const double x = ta[q] * rs[trow[q]];
      if (x > mx) { mx = x; best = q; }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const double om = __shfl_xor(mx, o, 64);
      const unsigned long long ob = __shfl_xor((unsigned long long)best, o, 64);
      if (om > mx || (om == mx && ob < best)) { mx = om; best = ob; }
    }
    if (lane == 0) { smx[w] = mx; sbest[w] = best; }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int q = 1; q < 4; q++)
        if (smx[q] > mx || (smx[q] == mx && sbest[q] < best)) { mx = smx[q]; best = sbest[q]; }
      pv[g] = mx;
      pp[g] = best;
    }
    __syncthreads();
  }
}
__global__ void k_fsl_fin(const uint32_t *trow, const uint64_t *perm, double *ta, double *a, const uint32_t *list,
                          const uint32_t *llist, const unsigned *nl, const uint64_t *choff, const double *pv,
                          const uint64_t *pp, uint32_t *si, uint32_t *sj, unsigned *removed) {
  const unsigned n = *nl;
  GRID_STRIDE(t, n) {
    const uint32_t r = llist[t], c = list[r];
    double mx = -DBL_MAX;
    uint64_t best = ~0ull;
    for (uint64_t g = choff[t]; g < choff[t + 1]; g++)
      if (pv[g] > mx) { mx = pv[g]; best = pp[g]; }        // chunks in order: the first wins ties
    si[r] = best != ~0ull ? trow[best] : 0u;
    sj[r] = c;
    if (best != ~0ull) { ta[best] = 0.0; if (perm) a[perm[best]] = 0.0; *removed = 1u; }
  }
}
// short rows: one thread per listed row, in order
__global__ void k_list_rowsum_t(const uint64_t *ro, const double *a, const uint32_t *list,
                                uint32_t n, double *out) {
  GRID_STRIDE(r, n) {
    const uint32_t i = list[r];
    double t = 0;
    for (uint64_t k = ro[i]; k < ro[i + 1]; k++) t += a[k];
    out[i] = t;
  }
}
// ordered row sums (from +0, left to right) of the listed rows: re-sums a row of R
// after an entry of it was removed (the removed entry is an exact zero now)
__global__ __launch_bounds__(256) void k_list_rowsum(const uint64_t *ro, const double *a,
                                                     const uint32_t *list, uint32_t n, double *out) {
  __shared__ double buf[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint64_t r = (uint64_t)blockIdx.x * 4 + w; r < n; r += (uint64_t)gridDim.x * 4) {
    const uint32_t i = list[r];
    const uint64_t k0 = ro[i], k1 = ro[i + 1];
    double t = 0;
    for (uint64_t c0 = k0; c0 < k1; c0 += 64) {
      if (c0 + lane < k1) buf[w][lane] = a[c0 + lane];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (lane == 0) {
        const int m = (int)min((uint64_t)64, k1 - c0);
        for (int q = 0; q < m; q++) t += buf[w][q];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (lane == 0) out[i] = t;
  }
}
// Incremental find_support sweeps: the distinct neighbours (columns of M) of the listed
// rows, first visit claimed by an exchange of the neighbour's stamp with `tag` (a plain
// load first skips the exchange for neighbours already claimed: most of them).
// Returns the count, which may exceed cap (the list is then incomplete: the caller
// falls back to full products).
__global__ void k_fs_expand(const uint64_t *ro, const uint32_t *col, const uint32_t *list,
                            uint32_t n, uint32_t *stamp, uint32_t tag, uint32_t *out,
                            unsigned *cnt, uint32_t cap) {
  GRID_STRIDE(r, n) {
    const uint32_t i = list[r];
    for (uint64_t k = ro[i]; k < ro[i + 1]; k++) {
      const uint32_t c = col[k];
      if (stamp[c] != tag && atomicExch(&stamp[c], tag) != tag) {
        const unsigned p = atomicAdd(cnt, 1u);
        if (p < cap) out[p] = c;
      }
    }
  }
}
__global__ void k_fs_expand_wave(const uint64_t *ro, const uint32_t *col, const uint32_t *list,
                                 uint32_t n, uint32_t *stamp, uint32_t tag, uint32_t *out,
                                 unsigned *cnt, uint32_t cap, uint32_t maxlen) {
  const int lane = threadIdx.x & 63;
  for (uint64_t r = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < n;
       r += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
    const uint32_t i = list[r];
    if (ro[i + 1] - ro[i] > maxlen) continue;     // k_fs_expand_long
    for (uint64_t k0 = ro[i]; k0 < ro[i + 1]; k0 += 64) {
      const uint64_t k = k0 + lane;
      bool fresh = false;
      uint32_t c = 0;
      if (k < ro[i + 1]) { c = col[k]; fresh = stamp[c] != tag && atomicExch(&stamp[c], tag) != tag; }
      const unsigned p = wave_append(cnt, fresh);
      if (fresh && p < cap) out[p] = c;
    }
  }
}
// Long rows (past fs_long() entries: the orphan coarse point's column, 10^4 - 10^5 rows)
// spread over the whole grid; k_fs_expand_wave skips them.
__global__ void k_fs_expand_long(const uint64_t *ro, const uint32_t *col, const uint32_t *llist,
                                 const unsigned *nl, uint32_t *stamp, uint32_t tag, uint32_t *out,
                                 unsigned *cnt, uint32_t cap) {
  const unsigned n = *nl;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (unsigned r = 0; r < n; r++) {
    const uint32_t i = llist[r];
    const uint64_t k1 = ro[i + 1];
    for (uint64_t b = ro[i] + (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); b < k1;
         b += stride) {                       // uniform per wavefront (wave_append)
      const uint64_t k = b + lane;
      bool fresh = false;
      uint32_t c = 0;
      if (k < k1) { c = col[k]; fresh = stamp[c] != tag && atomicExch(&stamp[c], tag) != tag; }
      const unsigned p = wave_append(cnt, fresh);
      if (fresh && p < cap) out[p] = c;
    }
  }
}
// entries r of list (n, or *nd when nd is given) whose row list[r] is longer than
// maxlen: the row (slot = 0) or the slot r (slot = 1) appended to out
__global__ void k_pick_long(const uint64_t *ro, const uint32_t *list, uint32_t n, const unsigned *nd,
                            uint32_t maxlen, int slot, uint32_t *out, unsigned *cnt) {
  const uint64_t m = nd ? *nd : n;
  GRID_STRIDE(r, m) {
    const uint32_t i = list[r];
    if (ro[i + 1] - ro[i] > maxlen) out[atomicAdd(cnt, 1u)] = slot ? (uint32_t)r : i;
  }
}
extern "C" uint32_t amgd_fs_expand(const dcsr *M, const uint32_t *list, uint32_t n, uint32_t *stamp,
                                   uint32_t tag, uint32_t *out, uint32_t cap) {
  if (!n) return 0;
  unsigned *cnt = (unsigned *)amgd_alloc(16);
  amgd_memset(cnt, 0, 8);
  if (M->rn && M->nnz >= 16ull * M->rn) {
    uint32_t *ll = (uint32_t *)amgd_alloc((size_t)n * 4 + 4);
    const uint32_t ml = fs_long(M);
    if (amgd_max_row_len(M) > ml) {                   // outlier rows present
      k_pick_long<<<grid_for(n), 256, 0, amgd_s()>>>(M->ro, list, n, nullptr, ml, 0, ll, cnt + 1);
      k_fs_expand_long<<<512, 256, 0, amgd_s()>>>(M->ro, M->col, ll, cnt + 1, stamp, tag, out, cnt, cap);
    }
    k_fs_expand_wave<<<grid_for((uint64_t)n * 64, 256, 16384), 256, 0, amgd_s()>>>(
        M->ro, M->col, list, n, stamp, tag, out, cnt, cap, ml);
    amgd_free(ll);
  } else {
    k_fs_expand<<<grid_for(n), 256, 0, amgd_s()>>>(M->ro, M->col, list, n, stamp, tag, out, cnt, cap);
  }
  KCHECK();
  unsigned h = 0;
  amgd_d2h(&h, cnt, 4);
  amgd_free(cnt);
  return h;
}

// ordered row sums (+0, left to right) of the listed rows of M into out[row]: one thread
// per row for short rows, the long-row SpMV kernels (amgd_spmv_rows) for long ones.  M may
// be a global-row view (other ranks' rows empty: their sums come out +0)
extern "C" void amgd_list_rowsum(const dcsr *M, const uint32_t *list, uint32_t n, double *out, int long_rows) {
  if (!n) return;
  if (!long_rows)
    k_list_rowsum_t<<<grid_for(n), 256, 0, amgd_s()>>>(M->ro, M->a, list, n, out);
  else
    amgd_spmv_rows(M, list, n, nullptr, out);
  KCHECK();
}
// One selection sweep: select + remove, then bring rs (row sums of R) and sumR
// (column sums) up to date for the rows / columns that lost an entry.
extern "C" uint32_t amgd_fs_select(const dcsr *Rl, const dcsr *Rt, const uint64_t *perm,
                                   double *rs, const double *w, double *sumR,
                                   double thr, uint32_t *sel_i, uint32_t *sel_j,
                                   uint32_t *nremoved) {
  return amgd_fs_select_ex(Rl, Rt, perm, rs, w, sumR, thr, sel_i, sel_j, nremoved, 0, 1);
}
// c0: Rt holds rows c0.. of R' (partitioned mode: sel_j gets the global column, w / sumR are
// the caller's pointers at c0); perm NULL: R's own copy is not touched; resum 0: rs / sumR
// are left to the caller
__global__ void k_add_u32(uint32_t *a, uint64_t n, uint32_t v) { GRID_STRIDE(i, n) a[i] += v; }
extern "C" uint32_t amgd_fs_select_ex(const dcsr *Rl, const dcsr *Rt, const uint64_t *perm,
                                      double *rs, const double *w, double *sumR,
                                      double thr, uint32_t *sel_i, uint32_t *sel_j,
                                      uint32_t *nremoved, uint32_t c0, int resum) {
  hipStream_t s = amgd_s();
  const uint32_t nc = Rt->rn;
  uint32_t *list = (uint32_t *)amgd_alloc(((size_t)nc + 1) * 4);
  unsigned *cnt = (unsigned *)amgd_alloc(16);
  amgd_memset(cnt, 0, 16);
  uint32_t *llist = nullptr;
  if (nc) {
    k_fs_badlist<<<grid_for(nc), 256, 0, s>>>(w, sumR, thr, nc, list, cnt + 2);
    llist = (uint32_t *)amgd_alloc(((size_t)nc + 1) * 4);
    const uint32_t ml = fs_long(Rt);
    if (amgd_max_row_len(Rt) > ml) {                  // outlier columns present
      k_pick_long<<<grid_for(nc, 256, 1024), 256, 0, s>>>(Rt->ro, list, nc, cnt + 2, ml, 1,
                                                         llist, cnt + 3);
      // long columns over the grid: at most nnz / (ml + 1) of them
      const uint64_t nmax = std::min<uint64_t>(nc, Rt->nnz / ((uint64_t)ml + 1) + 1);
      const uint64_t gmax = Rt->nnz / FSL_CH + nmax + 1;
      uint64_t *choff = (uint64_t *)amgd_alloc(8 * (nmax + 1) + 8), *pp = (uint64_t *)amgd_alloc(8 * gmax + 8);
      double *pv = (double *)amgd_alloc_f64(8 * gmax + 8);
      k_fsl_prep<<<1, 256, 0, s>>>(Rt->ro, list, llist, cnt + 3, choff);
      k_fsl_part<<<(int)std::min<uint64_t>(gmax, 4096), 256, 0, s>>>(Rt->ro, Rt->col, Rt->a, rs, list, llist,
                                                                     cnt + 3, choff, pv, pp);
      k_fsl_fin<<<grid_for(nmax), 256, 0, s>>>(Rt->col, perm, Rt->a, Rl->a, list, llist, cnt + 3, choff, pv, pp,
                                               sel_i, sel_j, cnt + 1);
      amgd_free(choff); amgd_free(pp); amgd_free(pv);
    }
    uint64_t avg = (Rt->nnz + nc - 1) / nc;
    int G = 4;
    while (G < 64 && (uint64_t)G * 2 <= avg) G <<= 1;
    const int gb = grid_for((uint64_t)nc * G, 256, 16384);
#define FS_SEL(GG)                                                                        \
    k_fs_select<GG><<<gb, 256, 0, s>>>(Rt->ro, Rt->col, perm, Rt->a, Rl->a, rs, list, cnt + 2, \
                                       sel_i, sel_j, cnt + 1, ml)
    switch (G) {
      case 4: FS_SEL(4); break;
      case 8: FS_SEL(8); break;
      case 16: FS_SEL(16); break;
      case 32: FS_SEL(32); break;
      default: FS_SEL(64); break;
    }
#undef FS_SEL
  }
  KCHECK();
  unsigned h[4];
  amgd_d2h(h, cnt, 12);
  h[0] = h[2];                    // selections = bad columns (one per column)
  if (c0 && h[0]) k_add_u32<<<grid_for(h[0]), 256, 0, s>>>(sel_j, h[0], c0);
  if (h[1] && resum) {
    amgd_list_rowsum(Rl, sel_i, h[0], rs, Rl->nnz > 32ull * Rl->rn);
    amgd_list_rowsum(Rt, sel_j, h[0], sumR, Rt->nnz > 32ull * Rt->rn);
  }
  amgd_free(list);
  amgd_free(cnt);
  if (llist) amgd_free(llist);
  *nremoved = h[1];
  return h[0];
}

// The selection when the sweep's w = R' rs product also produced each column's first
// largest product (amgd_spmv_amax on R'): the same (value, first position) maximum as
// k_fs_select's, taken from the product instead of a second pass over the bad columns.
__global__ void k_fs_pick_amx(const uint32_t *list, const unsigned *nlist, const uint64_t *amx,
                              const uint32_t *trow, const uint64_t *perm, double *ta, double *a,
                              uint32_t *si, uint32_t *sj, unsigned *removed) {
  const unsigned n = *nlist;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n;
       r += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t c = list[r];
    const uint64_t best = amx[c];
    si[r] = best != ~0ull ? trow[best] : 0u;
    sj[r] = c;
    if (best != ~0ull) { ta[best] = 0.0; if (perm) a[perm[best]] = 0.0; *removed = 1u; }
  }
}
extern "C" uint32_t amgd_fs_select_amx(const dcsr *Rl, const dcsr *Rt, const uint64_t *perm,
                                       double *rs, const double *w, double *sumR, double thr,
                                       const uint64_t *amx, uint32_t *sel_i, uint32_t *sel_j,
                                       uint32_t *nremoved) {
  hipStream_t s = amgd_s();
  const uint32_t nc = Rt->rn;
  uint32_t *list = (uint32_t *)amgd_alloc(((size_t)nc + 1) * 4);
  unsigned *cnt = (unsigned *)amgd_alloc(16);
  amgd_memset(cnt, 0, 16);
  if (nc) {
    k_fs_badlist<<<grid_for(nc), 256, 0, s>>>(w, sumR, thr, nc, list, cnt + 2);
    k_fs_pick_amx<<<grid_for(nc), 256, 0, s>>>(list, cnt + 2, amx, Rt->col, perm, Rt->a, Rl->a,
                                                sel_i, sel_j, cnt + 1);
  }
  KCHECK();
  unsigned h[4];
  amgd_d2h(h, cnt, 12);
  h[0] = h[2];
  if (h[1]) {
    amgd_list_rowsum(Rl, sel_i, h[0], rs, Rl->nnz > 32ull * Rl->rn);
    amgd_list_rowsum(Rt, sel_j, h[0], sumR, Rt->nnz > 32ull * Rt->rn);
  }
  amgd_free(list);
  amgd_free(cnt);
  *nremoved = h[1];
  return h[0];
}

// ---------------------------------------------------------------------------
// expand_support pieces (amg_setup.c:907)
// ---------------------------------------------------------------------------
__global__ void k_bad_rows(const uint64_t *ro, const double *a, uint32_t rn, uint8_t *bad,
                           unsigned *nbad) {
  GRID_STRIDE(i, rn) {
    uint8_t b = 0;
    for (uint64_t k = ro[i]; k < ro[i + 1]; k++)
      if (a[k] == 2.) { b = 1; break; }
    bad[i] = b;
    if (b) atomicAdd(nbad, 1u);
  }
}
extern "C" uint8_t *amgd_bad_rows(const dcsr *ns, uint32_t *nbad) {
  uint8_t *bad = (uint8_t *)amgd_alloc((size_t)ns->rn + 1);
  unsigned *c = (unsigned *)amgd_alloc(4);
  amgd_memset(c, 0, 4);
  if (ns->rn) k_bad_rows<<<grid_for(ns->rn), 256, 0, amgd_s()>>>(ns->ro, ns->a, ns->rn, bad, c);
  unsigned h;
  amgd_d2h(&h, c, 4);
  amgd_free(c);
  *nbad = h;
  return bad;
}

// Per bad row (one wavefront): |X| entries ranked by descending value, stable
// in column order (glibc qsort = merge sort, cmp_coo_v_revert amg_setup.c:1252);
// S = running sum over ranks, V = sum/2, N = 1 + #{S - V < 0}; pick ranks < N.
__global__ __launch_bounds__(64) void k_expand_pick(const uint64_t *ro, const uint32_t *col,
                                                    const double *a, uint32_t rn,
                                                    const uint8_t *bad, uint32_t *scol,
                                                    double *sval, uint32_t *pj, uint64_t *cnt,
                                                    int keep_unmasked) {
  const int lane = threadIdx.x;
  for (uint32_t i = blockIdx.x; i < rn; i += gridDim.x) {
    if (!bad[i]) { if (lane == 0 && !keep_unmasked) cnt[i] = 0; continue; }
    uint64_t r0 = ro[i];
    uint32_t L = (uint32_t)(ro[i + 1] - r0);
    for (uint32_t e = lane; e < L; e += 64) {
      double ve = fabs(a[r0 + e]);
      uint32_t rank = 0;
      for (uint32_t f = 0; f < L; f++) {
        double vf = fabs(a[r0 + f]);
        rank += (vf > ve) || (vf == ve && f < e);
      }
      scol[r0 + rank] = col[r0 + e];
      sval[r0 + rank] = ve;
    }
    __syncthreads();
    __shared__ uint32_t Nsh;
    if (lane == 0) {
      double tot = 0.0;
      for (uint32_t p = 0; p < L; p++) if (sval[r0 + p] != 0.) tot += sval[r0 + p];
      double V = tot * 0.5;
      uint32_t c = 0;
      if (V != 0.) {
        double s = 0.0;
        for (uint32_t p = 0; p < L; p++) {      // (monotone: see k_expand_pick_sort)
          if (sval[r0 + p] != 0.) s += sval[r0 + p];
          if (s - V < 0) c++;
          else break;
        }
      }
      uint32_t N = c + 1;
      Nsh = N < L ? N : L;
      cnt[i] = Nsh;
    }
    __syncthreads();
    uint32_t N = Nsh;
    for (uint32_t p = lane; p < N; p += 64) pj[r0 + p] = scol[r0 + p];
    __syncthreads();
  }
}
// Long bad rows: the same ranking by an LDS bitonic sort on (|value| descending,
// position ascending) -- a strict total order, so it equals the stable merge order
// of the reference's qsort -- instead of the O(L^2) rank count.  Rows longer than
// EP_MAXL keep the rank-count kernel.
#define EP_MAXL 4096
__global__ __launch_bounds__(256) void k_expand_pick_sort(const uint64_t *ro, const uint32_t *col,
                                                          const double *a, uint32_t rn,
                                                          const uint8_t *bad, uint32_t *scol,
                                                          double *sval, uint32_t *pj,
                                                          uint64_t *cnt, unsigned *longrows) {
  __shared__ double kv[EP_MAXL];
  __shared__ uint32_t kp[EP_MAXL];
  __shared__ uint32_t Nsh;
  const int t = threadIdx.x;
  for (uint32_t i = blockIdx.x; i < rn; i += gridDim.x) {
    if (!bad[i]) { if (t == 0) cnt[i] = 0; continue; }
    const uint64_t r0 = ro[i];
    const uint32_t L = (uint32_t)(ro[i + 1] - r0);
    if (L > EP_MAXL) { if (t == 0) { cnt[i] = ~0ull; atomicAdd(longrows, 1u); } continue; }
    uint32_t P = 1;
    while (P < L) P <<= 1;
    for (uint32_t e = t; e < P; e += 256) {
      kv[e] = e < L ? fabs(a[r0 + e]) : -1.0;
      kp[e] = e;
    }
    __syncthreads();
    for (uint32_t size = 2; size <= P; size <<= 1)
      for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
        for (uint32_t tt = t; tt < P / 2; tt += 256) {
          const uint32_t lo = 2 * tt - (tt & (stride - 1)), hi = lo + stride;
          const bool up = (lo & size) == 0;
          const double vl = kv[lo], vh = kv[hi];
          const uint32_t pl = kp[lo], ph = kp[hi];
          const bool hi_first = vh > vl || (vh == vl && ph < pl);   // hi ranks before lo
          if (hi_first == up) { kv[lo] = vh; kv[hi] = vl; kp[lo] = ph; kp[hi] = pl; }
        }
        __syncthreads();
      }
    for (uint32_t r = t; r < L; r += 256) {
      scol[r0 + r] = col[r0 + kp[r]];
      sval[r0 + r] = kv[r];
    }
    __syncthreads();
    if (t == 0) {
      double tot = 0.0;
      for (uint32_t p = 0; p < L; p++) if (kv[p] != 0.) tot += kv[p];
      double V = tot * 0.5;
      uint32_t c = 0;
      if (V != 0.) {
        // kv is sorted descending and >= 0, so the running sum -- and sum - V -- never
        // decreases: the count stops at the first prefix with sum - V >= 0
        double sum = 0.0;
        for (uint32_t p = 0; p < L; p++) {
          if (kv[p] != 0.) sum += kv[p];
          if (sum - V < 0) c++;
          else break;
        }
      }
      uint32_t N = c + 1;
      Nsh = N < L ? N : L;
      cnt[i] = Nsh;
    }
    __syncthreads();
    const uint32_t N = Nsh;
    for (uint32_t p = t; p < N; p += 256) pj[r0 + p] = col[r0 + kp[p]];
    __syncthreads();
  }
}
// rows the sort kernel left (cnt == ~0): the rank-count kernel on just those
__global__ void k_long_mask(const uint64_t *cnt, uint32_t rn, uint8_t *m) {
  GRID_STRIDE(i, rn) m[i] = cnt[i] == ~0ull ? 1 : 0;
}
__global__ void k_pick_compact(const uint64_t *ro, const uint64_t *off, const uint32_t *pj,
                               uint32_t rn, uint32_t *oi, uint32_t *oj) {
  GRID_STRIDE(i, rn) {
    uint64_t n = off[i + 1] - off[i];
    for (uint64_t t = 0; t < n; t++) {
      oi[off[i] + t] = (uint32_t)i;
      oj[off[i] + t] = pj[ro[i] + t];
    }
  }
}
extern "C" uint64_t amgd_expand_pick(const dcsr *Xf, const uint8_t *bad, uint32_t **pi,
                                     uint32_t **pj) {
  hipStream_t s = amgd_s();
  uint32_t *scol = (uint32_t *)amgd_alloc(Xf->nnz * 4 + 4);
  double *sval = (double *)amgd_alloc_f64(Xf->nnz * 8 + 8);
  uint32_t *tj = (uint32_t *)amgd_alloc(Xf->nnz * 4 + 4);
  uint64_t *cnt = (uint64_t *)amgd_alloc(((size_t)Xf->rn + 1) * 8);
  if (Xf->rn) {
    int g = (int)std::min<uint32_t>(Xf->rn, 65536u);
    if (Xf->nnz >= 64ull * Xf->rn) {      // long rows: LDS sort, then the few longer ones
      unsigned *nl = (unsigned *)amgd_alloc(4);
      amgd_memset(nl, 0, 4);
      k_expand_pick_sort<<<g, 256, 0, s>>>(Xf->ro, Xf->col, Xf->a, Xf->rn, bad, scol, sval, tj,
                                           cnt, nl);
      unsigned hl = 0;
      amgd_d2h(&hl, nl, 4);
      if (hl) {
        uint8_t *lm = (uint8_t *)amgd_alloc((size_t)Xf->rn + 1);
        k_long_mask<<<grid_for(Xf->rn), 256, 0, s>>>(cnt, Xf->rn, lm);
        k_expand_pick<<<g, 64, 0, s>>>(Xf->ro, Xf->col, Xf->a, Xf->rn, lm, scol, sval, tj, cnt, 1);
        amgd_free(lm);
      }
      amgd_free(nl);
    } else {
      k_expand_pick<<<g, 64, 0, s>>>(Xf->ro, Xf->col, Xf->a, Xf->rn, bad, scol, sval, tj, cnt, 0);
    }
    KCHECK();
  }
  uint64_t n = amgd_scan_u64(cnt, Xf->rn);
  uint32_t *oi = (uint32_t *)amgd_alloc(n * 4 + 4), *oj = (uint32_t *)amgd_alloc(n * 4 + 4);
  if (Xf->rn) k_pick_compact<<<grid_for(Xf->rn), 256, 0, s>>>(Xf->ro, cnt, tj, Xf->rn, oi, oj);
  KCHECK();
  amgd_free(scol); amgd_free(sval); amgd_free(tj); amgd_free(cnt);
  *pi = oi;
  *pj = oj;
  return n;
}

__global__ void k_binarize(double *a, uint64_t n, int mode) {
  GRID_STRIDE(k, n) {
    if (mode == 0) { if (a[k] == 2.) a[k] = 1.; }
    else if (a[k] != 0.) a[k] = 1.;
  }
}
extern "C" void amgd_skel_binarize(dcsr *A, int mode) {
  if (A->nnz) k_binarize<<<grid_for(A->nnz), 256, 0, amgd_s()>>>(A->a, A->nnz, mode);
}
// amg_setup.c:821-837: scale entries whose COLUMN equals the row index
__global__ void k_scale_diag_match(const uint64_t *ro, const uint32_t *col, double *a, uint32_t rn,
                                   const double *v, const double *wuc) {
  GRID_STRIDE(i, rn) {
    if (wuc[i] != 0.)
      for (uint64_t j = ro[i]; j < ro[i + 1]; j++)
        if (col[j] == i) {
          double vw = v[i] / wuc[i];
          a[j] = vw * a[j];
        }
  }
}
extern "C" void amgd_scale_diag_match(dcsr *W, const double *v, const double *wuc) {
  if (W->rn) k_scale_diag_match<<<grid_for(W->rn), 256, 0, amgd_s()>>>(W->ro, W->col, W->a, W->rn, v, wuc);
}

// partitioned mode: another rank's expansion rows claimed with the same tag (the union of
// the ranks' lists; count in *cnt, entries past cap not stored -- as k_fs_expand)
__global__ void k_fs_claim_ext(const uint32_t *ids, uint64_t n, uint32_t *stamp, uint32_t tag, uint32_t *out,
                               unsigned *cnt, uint32_t cap) {
  GRID_STRIDE(t, n) {
    const uint32_t c = ids[t];
    if (stamp[c] != tag && atomicExch(&stamp[c], tag) != tag) {
      const unsigned p = atomicAdd(cnt, 1u);
      if (p < cap) out[p] = c;
    }
  }
}
extern "C" uint32_t amgd_fs_claim_ext(const uint32_t *ids, uint64_t n, uint32_t *stamp, uint32_t tag, uint32_t *out,
                                      uint32_t have, uint32_t cap) {
  unsigned *cnt = (unsigned *)amgd_alloc(8);
  amgd_h2d(cnt, &have, 4);
  if (n) k_fs_claim_ext<<<grid_for(n), 256, 0, amgd_s()>>>(ids, n, stamp, tag, out, cnt, cap);
  KCHECK();
  unsigned h = 0;
  amgd_d2h(&h, cnt, 4);
  amgd_free(cnt);
  return h;
}
