// amgd_dev.h -- device-side helpers shared by the HIP translation units.
#ifndef AMGD_DEV_H
#define AMGD_DEV_H
#include <hip/hip_runtime.h>
#include <stdint.h>

void amgd_check(hipError_t e, const char *what, const char *file, int line);
#define HIPCK(x) amgd_check((x), #x, __FILE__, __LINE__)
#define KCHECK() amgd_check(hipGetLastError(), "kernel launch", __FILE__, __LINE__)
hipStream_t amgd_s();

static inline int grid_for(uint64_t n, int threads = 256, int cap = 8192) {
  uint64_t b = (n + threads - 1) / threads;
  if (b < 1) b = 1;
  if (b > (uint64_t)cap) b = cap;
  return (int)b;
}
// wave-aggregated append: one atomic per wavefront instead of one per lane
__device__ __forceinline__ unsigned wave_append(unsigned *counter, bool pred) {
  unsigned long long mask = __ballot(pred);
  if (!mask) return 0xffffffffu;
  const unsigned lane = threadIdx.x & 63;
  unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  int leader = __ffsll((long long)mask) - 1;
  unsigned base = 0;
  if ((int)lane == leader) base = atomicAdd(counter, (unsigned)__popcll(mask));
  base = __shfl(base, leader, 64);
  return pred ? base + (unsigned)__popcll(mask & lt) : 0xffffffffu;
}
// Ordered (left-to-right, from +0) sum of one row's products by a whole wavefront:
// the 64 products of a chunk are added on the integer grid of the running sum's
// binade while the running sum stays strictly inside it -- fl(s + p) = s + RN_u(p)
// there, so the sequential sum is s + u * (inclusive integer scan); the first
// product that leaves the binade (or is a tie, huge or non-finite) is added the
// ordinary way and the walk continues from the next one.  Bit-identical to the
// sequential loop (the argument of the reference-order dots, amgd_rt.hip).
// Every lane passes its own product `p` of the chunk (lanes >= m: ignored) and
// every lane returns the same updated sum.
__device__ __forceinline__ long long wave_incl_scan_i64(long long v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    long long y = __shfl_up(v, o, 64);
    if (lane >= o) v = (long long)((unsigned long long)v + (unsigned long long)y);
  }
  return v;
}
__device__ __forceinline__ double wave_chunk_add(double s, double p, int m, int lane) {
  const long long LO = 1ll << 52, HI = 1ll << 53;
  int j = 0;
  while (j < m) {
    const bool act = lane >= j && lane < m;
    if (s == 0.0) {                          // +0 + (+-0) = +0: jump to the first nonzero
      const unsigned long long nzm = __ballot(act && p != 0.0);
      if (!nzm) break;
      const int f = __ffsll((long long)nzm) - 1;
      s = __shfl(p, f, 64);                  // +0 + p == p exactly
      j = f + 1;
      continue;
    }
    if (!(fabs(s) >= 2.2250738585072014e-308) || !(fabs(s) < 1.0e300)) {
      for (int q = j; q < m; q++) s = s + __shfl(p, q, 64);   // subnormal / huge: one by one
      break;
    }
    const int e = ilogb(s);
    const long long S0 = (long long)ldexp(s, 52 - e);          // |S0| in [2^52, 2^53)
    const double xq = ldexp(p, 52 - e);
    const double r = rint(xq);
    const bool bad = act && (!(fabs(xq) < 7.2e16) || fabs(r - xq) == 0.5);
    const long long v = (act && !bad) ? (long long)r : 0ll;
    const long long P = wave_incl_scan_i64(v, lane);
    const long long run = (long long)((unsigned long long)S0 + (unsigned long long)P);
    const bool inside = S0 > 0 ? (run > LO && run < HI) : (run < -LO && run > -HI);
    const unsigned long long vm = __ballot(act && (bad || !inside));
    if (!vm) {
      const long long fin = __shfl(run, m - 1, 64);
      s = ldexp((double)fin, e - 52);
      break;
    }
    const int vl = __ffsll((long long)vm) - 1;                  // first violating product
    const long long before = __shfl(run, vl > 0 ? vl - 1 : 0, 64);
    const double sb = vl > j ? ldexp((double)before, e - 52) : s;
    s = sb + __shfl(p, vl, 64);
    j = vl + 1;
  }
  return s;
}
#define GRID_STRIDE(i, n) \
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (uint64_t)(n); \
       i += (uint64_t)gridDim.x * blockDim.x)
// inclusive block scan of one u32 per thread (NT = 64 or 256)
template <int NT>
__device__ __forceinline__ uint32_t block_incl_scan(uint32_t v, uint32_t *wtot) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t y = __shfl_up(v, o, 64);
    if (lane >= o) v += y;
  }
  if (NT == 64) return v;
  const int w = threadIdx.x >> 6;
  if (lane == 63) wtot[w] = v;
  __syncthreads();
  uint32_t add = 0;
  for (int q = 0; q < w; q++) add += wtot[q];
  __syncthreads();
  return v + add;
}
#endif
