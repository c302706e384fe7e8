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
