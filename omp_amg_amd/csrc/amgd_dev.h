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
#endif
