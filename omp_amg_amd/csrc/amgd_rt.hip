// amgd_rt.hip -- runtime for the MI355X AMG setup: stream, caching HBM pool,
// copies, event timers, scans (rocPRIM), deterministic reductions.
//
// Reductions are two-stage with a fixed grid, so every result is run-to-run
// reproducible; they are NOT the reference's left-to-right sums (amg_setup.c:3193),
// which is the one documented source of last-bit differences (DESIGN.md "Parity").
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_scan.hpp>

#include <cfloat>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <chrono>
#include <map>
#include <unordered_map>
#include <iterator>

#include "amgd.h"
#include "amgd_dev.h"

static hipStream_t g_stream = nullptr;
static bool g_inited = false;
static char g_err[512];

void amgd_check(hipError_t e, const char *what, const char *file, int line) {
  if (e != hipSuccess) {
    snprintf(g_err, sizeof g_err, "%s failed at %s:%d: %s", what, file, line, hipGetErrorString(e));
    fprintf(stderr, "omp_amg_amd: %s\n", g_err);
    fflush(stderr);
    abort();
  }
}

extern "C" const char *amgd_last_error(void) { return g_err; }
extern "C" void amgd_set_error(const char *msg) { snprintf(g_err, sizeof g_err, "%s", msg); }

// The reference's Lanczos start vector comes from the process-wide libc rand()
// stream (amg_setup.c:2447).  The HIP runtime may draw from that stream while it
// initialises, so runtime start-up runs on a scratch random(3) state and the
// caller's state is restored untouched afterwards.
static char g_rand_scratch[256];
extern "C" int amgd_rt_init(int device) {
  if (g_inited) return 0;
  char *saved = initstate(12345u, g_rand_scratch, sizeof g_rand_scratch);
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    snprintf(g_err, sizeof g_err, "no HIP device visible");
    setstate(saved);
    return -1;
  }
  HIPCK(hipSetDevice(device));
  HIPCK(hipStreamCreateWithFlags(&g_stream, hipStreamNonBlocking));
  // touch the device once so lazy code-object loading also happens here
  void *p = nullptr;
  HIPCK(hipMalloc(&p, 256));
  HIPCK(hipMemsetAsync(p, 0, 256, g_stream));
  HIPCK(hipStreamSynchronize(g_stream));
  HIPCK(hipFree(p));
  g_inited = true;
  setstate(saved);
  return 0;
}

hipStream_t amgd_s() {
  if (!g_inited && amgd_rt_init(0) != 0) {
    fprintf(stderr, "omp_amg_amd: HIP runtime unavailable: %s\n", g_err);
    abort();
  }
  return g_stream;
}
extern "C" void *amgd_stream(void) { return (void *)amgd_s(); }
extern "C" void amgd_set_stream(void *s) { amgd_s(); g_stream = (hipStream_t)s; }

// ---------------- HBM arena ----------------
// hipMalloc costs tens of microseconds to milliseconds (and hipFree synchronises
// the device); the setup makes ~10^4-10^5 short-lived allocations per run, of
// sizes from bytes to tens of GB.  One arena is reserved at the first allocation
// (all free HBM but a margin, AMGD_ARENA_GB overrides; 0 disables) and carved
// best-fit, with neighbouring free blocks coalesced on release.  Requests the
// arena cannot hold fall back to hipMalloc.  Blocks are recycled in stream order
// (one library stream; the Q-factor side stream is joined before its blocks are
// freed), so no block is reused while a kernel may still touch it.
static char *g_arena = nullptr;
static size_t g_arena_sz = 0;
static bool g_arena_tried = false;
static std::map<size_t, size_t> g_free_off;          // offset -> size
static std::multimap<size_t, size_t> g_free_sz;      // size -> offset
struct UsedBlock { size_t sz; uint64_t serial; };
static std::unordered_map<void *, UsedBlock> g_used; // live block -> size, allocation serial
static std::unordered_map<void *, size_t> g_direct;  // live hipMalloc fallbacks -> size
static size_t g_inuse = 0, g_peak = 0, g_ipeak = 0;
static uint64_t g_serial = 0;                         // allocations made so far
static size_t g_cap = (size_t)-1;                    // AMGD_HBM_CAP_GB / amgd_set_hbm_cap
static int g_cap_read = 0, g_try_depth = 0;
struct amgd_oom_error {};
// statistics (AMGD_PHASES report): driver allocations (arena + fallbacks), their time
static uint64_t g_nmalloc = 0, g_nrelease = 0;
static double g_tmalloc = 0, g_bmalloc = 0;
extern "C" { uint64_t amgd_route_ctr[32]; }
extern "C" void amgd_pool_stats(uint64_t *nmalloc, double *gbytes, double *ms, uint64_t *nrelease) {
  *nmalloc = g_nmalloc; *gbytes = g_bmalloc / 1e9; *ms = g_tmalloc * 1e3; *nrelease = g_nrelease;
}
static void free_insert(size_t off, size_t sz) {
  auto nx = g_free_off.lower_bound(off);
  if (nx != g_free_off.end() && nx->first == off + sz) {         // merge with the next block
    auto r = g_free_sz.equal_range(nx->second);
    for (auto it = r.first; it != r.second; ++it) if (it->second == nx->first) { g_free_sz.erase(it); break; }
    sz += nx->second;
    nx = g_free_off.erase(nx);
  }
  if (nx != g_free_off.begin()) {                                 // merge with the previous block
    auto pv = std::prev(nx);
    if (pv->first + pv->second == off) {
      auto r = g_free_sz.equal_range(pv->second);
      for (auto it = r.first; it != r.second; ++it) if (it->second == pv->first) { g_free_sz.erase(it); break; }
      off = pv->first;
      sz += pv->second;
      g_free_off.erase(pv);
    }
  }
  g_free_off[off] = sz;
  g_free_sz.insert({sz, off});
}
static void arena_init() {
  g_arena_tried = true;
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) { (void)hipGetLastError(); return; }
  const size_t margin = 24ull << 30;
  size_t want = fr > margin ? fr - margin : 0;
  const char *e = getenv("AMGD_ARENA_GB");
  if (e && *e) want = std::min<size_t>(want, (size_t)atoll(e) << 30);
  want &= ~((size_t)(2u << 20) - 1);
  auto t0 = std::chrono::steady_clock::now();
  while (want >= (1ull << 30)) {
    if (hipMalloc((void **)&g_arena, want) == hipSuccess) break;
    (void)hipGetLastError();
    g_arena = nullptr;
    want /= 2;
  }
  g_tmalloc += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (!g_arena) return;
  g_arena_sz = want;
  g_nmalloc++;
  g_bmalloc += (double)want;
  free_insert(0, want);
}

extern "C" void amgd_set_hbm_cap(size_t bytes) { g_cap = bytes ? bytes : (size_t)-1; g_cap_read = 1; }
// Out of HBM.  Inside amgd_try (the setup entry points) the setup is unwound: every
// block it allocated is released and the entry point returns an error with the text
// in amgd_error().  Elsewhere there is no caller to report to: abort as before.
static void oom(size_t sz) {
  snprintf(g_err, sizeof g_err, "out of HBM: request %.3f GB with %.3f GB live (peak %.3f GB, arena %.3f GB%s)",
           sz / 1e9, g_inuse / 1e9, g_peak / 1e9, g_arena_sz / 1e9,
           g_cap != (size_t)-1 ? ", capped" : "");
  fprintf(stderr, "omp_amg_amd: %s\n", g_err);
  // One rank unwinding alone would leave its peers blocked in the next collective:
  // with a multi-process communicator out of HBM stays fatal.
  // With the collective guard on (AMGD_COMM_CHECK) the failure is first announced to the
  // peers through it, and every rank unwinds together.
  if (g_try_depth > 0 && (amgd_comm_procs() <= 1 || amgd_comm_fail_agree())) throw amgd_oom_error();
  abort();
}
// a peer announced its failure through the collective guard: unwind this rank as well
extern "C" void amgd_throw_oom(void) {
  if (g_try_depth > 0) throw amgd_oom_error();
  abort();
}
extern "C" int amgd_try(int (*fn)(void *), void *arg) {
  const uint64_t mark = g_serial;
  g_try_depth++;
  int rc;
  try {
    rc = fn(arg);
  } catch (const amgd_oom_error &) {
    rc = -2;
    (void)hipDeviceSynchronize();      // the side stream of the Q factors as well
    amgd_spmv_split_clear();           // cached SpMV splits, pins and gather tables first
    std::vector<void *> live;
    for (auto &u : g_used)
      if (u.second.serial >= mark) live.push_back(u.first);
    g_try_depth--;
    for (void *p : live) amgd_free(p);
    amgd_reset_call_state();           // per-call flags the unwound frames had set
    return rc;
  }
  g_try_depth--;
  return rc;
}

extern "C" void *amgd_alloc(size_t bytes) {
  amgd_s();
  if (!g_arena_tried) arena_init();
  if (!g_cap_read) {
    g_cap_read = 1;
    const char *e = getenv("AMGD_HBM_CAP_GB");
    if (e && *e && atof(e) > 0) g_cap = (size_t)(atof(e) * 1073741824.0);
  }
  size_t sz = (bytes + 255) & ~(size_t)255;
  if (sz == 0) sz = 256;
  if (g_inuse + sz > g_cap) oom(sz);
  void *p = nullptr;
  auto it = g_free_sz.lower_bound(sz);                           // best fit
  if (it != g_free_sz.end()) {
    const size_t bsz = it->first, off = it->second;
    g_free_sz.erase(it);
    g_free_off.erase(off);
    if (bsz > sz) free_insert(off + sz, bsz - sz);
    p = g_arena + off;
  } else {                                                        // arena full: the driver
    auto t0 = std::chrono::steady_clock::now();
    if (hipMalloc(&p, sz) != hipSuccess) {
      (void)hipGetLastError();
      oom(sz);
    }
    g_tmalloc += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    g_nmalloc++;
    g_bmalloc += (double)sz;
    g_direct[p] = sz;
  }
  g_used[p] = UsedBlock{sz, g_serial++};
  g_inuse += sz;
  if (g_inuse > g_peak) g_peak = g_inuse;
  if (g_inuse > g_ipeak) g_ipeak = g_inuse;
  return p;
}

// Arrays of doubles.  AMGD_POISON=1 (tests): every such block starts as all-ones bytes, a NaN
// in every slot, instead of whatever the arena held -- a value read before it is written
// then turns the hierarchy into NaNs (a digest mismatch) instead of passing by luck
static int g_poison = -1;
extern "C" void amgd_set_poison(int on) { g_poison = on; }
extern "C" void *amgd_alloc_f64(size_t bytes) {
  void *p = amgd_alloc(bytes);
  if (g_poison < 0) { const char *e = getenv("AMGD_POISON"); g_poison = e && *e ? atoi(e) : 0; }
  if (g_poison > 0 && bytes) HIPCK(hipMemsetAsync(p, 0xff, bytes, amgd_s()));
  return p;
}
extern "C" void amgd_free(void *p) {
  if (!p) return;
  amgd_spmv_split_forget(p);
  auto it = g_used.find(p);
  if (it == g_used.end()) {
    fprintf(stderr, "omp_amg_amd: amgd_free of unknown pointer %p\n", p);
    abort();
  }
  const size_t sz = it->second.sz;
  g_used.erase(it);
  g_inuse -= sz;
  auto d = g_direct.find(p);
  if (d != g_direct.end()) {        // a fallback block goes back to the driver (stream-ordered)
    g_direct.erase(d);
    HIPCK(hipStreamSynchronize(g_stream));
    HIPCK(hipFree(p));
    g_nrelease++;
    return;
  }
  free_insert((size_t)((char *)p - g_arena), sz);
}

extern "C" void amgd_pool_release(void) {
  // the arena stays reserved for the process; nothing is cached outside it
  if (!g_inited) return;
  HIPCK(hipStreamSynchronize(g_stream));
}
extern "C" size_t amgd_pool_bytes_in_use(void) { return g_inuse; }
extern "C" size_t amgd_pool_peak_bytes(void) { return g_peak; }
extern "C" void amgd_pool_peak_reset(void) { g_peak = g_inuse; }
// the peak since the last call (phase tables: which phase holds the setup's peak)
extern "C" size_t amgd_pool_ipeak_take(void) {
  const size_t p = g_ipeak;
  g_ipeak = g_inuse;
  return p;
}

extern "C" void amgd_h2d(void *d, const void *h, size_t n) {
  if (n) HIPCK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, amgd_s()));
  HIPCK(hipStreamSynchronize(g_stream));
}
// Small readbacks (counts, scalars, flags: ~15 k per 256^3 setup) skip the runtime's
// copy + stream synchronisation: a one-wavefront kernel, ordered after all earlier work
// on the stream, stores the bytes and then a sequence number into host-coherent memory,
// and the host polls the sequence number.  A blocking hipMemcpyAsync + hipStreamSynchronize
// left the GPU idle ~28 us per readback (the copy's own launch, the completion signal,
// the host's wake-up); a polled store cuts that gap.  After ~0.5 s of polling the host
// falls back to hipStreamSynchronize, which reports a device fault as before.
// AMGD_D2H_POLL=0: the blocking copy for every readback.
#define PUB_MAX 256
static uint8_t *g_pub = nullptr;                 // [0, 8): sequence; [64, 64 + PUB_MAX): data
static uint64_t g_pub_seq = 0;
static int g_pub_on = -1;
__global__ void k_publish(const uint8_t *src, uint32_t n, uint8_t *dst, unsigned long long *flag,
                          unsigned long long seq) {
  for (uint32_t i = threadIdx.x; i < n; i += 64) dst[i] = src[i];
  __threadfence_system();
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
static bool pub_ready() {
  if (g_pub_on < 0) {
    const char *e = getenv("AMGD_D2H_POLL");
    g_pub_on = !(e && *e == '0');
    if (g_pub_on) {
      void *p = nullptr;
      if (hipHostMalloc(&p, 64 + PUB_MAX, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
        (void)hipGetLastError();
        g_pub_on = 0;
      } else {
        g_pub = (uint8_t *)p;
        memset(g_pub, 0, 64 + PUB_MAX);
      }
    }
  }
  return g_pub_on > 0;
}
// (A/B, tests) 0: blocking copies, 1: polled, -1: as AMGD_D2H_POLL says
extern "C" void amgd_set_d2h_poll(int on) {
  if (on == 0) { if (g_pub_on < 0) pub_ready(); if (g_pub_on > 0) g_pub_on = 2; return; }
  if (on == 1) {                        // polled, whatever AMGD_D2H_POLL said
    if (!g_pub) {
      void *p = nullptr;
      if (hipHostMalloc(&p, 64 + PUB_MAX, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
        (void)hipGetLastError();
        g_pub_on = 0;
        return;
      }
      g_pub = (uint8_t *)p;
      memset(g_pub, 0, 64 + PUB_MAX);
      g_pub_seq = 0;
    }
    g_pub_on = 1;
    return;
  }
  g_pub_on = -1;                        // -1: as the environment says (re-read on next use)
  if (g_pub) g_pub_on = 1;
  const char *e = getenv("AMGD_D2H_POLL");
  if (e && *e == '0') g_pub_on = g_pub ? 2 : 0;
}
extern "C" void amgd_d2h(void *h, const void *d, size_t n) {
  if (n && n <= PUB_MAX && pub_ready() && g_pub_on == 1) {
    const unsigned long long seq = ++g_pub_seq;
    k_publish<<<1, 64, 0, amgd_s()>>>((const uint8_t *)d, (uint32_t)n, g_pub + 64,
                                      (unsigned long long *)g_pub, seq);
    HIPCK(hipGetLastError());
    const volatile unsigned long long *flag = (const volatile unsigned long long *)g_pub;
    auto t0 = std::chrono::steady_clock::now();
    for (uint32_t it = 1; __atomic_load_n((const unsigned long long *)flag, __ATOMIC_ACQUIRE) != seq; it++) {
      __builtin_ia32_pause();
      if ((it & 4095u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(500)) {
        HIPCK(hipStreamSynchronize(g_stream));   // a long wait: block (reports faults)
        if (__atomic_load_n((const unsigned long long *)flag, __ATOMIC_ACQUIRE) != seq) {
          fprintf(stderr, "omp_amg_amd: readback flag not set after the stream drained\n");
          abort();
        }
        break;
      }
    }
    memcpy(h, g_pub + 64, n);
    return;
  }
  if (n) HIPCK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, amgd_s()));
  HIPCK(hipStreamSynchronize(g_stream));
}
extern "C" void amgd_d2d(void *d, const void *s, size_t n) {
  if (n) HIPCK(hipMemcpyAsync(d, s, n, hipMemcpyDeviceToDevice, amgd_s()));
}
extern "C" void amgd_memset(void *d, int v, size_t n) {
  if (n) HIPCK(hipMemsetAsync(d, v, n, amgd_s()));
}
extern "C" void amgd_sync(void) { HIPCK(hipStreamSynchronize(amgd_s())); }
extern "C" double amgd_wtime(void) {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

// ---------------- event timers ----------------
#define NTIMERS 16
static hipEvent_t g_t0[NTIMERS], g_t1[NTIMERS];
static std::vector<std::pair<hipEvent_t, hipEvent_t>> g_pend[NTIMERS];
static double g_acc[NTIMERS];
static bool g_tinit = false;
static void tinit() {
  if (g_tinit) return;
  for (int i = 0; i < NTIMERS; i++) g_acc[i] = 0;
  g_tinit = true;
}
static std::vector<hipEvent_t> g_evpool;   // recycled timing events (thousands per setup)
static hipEvent_t ev_get() {
  if (!g_evpool.empty()) { hipEvent_t e = g_evpool.back(); g_evpool.pop_back(); return e; }
  hipEvent_t e;
  HIPCK(hipEventCreate(&e));
  return e;
}
extern "C" void amgd_timer_start(int s) {
  tinit();
  hipEvent_t a = ev_get();
  HIPCK(hipEventRecord(a, amgd_s()));
  g_t0[s] = a;
}
extern "C" void amgd_timer_stop(int s) {
  hipEvent_t b = ev_get();
  HIPCK(hipEventRecord(b, amgd_s()));
  g_pend[s].push_back({g_t0[s], b});
}
// Two slots over the same interval (the long-row SpMV: all shapes + its own shape) share
// one event per end -- each timing event on the stream costs a few microseconds of GPU
// idle between kernels.  A shared event returns to the pool when both slots have read it.
static std::unordered_map<hipEvent_t, int> g_evshare;
extern "C" void amgd_timer_start2(int s, int s2) {
  amgd_timer_start(s);
  g_t0[s2] = g_t0[s];
}
extern "C" void amgd_timer_stop2(int s, int s2) {
  hipEvent_t b = ev_get();
  HIPCK(hipEventRecord(b, amgd_s()));
  g_pend[s].push_back({g_t0[s], b});
  g_pend[s2].push_back({g_t0[s2], b});
  g_evshare[g_t0[s]] += 2;
  g_evshare[b] += 2;
}
static void ev_put(hipEvent_t e) {
  auto it = g_evshare.find(e);
  if (it != g_evshare.end()) {
    if (--it->second > 0) return;
    g_evshare.erase(it);
  }
  g_evpool.push_back(e);
}
extern "C" double amgd_timer_ms(int s) {
  tinit();
  for (auto &pr : g_pend[s]) {
    HIPCK(hipEventSynchronize(pr.second));
    float ms = 0;
    HIPCK(hipEventElapsedTime(&ms, pr.first, pr.second));
    g_acc[s] += ms;
    ev_put(pr.first);
    ev_put(pr.second);
  }
  g_pend[s].clear();
  return g_acc[s];
}
extern "C" void amgd_timer_reset(void) {
  tinit();
  for (int i = 0; i < NTIMERS; i++) { (void)amgd_timer_ms(i); g_acc[i] = 0; }
}

// ---------------- dcsr helpers ----------------
extern "C" dcsr *dcsr_new(uint32_t rn, uint32_t cn, uint64_t nnz) {
  dcsr *A = (dcsr *)malloc(sizeof(dcsr));
  A->rn = rn; A->cn = cn; A->nnz = nnz;
  A->ro = (uint64_t *)amgd_alloc(((size_t)rn + 1) * 8);
  A->col = (uint32_t *)amgd_alloc(nnz * 4 + 4);
  A->a = (double *)amgd_alloc_f64(nnz * 8 + 8);
  return A;
}
extern "C" void dcsr_free(dcsr **A) {
  if (!A || !*A) return;
  amgd_free((*A)->ro); amgd_free((*A)->col); amgd_free((*A)->a);
  free(*A);
  *A = nullptr;
}
extern "C" dcsr *dcsr_copy(const dcsr *A) {
  dcsr *B = dcsr_new(A->rn, A->cn, A->nnz);
  amgd_d2d(B->ro, A->ro, ((size_t)A->rn + 1) * 8);
  amgd_d2d(B->col, A->col, A->nnz * 4);
  amgd_d2d(B->a, A->a, A->nnz * 8);
  return B;
}
extern "C" dcsr *dcsr_empty_like_pattern(const dcsr *A) {
  dcsr *B = dcsr_new(A->rn, A->cn, A->nnz);
  amgd_d2d(B->ro, A->ro, ((size_t)A->rn + 1) * 8);
  amgd_d2d(B->col, A->col, A->nnz * 4);
  return B;
}

// ---------------- scans ----------------
template <typename T>
static T scan_impl(T *counts, uint64_t n) {
  hipStream_t s = amgd_s();
  T *tmpout = (T *)amgd_alloc((n + 1) * sizeof(T));
  size_t tb = 0;
  HIPCK(rocprim::exclusive_scan(nullptr, tb, counts, tmpout, (T)0, (size_t)(n + 1),
                                rocprim::plus<T>(), s));
  void *tmp = amgd_alloc(tb + 16);
  // counts[n] must be a valid slot: callers allocate n+1; set it to 0 first
  HIPCK(hipMemsetAsync(counts + n, 0, sizeof(T), s));
  HIPCK(rocprim::exclusive_scan(tmp, tb, counts, tmpout, (T)0, (size_t)(n + 1),
                                rocprim::plus<T>(), s));
  HIPCK(hipMemcpyAsync(counts, tmpout, (n + 1) * sizeof(T), hipMemcpyDeviceToDevice, s));
  T total;
  amgd_d2h(&total, tmpout + n, sizeof(T));
  amgd_free(tmp);
  amgd_free(tmpout);
  return total;
}
extern "C" uint64_t amgd_scan_u64(uint64_t *c, uint64_t n) { return scan_impl<uint64_t>(c, n); }
extern "C" uint32_t amgd_scan_u32(uint32_t *c, uint64_t n) { return scan_impl<uint32_t>(c, n); }

__global__ void k_mask_to_u32(const uint8_t *m, uint32_t n, uint32_t *o) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    o[i] = m[i] ? 1u : 0u;
}
__global__ void k_rank_fix(const uint8_t *m, uint32_t n, uint32_t *o) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    if (!m[i]) o[i] = 0xffffffffu;
}
extern "C" uint32_t amgd_mask_rank(const uint8_t *mask, uint32_t n, uint32_t *map) {
  // map must hold n+1 entries
  k_mask_to_u32<<<grid_for(n), 256, 0, amgd_s()>>>(mask, n, map);
  uint32_t tot = amgd_scan_u32(map, n);
  k_rank_fix<<<grid_for(n), 256, 0, amgd_s()>>>(mask, n, map);
  return tot;
}

// ---------------- deterministic reductions ----------------
// Stage 1: RED_BLOCKS fixed blocks, grid-stride partial sums in a fixed order;
// stage 2: one block reduces the partials.  Same n -> same bits every run.
#define RED_BLOCKS 1024
#define RED_THREADS 256

template <typename Op>
__device__ double block_reduce(double v, Op op) {
  __shared__ double sh[RED_THREADS / 64];
  for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_down(v, o, 64));
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x < 64) {
    v = threadIdx.x < RED_THREADS / 64 ? sh[threadIdx.x] : 0.0;
    for (int o = 32; o > 0; o >>= 1) {
      double u = __shfl_down(v, o, 64);
      if (threadIdx.x + o < RED_THREADS / 64) v = op(v, u);
    }
  }
  return v;
}
struct AddOp { __device__ double operator()(double a, double b) const { return a + b; } };

__global__ void k_dot_partial(const double *a, const double *b, uint64_t n, double *part) {
  double s = 0.0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    s += a[i] * (b ? b[i] : a[i]);
  s = block_reduce(s, AddOp());
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}
__global__ void k_dot3_partial(const double *M, const double *b, uint64_t n, double *part) {
  double s = 0.0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    s += (M[i] * b[i]) * b[i];
  s = block_reduce(s, AddOp());
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}
__global__ void k_sum_final(const double *part, int np, double *out) {
  double s = 0.0;
  for (int i = threadIdx.x; i < np; i += blockDim.x) s += part[i];
  s = block_reduce(s, AddOp());
  if (threadIdx.x == 0) *out = s;
}
static double *g_red = nullptr;  // RED_BLOCKS partials + scalars
static double *g_red_h = nullptr;
static double *red_buf() {
  if (!g_red) {
    HIPCK(hipMalloc(&g_red, (RED_BLOCKS * 2 + 64) * sizeof(double)));
    HIPCK(hipHostMalloc(&g_red_h, 64 * sizeof(double)));
  }
  return g_red;
}
static int red_grid(uint64_t n) {
  uint64_t b = (n + RED_THREADS - 1) / RED_THREADS;
  return (int)std::max<uint64_t>(1, std::min<uint64_t>(b, RED_BLOCKS));
}
static double sum_finish(int nb) {
  double *p = red_buf();
  k_sum_final<<<1, RED_THREADS, 0, amgd_s()>>>(p, nb, p + 2 * RED_BLOCKS);
  amgd_d2h(g_red_h, p + 2 * RED_BLOCKS, 8);
  return g_red_h[0];
}
// Reference-order ("exact") dot products.  The reference sums left to right
// (vv_dot amg_setup.c:3193, norm2 :3309, pcg's rho_0 :2265-2267).  Its
// constraint solve runs PCG on an indefinite, non-symmetric S whenever
// sp_add lands off-pattern (DESIGN.md "Reference UB"); there the iteration is
// chaotic and only the reference's own summation order reproduces it.  In
// exact mode (default) one wavefront carries the sequential sum while three
// others stage the next tile of products through LDS: latency-bound
// (one dependent f64 add per element), bit-identical to the reference.
#define SEQ_TILE 2048
template <int MODE>   // 0: a.b  1: a.a  2: (M.*b).*b
__global__ __launch_bounds__(256) void k_dot_seq(const double *a, const double *b, uint64_t n,
                                                 double *out) {
  __shared__ double buf[2][SEQ_TILE];
  const int tid = threadIdx.x;
  double s = 0.0;
  uint64_t ntile = (n + SEQ_TILE - 1) / SEQ_TILE;
  // prologue: stage tile 0 with every thread
  for (uint64_t j = tid; j < SEQ_TILE && j < n; j += 256) {
    double x = a[j];
    buf[0][j] = MODE == 0 ? x * b[j] : MODE == 1 ? x * x : (x * b[j]) * b[j];
  }
  __syncthreads();
  for (uint64_t t = 0; t < ntile; t++) {
    int cur = (int)(t & 1);
    uint64_t base = t * SEQ_TILE;
    if (tid < 64) {
      if (tid == 0) {
        uint64_t m = n - base < SEQ_TILE ? n - base : SEQ_TILE;
        const double *p = buf[cur];
        uint64_t j = 0;
        // independent LDS loads first, then the dependent add chain in order
        for (; j + 16 <= m; j += 16) {
          double v[16];
#pragma unroll
          for (int q = 0; q < 16; q++) v[q] = p[j + q];
#pragma unroll
          for (int q = 0; q < 16; q++) s += v[q];
        }
        for (; j < m; j++) s += p[j];
      }
    } else if (t + 1 < ntile) {
      uint64_t nb = base + SEQ_TILE;
      for (uint64_t j = tid - 64; j < SEQ_TILE; j += 192) {
        uint64_t i = nb + j;
        if (i < n) {
          double x = a[i];
          buf[cur ^ 1][j] = MODE == 0 ? x * b[i] : MODE == 1 ? x * x : (x * b[i]) * b[i];
        }
      }
    }
    __syncthreads();
  }
  if (tid == 0) *out = s;
}
// ---------------------------------------------------------------------------
// Parallel bit-exact emulation of the sequential sum s = ((0 + p0) + p1) + ...
//
// While the running sum s stays strictly inside one binade [2^e, 2^(e+1)) (or
// its negative), every step rounds on the fixed grid u = 2^(e-52) and s is a
// multiple of u, so fl(s + p) = s + RN_u(p): the step is an integer addition
// of m = rint(p/u) in units of u.  One 1024-thread block streams tiles of
// products through LDS, computes the m's, block-scans them, and finds the first
// index where the candidate running value leaves the binade interior, where
// p/u is an exact tie (ties-to-even would depend on s), or where |p/u| is
// huge.  Everything before that index is committed at once; that element is
// added the ordinary way; the scan resumes after it.  The result is identical,
// bit for bit, to the left-to-right loop (tests/test_gpu_kernels.py checks it
// against k_dot_seq on adversarial inputs).
// ---------------------------------------------------------------------------
#define BN_THREADS 1024
#define BN_PER 4
#define BN_TILE (BN_THREADS * BN_PER)

__device__ __forceinline__ long long bn_block_excl_scan(long long v, long long *sh, long long *total) {
  // exclusive scan of one value per thread across the block (wrapping arithmetic)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned long long x = (unsigned long long)v;
  for (int o = 1; o < 64; o <<= 1) {
    unsigned long long y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[w] = (long long)x;
  __syncthreads();
  if (w == 0) {
    unsigned long long t = lane < BN_THREADS / 64 ? (unsigned long long)sh[lane] : 0ull;
    for (int o = 1; o < 64; o <<= 1) {
      unsigned long long y = __shfl_up(t, o, 64);
      if (lane >= o) t += y;
    }
    if (lane < BN_THREADS / 64) sh[lane] = (long long)t;   // inclusive per-wave totals
  }
  __syncthreads();
  unsigned long long before = w > 0 ? (unsigned long long)sh[w - 1] : 0ull;
  unsigned long long incl = before + x;
  *total = sh[BN_THREADS / 64 - 1];
  __syncthreads();
  return (long long)(incl - (unsigned long long)v);
}

__device__ __forceinline__ double bn_product(const double *a, const double *b, uint64_t i, int MODE_) {
  double x = a[i];
  return MODE_ == 0 ? x * b[i] : MODE_ == 1 ? x * x : (x * b[i]) * b[i];
}
// the whole block adds products [lo, hi) to the running sum s (uniform), in order
// MODE 0: a[i]*b[i], 1: a[i]^2, 2: (a[i]*b[i])*b[i], 3: a[i]*b[gcol[i]] (a row of a
// sparse matrix times a gathered vector), 4: a[i]
// AMGD_SEGSTAT=1 (analysis): exact-sum counters -- [0] k_seg_resolve rows, [1] chunks,
// [2] chunks that failed their speculation (binade_range), [3] binade_range rounds,
// [4] elements summed one by one (rounds > 48 or subnormal sums), [5] zero-skip steps;
// [6] chunks resolved by their split records; the exact dots: [7] chunks that failed their
// speculation, [8] of them resolved by their split records; printed at process exit
__device__ unsigned long long d_segstat[10];
__device__ int d_segstat_on = 0;
template <int MODE>
__device__ double binade_range(const double *a, const double *b, uint64_t lo, uint64_t hi, double s,
                               double *tile, long long *sh, double *s_sh, int *viol_sh,
                               const uint32_t *gcol = nullptr) {
  const int tid = threadIdx.x;
  for (uint64_t base = lo; base < hi; base += BN_TILE) {
    int tlen = (int)min((uint64_t)BN_TILE, hi - base);
    for (int q = tid; q < tlen; q += BN_THREADS) {
      uint64_t i = base + q;
      double x = a[i];
      tile[q] = MODE == 0 ? x * b[i] : MODE == 1 ? x * x : MODE == 2 ? (x * b[i]) * b[i]
              : MODE == 3 ? x * b[gcol[i]] : x;
    }
    __syncthreads();
    int j = 0, rounds = 0;
    while (j < tlen) {
      // sequential steps where the grid argument does not apply (s == 0,
      // subnormal s), or once a tile has needed too many re-scans
      if (s == 0.0 && rounds <= 48) {
        if (d_segstat_on && tid == 0) atomicAdd(&d_segstat[5], 1ull);
        // 0 + p == p exactly (and +0 for a zero p): jump to the first nonzero product
        if (tid == 0) (*viol_sh) = 0x7fffffff;
        __syncthreads();
        for (int q = j + tid; q < tlen; q += BN_THREADS)
          if (tile[q] != 0.0) { atomicMin(&(*viol_sh), q); break; }
        __syncthreads();
        int f = (*viol_sh);
        if (f == 0x7fffffff) { j = tlen; }
        else { s = s + tile[f]; j = f + 1; }
        __syncthreads();
        continue;
      }
      if (fabs(s) < 2.2250738585072014e-308 || rounds > 48) {
        if (tid == 0) {
          double t = s;
          int stop = rounds > 48 ? tlen : j + 1;
          if (d_segstat_on) atomicAdd(&d_segstat[4], (unsigned long long)(stop - j));
          for (int q = j; q < stop; q++) t += tile[q];
          (*s_sh) = t;
        }
        __syncthreads();
        s = (*s_sh);
        j = rounds > 48 ? tlen : j + 1;
        __syncthreads();
        continue;
      }
      rounds++;
      if (d_segstat_on && tid == 0) atomicAdd(&d_segstat[3], 1ull);
      int e = ilogb(s);
      double u = ldexp(1.0, e - 52);
      long long S0 = (long long)ldexp(s, 52 - e);       // |S0| in [2^52, 2^53)
      const long long LO = (1ll << 52), HI = (1ll << 53);
      // each thread owns BN_PER consecutive elements of [j, tlen)
      int first = j + tid * BN_PER;
      long long m[BN_PER];
      bool bad[BN_PER];
      long long loc = 0;
#pragma unroll
      for (int q = 0; q < BN_PER; q++) {
        int idx = first + q;
        m[q] = 0;
        bad[q] = false;
        if (idx < tlen) {
          double x = tile[idx] / u;                       // exact: power-of-two scaling
          double r = rint(x);
          if (!(fabs(x) < 4.6e18) || fabs(r - x) == 0.5) bad[q] = true;   // huge or tie
          else m[q] = (long long)r;
        }
        loc = (long long)((unsigned long long)loc + (unsigned long long)m[q]);
      }
      long long total;
      long long pre = bn_block_excl_scan(loc, sh, &total);
      // first violating index in my elements
      int myv = 0x7fffffff;
      long long run = (long long)((unsigned long long)S0 + (unsigned long long)pre);
#pragma unroll
      for (int q = 0; q < BN_PER; q++) {
        int idx = first + q;
        if (idx >= tlen || myv != 0x7fffffff) continue;
        if (bad[q]) { myv = idx; continue; }
        run = (long long)((unsigned long long)run + (unsigned long long)m[q]);
        bool inside = S0 > 0 ? (run > LO && run < HI) : (run < -LO && run > -HI);
        if (!inside) myv = idx;
      }
      if (tid == 0) (*viol_sh) = 0x7fffffff;
      __syncthreads();
      if (myv != 0x7fffffff) atomicMin(&(*viol_sh), myv);
      __syncthreads();
      int v = (*viol_sh);
      if (v == 0x7fffffff) {
        // whole remainder stays inside the binade
        long long fin = (long long)((unsigned long long)S0 + (unsigned long long)total);
        s = ldexp((double)fin, e - 52);
        j = tlen;
      } else {
        // commit [j, v) exactly, then add element v the ordinary way
        if (first <= v - 1 && v - 1 < first + BN_PER) {
          long long r2 = (long long)((unsigned long long)S0 + (unsigned long long)pre);
          for (int q = 0; first + q < v; q++) r2 = (long long)((unsigned long long)r2 + (unsigned long long)m[q]);
          (*s_sh) = ldexp((double)r2, e - 52) + tile[v];
        }
        if (v == j && tid == 0) (*s_sh) = s + tile[v];
        __syncthreads();
        s = (*s_sh);
        j = v + 1;
      }
      __syncthreads();
    }
    __syncthreads();
  }
  return s;
}

template <int MODE>
__global__ __launch_bounds__(BN_THREADS) void k_dot_binade(const double *a, const double *b,
                                                           uint64_t n, double *out) {
  __shared__ double tile[BN_TILE];
  __shared__ long long sh[BN_THREADS / 64 + 1];
  __shared__ double s_sh;
  __shared__ int viol_sh;
  double s = binade_range<MODE>(a, b, 0, n, 0.0, tile, sh, &s_sh, &viol_sh);
  if (threadIdx.x == 0) *out = s;
}

// ---------------------------------------------------------------------------
// Multi-CU speculation for long vectors.  The vector is cut into chunks of
// BN_TILE products.  (1) every chunk's plain sum, (2) an approximate prefix
// -> a guessed binade e_c of the running sum entering chunk c, (3) for that
// guess, in parallel over chunks: M_c = sum of rint(p/u_e) and the min / max
// of its prefixes (or a flag: tie, huge, no usable guess).  (4) one block walks
// the chunks in order with the exact running sum s: if s lies in binade e_c and
// s/u + every prefix stays strictly inside the binade, the chunk is exactly
// s + u*M_c (the same integer argument as above); otherwise its split record
// (one binade crossing inside the chunk, below -- a sum of squares crosses one at
// every 2^k-th chunk) is tried, and failing that the chunk is added by
// binade_range.  The result is the sequential sum, bit for bit.
// ---------------------------------------------------------------------------
#define SP_T 256
#define SP_PER (BN_TILE / SP_T)
template <int MODE>
__global__ __launch_bounds__(SP_T) void k_dot_csum(const double *a, const double *b, uint64_t n,
                                                   double *csum) {
  __shared__ double red[SP_T];
  uint64_t G = (n + BN_TILE - 1) / BN_TILE;
  for (uint64_t c = blockIdx.x; c < G; c += gridDim.x) {
    uint64_t lo = c * BN_TILE, hi = min(n, lo + BN_TILE);
    double t = 0;
    for (uint64_t i = lo + threadIdx.x; i < hi; i += SP_T) t += bn_product(a, b, i, MODE);
    red[threadIdx.x] = t;
    __syncthreads();
    for (int o = SP_T / 2; o > 0; o >>= 1) {
      if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) csum[c] = red[0];
    __syncthreads();
  }
}
// exclusive prefix of the chunk sums (any order: it is only a guess) -- wave scans of the
// 1024 threads' parts, then of the 16 wave totals
__global__ __launch_bounds__(1024) void k_dot_approx_prefix(double *csum, uint64_t G) {
  __shared__ double wtot[16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint64_t per = (G + 1023) / 1024;
  uint64_t lo = tid * per, hi = min(G, lo + per);
  double t = 0;
  for (uint64_t c = lo; c < hi; c++) t += csum[c];
  double x = t;
  for (int o = 1; o < 64; o <<= 1) {
    const double y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wtot[w] = x;
  __syncthreads();
  double ex = __shfl_up(x, 1, 64);
  if (lane == 0) ex = 0;
  double r = 0;
  for (int q = 0; q < w; q++) r += wtot[q];
  r += ex;
  for (uint64_t c = lo; c < hi; c++) { double v = csum[c]; csum[c] = r; r += v; }
}
struct SpecRec { long long M, mn, mx; int e, flag; };
// One binade crossing inside a chunk (round 6).  On the anisotropic orphan rows a strong
// entry jumps the running sum by ~10^3 -- into a higher binade -- so its chunk fails the
// whole-chunk record and was re-summed by binade_range (a tile load and 2-3 block rounds).
// The split record describes such a chunk as part 1 = [0, j) in the guessed binade e1, the
// crossing product p_j, and part 2 = (j, len) in the binade e2 of the guessed sum after it:
// the resolve checks part 1 against the exact running sum as a whole-chunk record is
// checked (s1 = (S + M1) u1 exactly), adds p_j the ordinary way (s2 = fl(s1 + p_j), the
// sequential loop's own step), checks part 2 against s2 in e2 and takes s3 = (S2 + M2) u2 --
// the sequential sum, O(1) per chunk.  A second crossing, a tie or a failed check: the
// chunk goes to binade_range as before.
struct SegSplit { long long M1, mn1, mx1, M2, mn2, mx2; double pj; int e1, e2, ok; };
__device__ __forceinline__ long long blk4_excl_scan(long long v, long long *sm, long long *total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  long long x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const long long y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sm[w] = x;
  __syncthreads();
  long long before = 0;
  for (int q = 0; q < w; q++) before += sm[q];
  *total = sm[0] + sm[1] + sm[2] + sm[3];
  __syncthreads();
  return before + x - v;
}
__device__ __forceinline__ void blk4_minmax(long long &mn, long long &mx, long long *sm) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const long long a = __shfl_xor(mn, o, 64), b = __shfl_xor(mx, o, 64);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  if (lane == 0) { sm[w] = mn; sm[4 + w] = mx; }
  __syncthreads();
  mn = sm[0]; mx = sm[4];
  for (int q = 1; q < 4; q++) { mn = sm[q] < mn ? sm[q] : mn; mx = sm[4 + q] > mx ? sm[4 + q] : mx; }
  __syncthreads();
}
// the split record of a chunk whose products are tile[0, tlen) (SP_T threads, PER each).
// The integer steps m = rint(p/u) are recomputed from the LDS tile on every pass instead of
// held per thread (PER = 16 for the dots' 4096-product chunks: arrays would spill)
__device__ __forceinline__ long long split_step(double p, double u, bool *bad) {
  const double v = p / u, rr = rint(v);           // exact: power-of-two scaling
  if (!(fabs(v) < 4.6e18) || fabs(rr - v) == 0.5) { *bad = true; return 0; }   // huge or tie
  return (long long)rr;
}
template <int PER>
__device__ void seg_split(const double *tile, int tlen, double gs, SegSplit *out, long long *sm, int *jsh) {
  const int tid = threadIdx.x;
  const long long LO = (1ll << 52), HI = (1ll << 53), NONE_MN = 0x7fffffffffffffffll, NONE_MX = -0x7fffffffffffffffll;
  SegSplit r;
  r.ok = 0;
  const bool normal = fabs(gs) >= 2.2250738585072014e-308 && fabs(gs) < 1e300;
  if (!normal) {                                  // uniform: no split record
    if (tid == 0) *out = r;
    return;
  }
  const int e1 = ilogb(gs);
  const double u1 = ldexp(1.0, e1 - 52);
  const long long Sg = (long long)ldexp(gs, 52 - e1);
  const int first = tid * PER, last = min(first + PER, tlen);
  long long loc = 0;
  for (int idx = first; idx < last; idx++) {
    bool b = false;
    loc += split_step(tile[idx], u1, &b);
  }
  long long tot;
  const long long pre = blk4_excl_scan(loc, sm, &tot);
  // the first index whose element is bad or whose guessed running value leaves the binade
  if (tid == 0) *jsh = 0x7fffffff;
  __syncthreads();
  {
    long long run = pre;
    for (int idx = first; idx < last; idx++) {
      bool b = false;
      const long long m = split_step(tile[idx], u1, &b);
      if (b) { atomicMin(jsh, idx); break; }
      run += m;
      const long long g = Sg + run;
      const bool inside = Sg > 0 ? (g > LO && g < HI) : (g < -LO && g > -HI);
      if (!inside) { atomicMin(jsh, idx); break; }
    }
  }
  __syncthreads();
  const int j = *jsh;
  __syncthreads();
  if (j >= tlen) {                               // no crossing under the guess
    if (tid == 0) *out = r;
    return;
  }
  // part 1: [0, j) relative to the entry value; M1 = its sum (the thread owning j - 1 knows it)
  long long mn1 = NONE_MN, mx1 = NONE_MX;
  if (tid == 0) sm[8] = 0;
  __syncthreads();
  {
    long long run = pre;
    for (int idx = first; idx < min(last, j); idx++) {
      bool b = false;
      run += split_step(tile[idx], u1, &b);
      mn1 = run < mn1 ? run : mn1;
      mx1 = run > mx1 ? run : mx1;
    }
    if (j > 0 && first <= j - 1 && j - 1 < last) sm[8] = run;
  }
  __syncthreads();
  const long long M1 = sm[8];
  __syncthreads();
  blk4_minmax(mn1, mx1, sm);
  const double pj = tile[j];
  const double gs2 = (double)(Sg + M1) * u1 + pj;   // a guess of the sum after the crossing
  const bool normal2 = fabs(gs2) >= 2.2250738585072014e-308 && fabs(gs2) < 1e300;
  const int e2 = normal2 ? ilogb(gs2) : 0;
  const double u2 = ldexp(1.0, e2 - 52);
  // part 2: (j, tlen) relative to the value after the crossing
  const int f2 = max(first, j + 1);
  long long loc2 = 0;
  bool bad2 = !normal2;
  for (int idx = f2; idx < last; idx++) loc2 += split_step(tile[idx], u2, &bad2);
  long long tot2;
  const long long pre2 = blk4_excl_scan(loc2, sm, &tot2);
  long long mn2 = NONE_MN, mx2 = NONE_MX;
  {
    long long run = pre2;
    for (int idx = f2; idx < last; idx++) {
      bool b = false;
      run += split_step(tile[idx], u2, &b);
      mn2 = run < mn2 ? run : mn2;
      mx2 = run > mx2 ? run : mx2;
    }
  }
  blk4_minmax(mn2, mx2, sm);
  if (tid == 0) *jsh = 0;
  __syncthreads();
  if (bad2) atomicOr(jsh, 1);
  __syncthreads();
  const int anybad2 = *jsh;
  if (tid == 0) {
    r.M1 = M1; r.mn1 = mn1; r.mx1 = mx1;
    r.M2 = tot2; r.mn2 = mn2; r.mx2 = mx2;
    r.pj = pj; r.e1 = e1; r.e2 = e2;
    r.ok = anybad2 ? 0 : 1;
    *out = r;
  }
  __syncthreads();
}
// the split chunk from the exact running sum s: the sum after it in *out, false if a check fails
__device__ __forceinline__ bool seg_split_apply(const SegSplit &r, double s, double *out) {
  const long long LO = (1ll << 52), HI = (1ll << 53), NONE_MN = 0x7fffffffffffffffll;
  if (!r.ok || !(fabs(s) >= 2.2250738585072014e-308 && fabs(s) < 1e300) || ilogb(s) != r.e1) return false;
  const long long S = (long long)ldexp(s, 52 - r.e1);
  if (r.mn1 != NONE_MN) {                          // part 1 non-empty: every partial sum inside
    const bool in1 = S > 0 ? (S + r.mn1 > LO && S + r.mx1 < HI) : (S + r.mx1 < -LO && S + r.mn1 > -HI);
    if (!in1) return false;
  }
  const double s1 = ldexp((double)(S + r.M1), r.e1 - 52);
  const double s2 = s1 + r.pj;                     // the crossing step, as the loop adds it
  if (r.mn2 == NONE_MN) { *out = s2; return true; }   // nothing after the crossing
  if (!(fabs(s2) >= 2.2250738585072014e-308 && fabs(s2) < 1e300) || ilogb(s2) != r.e2) return false;
  const long long S2 = (long long)ldexp(s2, 52 - r.e2);
  const bool in2 = S2 > 0 ? (S2 + r.mn2 > LO && S2 + r.mx2 < HI) : (S2 + r.mx2 < -LO && S2 + r.mn2 > -HI);
  if (!in2) return false;
  *out = ldexp((double)(S2 + r.M2), r.e2 - 52);
  return true;
}
template <int MODE>
__global__ __launch_bounds__(SP_T) void k_dot_spec(const double *a, const double *b, uint64_t n,
                                                   const double *approx, SpecRec *rec,
                                                   SegSplit *rec2) {
  __shared__ double tile[BN_TILE];
  __shared__ long long ssum[SP_T / 64], smin[SP_T / 64], smax[SP_T / 64];
  __shared__ int sflag;
  __shared__ long long ssm[9];
  __shared__ int sj, sneed;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  uint64_t G = (n + BN_TILE - 1) / BN_TILE;
  for (uint64_t c = blockIdx.x; c < G; c += gridDim.x) {
    uint64_t lo = c * BN_TILE, hi = min(n, lo + BN_TILE);
    int tlen = (int)(hi - lo);
    for (int q = tid; q < tlen; q += SP_T) tile[q] = bn_product(a, b, lo + q, MODE);
    if (tid == 0) sflag = 0;
    __syncthreads();
    double g = approx[c];
    int flag = !(fabs(g) >= 1e-290) || !(fabs(g) < 1e300);
    int e = flag ? 0 : ilogb(g);
    double u = ldexp(1.0, e - 52);
    long long loc = 0, lmin = 0x7fffffffffffffffll, lmax = -0x7fffffffffffffffll;
    int first = tid * SP_PER;
    for (int q = 0; q < SP_PER; q++) {
      int idx = first + q;
      if (idx >= tlen) break;
      double x = tile[idx] / u;
      double r = rint(x);
      if (!(fabs(x) < 4.6e18) || fabs(r - x) == 0.5) { flag = 1; break; }
      loc += (long long)r;
      lmin = loc < lmin ? loc : lmin;
      lmax = loc > lmax ? loc : lmax;
    }
    if (flag) atomicOr(&sflag, 1);
    // exclusive scan of loc over the block; prefix extremes = pre + local extremes
    long long x = loc;
    for (int o = 1; o < 64; o <<= 1) {
      long long y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    long long pre_w = x - loc;                // exclusive within the wave
    long long mn = first < tlen ? pre_w + lmin : 0x7fffffffffffffffll;
    long long mx = first < tlen ? pre_w + lmax : -0x7fffffffffffffffll;
    for (int o = 32; o > 0; o >>= 1) {
      long long m1 = __shfl_xor(mn, o, 64), m2 = __shfl_xor(mx, o, 64);
      mn = m1 < mn ? m1 : mn;
      mx = m2 > mx ? m2 : mx;
    }
    if (lane == 63) ssum[w] = x;
    if (lane == 0) { smin[w] = mn; smax[w] = mx; }
    __syncthreads();
    if (tid == 0) {
      long long run = 0, gmn = 0x7fffffffffffffffll, gmx = -0x7fffffffffffffffll;
      for (int q = 0; q < SP_T / 64; q++) {
        if (smin[q] != 0x7fffffffffffffffll) {
          gmn = run + smin[q] < gmn ? run + smin[q] : gmn;
          gmx = run + smax[q] > gmx ? run + smax[q] : gmx;
        }
        run += ssum[q];
      }
      SpecRec r;
      r.M = run; r.mn = gmn; r.mx = gmx; r.e = e; r.flag = sflag;
      rec[c] = r;
      // the whole-chunk record fails under the guess (a binade crossing of the running
      // sum, e.g. every 2^k-th chunk of a sum of squares): a split record as well
      const bool gnormal = fabs(g) >= 1e-290 && fabs(g) < 1e300;
      const long long Sg = gnormal ? (long long)ldexp(g, 52 - e) : 0;
      const long long LO = (1ll << 52), HI = (1ll << 53);
      const bool inside = !sflag && gnormal &&
                          (Sg > 0 ? (Sg + gmn > LO && Sg + gmx < HI) : (Sg + gmx < -LO && Sg + gmn > -HI));
      sneed = rec2 && !inside;
    }
    __syncthreads();
    if (sneed) seg_split<SP_PER>(tile, tlen, g, rec2 + c, ssm, &sj);
    else if (rec2 && tid == 0) rec2[c].ok = 0;
    __syncthreads();
  }
}
#define SP_BATCH 512
template <int MODE>
__global__ __launch_bounds__(BN_THREADS) void k_dot_resolve(const double *a, const double *b,
                                                            uint64_t n, const SpecRec *rec,
                                                            const SegSplit *rec2, double *out) {
  __shared__ double tile[BN_TILE];
  __shared__ long long sh[BN_THREADS / 64 + 1];
  __shared__ double s_sh;
  __shared__ int viol_sh;
  __shared__ SpecRec rb[SP_BATCH];
  const int tid = threadIdx.x;
  const uint64_t G = (n + BN_TILE - 1) / BN_TILE;
  const long long LO = (1ll << 52), HI = (1ll << 53);
  double s = 0.0;
  for (uint64_t cb = 0; cb < G; cb += SP_BATCH) {
    uint64_t ce = min(G, cb + SP_BATCH);
    for (uint64_t c = cb + tid; c < ce; c += BN_THREADS) rb[c - cb] = rec[c];
    __syncthreads();
    uint64_t c = cb;
    while (c < ce) {
      // The run of chunks from c guessed in the running sum's binade e is found by
      // all threads at once (one chunk per thread, SP_BATCH <= BN_THREADS): chunk q
      // passes if its guess is e and the running integer sum S + M_c + ... + M_{q-1}
      // plus its own prefix extremes stays strictly inside (2^52, 2^53); the sum
      // over the passing prefix is exact (every partial sum before the first failing
      // chunk is bounded by the binade), so s = (S + P) * 2^(e-52) exactly -- the
      // serial walk's result in one block scan.
      const bool normal = fabs(s) >= 2.2250738585072014e-308 && fabs(s) < 1.0e300;
      const int e = normal ? ilogb(s) : 0;
      const long long S = normal ? (long long)ldexp(s, 52 - e) : 0ll;
      const uint64_t q = c + (uint64_t)tid;
      SpecRec r;
      r.M = 0; r.mn = 0; r.mx = 0; r.e = 0; r.flag = 1;
      if (q < ce) r = rb[q - cb];
      bool ok = q < ce && normal && !r.flag && r.e == e;
      long long total;
      const long long pre = bn_block_excl_scan(ok ? r.M : 0ll, sh, &total);
      if (ok) {
        const long long base = (long long)((unsigned long long)S + (unsigned long long)pre);
        ok = S > 0 ? (base + r.mn > LO && base + r.mx < HI) : (base + r.mx < -LO && base + r.mn > -HI);
      }
      if (tid == 0) viol_sh = 0x7fffffff;
      __syncthreads();
      if (q < ce && !ok) atomicMin(&viol_sh, tid);
      __syncthreads();
      const int f = viol_sh;                                  // chunks c .. c+f-1 pass
      const uint64_t run_end = f == 0x7fffffff ? ce : c + (uint64_t)f;
      if (run_end > c && (uint64_t)tid == run_end - 1 - c)
        s_sh = ldexp((double)(long long)((unsigned long long)S + (unsigned long long)(pre + r.M)), e - 52);
      __syncthreads();
      if (run_end > c) s = s_sh;
      __syncthreads();
      c = run_end;
      if (c < ce) {                         // speculation failed: add this chunk exactly
        // one crossing inside the chunk: its split record, O(1) (thread 0)
        if (tid == 0) {
          double s3;
          const bool okk = rec2 && seg_split_apply(rec2[c], s, &s3);
          viol_sh = okk ? 1 : 0;
          if (okk) s_sh = s3;
        }
        __syncthreads();
        const bool split_done = viol_sh == 1;
        if (split_done) s = s_sh;
        if (d_segstat_on && tid == 0) { atomicAdd(&d_segstat[7], 1ull); if (split_done) atomicAdd(&d_segstat[8], 1ull); }
        __syncthreads();
        if (!split_done) {
          uint64_t lo = c * BN_TILE, hi = min(n, lo + BN_TILE);
          s = binade_range<MODE>(a, b, lo, hi, s, tile, sh, &s_sh, &viol_sh);
        }
        c++;
      }
    }
    __syncthreads();
  }
  if (tid == 0) *out = s;
}
// ---------------------------------------------------------------------------
// Long rows of a row-list product (amgd_spmv_rows): the ordered sums
// sum_k a[k]*x[col[k]] (MODE 3) or sum_k a[k] (MODE 4) of rows of 10^4 - 10^5 entries,
// bit for bit, by the speculation above applied per row: the rows' BN_TILE chunks are
// summed and speculated on by the whole grid, then one block per row walks its chunk
// records (binade_range for a chunk that fails).  The row list and its length live on
// the device; every kernel reads the length there.
// ---------------------------------------------------------------------------
// The long rows' chunks are SEG_TILE = 512 products (the dots keep BN_TILE = 4096): on the
// anisotropic levels' orphan rows every strong entry is a jump of the running sum into a
// higher binade, which fails its chunk's speculation -- ~9 of a row's 29 4096-chunks, each
// then re-summed by binade_range; finer chunks confine a jump to 512 products
#define SEG_TILE 512
#define SEG_PER (SEG_TILE / SP_T)
__device__ __forceinline__ double seg_product(const double *a, const double *x, const uint32_t *col,
                                             uint64_t k, int MODE_) {
  return MODE_ == 3 ? a[k] * x[col[k]] : a[k];
}
// chunk offsets of the listed rows (exclusive scan of ceil(len / BN_TILE)); one block
__global__ __launch_bounds__(BN_THREADS) void k_seg_prep(const uint64_t *ro, const uint32_t *list,
                                                         const unsigned *nl, uint64_t *choff) {
  __shared__ long long sh[BN_THREADS / 64 + 1];
  const unsigned n = *nl;
  long long run = 0;
  for (unsigned b = 0; b < n; b += BN_THREADS) {
    const unsigned r = b + threadIdx.x;
    long long c = 0;
    if (r < n) {
      const uint32_t i = list[r];
      c = (long long)((ro[i + 1] - ro[i] + SEG_TILE - 1) / SEG_TILE);
    }
    long long total;
    const long long pre = bn_block_excl_scan(c, sh, &total);
    if (r < n) choff[r] = (uint64_t)(run + pre);
    run += total;
  }
  if (threadIdx.x == 0) choff[n] = (uint64_t)run;
}
__device__ __forceinline__ unsigned seg_row_of(const uint64_t *choff, unsigned n, uint64_t g) {
  unsigned lo = 0, hi = n;                     // last r with choff[r] <= g
  while (hi - lo > 1) {
    const unsigned mid = (lo + hi) >> 1;
    if (choff[mid] <= g) lo = mid; else hi = mid;
  }
  return lo;
}
template <int MODE>
__global__ __launch_bounds__(SP_T) void k_seg_csum(const uint64_t *ro, const uint32_t *col,
                                                   const double *a, const double *x,
                                                   const uint32_t *list, const unsigned *nl,
                                                   const uint64_t *choff, double *csum) {
  __shared__ double red[SP_T];
  const unsigned n = *nl;
  const uint64_t G = choff[n];
  for (uint64_t g = blockIdx.x; g < G; g += gridDim.x) {
    const unsigned r = seg_row_of(choff, n, g);
    const uint32_t i = list[r];
    const uint64_t lo = ro[i] + (g - choff[r]) * SEG_TILE, hi = min(ro[i + 1], lo + SEG_TILE);
    double t = 0;
    for (uint64_t k = lo + threadIdx.x; k < hi; k += SP_T) t += seg_product(a, x, col, k, MODE);
    red[threadIdx.x] = t;
    __syncthreads();
    for (int o = SP_T / 2; o > 0; o >>= 1) {
      if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) csum[g] = red[0];
    __syncthreads();
  }
}
// per row: chunk sums -> exclusive prefixes (a guess of the running sum; any order), one
// block per row scanning 256 chunks at a time (one thread walking a row's ~230 chunks
// serially took 25 us per call, 1.0 s of the anisotropic 256^3 setup)
__global__ __launch_bounds__(256) void k_seg_prefix(const unsigned *nl, const uint64_t *choff, double *csum) {
  __shared__ double wsum[4];
  const unsigned n = *nl;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (unsigned r = blockIdx.x; r < n; r += gridDim.x) {
    double carry = 0.0;
    for (uint64_t g0 = choff[r]; g0 < choff[r + 1]; g0 += 256) {
      const uint64_t g = g0 + threadIdx.x;
      const double v = g < choff[r + 1] ? csum[g] : 0.0;
      double x = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const double y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
      }
      if (lane == 63) wsum[w] = x;
      __syncthreads();
      double add = carry;
      for (int q = 0; q < w; q++) add += wsum[q];
      const double tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
      if (g < choff[r + 1]) csum[g] = add + x - v;
      __syncthreads();
      carry += tot;
    }
  }
}
template <int MODE>
__global__ __launch_bounds__(SP_T) void k_seg_spec(const uint64_t *ro, const uint32_t *col,
                                                   const double *a, const double *x,
                                                   const uint32_t *list, const unsigned *nl,
                                                   const uint64_t *choff, const double *approx,
                                                   SpecRec *rec, SegSplit *rec2) {
  __shared__ double tile[SEG_TILE];
  __shared__ long long ssum[SP_T / 64], smin[SP_T / 64], smax[SP_T / 64];
  __shared__ int sflag;
  __shared__ long long ssm[9];
  __shared__ int sj, sneed;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const unsigned n = *nl;
  const uint64_t G = choff[n];
  for (uint64_t g = blockIdx.x; g < G; g += gridDim.x) {
    const unsigned r = seg_row_of(choff, n, g);
    const uint32_t i = list[r];
    const uint64_t lo = ro[i] + (g - choff[r]) * SEG_TILE, hi = min(ro[i + 1], lo + SEG_TILE);
    const int tlen = (int)(hi - lo);
    for (int q = tid; q < tlen; q += SP_T) tile[q] = seg_product(a, x, col, lo + q, MODE);
    if (tid == 0) sflag = 0;
    __syncthreads();
    const double gs = approx[g];
    int flag = !(fabs(gs) >= 1e-290) || !(fabs(gs) < 1e300);
    const int e = flag ? 0 : ilogb(gs);
    const double u = ldexp(1.0, e - 52);
    long long loc = 0, lmin = 0x7fffffffffffffffll, lmax = -0x7fffffffffffffffll;
    const int first = tid * SEG_PER;
    for (int q = 0; q < SEG_PER; q++) {
      const int idx = first + q;
      if (idx >= tlen) break;
      const double v = tile[idx] / u;
      const double rr = rint(v);
      if (!(fabs(v) < 4.6e18) || fabs(rr - v) == 0.5) { flag = 1; break; }
      loc += (long long)rr;
      lmin = loc < lmin ? loc : lmin;
      lmax = loc > lmax ? loc : lmax;
    }
    if (flag) atomicOr(&sflag, 1);
    long long xs = loc;
    for (int o = 1; o < 64; o <<= 1) {
      const long long y = __shfl_up(xs, o, 64);
      if (lane >= o) xs += y;
    }
    const long long pre_w = xs - loc;
    long long mn = first < tlen ? pre_w + lmin : 0x7fffffffffffffffll;
    long long mx = first < tlen ? pre_w + lmax : -0x7fffffffffffffffll;
    for (int o = 32; o > 0; o >>= 1) {
      const long long m1 = __shfl_xor(mn, o, 64), m2 = __shfl_xor(mx, o, 64);
      mn = m1 < mn ? m1 : mn;
      mx = m2 > mx ? m2 : mx;
    }
    if (lane == 63) ssum[w] = xs;
    if (lane == 0) { smin[w] = mn; smax[w] = mx; }
    __syncthreads();
    if (tid == 0) {
      long long run = 0, gmn = 0x7fffffffffffffffll, gmx = -0x7fffffffffffffffll;
      for (int q = 0; q < SP_T / 64; q++) {
        if (smin[q] != 0x7fffffffffffffffll) {
          gmn = run + smin[q] < gmn ? run + smin[q] : gmn;
          gmx = run + smax[q] > gmx ? run + smax[q] : gmx;
        }
        run += ssum[q];
      }
      SpecRec rc;
      rc.M = run; rc.mn = gmn; rc.mx = gmx; rc.e = e; rc.flag = sflag;
      rec[g] = rc;
      // under the guess, would the whole-chunk record fail?  then a split record
      const bool gnormal = fabs(gs) >= 1e-290 && fabs(gs) < 1e300;
      const long long Sg = gnormal ? (long long)ldexp(gs, 52 - e) : 0;
      const long long LO = (1ll << 52), HI = (1ll << 53);
      const bool inside = !sflag && gnormal &&
                          (Sg > 0 ? (Sg + gmn > LO && Sg + gmx < HI) : (Sg + gmx < -LO && Sg + gmn > -HI));
      sneed = rec2 && !inside;
    }
    __syncthreads();
    if (sneed) seg_split<SEG_PER>(tile, tlen, gs, rec2 + g, ssm, &sj);
    else if (rec2 && tid == 0) rec2[g].ok = 0;
    __syncthreads();
  }
}
// one block per row: the run of passing chunks found by a block scan (k_dot_resolve),
// a failing chunk added by binade_range
template <int MODE>
__global__ __launch_bounds__(BN_THREADS) void k_seg_resolve(const uint64_t *ro, const uint32_t *col,
                                                            const double *a, const double *x,
                                                            const uint32_t *list, const unsigned *nl,
                                                            const uint64_t *choff, const SpecRec *rec,
                                                            const SegSplit *rec2, double *z) {
  __shared__ double tile[BN_TILE];
  __shared__ long long sh[BN_THREADS / 64 + 1];
  __shared__ double s_sh;
  __shared__ int viol_sh;
  const int tid = threadIdx.x;
  const long long LO = (1ll << 52), HI = (1ll << 53);
  const unsigned n = *nl;
  for (unsigned r = blockIdx.x; r < n; r += gridDim.x) {
    const uint32_t i = list[r];
    const uint64_t c0 = choff[r], c1 = choff[r + 1], k0 = ro[i], k1 = ro[i + 1];
    if (d_segstat_on && tid == 0) { atomicAdd(&d_segstat[0], 1ull); atomicAdd(&d_segstat[1], c1 - c0); }
    double s = 0.0;
    uint64_t c = c0;
    while (c < c1) {
      const uint64_t ce = min(c1, c + (uint64_t)BN_THREADS);
      const bool normal = fabs(s) >= 2.2250738585072014e-308 && fabs(s) < 1.0e300;
      const int e = normal ? ilogb(s) : 0;
      const long long S = normal ? (long long)ldexp(s, 52 - e) : 0ll;
      const uint64_t q = c + (uint64_t)tid;
      SpecRec rc;
      rc.M = 0; rc.mn = 0; rc.mx = 0; rc.e = 0; rc.flag = 1;
      if (q < ce) rc = rec[q];
      bool ok = q < ce && normal && !rc.flag && rc.e == e;
      long long total;
      const long long pre = bn_block_excl_scan(ok ? rc.M : 0ll, sh, &total);
      if (ok) {
        const long long base = (long long)((unsigned long long)S + (unsigned long long)pre);
        ok = S > 0 ? (base + rc.mn > LO && base + rc.mx < HI) : (base + rc.mx < -LO && base + rc.mn > -HI);
      }
      if (tid == 0) viol_sh = 0x7fffffff;
      __syncthreads();
      if (q < ce && !ok) atomicMin(&viol_sh, tid);
      __syncthreads();
      const int f = viol_sh;
      const uint64_t run_end = f == 0x7fffffff ? ce : c + (uint64_t)f;
      if (run_end > c && (uint64_t)tid == run_end - 1 - c)
        s_sh = ldexp((double)(long long)((unsigned long long)S + (unsigned long long)(pre + rc.M)), e - 52);
      __syncthreads();
      if (run_end > c) s = s_sh;
      __syncthreads();
      c = run_end;
      if (c < ce) {
        if (d_segstat_on && tid == 0) atomicAdd(&d_segstat[2], 1ull);
        // one crossing inside the chunk: its split record, O(1) (thread 0)
        if (tid == 0) {
          double s3;
          const bool okk = rec2 && seg_split_apply(rec2[c], s, &s3);
          viol_sh = okk ? 1 : 0;
          if (okk) s_sh = s3;
          if (okk && d_segstat_on) atomicAdd(&d_segstat[6], 1ull);
        }
        __syncthreads();
        const bool split_done = viol_sh == 1;
        if (split_done) s = s_sh;
        __syncthreads();
        if (!split_done) {
          const uint64_t lo = k0 + (c - c0) * SEG_TILE, hi = min(k1, lo + SEG_TILE);
          s = binade_range<MODE>(a, x, lo, hi, s, tile, sh, &s_sh, &viol_sh, col);
        }
        c++;
      }
    }
    if (tid == 0) z[i] = s;
    __syncthreads();
  }
}
// ---------------------------------------------------------------------------
// Wavefront resolution (round 6).  The walks above take one 1024-thread block per row (per
// dot): every step -- a batch of chunk records, or a round of binade_range inside a chunk
// that failed its speculation -- costs a block scan and four to six barriers of 16
// wavefronts.  On the anisotropic levels' orphan rows (~119 K entries, 29 chunks, 30 % of
// them failing: every strong entry is a jump of ~10^3 over the running sum, a binade
// crossing) that was 184 us per row and 7 s of the anisotropic 256^3 setup
// (AMGD_SEGSTAT: 40 753 rows, 1.18 M chunks, 350 K failed, 1.40 M rounds;
// profiles/r06/aniso256_kernel_stats_r06d.csv).  Here one wavefront walks a row: the
// records 64 at a time (a wave scan of the chunks' integer sums, the first failing chunk
// by ballot), and a failed chunk 64 products at a time: the products scaled to the
// running sum's binade grid u = 2^(e-52) and rounded (exact power-of-two scaling), a wave
// scan of the integers, the first step that leaves the binade (or is a tie / too large) by
// ballot; the steps before it are exact (fl(s + p) = s + RN_u(p) while the sum stays in
// the binade), that step is added the ordinary way.  The same arithmetic as binade_range
// and k_dot_resolve with wave-level scans instead of block-level ones: the sequential sum,
// bit for bit.
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long wave_incl_scan_u64(unsigned long long v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(v, o, 64);
    if (lane >= o) v += y;
  }
  return v;
}
// s + p_lo + ... + p_{hi-1} in order (products by prod(k)), one wavefront
template <typename Prod>
__device__ double wave_binade_range(Prod prod, uint64_t lo, uint64_t hi, double s, int lane) {
  const long long LO = (1ll << 52), HI = (1ll << 53);
  for (uint64_t base = lo; base < hi; base += 64) {
    const uint32_t nv = (uint32_t)min((uint64_t)64, hi - base);
    const bool valid = (uint32_t)lane < nv;
    const double p = valid ? prod(base + lane) : 0.0;
    uint32_t j = 0;
    while (j < nv) {                                       // uniform over the wavefront
      if (s == 0.0) {                                      // 0 + p == p: to the first nonzero p
        const unsigned long long nz = __ballot(valid && (uint32_t)lane >= j && p != 0.0);
        if (!nz) break;
        const uint32_t f = (uint32_t)(__ffsll((long long)nz) - 1);
        s = s + __shfl(p, (int)f, 64);
        j = f + 1;
        continue;
      }
      if (!(fabs(s) >= 2.2250738585072014e-308) || !(fabs(s) < 1.0e300)) {
        s = s + __shfl(p, (int)j, 64);                     // subnormal / huge / non-finite: one step
        j++;
        continue;
      }
      const int e = ilogb(s);
      const double u = ldexp(1.0, e - 52);
      const long long S0 = (long long)ldexp(s, 52 - e);
      const bool act = valid && (uint32_t)lane >= j;
      long long m = 0;
      bool bad = false;
      if (act) {
        const double xq = p / u;                           // exact: power-of-two scaling
        const double r = rint(xq);
        if (!(fabs(xq) < 4.6e18) || fabs(r - xq) == 0.5) bad = true;
        else m = (long long)r;
      }
      const long long run = (long long)((unsigned long long)S0 + wave_incl_scan_u64((unsigned long long)m, lane));
      const bool inside = S0 > 0 ? (run > LO && run < HI) : (run < -LO && run > -HI);
      const unsigned long long viol = __ballot(act && (bad || !inside));
      if (!viol) {
        s = ldexp((double)__shfl(run, (int)nv - 1, 64), e - 52);
        j = nv;
      } else {
        const uint32_t v = (uint32_t)(__ffsll((long long)viol) - 1);
        const long long pre = __shfl(run, (int)(v > 0 ? v - 1 : 0), 64);
        const double sc = v > j ? ldexp((double)pre, e - 52) : s;   // the exact prefix
        s = sc + __shfl(p, (int)v, 64);
        j = v + 1;
      }
    }
  }
  return s;
}
// records [c0, c1) of one sum: the runs of passing chunks (wave scan, ballot), a failing
// chunk added by wave_binade_range (chunk c covers products [k0 + (c - c0) * BN_TILE, ..))
template <typename Prod>
__device__ double wave_resolve(Prod prod, const SpecRec *rec, uint64_t c0, uint64_t c1, uint64_t k0, uint64_t k1,
                               int lane, uint64_t tile) {
  const long long LO = (1ll << 52), HI = (1ll << 53);
  double s = 0.0;
  uint64_t c = c0;
  while (c < c1) {
    const uint64_t ce = min(c1, c + 64);
    const bool normal = fabs(s) >= 2.2250738585072014e-308 && fabs(s) < 1.0e300;
    const int e = normal ? ilogb(s) : 0;
    const long long S = normal ? (long long)ldexp(s, 52 - e) : 0ll;
    const uint64_t q = c + (uint64_t)lane;
    SpecRec rc;
    rc.M = 0; rc.mn = 0; rc.mx = 0; rc.e = 0; rc.flag = 1;
    if (q < ce) rc = rec[q];
    bool ok = q < ce && normal && !rc.flag && rc.e == e;
    const long long mv = ok ? rc.M : 0ll;
    const unsigned long long inc = wave_incl_scan_u64((unsigned long long)mv, lane);
    if (ok) {
      const long long base = (long long)((unsigned long long)S + inc - (unsigned long long)mv);
      ok = S > 0 ? (base + rc.mn > LO && base + rc.mx < HI) : (base + rc.mx < -LO && base + rc.mn > -HI);
    }
    const unsigned long long fails = __ballot(q < ce && !ok);
    const uint64_t f = fails ? (uint64_t)(__ffsll((long long)fails) - 1) : ce - c;   // chunks c .. c+f-1 pass
    const long long tot = (long long)((unsigned long long)S + __shfl(inc, (int)(f > 0 ? f - 1 : 0), 64));
    if (f > 0) s = ldexp((double)tot, e - 52);
    c += f;
    if (c < ce) {
      if (d_segstat_on && lane == 0) atomicAdd(&d_segstat[2], 1ull);
      const uint64_t lo = k0 + (c - c0) * tile, hi = min(k1, lo + tile);
      s = wave_binade_range(prod, lo, hi, s, lane);
      c++;
    }
  }
  return s;
}
template <int MODE>
__global__ __launch_bounds__(256) void k_seg_resolve_w(const uint64_t *ro, const uint32_t *col, const double *a,
                                                       const double *x, const uint32_t *list, const unsigned *nl,
                                                       const uint64_t *choff, const SpecRec *rec, double *z) {
  const int lane = threadIdx.x & 63;
  const unsigned n = *nl;
  auto prod = [&](uint64_t k) { return seg_product(a, x, col, k, MODE); };
  for (uint64_t r = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < n;
       r += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
    const uint32_t i = list[r];
    const uint64_t c0 = choff[r], c1 = choff[r + 1];
    if (d_segstat_on && lane == 0) { atomicAdd(&d_segstat[0], 1ull); atomicAdd(&d_segstat[1], c1 - c0); }
    const double s = wave_resolve(prod, rec, c0, c1, ro[i], ro[i + 1], lane, SEG_TILE);
    if (lane == 0) z[i] = s;
  }
}
template <int MODE>
__global__ __launch_bounds__(64) void k_dot_resolve_w(const double *a, const double *b, uint64_t n,
                                                      const SpecRec *rec, double *out) {
  const int lane = threadIdx.x & 63;
  auto prod = [&](uint64_t i) { return bn_product(a, b, i, MODE); };
  const double s = wave_resolve(prod, rec, 0, (n + BN_TILE - 1) / BN_TILE, 0, n, lane, BN_TILE);
  if (lane == 0) *out = s;
}
// AMGD_RESOLVE=wave (A/B): the wavefront walks above instead of the block-per-sum ones.  Off
// by default: they are bit-identical but slower -- one wavefront's loads (a failed chunk's
// products 64 at a time, the records 64 at a time) wait their latency step by step where
// the block has all of a tile's loads in flight: configs[4] 29.1 -> 44.9 s, configs[1]
// 24.5 -> 25.3 s (profiles/r06/resolve_wave_r06j.txt)
static int g_resolve_wave = -1;
extern "C" void amgd_set_resolve_wave(int on) { g_resolve_wave = on; }
static bool resolve_wave() {
  if (g_resolve_wave < 0) { const char *e = getenv("AMGD_RESOLVE"); g_resolve_wave = e && e[0] == 'w'; }
  return g_resolve_wave > 0;
}
// max_entries: an upper bound on the listed rows' total length (the matrix's nnz),
// nmax on their count: sizes the chunk records
static void segstat_report() {
  unsigned long long h[10];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(d_segstat), sizeof h) != hipSuccess) return;
  fprintf(stderr, "segstat rows %llu chunks %llu failed %llu rounds %llu serial %llu zeroskip %llu split %llu"
          " dot_failed %llu dot_split %llu\n", h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8]);
}
static void segstat_init() {
  static int done = 0;
  if (done) return;
  done = 1;
  const char *e = getenv("AMGD_SEGSTAT");
  if (!(e && *e && atoi(e))) return;
  const int one = 1;
  HIPCK(hipMemcpyToSymbol(HIP_SYMBOL(d_segstat_on), &one, sizeof one));
  atexit(segstat_report);
}
static int g_seg_split = -1;   // AMGD_SEG_SPLIT=0 / amgd_set_seg_split(0): no split records
static bool seg_split_on() {
  if (g_seg_split < 0) { const char *e = getenv("AMGD_SEG_SPLIT"); g_seg_split = e && *e ? atoi(e) : 1; }
  return g_seg_split != 0;
}
extern "C" void amgd_set_seg_split(int on) { g_seg_split = on < 0 ? -1 : on; }
// the exact dots' split records (A/B): AMGD_DOT_SPLIT=0 / amgd_set_dot_split(0) turns them off
// there alone; AMGD_SEG_SPLIT=0 turns off both
static int g_dot_split = -1;
static bool dot_split_on() {
  if (g_dot_split < 0) { const char *e = getenv("AMGD_DOT_SPLIT"); g_dot_split = e && *e ? atoi(e) : 1; }
  return g_dot_split != 0 && seg_split_on();
}
extern "C" void amgd_set_dot_split(int on) { g_dot_split = on < 0 ? -1 : on; }
extern "C" void amgd_rows_exact(const uint64_t *ro, const uint32_t *col, const double *a,
                                const double *x, const uint32_t *list, const unsigned *nlist,
                                uint32_t nmax, uint64_t max_entries, double *z) {
  if (!nmax) return;
  segstat_init();
  hipStream_t st = amgd_s();
  const uint64_t gmax = max_entries / SEG_TILE + nmax + 1;
  uint64_t *choff = (uint64_t *)amgd_alloc(((size_t)nmax + 1) * 8);
  double *csum = (double *)amgd_alloc_f64(gmax * 8);
  SpecRec *rec = (SpecRec *)amgd_alloc(gmax * sizeof(SpecRec));
  SegSplit *rec2 = seg_split_on() ? (SegSplit *)amgd_alloc(gmax * sizeof(SegSplit)) : nullptr;
  const int G = (int)std::min<uint64_t>(gmax, 1024);
  const int R = (int)std::min<uint32_t>(nmax, 256);
  k_seg_prep<<<1, BN_THREADS, 0, st>>>(ro, list, nlist, choff);
  if (x) {
    k_seg_csum<3><<<G, SP_T, 0, st>>>(ro, col, a, x, list, nlist, choff, csum);
    k_seg_prefix<<<(int)std::min<uint32_t>(nmax, 1024), 256, 0, st>>>(nlist, choff, csum);
    k_seg_spec<3><<<G, SP_T, 0, st>>>(ro, col, a, x, list, nlist, choff, csum, rec, rec2);
    if (resolve_wave())
      k_seg_resolve_w<3><<<(R + 3) / 4, 256, 0, st>>>(ro, col, a, x, list, nlist, choff, rec, z);
    else
      k_seg_resolve<3><<<R, BN_THREADS, 0, st>>>(ro, col, a, x, list, nlist, choff, rec, rec2, z);
  } else {
    k_seg_csum<4><<<G, SP_T, 0, st>>>(ro, col, a, x, list, nlist, choff, csum);
    k_seg_prefix<<<(int)std::min<uint32_t>(nmax, 1024), 256, 0, st>>>(nlist, choff, csum);
    k_seg_spec<4><<<G, SP_T, 0, st>>>(ro, col, a, x, list, nlist, choff, csum, rec, rec2);
    if (resolve_wave())
      k_seg_resolve_w<4><<<(R + 3) / 4, 256, 0, st>>>(ro, col, a, x, list, nlist, choff, rec, z);
    else
      k_seg_resolve<4><<<R, BN_THREADS, 0, st>>>(ro, col, a, x, list, nlist, choff, rec, rec2, z);
  }
  KCHECK();
  amgd_free(choff); amgd_free(csum); amgd_free(rec);
  if (rec2) amgd_free(rec2);
}
// dots of fewer than g_sp_min chunks: one block's binade scan (k_dot_binade); longer ones the
// chunk speculation (AMGD_DOT_SPEC_MIN / amgd_set_dot_spec_min: the threshold in chunks, A/B)
static int g_sp_min = -1;
static uint64_t sp_min_n() {
  if (g_sp_min < 0) { const char *e = getenv("AMGD_DOT_SPEC_MIN"); g_sp_min = e && *e ? atoi(e) : 16; }
  return (uint64_t)g_sp_min * BN_TILE;
}
extern "C" void amgd_set_dot_spec_min(int chunks) { g_sp_min = chunks; }
template <int MODE>
static void dot_exact_launch(const double *a, const double *b, uint64_t n, double *out) {
  hipStream_t st = amgd_s();
  if (n < sp_min_n()) {
    k_dot_binade<MODE><<<1, BN_THREADS, 0, st>>>(a, b, n, out);
    return;
  }
  segstat_init();
  uint64_t G = (n + BN_TILE - 1) / BN_TILE;
  double *csum = (double *)amgd_alloc_f64(G * 8 + 8);
  SpecRec *rec = (SpecRec *)amgd_alloc(G * sizeof(SpecRec) + 64);
  int g = (int)std::min<uint64_t>(G, 8192);
  k_dot_csum<MODE><<<g, SP_T, 0, st>>>(a, b, n, csum);
  k_dot_approx_prefix<<<1, 1024, 0, st>>>(csum, G);
  // split records for the block walk (the wavefront walk does not read them)
  SegSplit *rec2 = dot_split_on() && !resolve_wave() ? (SegSplit *)amgd_alloc(G * sizeof(SegSplit) + 64) : nullptr;
  k_dot_spec<MODE><<<g, SP_T, 0, st>>>(a, b, n, csum, rec, rec2);
  if (resolve_wave()) k_dot_resolve_w<MODE><<<1, 64, 0, st>>>(a, b, n, rec, out);
  else k_dot_resolve<MODE><<<1, BN_THREADS, 0, st>>>(a, b, n, rec, rec2, out);
  amgd_free(csum);
  amgd_free(rec);
  if (rec2) amgd_free(rec2);
}

static int g_exact = -1;
static int g_seq_plain = 0;      // 1: plain one-lane sequential loop (test reference)
extern "C" void amgd_set_seq_plain(int on) { g_seq_plain = on; }
extern "C" void amgd_set_exact(int on) { g_exact = on ? 1 : 0; }
extern "C" int amgd_get_exact(void) {
  if (g_exact < 0) {
    const char *e = getenv("AMGD_FAST_DOTS");
    g_exact = (e && *e && *e != '0') ? 0 : 1;
  }
  return g_exact;
}
static double seq_finish() {
  double *p = red_buf();
  amgd_d2h(g_red_h, p + 2 * RED_BLOCKS, 8);
  return g_red_h[0];
}
extern "C" double amgd_dot(const double *a, const double *b, uint64_t n) {
  if (n == 0) return 0.0;
  if (amgd_get_exact()) {
    if (g_seq_plain) {
      if (b) k_dot_seq<0><<<1, 256, 0, amgd_s()>>>(a, b, n, red_buf() + 2 * RED_BLOCKS);
      else k_dot_seq<1><<<1, 256, 0, amgd_s()>>>(a, a, n, red_buf() + 2 * RED_BLOCKS);
    } else if (b) {
      dot_exact_launch<0>(a, b, n, red_buf() + 2 * RED_BLOCKS);
    } else {
      dot_exact_launch<1>(a, a, n, red_buf() + 2 * RED_BLOCKS);
    }
    return seq_finish();
  }
  int nb = red_grid(n);
  k_dot_partial<<<nb, RED_THREADS, 0, amgd_s()>>>(a, b, n, red_buf());
  return sum_finish(nb);
}
extern "C" double amgd_norm2(const double *a, uint64_t n) { return sqrt(amgd_dot(a, nullptr, n)); }
extern "C" double amgd_dot3(const double *M, const double *b, uint64_t n) {
  if (n == 0) return 0.0;
  if (amgd_get_exact()) {
    if (g_seq_plain) k_dot_seq<2><<<1, 256, 0, amgd_s()>>>(M, b, n, red_buf() + 2 * RED_BLOCKS);
    else dot_exact_launch<2>(M, b, n, red_buf() + 2 * RED_BLOCKS);
    return seq_finish();
  }
  int nb = red_grid(n);
  k_dot3_partial<<<nb, RED_THREADS, 0, amgd_s()>>>(M, b, n, red_buf());
  return sum_finish(nb);
}

// first argmax: larger value wins, ties -> smaller index (extr_op, amg_setup.c:3281)
struct VI { double v; uint64_t i; };
__device__ inline VI vi_best(VI a, VI b) {
  if (b.v > a.v || (b.v == a.v && b.i < a.i)) return b;
  return a;
}
__global__ void k_argmax_partial(const double *a, const uint64_t *ia, uint64_t n, double *pv,
                                 uint64_t *pi) {
  VI best{-DBL_MAX, ~0ull};
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    VI c{a[i], ia ? ia[i] : i};
    best = vi_best(best, c);
  }
  __shared__ double sv[RED_THREADS];
  __shared__ uint64_t si[RED_THREADS];
  sv[threadIdx.x] = best.v; si[threadIdx.x] = best.i;
  __syncthreads();
  for (int o = RED_THREADS / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      VI x{sv[threadIdx.x], si[threadIdx.x]}, y{sv[threadIdx.x + o], si[threadIdx.x + o]};
      VI r = vi_best(x, y);
      sv[threadIdx.x] = r.v; si[threadIdx.x] = r.i;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) { pv[blockIdx.x] = sv[0]; pi[blockIdx.x] = si[0]; }
}
extern "C" double amgd_max_first(const double *a, uint64_t n, uint64_t *idx) {
  if (n == 0) { if (idx) *idx = 0; return -DBL_MAX; }
  int nb = red_grid(n);
  double *p = red_buf();
  uint64_t *pi = (uint64_t *)(p + RED_BLOCKS);
  k_argmax_partial<<<nb, RED_THREADS, 0, amgd_s()>>>(a, nullptr, n, p, pi);
  k_argmax_partial<<<1, RED_THREADS, 0, amgd_s()>>>(p, pi, nb, p + 2 * RED_BLOCKS,
                                                    (uint64_t *)(p + 2 * RED_BLOCKS + 1));
  amgd_d2h(g_red_h, p + 2 * RED_BLOCKS, 16);
  uint64_t gi;
  memcpy(&gi, &g_red_h[1], 8);
  if (idx) *idx = gi;
  return g_red_h[0];
}

// the first argmax of a and the max of b (same length) with one host round trip
extern "C" double amgd_max_first2(const double *a, const double *b, uint64_t n, uint64_t *idx,
                                  double *maxb) {
  if (n == 0) { if (idx) *idx = 0; *maxb = -DBL_MAX; return -DBL_MAX; }
  int nb = red_grid(n);
  double *p = red_buf();
  uint64_t *pi = (uint64_t *)(p + RED_BLOCKS);
  for (int q = 0; q < 2; q++) {          // partials reused in stream order
    k_argmax_partial<<<nb, RED_THREADS, 0, amgd_s()>>>(q ? b : a, nullptr, n, p, pi);
    k_argmax_partial<<<1, RED_THREADS, 0, amgd_s()>>>(p, pi, nb, p + 2 * RED_BLOCKS + 2 * q,
                                                      (uint64_t *)(p + 2 * RED_BLOCKS + 2 * q + 1));
  }
  amgd_d2h(g_red_h, p + 2 * RED_BLOCKS, 32);
  uint64_t gi;
  memcpy(&gi, &g_red_h[1], 8);
  if (idx) *idx = gi;
  *maxb = g_red_h[2];
  return g_red_h[0];
}

__global__ void k_count_gt(const double *a, uint64_t n, double thr, double *pc, double *pm) {
  double c = 0.0, m = 0.0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    c += a[i] > thr ? 1.0 : 0.0;
    m = a[i] > m ? a[i] : m;
  }
  c = block_reduce(c, AddOp());
  struct MaxOp { __device__ double operator()(double x, double y) const { return x > y ? x : y; } };
  __syncthreads();
  m = block_reduce(m, MaxOp());
  if (threadIdx.x == 0) { pc[blockIdx.x] = c; pm[blockIdx.x] = m; }
}
extern "C" uint64_t amgd_count_gt(const double *a, uint64_t n, double thr, double *maxv) {
  if (n == 0) { if (maxv) *maxv = 0; return 0; }
  int nb = red_grid(n);
  double *p = red_buf();
  k_count_gt<<<nb, RED_THREADS, 0, amgd_s()>>>(a, n, thr, p, p + RED_BLOCKS);
  std::vector<double> hc(nb), hm(nb);
  HIPCK(hipMemcpyAsync(hc.data(), p, nb * 8, hipMemcpyDeviceToHost, amgd_s()));
  HIPCK(hipMemcpyAsync(hm.data(), p + RED_BLOCKS, nb * 8, hipMemcpyDeviceToHost, amgd_s()));
  HIPCK(hipStreamSynchronize(amgd_s()));
  double c = 0, m = 0;
  for (int i = 0; i < nb; i++) { c += hc[i]; m = hm[i] > m ? hm[i] : m; }
  if (maxv) *maxv = m;
  return (uint64_t)c;
}

// ||A - I||_F^2 over stored values, I subtracted at the first diagonal entry
__global__ void k_fro_rows(const uint64_t *ro, const uint32_t *col, const double *a, uint32_t rn,
                           double *part) {
  double s = 0.0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < rn; i += gridDim.x * blockDim.x) {
    bool done = false;
    for (uint64_t j = ro[i]; j < ro[i + 1]; j++) {
      double v = a[j];
      if (!done && col[j] == i) { v = v - 1.0; done = true; }
      s += v * v;
    }
  }
  s = block_reduce(s, AddOp());
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}
extern "C" double amgd_fro_minus_eye(const dcsr *A) {
  int nb = red_grid(A->rn);
  k_fro_rows<<<nb, RED_THREADS, 0, amgd_s()>>>(A->ro, A->col, A->a, A->rn, red_buf());
  return sum_finish(nb);
}

// release every device resource of the library (pool, scratch, events, stream);
// any device pointer handed out before is invalid afterwards
extern "C" void amgd_rt_shutdown(void) {
  if (!g_inited) return;
  HIPCK(hipStreamSynchronize(g_stream));
  for (auto &d : g_direct) (void)hipFree(d.first);
  g_direct.clear();
  g_used.clear();
  amgd_spmv_split_clear();
  g_free_off.clear();
  g_free_sz.clear();
  if (g_arena) (void)hipFree(g_arena);
  g_arena = nullptr;
  g_arena_sz = 0;
  g_arena_tried = false;
  g_inuse = 0;
  if (g_red) { (void)hipFree(g_red); g_red = nullptr; }
  if (g_red_h) { (void)hipHostFree(g_red_h); g_red_h = nullptr; }
  if (g_pub) { (void)hipHostFree(g_pub); g_pub = nullptr; g_pub_on = -1; }
  if (g_tinit) {
    std::vector<hipEvent_t> all(g_evpool);
    for (int i = 0; i < NTIMERS; i++) {
      for (auto &pr : g_pend[i]) { all.push_back(pr.first); all.push_back(pr.second); }
      g_pend[i].clear();
    }
    std::sort(all.begin(), all.end());
    all.erase(std::unique(all.begin(), all.end()), all.end());   // shared events once
    for (hipEvent_t e : all) (void)hipEventDestroy(e);
    g_evpool.clear();
    g_evshare.clear();
    g_tinit = false;
  }
  (void)hipStreamDestroy(g_stream);
  g_stream = nullptr;
  g_inited = false;
}
