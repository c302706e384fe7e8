// amgd_comm.hip -- row sharding of the heavy setup kernels over the GPUs of one node.
//
// Design (DESIGN.md "Multi-GPU"): every rank keeps the whole hierarchy of the level
// being built in its own HBM (256^3 peaks at ~108 GB of 288 GB) and runs the
// setup's control flow redundantly -- coarsening sweeps, reference-order dots,
// Lanczos, the find_support loop -- so every host decision is taken identically
// everywhere without a collective.  The work-heavy, row-independent kernels are
// sharded: the Gustavson SpGEMMs (RAP, Af*W, the constraint pattern), the
// per-coarse-point Q factors and their application.  Rows (or coarse points) are
// split into contiguous ranges of equal WORK (products, nz^3, nz^2), each rank
// computes its ranges straight into the global output buffer, and one in-place
// allgatherv over xGMI completes it on every rank.  Each output row is computed
// by the same kernel from the same inputs, so the assembled result is
// bit-identical to the one-GPU result -- the parity contract does not change.
//
// Transports:
//   RCCL  -- the node's xGMI mesh is point-to-point (a link to every peer), so the
//            allgatherv is one ncclGroup of direct send/recv pairs with every peer
//            on the library stream (all links busy at once), not a ring.  librccl
//            is dlopen'ed from ROCm at amgd_comm_init_rccl so the library itself
//            loads (and its symbols export) without it.
//   host  -- a caller-supplied allgatherv callback (tests: gloo between processes
//            sharing one GPU; RCCL refuses two ranks on one device).
//   sim   -- one process computes every shard in turn (no communication): checks
//            the range splitting and assembly on a single GPU.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

#include "amgd.h"
#include "amgd_dev.h"
#include "omp_amg_amd.h"

#define API __attribute__((visibility("default")))

enum { COMM_NONE = 0, COMM_RCCL = 1, COMM_HOST = 2, COMM_SIM = 3 };
static int g_kind = COMM_NONE, g_rank = 0, g_size = 1;
// partitioned mode (amgd_psetup.c): the ranks own row blocks of every matrix; the
// replicated-hierarchy sharding of the kernels below is switched off (amgd_nshards() = 1)
// and the partitioned ops exchange rows / vectors through amgd_pcomm_* directly.
// g_part: -1 not chosen (crs_setup with np > 1 then runs partitioned), 0 off (the
// round-2 replicated hierarchy), 1 on.  The sim transport is never partitioned.
static int g_part = -1, g_part_susp = 0;
static int part_on(void) { return g_part == 1 && g_kind != COMM_SIM; }
static amgd_allgatherv_fn g_cb = nullptr;
static void *g_user = nullptr;
static double g_min_scale = 1.0;      // work thresholds x this (0: shard everything)
static uint64_t g_bytes = 0, g_calls = 0;
// by kind: [0] allgatherv of data (vector segments, gathered rows), [1] alltoallv (halo rows,
// transposes, routed entries), [2] allgathers of a few u64 (counts, flags, maxima); calls, bytes
static uint64_t g_kstat[3][2];
static int g_kind_small = 0;
static int g_inner = 0;        // host-transport alltoallv staging: its allgathervs are not counted
// set for a scope, restored on every exit -- also when a peer's FAIL record unwinds the setup
// through amgd_throw_oom inside the scope (a stuck flag would stop counting collectives)
struct FlagScope {
  int &f, old;
  explicit FlagScope(int &flag) : f(flag), old(flag) { f = 1; }
  ~FlagScope() { f = old; }
};
static uint64_t g_seq = 0, g_guard_calls = 0;   // collective guard: records exchanged (below)
static double g_ms = 0;

// ---- RCCL entry points (dlopen'ed) ----
struct Rccl {
  void *h = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId *);
  ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int);
  ncclResult_t (*CommDestroy)(ncclComm_t);
  ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*GroupStart)();
  ncclResult_t (*GroupEnd)();
  const char *(*GetErrorString)(ncclResult_t);
};
static Rccl R;
static ncclComm_t g_nc = nullptr;

static int rccl_load() {
  if (R.h) return 0;
  const char *names[] = {"/opt/rocm/lib/librccl.so.1", "librccl.so.1", "librccl.so"};
  for (const char *n : names)
    if ((R.h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
  if (!R.h) {
    fprintf(stderr, "omp_amg_amd: cannot load librccl: %s\n", dlerror());
    return -1;
  }
#define SYM(f)                                                       \
  *(void **)&R.f = dlsym(R.h, "nccl" #f);                            \
  if (!R.f) {                                                        \
    fprintf(stderr, "omp_amg_amd: librccl lacks nccl%s\n", #f);      \
    dlclose(R.h);                                                    \
    R = Rccl();                 /* not loaded: the next call retries */ \
    return -1;                                                       \
  }
  SYM(GetUniqueId) SYM(CommInitRank) SYM(CommDestroy) SYM(Send) SYM(Recv) SYM(GroupStart)
  SYM(GroupEnd) SYM(GetErrorString)
#undef SYM
  return 0;
}
#define NCCK(x)                                                                         \
  do {                                                                                  \
    ncclResult_t r_ = (x);                                                              \
    if (r_ != ncclSuccess) {                                                            \
      fprintf(stderr, "omp_amg_amd: %s failed at %s:%d: %s\n", #x, __FILE__, __LINE__, \
              R.GetErrorString(r_));                                                    \
      abort();                                                                          \
    }                                                                                   \
  } while (0)

extern "C" API int amgd_comm_rccl_uid(unsigned char *uid) {
  if (rccl_load()) return -1;
  ncclUniqueId id;
  if (R.GetUniqueId(&id) != ncclSuccess) return -2;
  memcpy(uid, id.internal, NCCL_UNIQUE_ID_BYTES);
  return 0;
}

extern "C" API int amgd_comm_init_rccl(int rank, int size, const unsigned char *uid) {
  amgd_comm_free();
  if (size < 1 || rank < 0 || rank >= size) return -3;
  if (rccl_load()) return -1;
  amgd_s();                                   // HIP device / stream first
  ncclUniqueId id;
  memcpy(id.internal, uid, NCCL_UNIQUE_ID_BYTES);
  if (R.CommInitRank(&g_nc, size, id, rank) != ncclSuccess) return -2;
  g_kind = COMM_RCCL;
  g_rank = rank;
  g_size = size;
  return 0;
}

extern "C" API int amgd_comm_init_host(int rank, int size, amgd_allgatherv_fn fn, void *user) {
  amgd_comm_free();
  if (size < 1 || rank < 0 || rank >= size || !fn) return -3;
  g_kind = COMM_HOST;
  g_rank = rank;
  g_size = size;
  g_cb = fn;
  g_user = user;
  return 0;
}

extern "C" API int amgd_comm_init_sim(int nshards) {
  amgd_comm_free();
  if (nshards < 1) return -3;
  g_kind = nshards > 1 ? COMM_SIM : COMM_NONE;
  g_size = nshards;
  return 0;
}

extern "C" API void amgd_comm_free(void) {
  if (g_kind == COMM_RCCL && g_nc) {
    amgd_sync();
    R.CommDestroy(g_nc);
    g_nc = nullptr;
  }
  g_kind = COMM_NONE;
  g_rank = 0;
  g_size = 1;
  g_seq = 0;
  g_part = -1;
  g_cb = nullptr;
  g_user = nullptr;
}

extern "C" API int amgd_comm_size(void) { return g_size; }
extern "C" API void amgd_comm_set_partitioned(int on) { g_part = on ? 1 : 0; }
extern "C" API int amgd_comm_partitioned(void) { return part_on() && !g_part_susp; }
// crs_setup's choice for np > 1: partitioned unless amgd_comm_set_partitioned(0) was called
int amgd_comm_part_default(void) { return g_part != 0 && g_kind != COMM_SIM; }
int amgd_comm_part_get(void) { return g_part; }
void amgd_comm_part_set(int v) { g_part = v; }
extern "C" API int amgd_comm_rank(void) { return g_rank; }
extern "C" API void amgd_comm_set_min_work(double scale) { g_min_scale = scale < 0 ? 1.0 : scale; }
extern "C" API void amgd_comm_stats(uint64_t *calls, uint64_t *bytes, double *ms) {
  *calls = g_calls;
  *bytes = g_bytes;
  *ms = g_ms;
}
extern "C" API void amgd_comm_stats_reset(void) {
  g_calls = g_bytes = 0;
  g_ms = 0;
  memset(g_kstat, 0, sizeof g_kstat);
}
void amgd_comm_stats_kind(uint64_t *out6) { memcpy(out6, g_kstat, sizeof g_kstat); }

// ---- internal API (amgd.h) ----
int amgd_nshards(void) { return g_kind == COMM_NONE || part_on() ? 1 : g_size; }
// a partitioned setup running one operation on gathered (whole) data on every rank:
// the kernels see neither partitioning nor sharding meanwhile
void amgd_comm_suspend_partition(int on) { g_part_susp = on ? 1 : 0; }
int amgd_comm_procs(void) { return g_kind == COMM_RCCL || g_kind == COMM_HOST ? g_size : 1; }
void amgd_my_shards(int *first, int *last) {
  if (g_kind == COMM_SIM) { *first = 0; *last = g_size; }
  else { *first = g_rank; *last = g_rank + 1; }
}
int amgd_shard_worth(uint64_t work, uint64_t min_work) {
  if (amgd_nshards() <= 1) return 0;
  static double env = -1;
  if (env < 0) {
    const char *e = getenv("AMGD_SHARD_MIN");
    env = e && *e ? atof(e) : 1.0;
  }
  return (double)work >= (double)min_work * env * g_min_scale;
}


// ---------------------------------------------------------------------------
// Collective-consistency guard (AMGD_COMM_CHECK=1, amgd_comm_set_check).  Every rank must
// enter the same collectives in the same order with matching sizes; a rank-local branch
// that skips one (round 4's r04e fault) leaves gloo failing on a size check and RCCL
// hanging or corrupting memory.  With the guard on, every collective first exchanges one
// fixed-size record per rank over the raw transport:
//   [seq, kind, call-site line, call-site file hash, offsets signature, send lengths[N],
//    receive lengths[N]]
// and every rank checks all records: same seq / kind / site / signature everywhere, and
// for an alltoallv the bytes any rank q sends any rank p equal the bytes p expects from
// q.  Every rank sees every record, so all of them abort together, naming the sites.  A record of kind FAIL is a rank that ran out
// of HBM inside its setup: every rank then unwinds (amgd_oom_error) and returns the same
// error, instead of the failing rank aborting the job.
// ---------------------------------------------------------------------------
enum { GK_AGV = 1, GK_A2A = 2, GK_FAIL = 3 };
static int g_check = -1;
static const char *g_site_f = nullptr;
static int g_site_l = 0, g_depth = 0;
static uint64_t *g_grec_d = nullptr;          // device records: N x (5 + N) u64 (outside the arena)
static int g_grec_n = 0;
extern "C" void amgd_comm_site(const char *f, int l) {
  if (!g_depth) { g_site_f = f; g_site_l = l; }
}
struct SiteScope {          // the outermost collective owns the recorded site
  SiteScope() { g_depth++; }
  ~SiteScope() { if (--g_depth == 0) { g_site_f = nullptr; g_site_l = 0; } }
};
extern "C" API void amgd_comm_set_check(int on) { g_check = on < 0 ? -1 : on ? 1 : 0; }
static int check_on(void) {
  if (g_check < 0) {
    const char *e = getenv("AMGD_COMM_CHECK");
    g_check = e && *e && atoi(e) ? 1 : 0;
  }
  return g_check;
}
extern "C" API uint64_t amgd_comm_guard_calls(void) { return g_guard_calls; }
// AMGD_COMM_SITES=1: calls and bytes per call site and kind (the outermost caller's
// file:line), printed by amgd_comm_site_report -- where a setup's collectives come from
#include <map>
#include <string>
static int g_sites = -1;
static std::map<std::string, std::pair<uint64_t, uint64_t>> g_site_stats;
static void site_count(const char *kind, uint64_t bytes) {
  if (g_sites < 0) { const char *e = getenv("AMGD_COMM_SITES"); g_sites = e && *e && atoi(e) ? 1 : 0; }
  if (!g_sites) return;
  char k[256];
  const char *f = g_site_f ? strrchr(g_site_f, '/') : nullptr;
  snprintf(k, sizeof k, "%s:%d %s", f ? f + 1 : g_site_f ? g_site_f : "?", g_site_l, kind);
  auto &v = g_site_stats[k];
  v.first++;
  v.second += bytes;
}
void amgd_comm_site_report(void) {
  if (g_sites <= 0 || g_site_stats.empty()) return;
  std::vector<std::pair<uint64_t, std::string>> v;
  uint64_t tot = 0;
  for (auto &e : g_site_stats) { v.push_back({e.second.first, e.first}); tot += e.second.first; }
  std::sort(v.rbegin(), v.rend());
  fprintf(stderr, "rank %d collectives by call site: %lu in total\n", g_rank, (unsigned long)tot);
  for (auto &e : v)
    fprintf(stderr, "rank %d site %-40s %8lu calls %10.3f MB\n", g_rank, e.second.c_str(), (unsigned long)e.first,
            g_site_stats[e.second].second / 1e6);
  g_site_stats.clear();
}
static uint64_t fnv(const void *p, size_t n, uint64_t h = 1469598103934665603ull) {
  const unsigned char *c = (const unsigned char *)p;
  for (size_t i = 0; i < n; i++) h = (h ^ c[i]) * 1099511628211ull;
  return h;
}
static const char *gk_name(uint64_t k) {
  return k == GK_AGV ? "allgatherv" : k == GK_A2A ? "alltoallv" : k == GK_FAIL ? "FAIL" : "?";
}
// every rank's record to every rank (fixed size: cannot itself mismatch); out: N x RL
static void guard_exchange(const uint64_t *mine, int RL, std::vector<uint64_t> &all) {
  const int N = g_size;
  all.assign((size_t)N * RL, 0);
  if (!g_grec_d || g_grec_n < N * RL) {
    if (g_grec_d) (void)hipFree(g_grec_d);
    HIPCK(hipMalloc(&g_grec_d, 8ull * N * RL));
    g_grec_n = N * RL;
  }
  HIPCK(hipMemcpyAsync(g_grec_d + (size_t)g_rank * RL, mine, 8ull * RL, hipMemcpyHostToDevice, amgd_s()));
  if (g_kind == COMM_HOST) {
    amgd_sync();
    std::vector<uint64_t> off(N + 1);
    for (int q = 0; q <= N; q++) off[q] = 8ull * q * RL;
    void *b = g_grec_d;
    if (g_cb(g_user, 1, &b, off.data(), g_rank, N) != 0) {
      fprintf(stderr, "omp_amg_amd: host transport failed in the collective guard\n");
      abort();
    }
  } else {
    hipStream_t st = amgd_s();
    NCCK(R.GroupStart());
    for (int p = 0; p < N; p++) {
      if (p == g_rank) continue;
      NCCK(R.Send(g_grec_d + (size_t)g_rank * RL, 8ull * RL, ncclChar, p, g_nc, st));
      NCCK(R.Recv(g_grec_d + (size_t)p * RL, 8ull * RL, ncclChar, p, g_nc, st));
    }
    NCCK(R.GroupEnd());
  }
  HIPCK(hipMemcpyAsync(all.data(), g_grec_d, 8ull * N * RL, hipMemcpyDeviceToHost, amgd_s()));
  amgd_sync();
  g_guard_calls++;
}
extern "C" void amgd_throw_oom(void);   // amgd_rt.hip: unwind the setup (inside amgd_try), abort elsewhere
// kind, offsets signature; A2A: send[p] / recv[p] byte counts
static void guard(int kind, uint64_t sig, const uint64_t *sendl, const uint64_t *recvl) {
  const int N = g_size;
  if (!check_on() || N == 1 || (g_kind != COMM_RCCL && g_kind != COMM_HOST)) return;
  const int RL = 5 + 2 * N;
  std::vector<uint64_t> mine(RL, 0), all;
  mine[0] = g_seq++;
  mine[1] = (uint64_t)kind;
  mine[2] = (uint64_t)g_site_l;
  mine[3] = g_site_f ? fnv(g_site_f, strlen(g_site_f)) : 0;
  mine[4] = sig;
  if (sendl) for (int p = 0; p < N; p++) { mine[5 + p] = sendl[p]; mine[5 + N + p] = recvl[p]; }
  guard_exchange(mine.data(), RL, all);
  for (int q = 0; q < N; q++) {
    const uint64_t *r = all.data() + (size_t)q * RL;
    if (r[1] == GK_FAIL) {
      char msg[256];
      snprintf(msg, sizeof msg, "rank %d failed (out of HBM) at collective %lu; rank %d unwinds with it", q,
               (unsigned long)r[0], g_rank);
      amgd_set_error(msg);
      fprintf(stderr, "omp_amg_amd: %s\n", msg);
      if (kind != GK_FAIL) amgd_throw_oom();
      return;
    }
  }
  for (int q = 0; q < N; q++) {
    const uint64_t *r = all.data() + (size_t)q * RL;
    bool bad = r[0] != mine[0] || r[1] != mine[1] || r[2] != mine[2] || r[3] != mine[3] ||
               (kind == GK_AGV && r[4] != mine[4]);
    uint64_t got = 0, want = 0;
    int to = -1;
    for (int p = 0; p < N && !bad && kind == GK_A2A; p++) {   // q -> p: sent == expected
      const uint64_t *rp = all.data() + (size_t)p * RL;
      if (p != q && r[5 + p] != rp[5 + N + q]) {
        bad = true;
        got = r[5 + p];
        want = rp[5 + N + q];
        to = p;
      }
    }
    if (bad) {
      fprintf(stderr,
              "omp_amg_amd: COLLECTIVE MISMATCH: rank %d at %s:%d (seq %lu, %s) vs rank %d at line %lu "
              "(seq %lu, %s)%s",
              g_rank, g_site_f ? g_site_f : "?", g_site_l, (unsigned long)mine[0], gk_name(mine[1]), q,
              (unsigned long)r[2], (unsigned long)r[0], gk_name(r[1]),
              r[3] != mine[3] ? ", other file" : r[4] != mine[4] && kind == GK_AGV ? ", offsets differ" : "");
      if (to >= 0) fprintf(stderr, ": rank %d sends %lu bytes to rank %d, which expects %lu", q,
                           (unsigned long)got, to, (unsigned long)want);
      fprintf(stderr, "\n");
      abort();
    }
  }
}
// out of HBM on this rank inside a setup: with the guard on, tell every rank (they are
// in, or will enter, their next collective's record exchange) and unwind together
extern "C" int amgd_comm_fail_agree(void) {
  if (g_size <= 1 || (g_kind != COMM_RCCL && g_kind != COMM_HOST) || !check_on()) return 0;
  guard(GK_FAIL, 0, nullptr, nullptr);
  return 1;
}

// Range s of the shards holds bytes [off[b*(N+1)+s], off[b*(N+1)+s+1]) of buffer b;
// every rank holds its own ranges, after the call every rank holds all of them.
void amgd_allgatherv_(int nbuf, void *const *bufs, const uint64_t *off) {
  SiteScope site_;
  const int N = g_size;
  if (g_kind == COMM_NONE || g_kind == COMM_SIM || N == 1) return;
  guard(GK_AGV, fnv(off, 8ull * nbuf * (N + 1), (uint64_t)nbuf), nullptr, nullptr);
  double t0 = amgd_wtime();
  uint64_t nb = 0;
  for (int b = 0; b < nbuf; b++) nb += off[b * (N + 1) + N] - off[b * (N + 1)];
  if (!g_inner) {             // counted as the collective an RCCL run makes
    g_bytes += nb;
    g_calls++;
    site_count(g_kind_small ? "u64" : "allgatherv", nb);
    g_kstat[g_kind_small ? 2 : 0][0]++;
    g_kstat[g_kind_small ? 2 : 0][1] += nb;
  }
  if (g_kind == COMM_HOST) {
    amgd_sync();
    if (g_cb(g_user, nbuf, bufs, off, g_rank, N) != 0) {
      fprintf(stderr, "omp_amg_amd: host allgatherv callback failed\n");
      abort();
    }
  } else {
    hipStream_t s = amgd_s();
    NCCK(R.GroupStart());
    for (int b = 0; b < nbuf; b++) {
      const uint64_t *o = off + (size_t)b * (N + 1);
      char *base = (char *)bufs[b];
      const uint64_t mlen = o[g_rank + 1] - o[g_rank];
      for (int p = 0; p < N; p++) {
        if (p == g_rank) continue;
        const uint64_t plen = o[p + 1] - o[p];
        if (mlen) NCCK(R.Send(base + o[g_rank], mlen, ncclChar, p, g_nc, s));
        if (plen) NCCK(R.Recv(base + o[p], plen, ncclChar, p, g_nc, s));
      }
    }
    NCCK(R.GroupEnd());
    // no host sync: the send/recv pairs run on the library stream, so every consumer
    // (kernels, copies, frees of the arena) is ordered after them already.  So on RCCL
    // g_ms (amgd_comm_stats' ms) is the host's enqueue time only, not the transfer time;
    // with more than one rank this stream-ordered path is unverified until an 8-GPU run
  }
  g_ms += (amgd_wtime() - t0) * 1e3;
}

// split[s] = first item whose exclusive work prefix reaches s*total/N (s = 0..N):
// contiguous ranges of equal work; prefix = exclusive scan, n+1 entries
__global__ void k_shard_split(const uint64_t *prefix, uint32_t n, int N, uint32_t *split) {
  const int s = threadIdx.x;
  if (s > N) return;
  const uint64_t total = prefix[n];
  if (s == N) { split[s] = n; return; }
  const unsigned __int128 t = (unsigned __int128)total * (unsigned)s;
  const uint64_t target = (uint64_t)(t / (unsigned)N);
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if (prefix[mid] < target) lo = mid + 1;
    else hi = mid;
  }
  split[s] = s == 0 ? 0 : lo;
}
void amgd_shard_split(const uint64_t *prefix, uint32_t n, uint32_t *split_h) {
  const int N = amgd_nshards();
  uint32_t *d = (uint32_t *)amgd_alloc(4 * (N + 1) + 4);
  k_shard_split<<<1, 64 * ((N + 64) / 64), 0, amgd_s()>>>(prefix, n, N, d);
  KCHECK();
  amgd_d2h(split_h, d, 4 * (size_t)(N + 1));
  amgd_free(d);
}

// per-shard u64 values gathered to every rank (in-place on a device buffer)
void amgd_allgather_u64_(uint64_t *vals_h) {
  SiteScope site_;
  if (part_on()) {                               // partitioned mode: one value per process
    amgd_pcomm_allgather_u64(vals_h, 1);
    return;
  }
  const int N = amgd_nshards();
  int f, l;
  amgd_my_shards(&f, &l);
  uint64_t *d = (uint64_t *)amgd_alloc(8 * (size_t)N + 8);
  amgd_h2d(d + f, vals_h + f, 8 * (size_t)(l - f));
  std::vector<uint64_t> off(N + 1);
  for (int s = 0; s <= N; s++) off[s] = 8 * (uint64_t)s;
  void *b = d;
  amgd_allgatherv(1, &b, off.data());
  amgd_d2h(vals_h, d, 8 * (size_t)N);
  amgd_free(d);
}

// host values of a device u64 array at the given indices
__global__ void k_gather_u64(const uint64_t *a, const uint32_t *idx, int n, uint64_t *o) {
  const int t = threadIdx.x;
  if (t < n) o[t] = a[idx[t]];
}
void amgd_gather_u64_at(const uint64_t *a, const uint32_t *idx_h, int n, uint64_t *out_h) {
  uint32_t *di = (uint32_t *)amgd_alloc(4 * (size_t)n + 4);
  uint64_t *dv = (uint64_t *)amgd_alloc(8 * (size_t)n + 8);
  amgd_h2d(di, idx_h, 4 * (size_t)n);
  k_gather_u64<<<1, 64 * ((n + 63) / 64), 0, amgd_s()>>>(a, di, n, dv);
  KCHECK();
  amgd_d2h(out_h, dv, 8 * (size_t)n);
  amgd_free(di);
  amgd_free(dv);
}

// ---------------------------------------------------------------------------
// Partitioned-mode collectives (amgd_part.hip / amgd_psetup.c): every process is one
// rank (sim is not a partitioned transport).  Ranks own contiguous row blocks, so these
// move rows and vector segments, never whole matrices.
// ---------------------------------------------------------------------------
int amgd_pcomm_rank(void) { return g_kind == COMM_RCCL || g_kind == COMM_HOST ? g_rank : 0; }
int amgd_pcomm_size(void) { return g_kind == COMM_RCCL || g_kind == COMM_HOST ? g_size : 1; }

// vals_h[N * rank .. N * rank + m) of this rank -> every rank (m u64 per rank)
void amgd_pcomm_allgather_u64_(uint64_t *vals_h, int m) {
  SiteScope site_;
  const int N = amgd_pcomm_size(), me = amgd_pcomm_rank();
  if (N == 1) return;
  uint64_t *d = (uint64_t *)amgd_alloc(8ull * N * m + 8);
  amgd_h2d(d + (size_t)me * m, vals_h + (size_t)me * m, 8ull * m);
  std::vector<uint64_t> off(N + 1);
  for (int s = 0; s <= N; s++) off[s] = 8ull * s * m;
  void *b = d;
  {
    FlagScope small_(g_kind_small);
    amgd_allgatherv(1, &b, off.data());
  }
  amgd_d2h(vals_h, d, 8ull * N * m);
  amgd_free(d);
}

// Personalised exchange: this rank sends bytes [soff[p], soff[p+1]) of `send` to rank p
// and receives rank p's bytes for it into [roff[p], roff[p+1]) of `recv` (the counts of
// both sides must agree: callers exchange counts first).  RCCL: one group of send/recv
// pairs with every peer (each xGMI link carries its own pair).  Host transport: staged
// through the allgatherv callback (every rank sees every send buffer; tests only).
// host transport (tests, several ranks on one GPU): N-1 rounds; in round k every rank
// contributes its piece for rank (r + k) mod N to one allgatherv and takes the piece of
// rank (r - k) mod N -- staging per round ~1/N of the data, not all of it
static void a2a_host(const void *send, const uint64_t *soff, void *recv, const uint64_t *roff) {
  const int N = amgd_pcomm_size(), me = amgd_pcomm_rank();
  FlagScope inner_(g_inner);
  std::vector<uint64_t> so((size_t)N * (N + 1));
  uint64_t *dt = (uint64_t *)amgd_alloc(8ull * N * (N + 1) + 8);
  amgd_h2d(dt + (size_t)me * (N + 1), soff, 8ull * (N + 1));
  {
    std::vector<uint64_t> o(N + 1);
    for (int q = 0; q <= N; q++) o[q] = 8ull * q * (N + 1);
    void *b = dt;
    amgd_allgatherv(1, &b, o.data());
  }
  amgd_d2h(so.data(), dt, 8ull * N * (N + 1));
  amgd_free(dt);
  for (int k = 1; k < N; k++) {
    std::vector<uint64_t> base(N + 1, 0);
    for (int r = 0; r < N; r++) {
      const int d = (r + k) % N;
      const uint64_t *sr = so.data() + (size_t)r * (N + 1);
      base[r + 1] = base[r] + (sr[d + 1] - sr[d]);
    }
    if (base[N] == 0) continue;
    char *stage = (char *)amgd_alloc(base[N] + 16);
    const int dst = (me + k) % N, src = (me - k + N) % N;
    const uint64_t mine = soff[dst + 1] - soff[dst];
    if (mine) HIPCK(hipMemcpyAsync(stage + base[me], (const char *)send + soff[dst], mine,
                                   hipMemcpyDeviceToDevice, amgd_s()));
    {
      std::vector<uint64_t> o(base.begin(), base.end());
      void *b = stage;
      amgd_allgatherv(1, &b, o.data());
    }
    const uint64_t len = base[src + 1] - base[src];
    if (len != roff[src + 1] - roff[src]) {
      fprintf(stderr, "omp_amg_amd: alltoallv: rank %d expects %lu bytes from %d, which sends %lu\n", me,
              (unsigned long)(roff[src + 1] - roff[src]), src, (unsigned long)len);
      abort();
    }
    if (len) HIPCK(hipMemcpyAsync((char *)recv + roff[src], stage + base[src], len, hipMemcpyDeviceToDevice,
                                  amgd_s()));
    g_bytes += len;
    amgd_sync();
    amgd_free(stage);
  }
}

// nb personalised exchanges in one collective (RCCL: one group of send/recv pairs)
void amgd_pcomm_alltoallv_n_(int nb, const void *const *send, const uint64_t *const *soff, void *const *recv,
                             const uint64_t *const *roff) {
  SiteScope site_;
  const int N = amgd_pcomm_size(), me = amgd_pcomm_rank();
  for (int b = 0; b < nb && N > 1 && check_on(); b++) {
    std::vector<uint64_t> sl(N), rl(N);
    for (int p = 0; p < N; p++) { sl[p] = soff[b][p + 1] - soff[b][p]; rl[p] = roff[b][p + 1] - roff[b][p]; }
    guard(GK_A2A, 0, sl.data(), rl.data());
  }
  for (int b = 0; b < nb; b++) {
    const uint64_t own = soff[b][me + 1] - soff[b][me];
    if (own) HIPCK(hipMemcpyAsync((char *)recv[b] + roff[b][me], (const char *)send[b] + soff[b][me], own,
                                  hipMemcpyDeviceToDevice, amgd_s()));
  }
  if (N == 1) return;
  double t0 = amgd_wtime();
  g_calls++;
  uint64_t rb = 0;
  for (int b = 0; b < nb; b++)
    for (int p = 0; p < N; p++) if (p != me) rb += roff[b][p + 1] - roff[b][p];
  site_count("alltoallv", rb);
  g_kstat[1][0]++;
  g_kstat[1][1] += rb;
  if (g_kind == COMM_RCCL) {
    hipStream_t s = amgd_s();
    NCCK(R.GroupStart());
    for (int b = 0; b < nb; b++)
      for (int p = 0; p < N; p++) {
        if (p == me) continue;
        const uint64_t sl = soff[b][p + 1] - soff[b][p], rl = roff[b][p + 1] - roff[b][p];
        if (sl) NCCK(R.Send((const char *)send[b] + soff[b][p], sl, ncclChar, p, g_nc, s));
        if (rl) NCCK(R.Recv((char *)recv[b] + roff[b][p], rl, ncclChar, p, g_nc, s));
        g_bytes += rl;
      }
    NCCK(R.GroupEnd());          // stream-ordered like amgd_allgatherv: no host sync
  } else {
    for (int b = 0; b < nb; b++) a2a_host(send[b], soff[b], recv[b], roff[b]);
  }
  g_ms += (amgd_wtime() - t0) * 1e3;
}
void amgd_pcomm_alltoallv_(const void *send, const uint64_t *soff, void *recv, const uint64_t *roff) {
  amgd_pcomm_alltoallv_n_(1, &send, &soff, &recv, &roff);
}
