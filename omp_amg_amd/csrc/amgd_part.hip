// amgd_part.hip -- row-partitioned matrices: halo exchange, distributed transpose,
// vector completion (amgd_part.h).
//
// Reference: the reference distributes a level's rows with the crystal router
// (amg_setup_aux, /root/reference/amg.c:399-468) and its serial setup (amg_setup.c)
// defines every value.  Here each rank keeps its row block of every matrix and the
// one-GPU kernels run unchanged on it: an operation that reads rows of another operand
// by global index (the B of a product, the A of the Q factors) gets those rows through
// pm_halo_rows; one whose output is a vector completes it with pm_allgather_vec.  Every
// row is produced by the same kernel from the same row data as on one GPU, so the
// partitioned hierarchy is bit-identical to the one-GPU (and the reference's) hierarchy.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "amgd.h"
#include "amgd_dev.h"
#include "amgd_part.h"

// ---------------------------------------------------------------------------
// partitions
// ---------------------------------------------------------------------------
extern "C" apart *apart_even(uint32_t n, int N) {
  apart *P = (apart *)calloc(1, sizeof(apart));
  P->N = N;
  P->n = n;
  P->split = (uint32_t *)malloc(sizeof(uint32_t) * (N + 1));
  for (int p = 0; p <= N; p++) P->split[p] = (uint32_t)(((uint64_t)n * p) / N);
  return P;
}
__global__ void k_range_count(const uint8_t *m, const uint32_t *split, unsigned long long *cnt) {
  const uint32_t a = split[blockIdx.x], b = split[blockIdx.x + 1];
  unsigned long long c = 0;
  for (uint32_t i = a + threadIdx.x; i < b; i += blockDim.x) c += m[i] ? 1 : 0;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
  __shared__ unsigned long long sh[4];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}
extern "C" apart *apart_induced(const apart *P, const uint8_t *mask) {
  const int N = P->N;
  uint32_t *ds = (uint32_t *)amgd_alloc(4ull * (N + 1) + 4);
  unsigned long long *dc = (unsigned long long *)amgd_alloc(8ull * N + 8);
  amgd_h2d(ds, P->split, 4ull * (N + 1));
  k_range_count<<<N, 256, 0, amgd_s()>>>(mask, ds, dc);
  KCHECK();
  std::vector<unsigned long long> c(N);
  amgd_d2h(c.data(), dc, 8ull * N);
  amgd_free(ds);
  amgd_free(dc);
  apart *Q = (apart *)calloc(1, sizeof(apart));
  Q->N = N;
  Q->split = (uint32_t *)malloc(sizeof(uint32_t) * (N + 1));
  Q->split[0] = 0;
  for (int p = 0; p < N; p++) Q->split[p + 1] = Q->split[p] + (uint32_t)c[p];
  Q->n = Q->split[N];
  return Q;
}
extern "C" void apart_free(apart **P) {
  if (!P || !*P) return;
  free((*P)->split);
  free(*P);
  *P = nullptr;
}

extern "C" pmat *pm_new(dcsr *m, const apart *rp, const apart *cp) {
  pmat *A = (pmat *)malloc(sizeof(pmat));
  A->m = m;
  A->rp = rp;
  A->cp = cp;
  return A;
}
extern "C" void pm_free(pmat **A) {
  if (!A || !*A) return;
  dcsr_free(&(*A)->m);
  free(*A);
  *A = nullptr;
}
extern "C" pmat *pm_copy(const pmat *A) { return pm_new(dcsr_copy(A->m), A->rp, A->cp); }

static inline uint32_t my_r0(const apart *P) { return P->split[amgd_pcomm_rank()]; }
__global__ void k_len_to_u64(const uint32_t *len, uint64_t n, uint64_t *o) { GRID_STRIDE(i, n) o[i] = len[i]; }

// ---------------------------------------------------------------------------
// vectors
// ---------------------------------------------------------------------------
extern "C" void pm_allgather_vec(void *v, size_t elem, const apart *P) {
  if (P->N == 1) return;
  std::vector<uint64_t> off(P->N + 1);
  for (int p = 0; p <= P->N; p++) off[p] = (uint64_t)P->split[p] * elem;
  void *b = v;
  amgd_allgatherv(1, &b, off.data());
}

// (row, value) of the listed rows this rank owns
__global__ void k_list_own(const uint32_t *list, uint32_t n, uint32_t lo, uint32_t hi, const double *z,
                           uint32_t *oi, double *ov, unsigned *cnt) {
  for (uint64_t r0 = (uint64_t)blockIdx.x * blockDim.x; r0 < n; r0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = r0 + threadIdx.x;
    const uint32_t i = r < n ? list[r] : 0u;
    const bool mine = r < n && i >= lo && i < hi;
    const unsigned p = wave_append(cnt, mine);
    if (mine) { oi[p] = i; ov[p] = z[i]; }
  }
}
__global__ void k_list_scatter(const uint32_t *oi, const double *ov, uint64_t n, double *z) {
  GRID_STRIDE(t, n) z[oi[t]] = ov[t];
}
// listed rows per owner rank, counted on every rank alike (every rank holds the same list
// content): the exchange needs no count round of its own
__global__ void k_owner_hist(const uint32_t *list, uint32_t n, const uint32_t *split, int N,
                             unsigned long long *cnt) {
  GRID_STRIDE(r, n) {
    const uint32_t i = list[r];
    int lo = 0, hi = N;                       // owner: split[p] <= i < split[p+1]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (split[mid] <= i) lo = mid;
      else hi = mid;
    }
    atomicAdd(&cnt[lo], 1ull);
  }
}
// Several lists at once (nv vectors, each with its list and partition): one allgatherv of
// (row, value) pairs for all of them.  The counts come from k_owner_hist on every rank.
extern "C" void pm_list_sync_n(int nv, double *const *z, const uint32_t *const *list, const uint32_t *n,
                               const apart *const *P) {
  const int N = P[0]->N, me = amgd_pcomm_rank();
  if (N == 1) return;
  hipStream_t s = amgd_s();
  std::vector<uint64_t> cnt((size_t)nv * N);
  {
    unsigned long long *dc = (unsigned long long *)amgd_alloc(8ull * nv * N + 8);
    uint32_t *dsp = (uint32_t *)amgd_alloc(4ull * nv * (N + 1) + 4);
    amgd_memset(dc, 0, 8ull * nv * N);
    for (int v = 0; v < nv; v++) {
      amgd_h2d(dsp + (size_t)v * (N + 1), P[v]->split, 4ull * (N + 1));
      if (n[v]) k_owner_hist<<<grid_for(n[v]), 256, 0, s>>>(list[v], n[v], dsp + (size_t)v * (N + 1), N,
                                                           dc + (size_t)v * N);
    }
    KCHECK();
    amgd_d2h(cnt.data(), dc, 8ull * nv * N);
    amgd_free(dc);
    amgd_free(dsp);
  }
  // buffers: per vector (ids, values); rank p's pairs of vector v at pre_v[p]
  std::vector<void *> bufs(2 * nv);
  std::vector<uint64_t> off((size_t)2 * nv * (N + 1));
  std::vector<uint64_t> tot(nv);
  std::vector<uint32_t *> oi(nv);
  std::vector<double *> ov(nv);
  unsigned *c = (unsigned *)amgd_alloc(8ull * nv + 8);
  amgd_memset(c, 0, 8ull * nv);
  for (int v = 0; v < nv; v++) {
    uint64_t t = 0;
    for (int p = 0; p < N; p++) {
      off[(size_t)(2 * v) * (N + 1) + p] = 4 * t;
      off[(size_t)(2 * v + 1) * (N + 1) + p] = 8 * t;
      t += cnt[(size_t)v * N + p];
    }
    off[(size_t)(2 * v) * (N + 1) + N] = 4 * t;
    off[(size_t)(2 * v + 1) * (N + 1) + N] = 8 * t;
    tot[v] = t;
    oi[v] = (uint32_t *)amgd_alloc(4 * t + 8);
    ov[v] = (double *)amgd_alloc_f64(8 * t + 8);
    bufs[2 * v] = oi[v];
    bufs[2 * v + 1] = ov[v];
    const uint64_t at = off[(size_t)(2 * v) * (N + 1) + me] / 4;
    if (n[v]) k_list_own<<<grid_for(n[v]), 256, 0, s>>>(list[v], n[v], P[v]->split[me], P[v]->split[me + 1], z[v],
                                                       oi[v] + at, ov[v] + at, c + v);
  }
  KCHECK();
  amgd_allgatherv(2 * nv, bufs.data(), off.data());
  for (int v = 0; v < nv; v++) {
    if (tot[v]) k_list_scatter<<<grid_for(tot[v]), 256, 0, s>>>(oi[v], ov[v], tot[v], z[v]);
    amgd_free(oi[v]);
    amgd_free(ov[v]);
  }
  KCHECK();
  amgd_free(c);
}
extern "C" void pm_list_sync(double *z, const uint32_t *list, uint32_t n, const apart *P) {
  pm_list_sync_n(1, &z, &list, &n, &P);
}

// Every rank's `bytes` (device, at mine) and one u64 `user` value to every rank, in rank
// order.  One collective when every rank's share fits the call site's eager slot: the
// share travels with its length in a fixed-size record; past it a second, exact round
// moves the rest.  After every call the site's slot is set to 5/4 of that call's largest
// share, within [4 KB, 1 MB] -- the same decision on every rank, since every rank sees
// every length; callers keep one state per recurring exchange (a BFS hop, an expansion
// step), whose share is like the previous sweep's.  N x 1 MB at most per record exchange
// (~20 us over xGMI at N = 8: comparable to the latency of the round it saves).
__global__ void k_eager_hdr(const uint64_t *rec, int N, uint64_t rs8, uint64_t *out) {
  const int p = threadIdx.x;
  if (p < N) { out[2 * p] = rec[p * rs8]; out[2 * p + 1] = rec[p * rs8 + 1]; }
}
static uint64_t g_eager_gen = 1;
static uint64_t g_eager_calls = 0, g_eager_second = 0;
extern "C" void pm_eager_new_setup(void) { g_eager_gen++; }
// AMGD_EAGER_SLOT=<bytes> / pm_eager_force_slot (tests): every call site's slot fixed at that
// size (>= 8), below the usual shares, so the exact second round runs on nearly every call
static int64_t g_eager_forced = -1;
extern "C" void pm_eager_force_slot(int64_t bytes) { g_eager_forced = bytes; }
static uint64_t eager_forced() {
  if (g_eager_forced < 0) {
    const char *e = getenv("AMGD_EAGER_SLOT");
    g_eager_forced = e && *e ? atoll(e) : 0;
  }
  return g_eager_forced > 0 ? (uint64_t)(g_eager_forced < 8 ? 8 : g_eager_forced) : 0;
}
extern "C" void pm_eager_stats(uint64_t *calls, uint64_t *second) { *calls = g_eager_calls; *second = g_eager_second; }
extern "C" char *pm_allgather_dyn(pm_eager *e, const void *mine, uint64_t bytes, uint64_t user, uint64_t *len,
                                  uint64_t *users, uint64_t *total) {
  // slots adapt within one setup only: a rank's earlier setups must not change its record
  // size in this one (all ranks start every partitioned setup from the same default)
  if (e->gen != g_eager_gen) { e->gen = g_eager_gen; e->slot = 0; }
  const int N = amgd_pcomm_size(), me = amgd_pcomm_rank();
  hipStream_t s = amgd_s();
  if (N == 1) {
    char *out = (char *)amgd_alloc(bytes + 8);
    if (bytes) HIPCK(hipMemcpyAsync(out, mine, bytes, hipMemcpyDeviceToDevice, s));
    len[0] = bytes; users[0] = user; *total = bytes;
    return out;
  }
  if (e->slot == 0) e->slot = 4096;
  if (eager_forced()) e->slot = eager_forced();
  g_eager_calls++;
  const uint64_t slot = (e->slot + 7) & ~7ull, rs = 16 + slot;       // record bytes
  char *rec = (char *)amgd_alloc((uint64_t)N * rs + 8);
  const uint64_t hdr[2] = {bytes, user};
  amgd_h2d(rec + (uint64_t)me * rs, hdr, 16);
  const uint64_t eb = bytes < slot ? bytes : slot;
  if (eb) HIPCK(hipMemcpyAsync(rec + (uint64_t)me * rs + 16, mine, eb, hipMemcpyDeviceToDevice, s));
  {
    std::vector<uint64_t> off(N + 1);
    for (int p = 0; p <= N; p++) off[p] = (uint64_t)p * rs;
    void *b = rec;
    amgd_allgatherv(1, &b, off.data());
  }
  std::vector<uint64_t> h(2 * N);
  {
    uint64_t *dh = (uint64_t *)amgd_alloc(16ull * N + 8);
    k_eager_hdr<<<1, 64 * ((N + 63) / 64), 0, s>>>((const uint64_t *)rec, N, rs / 8, dh);
    KCHECK();
    amgd_d2h(h.data(), dh, 16ull * N);
    amgd_free(dh);
  }
  std::vector<uint64_t> pre(N + 1, 0);
  uint64_t mx = 0, over = 0;
  for (int p = 0; p < N; p++) {
    len[p] = h[2 * p];
    users[p] = h[2 * p + 1];
    pre[p + 1] = pre[p] + len[p];
    mx = len[p] > mx ? len[p] : mx;
    over += len[p] > slot ? len[p] - slot : 0;
  }
  *total = pre[N];
  char *out = (char *)amgd_alloc(pre[N] + 8);
  for (int p = 0; p < N; p++) {
    const uint64_t c = len[p] < slot ? len[p] : slot;
    if (c) HIPCK(hipMemcpyAsync(out + pre[p], rec + (uint64_t)p * rs + 16, c, hipMemcpyDeviceToDevice, s));
  }
  amgd_free(rec);
  if (over) {                          // the rest of the long shares, exactly
    g_eager_second++;
    std::vector<uint64_t> ro(N + 1, 0);
    for (int p = 0; p < N; p++) ro[p + 1] = ro[p] + (len[p] > slot ? len[p] - slot : 0);
    char *rem = (char *)amgd_alloc(ro[N] + 8);
    if (bytes > slot)
      HIPCK(hipMemcpyAsync(rem + ro[me], (const char *)mine + slot, bytes - slot, hipMemcpyDeviceToDevice, s));
    void *b = rem;
    amgd_allgatherv(1, &b, ro.data());
    for (int p = 0; p < N; p++)
      if (len[p] > slot)
        HIPCK(hipMemcpyAsync(out + pre[p] + slot, rem + ro[p], len[p] - slot, hipMemcpyDeviceToDevice, s));
    amgd_free(rem);
  }
  {
    uint64_t ns = mx + mx / 4;
    e->slot = ns < 4096 ? 4096 : ns > (1u << 20) ? (1u << 20) : ns;
  }
  return out;
}

// ---------------------------------------------------------------------------
// global-row views
// ---------------------------------------------------------------------------
__global__ void k_gro_fill(const uint64_t *lro, uint32_t r0, uint32_t r1, uint32_t n, uint64_t nnz,
                           uint64_t *gro) {
  GRID_STRIDE(i, (uint64_t)n + 1) gro[i] = i <= r0 ? 0 : i >= r1 ? nnz : lro[i - r0];
}
extern "C" dcsr pm_gview(const pmat *A) {
  const uint32_t r0 = my_r0(A->rp), n = A->rp->n;
  dcsr g = *A->m;
  g.rn = n;
  g.ro = (uint64_t *)amgd_alloc(((size_t)n + 1) * 8);
  k_gro_fill<<<grid_for((uint64_t)n + 1), 256, 0, amgd_s()>>>(A->m->ro, r0, r0 + A->m->rn, n, A->m->nnz, g.ro);
  KCHECK();
  return g;
}
extern "C" void pm_gview_free(dcsr *g) {
  amgd_free(g->ro);
  g->ro = nullptr;
}
extern "C" dcsr *pm_localize(dcsr *G, uint32_t r0, uint32_t r1) {
  dcsr *L = (dcsr *)malloc(sizeof(dcsr));
  L->rn = r1 - r0;
  L->cn = G->cn;
  L->nnz = G->nnz;
  L->ro = (uint64_t *)amgd_alloc(((size_t)L->rn + 1) * 8);
  amgd_d2d(L->ro, G->ro + r0, ((size_t)L->rn + 1) * 8);    // rows < r0 are empty: starts at 0
  L->col = G->col;
  L->a = G->a;
  amgd_free(G->ro);
  free(G);
  return L;
}

// ---------------------------------------------------------------------------
// vector-valued row ops
// ---------------------------------------------------------------------------
extern "C" void pm_spmv(const pmat *M, const double *x, double *z, double alpha, const double *y,
                        double beta, const uint8_t *f) {
  const uint32_t r0 = my_r0(M->rp);
  amgd_spmv(M->m, x, z + r0, alpha, y ? y + r0 : nullptr, beta, f ? f + r0 : nullptr);
  pm_allgather_vec(z, 8, M->rp);
}
extern "C" void pm_spmvt(const pmat *Mt, const double *x, double *z) {
  amgd_spmvt(Mt->m, x, z + my_r0(Mt->rp));
  pm_allgather_vec(z, 8, Mt->rp);
}
extern "C" void pm_colsum(const pmat *Mt, double *z) {
  amgd_colsum(Mt->m, z + my_r0(Mt->rp));
  pm_allgather_vec(z, 8, Mt->rp);
}
extern "C" void pm_diag(const pmat *A, double *D) {
  dcsr g = pm_gview(A);             // the diagonal is found by global row index
  amgd_diag(&g, D);
  pm_gview_free(&g);
  pm_allgather_vec(D, 8, A->rp);
}
extern "C" void pm_rowsum_sq_inv(const pmat *A, double *s) {
  amgd_rowsum_sq_inv(A->m, s + my_r0(A->rp));
  pm_allgather_vec(s, 8, A->rp);
}
// ||A - I||_F^2: the per-rank partial sums added in rank order (the one-GPU value is a
// fixed-order tree sum as well; it only decides the Lanczos shortcut fro < 1e-11)
extern "C" double pm_fro_minus_eye(const pmat *A) {
  dcsr g = pm_gview(A);
  const double part = amgd_fro_minus_eye(&g);
  pm_gview_free(&g);
  const int N = A->rp->N, me = amgd_pcomm_rank();
  std::vector<uint64_t> v(N, 0);
  memcpy(&v[me], &part, 8);
  amgd_pcomm_allgather_u64(v.data(), 1);
  double s = 0;
  for (int p = 0; p < N; p++) { double d; memcpy(&d, &v[p], 8); s += d; }
  return s;
}

// ---------------------------------------------------------------------------
// matrix-valued row ops
// ---------------------------------------------------------------------------
extern "C" pmat *pm_mpm(double alpha, const pmat *A, double beta, const pmat *B) {
  return pm_new(amgd_mpm(alpha, A->m, beta, B->m), A->rp, A->cp);
}
extern "C" pmat *pm_mxmpoint(const pmat *A, const pmat *B) {
  return pm_new(amgd_mxmpoint(A->m, B->m), A->rp, A->cp);
}
extern "C" pmat *pm_drop_zeros(const pmat *A) { return pm_new(amgd_drop_zeros(A->m), A->rp, A->cp); }
extern "C" pmat *pm_rows_masked(const pmat *A, const uint8_t *mask) {
  return pm_new(amgd_rows_masked(A->m, mask + my_r0(A->rp)), A->rp, A->cp);
}
extern "C" pmat *pm_sub_mat(const pmat *A, const uint8_t *vr, const uint8_t *vc, const apart *rp_out,
                            const apart *cp_out) {
  return pm_new(amgd_sub_mat(A->m, vr + my_r0(A->rp), vc), rp_out, cp_out);
}
extern "C" void pm_diag_op(pmat *A, const double *D, int op) {
  dcsr g = pm_gview(A);
  amgd_diag_op(&g, D, op);
  pm_gview_free(&g);
}
extern "C" void pm_diag_op2(pmat *A, const double *Dl, const double *Dr, int op) {
  dcsr g = pm_gview(A);
  amgd_diag_op2(&g, Dl, Dr, op);
  pm_gview_free(&g);
}

// ---------------------------------------------------------------------------
// transpose: every rank transposes its rows (rows of A^T = all columns, entries in
// ascending local row = ascending global row), sends the rows of A^T that rank p owns
// to p, and p concatenates the pieces of each row in rank order -- ascending global row,
// the order of the one-GPU stable transpose (amg_setup.c:2000)
// ---------------------------------------------------------------------------
__global__ void k_row_lens_u32(const uint64_t *ro, uint32_t n, uint32_t *len) {
  GRID_STRIDE(i, n) len[i] = (uint32_t)(ro[i + 1] - ro[i]);
}
__global__ void k_sum_lens(const uint32_t *lens, int N, uint32_t n, uint64_t *cnt) {
  GRID_STRIDE(j, n) {
    uint64_t c = 0;
    for (int s = 0; s < N; s++) c += lens[(uint64_t)s * n + j];
    cnt[j] = c;
  }
}
// piece of source s: rows j with lens_s[j] entries at src (consecutive rows), placed after
// the pieces of the earlier sources (cur[j] = entries already placed in row j); one
// wavefront per row, lanes copying consecutive entries (coalesced for long rows)
__global__ void k_place_piece(const uint32_t *lens, const uint64_t *soff, uint32_t n, const uint32_t *scol,
                              const double *sa, uint32_t cadd, const uint64_t *ro, uint32_t *cur,
                              uint32_t *col, double *a) {
  const int lane = threadIdx.x & 63;
  for (uint64_t j = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; j < n;
       j += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
    const uint32_t l = lens[j];
    if (!l) continue;
    const uint64_t s0 = soff[j], d0 = ro[j] + cur[j];
    for (uint32_t t = lane; t < l; t += 64) { col[d0 + t] = scol[s0 + t] + cadd; a[d0 + t] = sa[s0 + t]; }
    if (lane == 0) cur[j] += l;
  }
}
static inline int wave_rows_grid(uint64_t n) { return grid_for(n * 64, 256, 65536); }
static void gather_at(const uint64_t *d, const uint32_t *idx, int n, uint64_t *out) {
  amgd_gather_u64_at(d, idx, n, out);
}
extern "C" pmat *pm_transpose(const pmat *A) {
  const apart *RP = A->rp, *CP = A->cp;
  const int N = RP->N, me = amgd_pcomm_rank();
  hipStream_t s = amgd_s();
  dcsr *T = amgd_transpose(A->m, nullptr);                // rows: all columns of A
  if (N == 1) {                     // one rank: the local transpose is the whole one
    T->cn = RP->n;
    return pm_new(T, CP, RP);
  }
  const uint32_t nc = CP->n, c0 = CP->split[me], c1 = CP->split[me + 1], nl = c1 - c0;
  // entry ranges of the pieces
  std::vector<uint64_t> tro(N + 1);
  gather_at(T->ro, CP->split, N + 1, tro.data());
  uint32_t *lens = (uint32_t *)amgd_alloc(4ull * nc + 8);
  if (nc) k_row_lens_u32<<<grid_for(nc), 256, 0, s>>>(T->ro, nc, lens);
  KCHECK();
  // 1. row lengths: rank p gets lens[c0_p .. c1_p) from every rank (nl_p per source)
  uint32_t *rlens = (uint32_t *)amgd_alloc(4ull * N * nl + 8);
  std::vector<uint64_t> so(N + 1), ro(N + 1);
  for (int p = 0; p <= N; p++) { so[p] = 4ull * CP->split[p]; ro[p] = 4ull * p * nl; }
  amgd_pcomm_alltoallv(lens, so.data(), rlens, ro.data());
  // 2. entries: counts of the pieces coming here
  std::vector<uint64_t> cnt((size_t)N * N, 0);
  for (int p = 0; p < N; p++) cnt[(size_t)me * N + p] = tro[p + 1] - tro[p];
  amgd_pcomm_allgather_u64(cnt.data(), N);
  std::vector<uint64_t> rpre(N + 1, 0);
  for (int q = 0; q < N; q++) rpre[q + 1] = rpre[q] + cnt[(size_t)q * N + me];
  const uint64_t nz = rpre[N];
  uint32_t *rcol = (uint32_t *)amgd_alloc(4 * nz + 8);
  double *ra = (double *)amgd_alloc_f64(8 * nz + 8);
  std::vector<uint64_t> s4(N + 1), r4(N + 1), s8(N + 1), r8(N + 1);
  for (int p = 0; p <= N; p++) {
    s4[p] = 4 * tro[p]; s8[p] = 8 * tro[p];
    r4[p] = 4 * rpre[p]; r8[p] = 8 * rpre[p];
  }
  {                                       // columns and values in one exchange
    const void *sb[2] = {T->col, T->a};
    const uint64_t *so2[2] = {s4.data(), s8.data()}, *ro2[2] = {r4.data(), r8.data()};
    void *rb[2] = {rcol, ra};
    amgd_pcomm_alltoallv_n(2, sb, so2, rb, ro2);
  }
  dcsr_free(&T);
  amgd_free(lens);
  // 3. assemble: row j = the pieces of ranks 0..N-1 in order
  dcsr *X = (dcsr *)malloc(sizeof(dcsr));
  X->rn = nl;
  X->cn = RP->n;
  X->nnz = nz;
  X->ro = (uint64_t *)amgd_alloc(((size_t)nl + 1) * 8);
  X->col = (uint32_t *)amgd_alloc(4 * nz + 8);
  X->a = (double *)amgd_alloc_f64(8 * nz + 8);
  if (nl) k_sum_lens<<<grid_for(nl), 256, 0, s>>>(rlens, N, nl, X->ro);
  KCHECK();
  amgd_scan_u64(X->ro, nl);
  uint32_t *cur = (uint32_t *)amgd_alloc(4ull * nl + 8);
  uint64_t *soff = (uint64_t *)amgd_alloc(8ull * nl + 16);
  amgd_memset(cur, 0, 4ull * nl);
  for (int q = 0; q < N && nl; q++) {
    if (rpre[q + 1] == rpre[q]) continue;
    // offsets of source q's rows inside its piece
    k_len_to_u64<<<grid_for(nl), 256, 0, s>>>(rlens + (size_t)q * nl, nl, soff);
    amgd_scan_u64(soff, nl);
    k_place_piece<<<wave_rows_grid(nl), 256, 0, s>>>(rlens + (size_t)q * nl, soff, nl, rcol + rpre[q], ra + rpre[q],
                                               RP->split[q], X->ro, cur, X->col, X->a);
    KCHECK();
  }
  amgd_free(cur); amgd_free(soff); amgd_free(rlens); amgd_free(rcol); amgd_free(ra);
  return pm_new(X, CP, RP);
}

// ---------------------------------------------------------------------------
// halo rows: B's rows referenced by the columns of L, next to B's own rows, in a
// global-row view (offsets for all B rows; rows neither own nor referenced are empty)
// ---------------------------------------------------------------------------
__global__ void k_mark_cols(const uint32_t *col, uint64_t nnz, uint8_t *mark) {
  GRID_STRIDE(k, nnz) mark[col[k]] = 1;
}
__global__ void k_unmark_range(uint8_t *mark, uint32_t lo, uint32_t hi) {
  GRID_STRIDE(i, (uint64_t)(hi - lo)) mark[lo + i] = 0;
}
__global__ void k_compact_marked(const uint8_t *mark, const uint32_t *rank, uint32_t n, uint32_t *list) {
  GRID_STRIDE(i, n) if (mark[i]) list[rank[i]] = (uint32_t)i;
}
// lower bound of each split point in the sorted list
__global__ void k_split_bounds(const uint32_t *list, uint32_t n, const uint32_t *split, int N, uint64_t *pos) {
  const int p = threadIdx.x;
  if (p > N) return;
  const uint32_t x = split[p];
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if (list[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  pos[p] = lo;
}
// owner side: lengths of the requested rows (global ids in the own range)
__global__ void k_req_lens(const uint32_t *req, uint64_t n, uint32_t r0, const uint64_t *ro, uint32_t *len) {
  GRID_STRIDE(t, n) {
    const uint32_t i = req[t] - r0;
    len[t] = (uint32_t)(ro[i + 1] - ro[i]);
  }
}
__global__ void k_req_copy(const uint32_t *req, uint64_t n, uint32_t r0, const uint64_t *ro,
                           const uint32_t *col, const double *a, const uint64_t *off, uint32_t *ocol, double *oa) {
  const int lane = threadIdx.x & 63;       // one wavefront per requested row
  for (uint64_t t = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; t < n;
       t += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
    const uint32_t i = req[t] - r0;
    const uint64_t k0 = ro[i], l = ro[i + 1] - k0, o = off[t];
    if (col) for (uint64_t q = lane; q < l; q += 64) ocol[o + q] = col[k0 + q];
    for (uint64_t q = lane; q < l; q += 64) oa[o + q] = a[k0 + q];
  }
}
// requester side: row lengths of the extended matrix
__global__ void k_ext_lens_own(const uint64_t *ro, uint32_t r0, uint32_t nl, uint64_t *len) {
  GRID_STRIDE(i, nl) len[r0 + i] = ro[i + 1] - ro[i];
}
__global__ void k_ext_lens_halo(const uint32_t *need, const uint32_t *hlen, uint64_t n, uint64_t *len) {
  GRID_STRIDE(t, n) len[need[t]] = hlen[t];
}
// Halo views that are B itself (one rank: no row is another rank's) alias B's arrays;
// pm_ext_free releases only their header.
#include <unordered_set>
static std::unordered_set<const dcsr *> g_views;
extern "C" int pm_ext_is_view(const dcsr *E) { return g_views.count(E) ? 1 : 0; }
extern "C" dcsr *pm_halo_rows(const pmat *B, const dcsr *L) {
  const apart *P = B->rp;
  const int N = P->N, me = amgd_pcomm_rank();
  const uint32_t n = P->n, r0 = P->split[me], r1 = P->split[me + 1], nl = r1 - r0;
  hipStream_t s = amgd_s();
  if (N == 1) {
    dcsr *E = (dcsr *)malloc(sizeof(dcsr));
    *E = *B->m;
    g_views.insert(E);
    return E;
  }
  // 1. the rows L references outside the own range, ascending
  uint8_t *mark = (uint8_t *)amgd_alloc((size_t)n + 8);
  uint32_t *rank = (uint32_t *)amgd_alloc(4ull * n + 8);
  amgd_memset(mark, 0, n);
  if (L->nnz) k_mark_cols<<<grid_for(L->nnz), 256, 0, s>>>(L->col, L->nnz, mark);
  if (nl) k_unmark_range<<<grid_for(nl), 256, 0, s>>>(mark, r0, r1);
  KCHECK();
  const uint32_t nneed = amgd_mask_rank(mark, n, rank);
  uint32_t *need = (uint32_t *)amgd_alloc(4ull * nneed + 8);
  if (n) k_compact_marked<<<grid_for(n), 256, 0, s>>>(mark, rank, n, need);
  KCHECK();
  amgd_free(mark);
  amgd_free(rank);
  std::vector<uint64_t> pos(N + 1);
  {
    uint32_t *ds = (uint32_t *)amgd_alloc(4ull * (N + 1) + 4);
    uint64_t *dp = (uint64_t *)amgd_alloc(8ull * (N + 1) + 8);
    amgd_h2d(ds, P->split, 4ull * (N + 1));
    k_split_bounds<<<1, 64 * ((N + 64) / 64), 0, s>>>(need, nneed, ds, N, dp);
    KCHECK();
    amgd_d2h(pos.data(), dp, 8ull * (N + 1));
    amgd_free(ds);
    amgd_free(dp);
  }
  // 2. request counts (rows) between every pair of ranks
  std::vector<uint64_t> cnt((size_t)N * N, 0);
  for (int p = 0; p < N; p++) cnt[(size_t)me * N + p] = pos[p + 1] - pos[p];
  amgd_pcomm_allgather_u64(cnt.data(), N);
  std::vector<uint64_t> qpre(N + 1, 0);                 // requests arriving here, by requester
  for (int q = 0; q < N; q++) qpre[q + 1] = qpre[q] + cnt[(size_t)q * N + me];
  const uint64_t nreq = qpre[N];
  uint32_t *req = (uint32_t *)amgd_alloc(4 * nreq + 8);
  std::vector<uint64_t> so(N + 1), ro(N + 1);
  for (int p = 0; p <= N; p++) { so[p] = 4 * pos[p]; ro[p] = 4 * qpre[p]; }
  amgd_pcomm_alltoallv(need, so.data(), req, ro.data());
  // 3. lengths of the requested rows back to the requesters
  const dcsr *Bm = B->m;
  uint32_t *rlen = (uint32_t *)amgd_alloc(4 * nreq + 8);
  if (nreq) k_req_lens<<<grid_for(nreq), 256, 0, s>>>(req, nreq, r0, Bm->ro, rlen);
  KCHECK();
  uint32_t *hlen = (uint32_t *)amgd_alloc(4ull * nneed + 8);
  amgd_pcomm_alltoallv(rlen, ro.data(), hlen, so.data());
  // 4. the rows themselves: send offsets from the requested lengths, receive offsets from
  //    the lengths that came back
  uint64_t *roff = (uint64_t *)amgd_alloc(8 * nreq + 16);
  if (nreq) k_len_to_u64<<<grid_for(nreq), 256, 0, s>>>(rlen, nreq, roff);
  const uint64_t nsend = amgd_scan_u64(roff, nreq);
  uint64_t *hoff = (uint64_t *)amgd_alloc(8ull * nneed + 16);
  if (nneed) k_len_to_u64<<<grid_for(nneed), 256, 0, s>>>(hlen, nneed, hoff);
  const uint64_t nhalo = amgd_scan_u64(hoff, nneed);
  std::vector<uint64_t> sb(N + 1), rb(N + 1);
  {
    std::vector<uint32_t> qi(N + 1), ni(N + 1);
    for (int p = 0; p <= N; p++) { qi[p] = (uint32_t)qpre[p]; ni[p] = (uint32_t)pos[p]; }
    gather_at(roff, qi.data(), N + 1, sb.data());
    gather_at(hoff, ni.data(), N + 1, rb.data());
  }
  const bool cols = Bm->col != nullptr;     // NULL: a values-only pseudo-matrix (Q factors)
  uint32_t *scol = cols ? (uint32_t *)amgd_alloc(4 * nsend + 8) : nullptr;
  double *sa = (double *)amgd_alloc_f64(8 * nsend + 8);
  if (nreq) k_req_copy<<<wave_rows_grid(nreq), 256, 0, s>>>(req, nreq, r0, Bm->ro, Bm->col, Bm->a, roff, scol, sa);
  KCHECK();
  // 5. the extended matrix: row offsets first, then the halo rows received straight into
  //    it -- the rows of the ranks below come before the own rows, those above after them,
  //    each rank's in ascending order (need is ascending), so the receive offsets are the
  //    halo offsets shifted past the own entries for the ranks above
  (void)nhalo;
  dcsr *E = (dcsr *)malloc(sizeof(dcsr));
  E->rn = n;
  E->cn = Bm->cn;
  E->ro = (uint64_t *)amgd_alloc(((size_t)n + 1) * 8);
  amgd_memset(E->ro, 0, ((size_t)n + 1) * 8);
  if (nl) k_ext_lens_own<<<grid_for(nl), 256, 0, s>>>(Bm->ro, r0, nl, E->ro);
  if (nneed) k_ext_lens_halo<<<grid_for(nneed), 256, 0, s>>>(need, hlen, nneed, E->ro);
  KCHECK();
  E->nnz = amgd_scan_u64(E->ro, n);
  const uint64_t ownnz = Bm->nnz;
  E->col = cols ? (uint32_t *)amgd_alloc(4 * E->nnz + 8) : nullptr;
  E->a = (double *)amgd_alloc_f64(8 * E->nnz + 8);
  std::vector<uint64_t> s4(N + 1), r4(N + 1), s8(N + 1), r8(N + 1);
  for (int p = 0; p <= N; p++) {
    const uint64_t at = rb[p] + (p > me ? ownnz : 0);
    s4[p] = 4 * sb[p]; s8[p] = 8 * sb[p]; r4[p] = 4 * at; r8[p] = 8 * at;
  }
  {                                       // values (and columns) in one exchange
    const void *sb[2] = {sa, scol};
    const uint64_t *so2[2] = {s8.data(), s4.data()}, *ro2[2] = {r8.data(), r4.data()};
    void *rb[2] = {E->a, E->col};
    amgd_pcomm_alltoallv_n(cols ? 2 : 1, sb, so2, rb, ro2);
  }
  amgd_free(req); amgd_free(rlen); amgd_free(roff); amgd_free(scol); amgd_free(sa);
  // the own rows: one contiguous block of B's arrays into one contiguous block of E's
  if (ownnz) {
    uint64_t at = 0;
    amgd_d2h(&at, E->ro + r0, 8);
    if (cols) HIPCK(hipMemcpyAsync(E->col + at, Bm->col, 4 * ownnz, hipMemcpyDeviceToDevice, s));
    HIPCK(hipMemcpyAsync(E->a + at, Bm->a, 8 * ownnz, hipMemcpyDeviceToDevice, s));
  }
  amgd_free(need); amgd_free(hlen); amgd_free(hoff);
  return E;
}
extern "C" void pm_ext_free(dcsr **E) {
  if (!E || !*E) return;
  if (g_views.erase(*E)) {
    free(*E);
    *E = nullptr;
    return;
  }
  dcsr_free(E);
}

extern "C" pmat *pm_spgemm(const pmat *A, const pmat *B, int pattern) {
  dcsr *E = pm_halo_rows(B, A->m);
  dcsr *X = pattern ? amgd_spgemm_pattern(A->m, E) : amgd_spgemm(A->m, E);
  pm_ext_free(&E);
  return pm_new(X, A->rp, B->cp);
}

// ---------------------------------------------------------------------------
// whole matrix on every rank (the partitioned interp_lmop falls back to it when the
// general walk is needed: that walk follows sp_add past the end of a row into the next
// rows, amg_setup.c:1665-1677, which may belong to another rank)
// ---------------------------------------------------------------------------
__global__ void k_ro_place(const uint64_t *lro, uint32_t nl, uint64_t base, uint64_t *dst) {
  GRID_STRIDE(i, nl) dst[i] = lro[i + 1] + base;
}
static dcsr *gather_rows(const pmat *A, bool vals) {
  const apart *P = A->rp;
  const int N = P->N, me = amgd_pcomm_rank();
  const bool cols = A->m->col != nullptr;     // NULL: a values-only pseudo-matrix (Q factors)
  std::vector<uint64_t> nz(N, 0);
  nz[me] = A->m->nnz;
  amgd_pcomm_allgather_u64(nz.data(), 1);
  std::vector<uint64_t> base(N + 1, 0);
  for (int p = 0; p < N; p++) base[p + 1] = base[p] + nz[p];
  dcsr *F = (dcsr *)malloc(sizeof(dcsr));
  F->rn = P->n; F->cn = A->m->cn; F->nnz = base[N];
  F->ro = (uint64_t *)amgd_alloc(((size_t)P->n + 1) * 8);
  F->col = cols ? (uint32_t *)amgd_alloc(base[N] * 4 + 4) : nullptr;
  F->a = vals ? (double *)amgd_alloc_f64(base[N] * 8 + 8) : nullptr;
  amgd_memset(F->ro, 0, 8);
  const uint32_t r0 = P->split[me], nl = A->m->rn;
  if (nl) k_ro_place<<<grid_for(nl), 256, 0, amgd_s()>>>(A->m->ro, nl, base[me], F->ro + r0 + 1);
  KCHECK();
  if (nz[me]) {
    if (cols) amgd_d2d(F->col + base[me], A->m->col, 4 * nz[me]);
    if (vals) amgd_d2d(F->a + base[me], A->m->a, 8 * nz[me]);
  }
  std::vector<uint64_t> off(3 * (N + 1));
  void *bufs[3];
  int nb = 0;
  auto add = [&](void *buf, uint64_t elem, bool rows) {
    for (int p = 0; p <= N; p++) off[nb * (N + 1) + p] = rows ? ((uint64_t)P->split[p] + 1) * 8 : base[p] * elem;
    bufs[nb++] = buf;
  };
  add(F->ro, 8, true);
  if (cols) add(F->col, 4, false);
  if (vals) add(F->a, 8, false);
  amgd_allgatherv(nb, bufs, off.data());
  return F;
}
extern "C" dcsr *pm_gather_full(const pmat *A) { return gather_rows(A, true); }
extern "C" dcsr *pm_gather_pattern(const pmat *A) { return gather_rows(A, false); }


// kpos[e] of W_skel entry e = (row i, column c): the position of i in support c (row c of
// the extended W_skel^T): the support is sorted, so a binary search (the one-GPU path reads
// the same number off the transpose's permutation)
__global__ void k_kpos_search(const uint64_t *ro, const uint32_t *col, uint32_t nl, uint32_t r0,
                              const uint64_t *tro, const uint32_t *tcol, uint32_t *kpos) {
  GRID_STRIDE(i, nl) {
    const uint32_t gi = r0 + (uint32_t)i;
    for (uint64_t e = ro[i]; e < ro[i + 1]; e++) {
      const uint32_t c = col[e];
      uint64_t lo = tro[c], hi = tro[c + 1];
      const uint64_t b = lo;
      while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (tcol[mid] < gi) lo = mid + 1;
        else hi = mid;
      }
      kpos[e] = (uint32_t)(lo - b);
    }
  }
}
extern "C" uint32_t *pm_kpos(const pmat *Wskel, const dcsr *WtE) {
  const dcsr *W = Wskel->m;
  uint32_t *kp = (uint32_t *)amgd_alloc(4 * W->nnz + 8);
  if (W->rn)
    k_kpos_search<<<grid_for(W->rn), 256, 0, amgd_s()>>>(W->ro, W->col, W->rn, my_r0(Wskel->rp), WtE->ro,
                                                         WtE->col, kp);
  KCHECK();
  return kp;
}

// entries (ri[t], cj[t]) of the own rows set to 0 (each is present: find_support's
// selections come from R' and R has the same entries)
__global__ void k_zero_entries(const uint64_t *ro, const uint32_t *col, double *a, uint32_t r0, uint32_t r1,
                               const uint32_t *ri, const uint32_t *cj, uint64_t n) {
  GRID_STRIDE(t, n) {
    const uint32_t i = ri[t];
    if (i < r0 || i >= r1) continue;
    uint64_t lo = ro[i - r0], hi = ro[i - r0 + 1];
    const uint32_t c = cj[t];
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (col[mid] < c) lo = mid + 1;
      else hi = mid;
    }
    if (lo < ro[i - r0 + 1] && col[lo] == c) a[lo] = 0.0;
  }
}
extern "C" void pm_zero_entries(pmat *M, const uint32_t *ri, const uint32_t *cj, uint64_t n) {
  const uint32_t r0 = my_r0(M->rp);
  if (n) k_zero_entries<<<grid_for(n), 256, 0, amgd_s()>>>(M->m->ro, M->m->col, M->m->a, r0, r0 + M->m->rn, ri,
                                                          cj, n);
  KCHECK();
}

// ordered row sums (from +0, left to right -- amgd_spmv_rows' sums) of the listed rows this
// rank owns, then every rank gets all of them
// (the one-GPU kernels on the global-row view: rows of other ranks are empty there and sum
// to +0, which pm_list_sync then overwrites with their owners' values)
// rows si of Rl and rows sj of Rt (find_support's re-sums after a selection) in one exchange
extern "C" void pm_list_rowsum2(const pmat *A, const uint32_t *la, double *oa, const pmat *B, const uint32_t *lb,
                                double *ob, uint32_t n) {
  const pmat *M[2] = {A, B};
  const uint32_t *L[2] = {la, lb};
  double *O[2] = {oa, ob};
  for (int q = 0; q < 2 && n; q++) {
    dcsr g = pm_gview(M[q]);
    amgd_list_rowsum(&g, L[q], n, O[q], M[q]->m->nnz > 32ull * M[q]->m->rn);
    pm_gview_free(&g);
  }
  const uint32_t nn[2] = {n, n};
  const apart *P[2] = {A->rp, B->rp};
  pm_list_sync_n(2, O, L, nn, P);
}
extern "C" void pm_list_rowsum(const pmat *M, const uint32_t *list, uint32_t n, double *out) {
  if (n) {
    dcsr g = pm_gview(M);
    amgd_list_rowsum(&g, list, n, out, M->m->nnz > 32ull * M->m->rn);
    pm_gview_free(&g);
  }
  pm_list_sync(out, list, n, M->rp);
}

// the entries of a whole COO (row ri, column cj, value 1; the same list on every rank)
// that fall in the own rows, as local rows (coo2csr: sorted, duplicates summed)
__global__ void k_own_coo(const uint32_t *ri, const uint32_t *cj, uint64_t n, uint32_t r0, uint32_t r1,
                          uint32_t *oi, uint32_t *oj, unsigned *cnt) {
  for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x; b < n; b += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t t = b + threadIdx.x;
    const bool mine = t < n && ri[t] >= r0 && ri[t] < r1;
    const unsigned p = wave_append(cnt, mine);
    if (mine) { oi[p] = ri[t] - r0; oj[p] = cj[t]; }
  }
}
__global__ void k_fill1(double *a, uint64_t n) { GRID_STRIDE(i, n) a[i] = 1.0; }
extern "C" pmat *pm_coo_ones(const uint32_t *ri, const uint32_t *cj, uint64_t n, const apart *rp,
                             const apart *cp) {
  const int me = amgd_pcomm_rank();
  const uint32_t r0 = rp->split[me], r1 = rp->split[me + 1];
  uint32_t *oi = (uint32_t *)amgd_alloc(4 * n + 8), *oj = (uint32_t *)amgd_alloc(4 * n + 8);
  unsigned *cnt = (unsigned *)amgd_alloc(8);
  amgd_memset(cnt, 0, 4);
  if (n) k_own_coo<<<grid_for(n), 256, 0, amgd_s()>>>(ri, cj, n, r0, r1, oi, oj, cnt);
  KCHECK();
  unsigned h = 0;
  amgd_d2h(&h, cnt, 4);
  double *ones = (double *)amgd_alloc_f64(8ull * h + 8);
  if (h) k_fill1<<<grid_for(h), 256, 0, amgd_s()>>>(ones, h);
  KCHECK();
  dcsr *X = amgd_coo2csr(h, oi, oj, ones, r1 - r0, cp->n, 1);
  amgd_free(oi); amgd_free(oj); amgd_free(cnt); amgd_free(ones);
  return pm_new(X, rp, cp);
}

// ---------------------------------------------------------------------------
// level-0 entries to the owners of their rows: a stable sort by owner rank (entries of
// one owner keep their order), one alltoallv per array; the receiver holds the pieces in
// source-rank order -- the order an allgatherv of every rank's entries would give, so
// duplicates are summed by build_csr / coo2csr in the same order
// ---------------------------------------------------------------------------
__global__ void k_owner_key(const uint32_t *I, uint64_t nz, const uint32_t *split, int N, uint32_t *key,
                            uint32_t *idx) {
  GRID_STRIDE(t, nz) {
    const uint32_t i = I[t];
    int lo = 0, hi = N;                   // last p with split[p] <= i
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (split[mid] <= i) lo = mid;
      else hi = mid;
    }
    key[t] = (uint32_t)lo;
    idx[t] = (uint32_t)t;
  }
}
template <typename T>
__global__ void k_permute(const T *src, const uint32_t *perm, uint64_t n, T *dst) {
  GRID_STRIDE(t, n) dst[t] = src[perm[t]];
}
__global__ void k_owner_bounds(const uint32_t *key, uint64_t n, int N, uint64_t *pos) {
  const int p = threadIdx.x;
  if (p > N) return;
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (key[mid] < (uint32_t)p) lo = mid + 1;
    else hi = mid;
  }
  pos[p] = lo;
}
extern "C" uint64_t pm_route_coo(uint64_t nz, const uint32_t *I, const uint32_t *J, const double *V,
                                 const apart *P, uint32_t **Io, uint32_t **Jo, double **Vo) {
  const int N = P->N, me = amgd_pcomm_rank();
  hipStream_t s = amgd_s();
  uint32_t *ds = (uint32_t *)amgd_alloc(4ull * (N + 1) + 4);
  amgd_h2d(ds, P->split, 4ull * (N + 1));
  uint32_t *key = (uint32_t *)amgd_alloc(4 * nz + 8), *idx = (uint32_t *)amgd_alloc(4 * nz + 8);
  uint32_t *key2 = (uint32_t *)amgd_alloc(4 * nz + 8), *perm = (uint32_t *)amgd_alloc(4 * nz + 8);
  std::vector<uint64_t> pos(N + 1, 0);
  if (nz) {
    k_owner_key<<<grid_for(nz), 256, 0, s>>>(I, nz, ds, N, key, idx);
    KCHECK();
    int eb = 1;
    while ((1 << eb) < N) eb++;
    size_t tb = 0;
    HIPCK(rocprim::radix_sort_pairs(nullptr, tb, key, key2, idx, perm, (size_t)nz, 0, eb, s));
    void *tmp = amgd_alloc(tb + 16);
    HIPCK(rocprim::radix_sort_pairs(tmp, tb, key, key2, idx, perm, (size_t)nz, 0, eb, s));
    amgd_free(tmp);
    uint64_t *dp = (uint64_t *)amgd_alloc(8ull * (N + 1) + 8);
    k_owner_bounds<<<1, 64 * ((N + 64) / 64), 0, s>>>(key2, nz, N, dp);
    KCHECK();
    amgd_d2h(pos.data(), dp, 8ull * (N + 1));
    amgd_free(dp);
  }
  uint32_t *sI = (uint32_t *)amgd_alloc(4 * nz + 8), *sJ = (uint32_t *)amgd_alloc(4 * nz + 8);
  double *sV = (double *)amgd_alloc_f64(8 * nz + 8);
  if (nz) {
    k_permute<uint32_t><<<grid_for(nz), 256, 0, s>>>(I, perm, nz, sI);
    k_permute<uint32_t><<<grid_for(nz), 256, 0, s>>>(J, perm, nz, sJ);
    k_permute<double><<<grid_for(nz), 256, 0, s>>>(V, perm, nz, sV);
    KCHECK();
  }
  amgd_free(ds); amgd_free(key); amgd_free(idx); amgd_free(key2); amgd_free(perm);
  std::vector<uint64_t> cnt((size_t)N * N, 0);
  for (int p = 0; p < N; p++) cnt[(size_t)me * N + p] = pos[p + 1] - pos[p];
  amgd_pcomm_allgather_u64(cnt.data(), N);
  std::vector<uint64_t> rp(N + 1, 0);
  for (int q = 0; q < N; q++) rp[q + 1] = rp[q] + cnt[(size_t)q * N + me];
  const uint64_t m = rp[N];
  *Io = (uint32_t *)amgd_alloc(4 * m + 8);
  *Jo = (uint32_t *)amgd_alloc(4 * m + 8);
  *Vo = (double *)amgd_alloc_f64(8 * m + 8);
  std::vector<uint64_t> s4(N + 1), r4(N + 1), s8(N + 1), r8(N + 1);
  for (int p = 0; p <= N; p++) { s4[p] = 4 * pos[p]; s8[p] = 8 * pos[p]; r4[p] = 4 * rp[p]; r8[p] = 8 * rp[p]; }
  amgd_pcomm_alltoallv(sI, s4.data(), *Io, r4.data());
  amgd_pcomm_alltoallv(sJ, s4.data(), *Jo, r4.data());
  amgd_pcomm_alltoallv(sV, s8.data(), *Vo, r8.data());
  amgd_free(sI); amgd_free(sJ); amgd_free(sV);
  return m;
}

// ---------------------------------------------------------------------------
// level-0 helpers of the partitioned build
// ---------------------------------------------------------------------------
__global__ void k_pmax_ij(const uint32_t *I, const uint32_t *J, uint64_t nz, unsigned *mx) {
  unsigned a = 0, b = 0;
  GRID_STRIDE(k, nz) {
    a = max(a, I[k] + 1);
    b = max(b, J[k] + 1);
  }
  atomicMax(&mx[0], a);
  atomicMax(&mx[1], b);
}
extern "C" void amgd_max_ij(uint64_t nz, const uint32_t *I, const uint32_t *J, uint32_t *mx) {
  unsigned *d = (unsigned *)amgd_alloc(16);
  amgd_memset(d, 0, 8);
  if (nz) k_pmax_ij<<<grid_for(nz), 256, 0, amgd_s()>>>(I, J, nz, d);
  KCHECK();
  amgd_d2h(mx, d, 8);
  amgd_free(d);
}
__global__ void k_vadd_u32(uint32_t *a, uint64_t n, uint32_t v) { GRID_STRIDE(i, n) a[i] += v; }
extern "C" void amgd_vadd_u32(uint32_t *a, uint64_t n, uint32_t v) {
  if (n) k_vadd_u32<<<grid_for(n), 256, 0, amgd_s()>>>(a, n, v);
  KCHECK();
}
__global__ void k_nonempty_rows(const uint64_t *ro, uint32_t rn, uint8_t *m) {
  GRID_STRIDE(i, rn) m[i] = ro[i + 1] != ro[i] ? 1 : 0;
}
extern "C" void amgd_nonempty_rows(const dcsr *T, uint8_t *out) {
  if (T->rn) k_nonempty_rows<<<grid_for(T->rn), 256, 0, amgd_s()>>>(T->ro, T->rn, out);
  KCHECK();
}
