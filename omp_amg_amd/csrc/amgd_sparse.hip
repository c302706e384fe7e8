// amgd_sparse.hip -- CSR kernels for the MI355X AMG setup.
//
// Every kernel reproduces the reference's floating-point operation order
// (nicooff/omp_amg amg_setup.c / amg_tools.c) so that integer structure is
// bit-identical and values agree to the last bit wherever the reference's
// order is local to a row:
//   * SpMV (apply_M, amg_tools.c:76): each row summed left-to-right from +0.0;
//   * M^T x (apply_Mt, amg_tools.c:102): scattered in row order => per column
//     ascending rows, done here as an ordered gather over the transpose;
//   * SpGEMM (mxm, amg_setup.c:1894): X[i][j] accumulated over k ascending,
//     exact zeros dropped, columns ascending;
//   * mpm / mxmpoint (amg_setup.c:1684 / 1807): sorted merges, zero-drop rule.
// Compiled with -ffp-contract=off: no FMA contraction (the reference is ISO C).
#include <hip/hip_runtime.h>
#include <cfloat>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#include "amgd.h"
#include "amgd_dev.h"

static int bits_for(uint64_t v) {  // bits needed to represent v
  int b = 0;
  while (b < 64 && (v >> b) != 0) b++;
  return b < 1 ? 1 : b;
}

// ---------------------------------------------------------------------------
// generic helpers
// ---------------------------------------------------------------------------
__global__ void k_row_of_entry(const uint64_t *ro, uint32_t rn, uint32_t *row) {
  GRID_STRIDE(i, rn) {
    for (uint64_t k = ro[i]; k < ro[i + 1]; k++) row[k] = (uint32_t)i;
  }
}
// long rows: one wavefront per row (coalesced writes)
__global__ void k_row_of_entry_wave(const uint64_t *ro, uint32_t rn, uint32_t *row) {
  const int lane = threadIdx.x & 63;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < rn;
       i += ((uint64_t)gridDim.x * blockDim.x) >> 6)
    for (uint64_t k = ro[i] + lane; k < ro[i + 1]; k += 64) row[k] = (uint32_t)i;
}
#define WAVE_ROWS_MIN_MEAN 16   // mean row length from which per-row loops go wave-per-row
static inline bool long_rows(uint64_t nnz, uint32_t rn) {
  return rn && nnz >= (uint64_t)WAVE_ROWS_MIN_MEAN * rn;
}
static inline int wave_grid(uint32_t rn) { return grid_for((uint64_t)rn * 64, 256, 65536); }
__global__ void k_fill_u64(uint64_t *p, uint64_t n, uint64_t v) { GRID_STRIDE(i, n) p[i] = v; }
void amgd_row_of_entry_launch(const uint64_t *ro, uint32_t rn, uint32_t *row) {
  if (rn) k_row_of_entry<<<grid_for(rn), 256, 0, amgd_s()>>>(ro, rn, row);
}

// ---------------------------------------------------------------------------
// COO -> CSR, stable by (i, j): coo2csr (amg_setup.c:3684) sorts with the
// stable sarray_sort_2(i, j); here a stable LSD radix sort on the 64-bit key
// (i<<32 | j) carries the values.  Zero values (build_csr_dim drops them,
// amg_setup.c:3666) get the sentinel row rn and sort past the end.
// ---------------------------------------------------------------------------
__global__ void k_coo_keys(const uint32_t *I, const uint32_t *J, const double *V, uint64_t nz,
                           uint32_t rn, int drop_zero, uint64_t *key, uint64_t *cnt) {
  GRID_STRIDE(k, nz) {
    bool keep = !drop_zero || V[k] != 0.0;
    uint64_t r = keep ? I[k] : rn;
    key[k] = (r << 32) | (uint64_t)J[k];
    if (keep) atomicAdd((unsigned long long *)&cnt[I[k]], 1ull);
  }
}
__global__ void k_coo_split(const uint64_t *key, const double *vs, uint64_t nz, uint32_t *col,
                            double *a) {
  GRID_STRIDE(k, nz) {
    col[k] = (uint32_t)(key[k] & 0xffffffffull);
    a[k] = vs[k];
  }
}

extern "C" dcsr *amgd_coo2csr(uint64_t nz, const uint32_t *I, const uint32_t *J, const double *V,
                              uint32_t rn, uint32_t cn, int drop_zero) {
  hipStream_t s = amgd_s();
  uint64_t *cnt = (uint64_t *)amgd_alloc(((size_t)rn + 1) * 8);
  HIPCK(hipMemsetAsync(cnt, 0, ((size_t)rn + 1) * 8, s));
  uint64_t *key = (uint64_t *)amgd_alloc(nz * 8 + 8), *key2 = (uint64_t *)amgd_alloc(nz * 8 + 8);
  double *v2 = (double *)amgd_alloc_f64(nz * 8 + 8);
  if (nz) {
    k_coo_keys<<<grid_for(nz), 256, 0, s>>>(I, J, V, nz, rn, drop_zero, key, cnt);
    KCHECK();
    size_t tb = 0;
    int eb = 32 + bits_for(rn);
    HIPCK(rocprim::radix_sort_pairs(nullptr, tb, key, key2, V, v2, (size_t)nz, 0, eb, s));
    void *tmp = amgd_alloc(tb + 16);
    HIPCK(rocprim::radix_sort_pairs(tmp, tb, key, key2, V, v2, (size_t)nz, 0, eb, s));
    amgd_free(tmp);
  }
  uint64_t kept = amgd_scan_u64(cnt, rn);
  dcsr *A = (dcsr *)malloc(sizeof(dcsr));
  A->rn = rn; A->cn = cn; A->nnz = kept;
  A->ro = cnt;
  A->col = (uint32_t *)amgd_alloc(kept * 4 + 4);
  A->a = (double *)amgd_alloc_f64(kept * 8 + 8);
  if (kept) {
    k_coo_split<<<grid_for(kept), 256, 0, s>>>(key2, v2, kept, A->col, A->a);
    KCHECK();
  }
  amgd_free(key); amgd_free(key2); amgd_free(v2);
  return A;
}

// ---------------------------------------------------------------------------
// build_csr (amg_setup.c:3612): drop exact zeros, sort, then remove the empty
// rows and the same-index columns with sub_mat(A, nonempty, nonempty).
// ---------------------------------------------------------------------------
__global__ void k_max_ij(const uint32_t *I, const uint32_t *J, uint64_t nz, unsigned *mx) {
  unsigned a = 0, b = 0;
  GRID_STRIDE(k, nz) {
    a = max(a, I[k] + 1);
    b = max(b, J[k] + 1);
  }
  atomicMax(&mx[0], a);
  atomicMax(&mx[1], b);
}
__global__ void k_nonempty(const uint64_t *ro, uint32_t rn, uint32_t n, uint8_t *m) {
  GRID_STRIDE(i, n) m[i] = (i < rn && ro[i + 1] != ro[i]) ? 1 : 0;
}
extern "C" dcsr *amgd_build_csr(uint64_t nz, const uint32_t *Ai, const uint32_t *Aj,
                                const double *Av) {
  hipStream_t s = amgd_s();
  unsigned *mx = (unsigned *)amgd_alloc(8);
  HIPCK(hipMemsetAsync(mx, 0, 8, s));
  if (nz) k_max_ij<<<grid_for(nz), 256, 0, s>>>(Ai, Aj, nz, mx);
  unsigned hm[2];
  amgd_d2h(hm, mx, 8);
  amgd_free(mx);
  dcsr *T = amgd_coo2csr(nz, Ai, Aj, Av, hm[0], hm[1], 1);
  uint32_t n = std::max(hm[0], hm[1]);
  uint8_t *zr = (uint8_t *)amgd_alloc(n + 1);
  k_nonempty<<<grid_for(n), 256, 0, s>>>(T->ro, T->rn, n, zr);
  dcsr *A = amgd_sub_mat(T, zr, zr);
  amgd_free(zr);
  dcsr_free(&T);
  return A;
}

// ---------------------------------------------------------------------------
// sub_mat (amg_setup.c:3058)
// ---------------------------------------------------------------------------
__global__ void k_sub_count(const uint64_t *ro, const uint32_t *col, uint32_t rn, const uint8_t *vr,
                            const uint8_t *vc, const uint32_t *rmap, uint64_t *cnt) {
  GRID_STRIDE(i, rn) {
    if (!vr[i]) continue;
    uint64_t c = 0;
    for (uint64_t k = ro[i]; k < ro[i + 1]; k++) c += vc[col[k]] ? 1 : 0;
    cnt[rmap[i]] = c;
  }
}
__global__ void k_sub_fill(const uint64_t *ro, const uint32_t *col, const double *a, uint32_t rn,
                           const uint8_t *vr, const uint8_t *vc, const uint32_t *rmap,
                           const uint32_t *cmap, const uint64_t *sro, uint32_t *scol, double *sa) {
  GRID_STRIDE(i, rn) {
    if (!vr[i]) continue;
    uint64_t o = sro[rmap[i]];
    for (uint64_t k = ro[i]; k < ro[i + 1]; k++) {
      uint32_t c = col[k];
      if (vc[c]) { scol[o] = cmap[c]; sa[o] = a[k]; o++; }
    }
  }
}
// long rows: one wavefront per row -- the kept entries of a 64-entry chunk are
// placed by a ballot prefix, in order
__global__ void k_sub_count_wave(const uint64_t *ro, const uint32_t *col, uint32_t rn,
                                 const uint8_t *vr, const uint8_t *vc, const uint32_t *rmap,
                                 uint64_t *cnt) {
  const int lane = threadIdx.x & 63;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < rn;
       i += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
    if (!vr[i]) continue;
    uint64_t c = 0;
    for (uint64_t k0 = ro[i]; k0 < ro[i + 1]; k0 += 64) {
      const uint64_t k = k0 + lane;
      c += __popcll(__ballot(k < ro[i + 1] && vc[col[k]]));
    }
    if (lane == 0) cnt[rmap[i]] = c;
  }
}
__global__ void k_sub_fill_wave(const uint64_t *ro, const uint32_t *col, const double *a,
                                uint32_t rn, const uint8_t *vr, const uint8_t *vc,
                                const uint32_t *rmap, const uint32_t *cmap, const uint64_t *sro,
                                uint32_t *scol, double *sa) {
  const int lane = threadIdx.x & 63;
  const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < rn;
       i += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
    if (!vr[i]) continue;
    uint64_t o = sro[rmap[i]];
    for (uint64_t k0 = ro[i]; k0 < ro[i + 1]; k0 += 64) {
      const uint64_t k = k0 + lane;
      uint32_t c = 0;
      bool keep = false;
      if (k < ro[i + 1]) { c = col[k]; keep = vc[c] != 0; }
      const unsigned long long m = __ballot(keep);
      if (keep) {
        const uint64_t q = o + __popcll(m & below);
        scol[q] = cmap[c];
        sa[q] = a[k];
      }
      o += __popcll(m);
    }
  }
}
extern "C" dcsr *amgd_sub_mat(const dcsr *A, const uint8_t *vr, const uint8_t *vc) {
  hipStream_t s = amgd_s();
  uint32_t *rmap = (uint32_t *)amgd_alloc(((size_t)A->rn + 1) * 4);
  uint32_t *cmap = (uint32_t *)amgd_alloc(((size_t)A->cn + 1) * 4);
  uint32_t srn = amgd_mask_rank(vr, A->rn, rmap);
  uint32_t scn = amgd_mask_rank(vc, A->cn, cmap);
  uint64_t *cnt = (uint64_t *)amgd_alloc(((size_t)srn + 1) * 8);
  const bool lr = long_rows(A->nnz, A->rn);
  if (A->rn && lr)
    k_sub_count_wave<<<wave_grid(A->rn), 256, 0, s>>>(A->ro, A->col, A->rn, vr, vc, rmap, cnt);
  else if (A->rn)
    k_sub_count<<<grid_for(A->rn), 256, 0, s>>>(A->ro, A->col, A->rn, vr, vc, rmap, cnt);
  KCHECK();
  uint64_t nz = amgd_scan_u64(cnt, srn);
  dcsr *S = (dcsr *)malloc(sizeof(dcsr));
  S->rn = srn; S->cn = scn; S->nnz = nz; S->ro = cnt;
  S->col = (uint32_t *)amgd_alloc(nz * 4 + 4);
  S->a = (double *)amgd_alloc_f64(nz * 8 + 8);
  if (A->rn && lr)
    k_sub_fill_wave<<<wave_grid(A->rn), 256, 0, s>>>(A->ro, A->col, A->a, A->rn, vr, vc, rmap, cmap,
                                                      S->ro, S->col, S->a);
  else if (A->rn)
    k_sub_fill<<<grid_for(A->rn), 256, 0, s>>>(A->ro, A->col, A->a, A->rn, vr, vc, rmap, cmap,
                                                S->ro, S->col, S->a);
  KCHECK();
  amgd_free(rmap); amgd_free(cmap);
  return S;
}

// ---------------------------------------------------------------------------
// transpose (amg_setup.c:2000): sort by (j, i); a stable radix sort of the
// column keys over entries already in row order gives exactly that order.
// perm_out (optional) maps CSC position -> CSR position.
// ---------------------------------------------------------------------------
__global__ void k_iota_u64(uint64_t *p, uint64_t n) { GRID_STRIDE(i, n) p[i] = i; }
__global__ void k_iota_u32(uint32_t *p, uint64_t n) { GRID_STRIDE(i, n) p[i] = (uint32_t)i; }
// P = u64 (perm handed back to the caller) or u32 (nnz < 2^32, perm internal:
// a third less radix-sort traffic and a narrower perm read here)
// (four entries per thread per step: their perm loads, then all eight gathers, in flight
// together -- the gathers are the cost)
template <typename P>
__global__ void k_tr_fill(const P *perm, const uint32_t *row, const double *a, uint64_t nz,
                          uint32_t *tcol, double *ta) {
  const uint64_t S = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t0 < nz; t0 += 4 * S) {
    uint64_t p[4];
#pragma unroll
    for (int u = 0; u < 4; u++) p[u] = t0 + u * S < nz ? (uint64_t)perm[t0 + u * S] : 0;
    uint32_t r[4];
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      if (t0 + u * S < nz) { r[u] = row[p[u]]; v[u] = a[p[u]]; }
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      if (t0 + u * S < nz) { tcol[t0 + u * S] = r[u]; ta[t0 + u * S] = v[u]; }
    }
  }
}
// row offsets of the transpose from the sorted column keys: ro[c] = #keys < c, i.e.
// every c in (keys[t-1], keys[t]] starts at t (no atomics, no scan)
// (runs of more than RO_GAP empty columns are queued and filled block-wide)
#define RO_GAP 64
__global__ void k_ro_from_sorted(const uint32_t *keys, uint64_t nz, uint32_t cn, uint64_t *ro,
                                 unsigned *ngap, uint64_t *gaps) {
  GRID_STRIDE(t, nz + 1) {
    const uint64_t lo = t == 0 ? 0 : (uint64_t)keys[t - 1] + 1;
    const uint64_t hi = t == nz ? (uint64_t)cn : (uint64_t)keys[t];
    if (hi + 1 > lo + RO_GAP) {
      const unsigned g = atomicAdd(ngap, 1u);
      gaps[3 * (uint64_t)g] = lo;
      gaps[3 * (uint64_t)g + 1] = hi;
      gaps[3 * (uint64_t)g + 2] = t;
      continue;
    }
    for (uint64_t c = lo; c <= hi; c++) ro[c] = t;
  }
}
__global__ void k_ro_gaps(const unsigned *ngap, const uint64_t *gaps, uint64_t *ro) {
  const unsigned n = *ngap;
  for (unsigned g = blockIdx.x; g < n; g += gridDim.x) {
    const uint64_t lo = gaps[3 * (uint64_t)g], hi = gaps[3 * (uint64_t)g + 1],
                   t = gaps[3 * (uint64_t)g + 2];
    for (uint64_t c = lo + threadIdx.x; c <= hi; c += blockDim.x) ro[c] = t;
  }
}
extern "C" dcsr *amgd_transpose(const dcsr *A, uint64_t **perm_out) {
  hipStream_t s = amgd_s();
  uint64_t nz = A->nnz;
  const bool narrow = !perm_out && nz < (1ull << 32);
  uint64_t *cnt = (uint64_t *)amgd_alloc(((size_t)A->cn + 1) * 8);
  void *perm = amgd_alloc(nz * (narrow ? 4 : 8) + 8);
  if (!nz) HIPCK(hipMemsetAsync(cnt, 0, ((size_t)A->cn + 1) * 8, s));
  if (nz) {
    void *iota = amgd_alloc(nz * (narrow ? 4 : 8) + 8);
    uint32_t *kout = (uint32_t *)amgd_alloc(nz * 4 + 4);
    size_t tb = 0;
    int eb = bits_for(A->cn);
    void *tmp;
    if (narrow) {
      k_iota_u32<<<grid_for(nz), 256, 0, s>>>((uint32_t *)iota, nz);
      HIPCK(rocprim::radix_sort_pairs(nullptr, tb, A->col, kout, (uint32_t *)iota,
                                      (uint32_t *)perm, (size_t)nz, 0, eb, s));
      tmp = amgd_alloc(tb + 16);
      HIPCK(rocprim::radix_sort_pairs(tmp, tb, A->col, kout, (uint32_t *)iota, (uint32_t *)perm,
                                      (size_t)nz, 0, eb, s));
    } else {
      k_iota_u64<<<grid_for(nz), 256, 0, s>>>((uint64_t *)iota, nz);
      HIPCK(rocprim::radix_sort_pairs(nullptr, tb, A->col, kout, (uint64_t *)iota,
                                      (uint64_t *)perm, (size_t)nz, 0, eb, s));
      tmp = amgd_alloc(tb + 16);
      HIPCK(rocprim::radix_sort_pairs(tmp, tb, A->col, kout, (uint64_t *)iota, (uint64_t *)perm,
                                      (size_t)nz, 0, eb, s));
    }
    {
      // a run of > RO_GAP empty columns needs > RO_GAP columns: at most cn / RO_GAP + 1 runs
      const uint64_t maxg = (uint64_t)A->cn / RO_GAP + 2;
      uint64_t *gaps = (uint64_t *)amgd_alloc(maxg * 24 + 16);
      unsigned *ngap = (unsigned *)amgd_alloc(16);
      HIPCK(hipMemsetAsync(ngap, 0, 4, s));
      k_ro_from_sorted<<<grid_for(nz + 1), 256, 0, s>>>(kout, nz, A->cn, cnt, ngap, gaps);
      k_ro_gaps<<<1024, 256, 0, s>>>(ngap, gaps, cnt);
      KCHECK();
      amgd_free(gaps);
      amgd_free(ngap);
    }
    amgd_free(tmp); amgd_free(iota); amgd_free(kout);
  }
  dcsr *T = (dcsr *)malloc(sizeof(dcsr));
  T->rn = A->cn; T->cn = A->rn; T->nnz = nz; T->ro = cnt;
  T->col = (uint32_t *)amgd_alloc(nz * 4 + 4);
  T->a = (double *)amgd_alloc_f64(nz * 8 + 8);
  if (nz) {
    uint32_t *row = (uint32_t *)amgd_alloc(nz * 4 + 4);
    if (long_rows(nz, A->rn)) k_row_of_entry_wave<<<wave_grid(A->rn), 256, 0, s>>>(A->ro, A->rn, row);
    else k_row_of_entry<<<grid_for(A->rn), 256, 0, s>>>(A->ro, A->rn, row);
    if (narrow)
      k_tr_fill<uint32_t><<<grid_for((nz + 3) / 4, 256, 16384), 256, 0, s>>>((const uint32_t *)perm, row, A->a, nz,
                                                       T->col, T->a);
    else
      k_tr_fill<uint64_t><<<grid_for((nz + 3) / 4, 256, 16384), 256, 0, s>>>((const uint64_t *)perm, row, A->a, nz,
                                                       T->col, T->a);
    KCHECK();
    amgd_free(row);
  }
  if (perm_out) *perm_out = (uint64_t *)perm;
  else amgd_free(perm);
  return T;
}

// A without its exactly-zero entries (shape unchanged)
__global__ void k_nz_count(const uint64_t *ro, const double *a, uint32_t rn, uint64_t *cnt) {
  GRID_STRIDE(i, rn) {
    uint64_t c = 0;
    for (uint64_t k = ro[i]; k < ro[i + 1]; k++) c += a[k] != 0.0 ? 1 : 0;
    cnt[i] = c;
  }
}
__global__ void k_nz_fill(const uint64_t *ro, const uint32_t *col, const double *a, uint32_t rn,
                          const uint64_t *xro, uint32_t *xcol, double *xa) {
  GRID_STRIDE(i, rn) {
    uint64_t o = xro[i];
    for (uint64_t k = ro[i]; k < ro[i + 1]; k++)
      if (a[k] != 0.0) { xcol[o] = col[k]; xa[o] = a[k]; o++; }
  }
}
extern "C" dcsr *amgd_drop_zeros(const dcsr *A) {
  hipStream_t s = amgd_s();
  uint64_t *cnt = (uint64_t *)amgd_alloc(((size_t)A->rn + 1) * 8);
  if (A->rn) k_nz_count<<<grid_for(A->rn), 256, 0, s>>>(A->ro, A->a, A->rn, cnt);
  const uint64_t nz = amgd_scan_u64(cnt, A->rn);
  dcsr *X = (dcsr *)malloc(sizeof(dcsr));
  X->rn = A->rn; X->cn = A->cn; X->nnz = nz; X->ro = cnt;
  X->col = (uint32_t *)amgd_alloc(nz * 4 + 4);
  X->a = (double *)amgd_alloc_f64(nz * 8 + 8);
  if (A->rn && nz) k_nz_fill<<<grid_for(A->rn), 256, 0, s>>>(A->ro, A->col, A->a, A->rn, X->ro, X->col, X->a);
  KCHECK();
  return X;
}

// rows of A kept where mask != 0, the others emptied (shape unchanged)
__global__ void k_rowmask_count(const uint64_t *ro, uint32_t rn, const uint8_t *m, uint64_t *cnt) {
  GRID_STRIDE(i, rn) cnt[i] = m[i] ? ro[i + 1] - ro[i] : 0;
}
__global__ void k_rowmask_fill(const uint64_t *ro, const uint32_t *col, const double *a, uint32_t rn,
                               const uint8_t *m, const uint64_t *xro, uint32_t *xcol, double *xa) {
  GRID_STRIDE(i, rn) {
    if (!m[i]) continue;
    uint64_t o = xro[i];
    for (uint64_t k = ro[i]; k < ro[i + 1]; k++, o++) { xcol[o] = col[k]; xa[o] = a[k]; }
  }
}
__global__ void k_rowmask_fill_wave(const uint64_t *ro, const uint32_t *col, const double *a,
                                    uint32_t rn, const uint8_t *m, const uint64_t *xro,
                                    uint32_t *xcol, double *xa) {
  const int lane = threadIdx.x & 63;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < rn;
       i += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
    if (!m[i]) continue;
    const uint64_t k0 = ro[i], o = xro[i], n = ro[i + 1] - k0;
    for (uint64_t t = lane; t < n; t += 64) { xcol[o + t] = col[k0 + t]; xa[o + t] = a[k0 + t]; }
  }
}
extern "C" dcsr *amgd_rows_masked(const dcsr *A, const uint8_t *mask) {
  hipStream_t s = amgd_s();
  uint64_t *cnt = (uint64_t *)amgd_alloc(((size_t)A->rn + 1) * 8);
  if (A->rn) k_rowmask_count<<<grid_for(A->rn), 256, 0, s>>>(A->ro, A->rn, mask, cnt);
  uint64_t nz = amgd_scan_u64(cnt, A->rn);
  dcsr *X = (dcsr *)malloc(sizeof(dcsr));
  X->rn = A->rn; X->cn = A->cn; X->nnz = nz; X->ro = cnt;
  X->col = (uint32_t *)amgd_alloc(nz * 4 + 4);
  X->a = (double *)amgd_alloc_f64(nz * 8 + 8);
  if (A->rn && nz && long_rows(A->nnz, A->rn))
    k_rowmask_fill_wave<<<wave_grid(A->rn), 256, 0, s>>>(A->ro, A->col, A->a, A->rn, mask, X->ro,
                                                          X->col, X->a);
  else if (A->rn && nz)
    k_rowmask_fill<<<grid_for(A->rn), 256, 0, s>>>(A->ro, A->col, A->a, A->rn, mask, X->ro, X->col, X->a);
  KCHECK();
  return X;
}

// inverse of a permutation of 0..n-1: q[p[t]] = t
__global__ void k_perm_inv(const uint64_t *p, uint64_t n, uint64_t *q) { GRID_STRIDE(t, n) q[p[t]] = t; }
extern "C" uint64_t *amgd_perm_inverse(const uint64_t *p, uint64_t n) {
  uint64_t *q = (uint64_t *)amgd_alloc(n * 8 + 8);
  if (n) k_perm_inv<<<grid_for(n), 256, 0, amgd_s()>>>(p, n, q);
  KCHECK();
  return q;
}
// entries of A kept where mask[col] != 0 (shape unchanged, order within rows kept):
// the transpose of rows_masked(B, mask) is cols_masked(B', mask), without a sort
__global__ void k_colmask_count(const uint64_t *ro, const uint32_t *col, uint32_t rn,
                                const uint8_t *m, uint64_t *cnt) {
  const int lane = threadIdx.x & 63;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < rn;
       i += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
    uint64_t c = 0;
    for (uint64_t k = ro[i] + lane; k < ro[i + 1]; k += 64) c += m[col[k]] ? 1 : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if (lane == 0) cnt[i] = c;
  }
}
__global__ void k_colmask_fill(const uint64_t *ro, const uint32_t *col, const double *a, uint32_t rn,
                               const uint8_t *m, const uint64_t *xro, uint32_t *xcol, double *xa) {
  const int lane = threadIdx.x & 63;
  const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < rn;
       i += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
    uint64_t o = xro[i];
    const uint64_t k1 = ro[i + 1];
    for (uint64_t k0 = ro[i]; k0 < k1; k0 += 64) {       // uniform trip count per wave
      const uint64_t k = k0 + lane;
      const bool keep = k < k1 && m[col[k]];
      const unsigned long long b = __ballot(keep);
      if (keep) {
        const uint64_t p = o + (uint64_t)__popcll(b & below);
        xcol[p] = col[k];
        xa[p] = a[k];
      }
      o += (uint64_t)__popcll(b);
    }
  }
}
extern "C" dcsr *amgd_cols_masked(const dcsr *A, const uint8_t *mask) {
  hipStream_t s = amgd_s();
  uint64_t *cnt = (uint64_t *)amgd_alloc(((size_t)A->rn + 1) * 8);
  if (A->rn) k_colmask_count<<<wave_grid(A->rn), 256, 0, s>>>(A->ro, A->col, A->rn, mask, cnt);
  uint64_t nz = amgd_scan_u64(cnt, A->rn);
  dcsr *X = (dcsr *)malloc(sizeof(dcsr));
  X->rn = A->rn; X->cn = A->cn; X->nnz = nz; X->ro = cnt;
  X->col = (uint32_t *)amgd_alloc(nz * 4 + 4);
  X->a = (double *)amgd_alloc_f64(nz * 8 + 8);
  if (A->rn && nz)
    k_colmask_fill<<<wave_grid(A->rn), 256, 0, s>>>(A->ro, A->col, A->a, A->rn, mask, X->ro, X->col, X->a);
  KCHECK();
  return X;
}

// ---------------------------------------------------------------------------
// SpMV: t_i = sum_j a_ij x_col(j), left to right from +0.0 (apply_M).
// CSR-stream: a 256-thread block owns 256 consecutive rows and walks their
// nnz range in LDS-sized chunks: all threads compute the products of a chunk
// with coalesced loads of (col, a), then each thread adds the part of its own
// row inside the chunk, in order.  Chunks are visited in order, so every row
// sum is the reference's left-to-right sum whatever the row lengths.
// ---------------------------------------------------------------------------
#define SPMV_ROWS 256
#define SPMV_CH 4096
__global__ __launch_bounds__(256) void k_spmv(const uint64_t *ro, const uint32_t *col,
                                              const double *a, uint32_t rn, const double *x,
                                              double *z, double alpha, const double *y,
                                              double beta, const uint8_t *f,
                                              const uint32_t *fs = nullptr, uint32_t fb = 0,
                                              uint32_t fr = 0) {
  __shared__ double pv[SPMV_CH];
  const int tid = threadIdx.x;
  for (uint64_t r0 = (uint64_t)blockIdx.x * SPMV_ROWS; r0 < rn;
       r0 += (uint64_t)gridDim.x * SPMV_ROWS) {
    const uint64_t r1 = min((uint64_t)rn, r0 + SPMV_ROWS);
    const uint64_t i = r0 + tid;
    const bool own = i < r1;
    // row filter (incremental coarsening): a block with no row within fr hops
    // of the last sweep's changes skips; the others recompute every row
    // (identical arithmetic, so clean rows are rewritten with their own values)
    if (fs && !__syncthreads_or(own && fs[i] - fb <= fr)) continue;
    const uint64_t b0 = ro[r0], b1 = ro[r1];
    const uint64_t k0 = own ? ro[i] : 0, k1 = own ? ro[i + 1] : 0;
    double t = 0;
    for (uint64_t c0 = b0; c0 < b1; c0 += SPMV_CH) {
      const uint64_t c1 = min(b1, c0 + SPMV_CH);
      // eight (value, column) loads, then eight gathers, in flight per thread
      for (uint64_t kb = c0 + tid; kb < c1; kb += 256 * 8) {
        double av[8];
        uint32_t cv[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const uint64_t k = kb + 256 * u;
          av[u] = 0.0;
          cv[u] = 0;
          if (k < c1) {
            av[u] = a[k];
            if (x) cv[u] = col[k];
          }
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const uint64_t k = kb + 256 * u;
          if (k < c1) pv[k - c0] = x ? av[u] * x[cv[u]] : av[u];
        }
      }
      __syncthreads();
      const uint64_t lo = max(k0, c0), hi = min(k1, c1);
#pragma unroll 8
      for (uint64_t k = lo; k < hi; k++) t += pv[k - c0];
      __syncthreads();
    }
    if (own) {
      double v = (alpha == 0.0 || y == nullptr) ? beta * t : alpha * y[i] + beta * t;
      if (f) v = v * (f[i] ? 1.0 : 0.0);
      z[i] = v;
    }
  }
}
// long rows: one wavefront per row; the 64 lanes load and multiply a chunk
// (coalesced) into LDS, lane 0 adds the chunk in order -- same sum, same order.
// The next chunk's loads are issued before lane 0's adds (double buffering), and
// lane 0 reads its chunk 8 products at a time.
__device__ __forceinline__ double wave_row_sum(const uint32_t *col, const double *a,
                                               const double *x, uint64_t k0, uint64_t k1,
                                               double *buf, int lane) {
  double t = 0;
  uint64_t k = k0 + lane;
  double p = 0.0;
  if (k < k1) p = x ? a[k] * x[col[k]] : a[k];
  for (uint64_t c0 = k0; c0 < k1; c0 += 64) {
    buf[lane] = p;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint64_t kn = c0 + 64 + lane;
    uint32_t cn = 0;
    double an = 0.0;
    if (kn < k1) {
      an = a[kn];
      if (x) cn = col[kn];
    }
    if (lane == 0) {
      const int m = (int)min((uint64_t)64, k1 - c0);
      int q = 0;
      for (; q + 8 <= m; q += 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = buf[q + u];
#pragma unroll
        for (int u = 0; u < 8; u++) t += v[u];
      }
      for (; q < m; q++) t += buf[q];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    p = 0.0;
    if (kn < k1) p = x ? an * x[cn] : an;
  }
  return t;
}
__global__ __launch_bounds__(256) void k_spmv_wave(const uint64_t *ro, const uint32_t *col,
                                                   const double *a, uint32_t rn, const double *x,
                                                   double *z, double alpha, const double *y,
                                                   double beta, const uint8_t *f) {
  __shared__ double buf[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + w; i < rn; i += (uint64_t)gridDim.x * 4) {
    const double t = wave_row_sum(col, a, x, ro[i], ro[i + 1], buf[w], lane);
    if (lane == 0) {
      double v = (alpha == 0.0 || y == nullptr) ? beta * t : alpha * y[i] + beta * t;
      if (f) v = v * (f[i] ? 1.0 : 0.0);
      z[i] = v;
    }
  }
}
// long rows, one row per LANE (RW = 64; fewer rows per wavefront below): each wavefront owns 64 rows and walks them in
// rounds of 16 entries; a round is loaded cooperatively (each load instruction
// covers four 16-entry row segments, 128 B each) into an LDS tile, and every lane
// then adds its own row's 16 products in order.  The sum is the reference's
// left-to-right sum and all 64 lanes add at once (k_spmv_wave leaves 63 idle).
// LIST: the rows are list[0..n) instead of 0..n.
// Long rows (mean >= 32): the lane kernel from 4096 rows on, with RW = 4 / 16 / 64
// rows per wavefront by row count (lane_rw); wave-per-row (lane 0 adds) below
// AMGD_SL_MIN_ROWS / AMGD_SL_LIST_MIN_ROWS (default 4096).  Chosen from the
// micro-benchmark on the 256^3 setup's matrix shapes (tools/spmv_bench.py,
// profiles/r02/spmv_bench.txt).  The sums are the same either way.
// amgd_spmv_set_sl_min() (tests) forces both; -1 returns to the environment/default.
static int64_t g_sl_forced = -1;
static int64_t sl_env(const char *name, int64_t dflt) {
  const char *e = getenv(name);
  return e && *e ? atoll(e) : dflt;
}
static int64_t sl_min_whole() { return g_sl_forced >= 0 ? g_sl_forced : sl_env("AMGD_SL_MIN_ROWS", 4096); }
static int64_t sl_min_list() { return g_sl_forced >= 0 ? g_sl_forced : sl_env("AMGD_SL_LIST_MIN_ROWS", 4096); }
extern "C" void amgd_spmv_set_sl_min(int64_t n) { g_sl_forced = n < 0 ? -1 : n; }
// RW rows per wavefront (64: one row per lane; 16 / 4 for matrices with fewer, longer
// rows -- more wavefronts in flight, the first RW lanes add).
// Long-row SpMV, the x gather one round ahead (round 3).  A wavefront owns RW rows; a
// round is PER x 64 entries (SEG = 64 PER / RW per row), each load instruction
// covering whole >= 128 B row segments, transposed through LDS so that lane r of the
// first RW adds row r's segment left to right.  During the adds of round r the gather
// x[col] of round r+1 (its columns arrived during round r-1) and the (value, column)
// loads of round r+2 are in flight.  Every row is summed left to right from +0: the
// reference's row sum.  LIST: the rows are list[0..n) instead of 0..n (rows longer
// than maxlen are left to k_rows_exact).
//
// Round 5: every load is unconditional and straight-line.  Round 4's loads sat behind
// per-lane bounds branches and a uniform "last round" branch, so the load counts between
// the waits were not static and the compiler waited for ALL outstanding loads
// (s_waitcnt vmcnt(0)) before the products of every round -- the two rounds meant to be
// in flight drained to one.  Now a lane past its row's end loads a valid dummy entry
// (index 0: the kernel only runs on matrices with entries) and its product is dropped by
// a per-round bit mask applied when the product is formed, after the data arrived; the
// same entries enter the same ordered sums.  HASX: products with x (x == nullptr:
// ordered row sums) as a template parameter, so no load sits behind a runtime branch.
template <bool LIST, int RW, int PER = 16, bool HASX = true>
__global__ __launch_bounds__(256) void k_spmv_pipe(const uint64_t *ro, const uint32_t *col,
                                                   const double *a, uint32_t n,
                                                   const uint32_t *list, const double *x,
                                                   double *z, double alpha, const double *y,
                                                   double beta, const uint8_t *f,
                                                   uint32_t maxlen = 0xffffffffu) {
  constexpr int SEG = 64 * PER / RW;
  static_assert(PER <= 32, "k_spmv_pipe: the round mask holds PER bits");
  __shared__ double buf[4][RW][SEG + 1];
  __shared__ uint64_t rk0[4][RW];
  __shared__ uint32_t rlen[4][RW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint64_t rb = ((uint64_t)blockIdx.x * 4 + w) * RW; rb < n;
       rb += (uint64_t)gridDim.x * 4 * RW) {
    const uint64_t r = rb + lane;
    const bool own = lane < RW && r < n;
    const uint32_t i = own ? (LIST ? list[r] : (uint32_t)r) : 0u;
    uint64_t k0 = own ? ro[i] : 0, k1 = own ? ro[i + 1] : 0;
    if (LIST && k1 - k0 > maxlen) k1 = k0;      // a long row: left to k_rows_exact
    const uint32_t len = (uint32_t)(k1 - k0);
    if (lane < RW) {
      rk0[w][lane] = k0;
      rlen[w][lane] = len;
    }
    uint32_t mx = len;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { uint32_t u = __shfl_xor(mx, o, 64); mx = u > mx ? u : mx; }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // (value, column) of round `off`: lane L's q-th entry is flat entry q*64 + L; a lane
    // past its row's end loads entry 0 and clears its bit of the round mask
    auto ld = [&](uint32_t off, double *av, uint32_t *cv) -> uint32_t {
      uint32_t m = 0;
#pragma unroll
      for (int q = 0; q < PER; q++) {
        const int fl = q * 64 + lane, rr = fl / SEG, sub = fl % SEG;
        const uint32_t en = off + sub;
        const bool ok = en < rlen[w][rr];
        const uint64_t k = ok ? rk0[w][rr] + en : 0;
        m |= ok ? 1u << q : 0u;
        av[q] = a[k];
        if (HASX) cv[q] = col[k];
      }
      return m;
    };
    double a0[PER], g0[PER], a1[PER];
    uint32_t c0[PER], c1[PER];
    const uint32_t m0i = ld(0, a0, c0);
    if (HASX) {
#pragma unroll
      for (int q = 0; q < PER; q++) g0[q] = x[c0[q]];
    }
    uint32_t m0 = m0i, m1 = ld(SEG, a1, c1);
    double t = 0;
    for (uint32_t off = 0; off < mx; off += SEG) {
#pragma unroll
      for (int q = 0; q < PER; q++) {
        const int fl = q * 64 + lane;
        const double pr = HASX ? a0[q] * g0[q] : a0[q];
        buf[w][fl / SEG][fl % SEG] = (m0 >> q) & 1u ? pr : 0.0;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      double g1[PER], a2[PER];
      uint32_t c2[PER];
      if (HASX) {
#pragma unroll
        for (int q = 0; q < PER; q++) g1[q] = x[c1[q]];              // round off + SEG
      }
      const uint32_t m2 = ld(off + 2 * SEG, a2, c2);                 // round off + 2 SEG
      if (lane < RW && off < len) {
        const uint32_t m = min((uint32_t)SEG, len - off);
        if (m == SEG) {
          constexpr int U = SEG < 16 ? SEG : 16;
#pragma unroll
          for (int e0 = 0; e0 < SEG; e0 += U) {
            double u[U];
#pragma unroll
            for (int e = 0; e < U; e++) u[e] = buf[w][lane][e0 + e];
#pragma unroll
            for (int e = 0; e < U; e++) t += u[e];
          }
        } else {
          for (uint32_t e = 0; e < m; e++) t += buf[w][lane][e];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int q = 0; q < PER; q++) {
        a0[q] = a1[q]; a1[q] = a2[q];
        if (HASX) { g0[q] = g1[q]; c1[q] = c2[q]; }
      }
      m0 = m1;
      m1 = m2;
    }
    if (own && (!LIST || ro[i + 1] - ro[i] <= maxlen)) {
      double v = (alpha == 0.0 || y == nullptr) ? beta * t : alpha * y[i] + beta * t;
      if (f) v = v * (f[i] ? 1.0 : 0.0);
      z[i] = v;
    }
  }
}
// k_spmv_pipe with paired loads (products with x only): lane L's p-th load covers the two
// consecutive entries 2 (p 64 + L) and 2 (p 64 + L) + 1 of the round, one 16 B value load
// and one 8 B column load for both -- two thirds of the memory instructions of k_spmv_pipe
// per entry.  For the pairs to be aligned a row is walked from the even offset k0 & ~1:
// when its first entry sits at an odd offset, the leading slot holds a masked product
// (+0) that enters the row's sum before its first product, which leaves the reference's
// ordered sum unchanged ((+0) + p == p for every p, -0 included).  A slot past a row's
// end, or the masked leading slot, gathers x[0] (its column may be another row's or the
// allocation's padding).  Needs a 16 B aligned value array and an 8 B aligned column
// array (the launcher checks: arena blocks are 256 B aligned; views fall back).
// Depths (rounds ahead of the round whose products are formed): CA for the columns, GA
// for the x gathers (issued when a round's columns have arrived, CA - GA rounds after
// them), VA for the values (VA == CA: loaded with the columns; else on their own, the
// pair index recomputed).  CA 2, GA 1, VA 2 (other depths measured slower).
// AMX (whole-matrix products only): per row also the position of its first largest
// product (strict >, from -DBL_MAX: find_support's selection rule, k_fs_select) as the
// global entry index into amx[row] (~0 when no product beats -DBL_MAX).  Every round's
// maximum is found by all 64 lanes (the adds use only RW of them); tracking it in the adding
// lane alone measured 0.1 s slower per 256^3 setup (profiles/r05/ab256_r05aj_parallel_max.txt).
template <bool LIST, int RW, int PER, int CA, int GA, int VA, bool AMX = false>
__device__ __forceinline__ void spmv_pair_body(const uint64_t *ro, const uint32_t *col,
                                               const double *a, uint32_t n,
                                               const uint32_t *list, const double *x,
                                               double *z, double alpha, const double *y,
                                               double beta, const uint8_t *f, uint32_t maxlen,
                                               uint64_t *amx = nullptr) {
  constexpr int SEG = 64 * PER / RW, PH = PER / 2, NC = CA - GA;
  static_assert(PER <= 32 && PER % 2 == 0 && SEG % 2 == 0, "k_spmv_pair: round shape");
  static_assert(GA >= 1 && NC >= 1 && VA >= 1 && VA <= CA, "k_spmv_pair: depths");
  __shared__ double buf[4][RW][SEG + 1];
  __shared__ uint64_t rk0[4][RW];
  __shared__ uint32_t rlen[4][RW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const double2 *a2p = reinterpret_cast<const double2 *>(a);
  const uint2 *c2p = reinterpret_cast<const uint2 *>(col);
  for (uint64_t rb = ((uint64_t)blockIdx.x * 4 + w) * RW; rb < n;
       rb += (uint64_t)gridDim.x * 4 * RW) {
    const uint64_t r = rb + lane;
    const bool own = lane < RW && r < n;
    const uint32_t i = own ? (LIST ? list[r] : (uint32_t)r) : 0u;
    uint64_t k0 = own ? ro[i] : 0, k1 = own ? ro[i + 1] : 0;
    if (LIST && k1 - k0 > maxlen) k1 = k0;
    const uint32_t lead = k1 > k0 ? (uint32_t)(k0 & 1) : 0u;
    const uint32_t vlen = (uint32_t)(k1 - k0) + lead;     // slots from the even start
    if (lane < RW) {
      rk0[w][lane] = (k0 - lead) >> 1;                    // in pairs
      rlen[w][lane] = vlen | lead << 31;
    }
    uint32_t mx = vlen;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { uint32_t u = __shfl_xor(mx, o, 64); mx = u > mx ? u : mx; }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // row and slot of lane's p-th pair in a round: 64 consecutive pairs per load (a row's
    // segment, 128 B and more per row)
    auto slot = [&](int p, int &rr, int &sub) {
      const int fl = 2 * (p * 64 + lane);
      rr = fl / SEG; sub = fl % SEG;
    };
    // pair index of lane's p-th pair of round `off` (0 past the row's end) and its two
    // mask bits (first slot: a real entry, not the masked leading slot; second: in the row)
    auto pk = [&](uint32_t off, int p, uint32_t &m) -> uint64_t {
      int rr, sub;
      slot(p, rr, sub);
      const uint32_t en = off + sub, info = rlen[w][rr], vl = info & 0x7fffffffu;
      const bool any = en < vl;
      m |= (any && en >= (info >> 31) ? 1u : 0u) << (2 * p);
      m |= (en + 1 < vl ? 1u : 0u) << (2 * p + 1);
      return any ? rk0[w][rr] + (en >> 1) : 0;
    };
    // columns (and, VA == CA, values) of round `off`; its mask
    auto ldc = [&](uint32_t off, double *av, uint32_t *cv) -> uint32_t {
      uint32_t m = 0;
#pragma unroll
      for (int p = 0; p < PH; p++) {
        const uint64_t k = pk(off, p, m);
        if (VA == CA) {
          const double2 v = a2p[k];
          av[2 * p] = v.x; av[2 * p + 1] = v.y;
        }
        const uint2 c = c2p[k];
        cv[2 * p] = c.x; cv[2 * p + 1] = c.y;
      }
      return m;
    };
    auto lda = [&](uint32_t off, double *av) {
      uint32_t m = 0;
#pragma unroll
      for (int p = 0; p < PH; p++) {
        const double2 v = a2p[pk(off, p, m)];
        av[2 * p] = v.x; av[2 * p + 1] = v.y;
      }
    };
    auto gat = [&](const uint32_t *cv, uint32_t m, double *gv) {
#pragma unroll
      for (int q = 0; q < PER; q++) gv[q] = x[(m >> q) & 1u ? cv[q] : 0u];
    };
    // ring state at the top of round r: va[j] values of round r + j (j < VA), gv[j] gathers
    // of round r + j (j < GA), cq[j] columns of round r + GA + j (j < NC), ms[j] the mask of
    // round r + j (j < CA)
    double va[VA][PER], gv[GA][PER];
    uint32_t cq[NC][PER], ms[CA];
    {
      double vt[PER];
      uint32_t ct[PER];
#pragma unroll
      for (int j = 0; j < CA; j++) {
        if (j < GA) {
          ms[j] = ldc(j * SEG, j < VA ? va[j] : vt, ct);
          gat(ct, ms[j], gv[j]);
        } else {
          ms[j] = ldc(j * SEG, j < VA ? va[j] : vt, cq[j - GA]);
        }
        if (VA < CA && j < VA) lda(j * SEG, va[j]);
      }
    }
    double t = 0, mxv = -DBL_MAX;
    uint32_t mxp = 0xffffffffu;
    for (uint32_t off = 0; off < mx; off += SEG) {
#pragma unroll
      for (int p = 0; p < PH; p++) {
        int rr, sub;
        slot(p, rr, sub);
        buf[w][rr][sub] = (ms[0] >> (2 * p)) & 1u ? va[0][2 * p] * gv[0][2 * p] : 0.0;
        buf[w][rr][sub + 1] = (ms[0] >> (2 * p + 1)) & 1u ? va[0][2 * p + 1] * gv[0][2 * p + 1] : 0.0;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (AMX) {
        // the round's first largest product of every row, by all 64 lanes: 64 / RW lanes
        // per row scan SEG / (64 / RW) consecutive slots each in order, then combine --
        // larger value, or equal value at the smaller position -- which is the sequential
        // "first x > max" (NaN, -inf and -DBL_MAX never enter); earlier rounds keep ties
        constexpr int LPR = 64 / RW, EPL = SEG / LPR;
        const int rr = lane / LPR, part = lane % LPR;
        const uint32_t info = rlen[w][rr], vl = info & 0x7fffffffu, ld0 = info >> 31;
        double bv = -DBL_MAX;
        uint32_t bp = 0xffffffffu;
#pragma unroll
        for (int e = 0; e < EPL; e++) {
          const uint32_t sub = (uint32_t)(part * EPL + e), pos = off + sub;
          const double v = buf[w][rr][sub];
          if (pos < vl && pos >= ld0 && v > bv) { bv = v; bp = pos; }
        }
#pragma unroll
        for (int o = LPR / 2; o > 0; o >>= 1) {
          const double ov = __shfl_xor(bv, o, 64);
          const uint32_t op = (uint32_t)__shfl_xor((int)bp, o, 64);
          if (ov > bv || (ov == bv && op < bp)) { bv = ov; bp = op; }
        }
        const double sv = __shfl(bv, (lane % RW) * LPR, 64);
        const uint32_t sp = (uint32_t)__shfl((int)bp, (lane % RW) * LPR, 64);
        if (lane < RW && sv > mxv) { mxv = sv; mxp = sp; }
      }
      // shift the rings down one round, then fill the new last slots
#pragma unroll
      for (int j = 0; j + 1 < VA; j++)
#pragma unroll
        for (int q = 0; q < PER; q++) va[j][q] = va[j + 1][q];
#pragma unroll
      for (int j = 0; j + 1 < GA; j++)
#pragma unroll
        for (int q = 0; q < PER; q++) gv[j][q] = gv[j + 1][q];
#pragma unroll
      for (int j = 0; j + 1 < CA; j++) ms[j] = ms[j + 1];
      gat(cq[0], ms[GA - 1], gv[GA - 1]);                     // round off + GA SEG
#pragma unroll
      for (int j = 0; j + 1 < NC; j++)
#pragma unroll
        for (int q = 0; q < PER; q++) cq[j][q] = cq[j + 1][q];
      if (VA < CA) lda(off + VA * SEG, va[VA - 1]);           // round off + VA SEG
      ms[CA - 1] = ldc(off + CA * SEG, va[VA - 1], cq[NC - 1]);   // round off + CA SEG
      if (lane < RW && off < vlen) {
        const uint32_t m = min((uint32_t)SEG, vlen - off);
        if (m == SEG) {
          constexpr int U = SEG < (VA < CA ? 8 : 16) ? SEG : (VA < CA ? 8 : 16);
#pragma unroll
          for (int e0 = 0; e0 < SEG; e0 += U) {
            double u[U];
#pragma unroll
            for (int e = 0; e < U; e++) u[e] = buf[w][lane][e0 + e];
#pragma unroll
            for (int e = 0; e < U; e++) t += u[e];
          }
        } else {
          for (uint32_t e = 0; e < m; e++) t += buf[w][lane][e];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (own && (!LIST || ro[i + 1] - ro[i] <= maxlen)) {
      double v = (alpha == 0.0 || y == nullptr) ? beta * t : alpha * y[i] + beta * t;
      if (f) v = v * (f[i] ? 1.0 : 0.0);
      z[i] = v;
    }
    if (AMX && own) amx[i] = mxp == 0xffffffffu ? ~0ull : k0 - lead + mxp;
  }
}
template <bool LIST, int RW, int PER, int CA = 2, int GA = 1, int VA = 2>
__global__ __launch_bounds__(256) void k_spmv_pair(const uint64_t *ro, const uint32_t *col,
                                                   const double *a, uint32_t n,
                                                   const uint32_t *list, const double *x,
                                                   double *z, double alpha, const double *y,
                                                   double beta, const uint8_t *f,
                                                   uint32_t maxlen = 0xffffffffu) {
  spmv_pair_body<LIST, RW, PER, CA, GA, VA>(ro, col, a, n, list, x, z, alpha, y, beta, f, maxlen);
}
template <int RW, int PER>
__global__ __launch_bounds__(256) void k_spmv_pair_amx(const uint64_t *ro, const uint32_t *col,
                                                       const double *a, uint32_t n, const double *x,
                                                       double *z, uint64_t *amx) {
  spmv_pair_body<false, RW, PER, 2, 1, 2, true>(ro, col, a, n, nullptr, x, z, 0.0, nullptr, 1.0, nullptr,
                                                0xffffffffu, amx);
}
// ---------------------------------------------------------------------------
// Tabled long-row SpMV (round 6).  The lane kernels above are bound by texture-address
// work on the x gathers: ~30 distinct 128-B lines per 64-lane gather instruction, TA busy
// 87-96 % (profiles/r05/mvctr/).  But a tile of consecutive rows gathers from few
// distinct x entries: at 256^3, 256 rows of level 1's R gather 2.7-3.3 K distinct columns
// for 11-15 K entries (~250 lines), 16-64 rows of levels 3-5 3-7 K for 20-120 K entries
// (profiles/r06/mvstat256_r06d.txt, AMGD_MVSTAT=1).  find_support multiplies the same
// patterns 35-240 times per call (only values change: removed entries are zeroed), so
// per pinned matrix (amgd_rowmax_pin) the rows are cut into tiles of TR rows and for each
// tile its distinct columns (ascending: `tab`) and, per entry, the 16-bit slot of its
// column in them are built once (k_tab_count / k_tab_fill: a bit map over the tile's
// column span in LDS).  A product then loads the tile's x[tab] into LDS once (sorted
// columns: whole lines) and every entry gathers xs[slot] from LDS instead of x[col] --
// the same value, so the same products summed in the same order (the lane kernel's
// rounds, rows and ordered adds are unchanged): bit-identical.  Entry stream: 8 B value +
// 2 B slot instead of 8 B + 4 B.  A tile whose distinct columns exceed the LDS table, or
// whose column span exceeds the build's bit map, runs the plain gathers ("direct").
// AMGD_MV_TAB=1 / amgd_spmv_set_tab(1): on (off by default, measured below).
// ---------------------------------------------------------------------------
#define TAB_BM_WORDS 16384                // build bit map: 524288 columns of span
#define TAB_DIRECT 0xffffffffu
template <int RW> struct TabShape;
template <> struct TabShape<64> { static constexpr int PER = 16, TMAX = 5120; };
template <> struct TabShape<16> { static constexpr int PER = 16, TMAX = 5632; };
template <> struct TabShape<4> { static constexpr int PER = 8, TMAX = 7680; };
// per tile: distinct columns (or TAB_DIRECT) and the smallest column
__global__ __launch_bounds__(256) void k_tab_count(const uint64_t *ro, const uint32_t *col, uint32_t n,
                                                   uint32_t TR, uint32_t ntiles, uint32_t tmax,
                                                   uint32_t *nd_out, uint2 *span_out) {
  extern __shared__ uint32_t bm[];                // TAB_BM_WORDS
  __shared__ uint32_t red[4][2];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint32_t r0 = t * TR, r1 = min(n, r0 + TR);
    uint32_t lo = 0xffffffffu, hi = 0;
    for (uint32_t r = r0 + tid; r < r1; r += 256)
      if (ro[r + 1] > ro[r]) { lo = min(lo, col[ro[r]]); hi = max(hi, col[ro[r + 1] - 1]); }
    for (int o = 32; o; o >>= 1) { lo = min(lo, (uint32_t)__shfl_xor((int)lo, o, 64)); hi = max(hi, (uint32_t)__shfl_xor((int)hi, o, 64)); }
    if (lane == 0) { red[w][0] = lo; red[w][1] = hi; }
    __syncthreads();
    lo = min(min(red[0][0], red[1][0]), min(red[2][0], red[3][0]));
    hi = max(max(red[0][1], red[1][1]), max(red[2][1], red[3][1]));
    __syncthreads();
    uint32_t nd = 0;
    if (lo <= hi) {
      const uint64_t span = (uint64_t)hi - lo + 1;
      if (span > 32ull * TAB_BM_WORDS) {
        nd = TAB_DIRECT;
      } else {
        const uint32_t nw = (uint32_t)((span + 31) >> 5);
        for (uint32_t q = tid; q < nw; q += 256) bm[q] = 0;
        __syncthreads();
        for (uint64_t k = ro[r0] + tid; k < ro[r1]; k += 256) {
          const uint32_t c = col[k] - lo;
          atomicOr(&bm[c >> 5], 1u << (c & 31));
        }
        __syncthreads();
        uint32_t s = 0;
        for (uint32_t q = tid; q < nw; q += 256) s += __popc(bm[q]);
        for (int o = 32; o; o >>= 1) s += (uint32_t)__shfl_xor((int)s, o, 64);
        if (lane == 0) red[w][0] = s;
        __syncthreads();
        nd = red[0][0] + red[1][0] + red[2][0] + red[3][0];
        if (nd > tmax) nd = TAB_DIRECT;
        __syncthreads();
      }
    }
    if (tid == 0) { nd_out[t] = nd; span_out[t] = make_uint2(lo, hi); }
  }
}
// tab (the tile's distinct columns, ascending) and every entry's slot in it
__global__ __launch_bounds__(256) void k_tab_fill(const uint64_t *ro, const uint32_t *col, uint32_t n,
                                                  uint32_t TR, uint32_t ntiles, const uint32_t *nd_in,
                                                  const uint2 *span_in, const uint64_t *toff,
                                                  uint32_t *tab, uint16_t *slot) {
  extern __shared__ uint32_t tab_sh[];         // bm[TAB_BM_WORDS] then pre (u16)[TAB_BM_WORDS]
  uint32_t *bm = tab_sh;
  uint16_t *pre = reinterpret_cast<uint16_t *>(tab_sh + TAB_BM_WORDS);
  __shared__ uint32_t wtot[4];
  const int tid = threadIdx.x;
  for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint32_t nd = nd_in[t];
    if (nd == 0 || nd == TAB_DIRECT) continue;            // uniform per block
    const uint32_t r0 = t * TR, r1 = min(n, r0 + TR), lo = span_in[t].x, hi = span_in[t].y;
    const uint32_t nw = (hi - lo + 32) >> 5;
    for (uint32_t q = tid; q < nw; q += 256) bm[q] = 0;
    __syncthreads();
    const uint64_t e0 = ro[r0], e1 = ro[r1];
    for (uint64_t k = e0 + tid; k < e1; k += 256) {
      const uint32_t c = col[k] - lo;
      atomicOr(&bm[c >> 5], 1u << (c & 31));
    }
    __syncthreads();
    // exclusive prefix of the words' popcounts: contiguous chunks per thread, then a block scan
    const uint32_t per = (nw + 255) / 256, q0 = min(nw, tid * per), q1 = min(nw, q0 + per);
    uint32_t s = 0;
    for (uint32_t q = q0; q < q1; q++) s += __popc(bm[q]);
    const uint32_t incl = block_incl_scan<256>(s, wtot);
    uint32_t run = incl - s;
    for (uint32_t q = q0; q < q1; q++) { pre[q] = (uint16_t)run; run += __popc(bm[q]); }
    __syncthreads();
    uint32_t *tb = tab + toff[t];
    for (uint32_t q = tid; q < nw; q += 256) {
      uint32_t b = bm[q], p = pre[q];
      while (b) {
        const int bit = __ffs(b) - 1;
        tb[p++] = lo + 32 * q + bit;
        b &= b - 1;
      }
    }
    for (uint64_t k = e0 + tid; k < e1; k += 256) {
      const uint32_t c = col[k] - lo, q = c >> 5;
      slot[k] = (uint16_t)(pre[q] + __popc(bm[q] & ((1u << (c & 31)) - 1u)));
    }
    __syncthreads();
  }
}
// One tile of rows [r0, r1) for a workgroup of 4 wavefronts: k_spmv_pair's rounds (pair
// loads, masked leading / trailing slots, ordered adds, AMX maxima), the gather from the
// LDS table xs (TAB: loaded by the caller) or from x (direct tiles).
template <int RW, int PER, int TMAX, bool TAB, bool AMX>
__device__ __forceinline__ void spmv_tab_rows(const uint64_t *ro, const uint32_t *col, const uint16_t *slot,
                                              const double *a, uint32_t r0, uint32_t r1, const double *x,
                                              const uint32_t *tb, uint32_t nd, double *xs, double *z,
                                              double alpha, const double *y, double beta, const uint8_t *f,
                                              uint64_t *amx, double (*buf)[RW][64 * PER / RW + 1],
                                              uint64_t (*rk0)[RW], uint32_t (*rlen)[RW]) {
  constexpr int SEG = 64 * PER / RW, PH = PER / 2;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const double2 *a2p = reinterpret_cast<const double2 *>(a);
  const uint2 *c2p = reinterpret_cast<const uint2 *>(col);
  const uint32_t *s2p = reinterpret_cast<const uint32_t *>(slot);
  auto pk = [&](uint32_t off, int p, uint32_t &m) -> uint64_t {
    const int fl = 2 * (p * 64 + lane), rr = fl / SEG, sub = fl % SEG;
    const uint32_t en = off + sub, info = rlen[w][rr], vl = info & 0x7fffffffu;
    const bool any = en < vl;
    m |= (any && en >= (info >> 31) ? 1u : 0u) << (2 * p);
    m |= (en + 1 < vl ? 1u : 0u) << (2 * p + 1);
    return any ? rk0[w][rr] + (en >> 1) : 0;
  };
  // values and gather indices (slots or columns) of round `off`
  auto ldc = [&](uint32_t off, double *av, uint32_t *cv) -> uint32_t {
    uint32_t m = 0;
#pragma unroll
    for (int p = 0; p < PH; p++) {
      const uint64_t k = pk(off, p, m);
      const double2 v = a2p[k];
      av[2 * p] = v.x; av[2 * p + 1] = v.y;
      if (TAB) {
        const uint32_t s = s2p[k];
        cv[2 * p] = s & 0xffffu; cv[2 * p + 1] = s >> 16;
      } else {
        const uint2 c = c2p[k];
        cv[2 * p] = c.x; cv[2 * p + 1] = c.y;
      }
    }
    return m;
  };
  auto gat = [&](const uint32_t *cv, uint32_t m, double *gv) {
#pragma unroll
    for (int q = 0; q < PER; q++) {
      const uint32_t c = (m >> q) & 1u ? cv[q] : 0u;
      gv[q] = TAB ? xs[c] : x[c];
    }
  };
  for (uint64_t rb = (uint64_t)r0 + (uint64_t)w * RW; rb < r1; rb += 4 * RW) {
    const uint64_t r = rb + lane;
    const bool own = lane < RW && r < r1;
    const uint32_t i = own ? (uint32_t)r : 0u;
    const uint64_t k0 = own ? ro[i] : 0, k1 = own ? ro[i + 1] : 0;
    const uint32_t lead = k1 > k0 ? (uint32_t)(k0 & 1) : 0u;
    const uint32_t vlen = (uint32_t)(k1 - k0) + lead;
    if (lane < RW) {
      rk0[w][lane] = (k0 - lead) >> 1;
      rlen[w][lane] = vlen | lead << 31;
    }
    uint32_t mx = vlen;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { uint32_t u = __shfl_xor(mx, o, 64); mx = u > mx ? u : mx; }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double va[2][PER], gv[PER];
    uint32_t cq[PER], ct[PER], ms[2];
    ms[0] = ldc(0, va[0], ct);
    ms[1] = ldc(SEG, va[1], cq);
    gat(ct, ms[0], gv);
    double t = 0, mxv = -DBL_MAX;
    uint32_t mxp = 0xffffffffu;
    for (uint32_t off = 0; off < mx; off += SEG) {
#pragma unroll
      for (int p = 0; p < PH; p++) {
        const int fl = 2 * (p * 64 + lane), rr = fl / SEG, sub = fl % SEG;
        buf[w][rr][sub] = (ms[0] >> (2 * p)) & 1u ? va[0][2 * p] * gv[2 * p] : 0.0;
        buf[w][rr][sub + 1] = (ms[0] >> (2 * p + 1)) & 1u ? va[0][2 * p + 1] * gv[2 * p + 1] : 0.0;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (AMX) {
        constexpr int LPR = 64 / RW, EPL = SEG / LPR;
        const int rr = lane / LPR, part = lane % LPR;
        const uint32_t info = rlen[w][rr], vl = info & 0x7fffffffu, ld0 = info >> 31;
        double bv = -DBL_MAX;
        uint32_t bp = 0xffffffffu;
#pragma unroll
        for (int e = 0; e < EPL; e++) {
          const uint32_t sub = (uint32_t)(part * EPL + e), pos = off + sub;
          const double v = buf[w][rr][sub];
          if (pos < vl && pos >= ld0 && v > bv) { bv = v; bp = pos; }
        }
#pragma unroll
        for (int o = LPR / 2; o > 0; o >>= 1) {
          const double ov = __shfl_xor(bv, o, 64);
          const uint32_t op = (uint32_t)__shfl_xor((int)bp, o, 64);
          if (ov > bv || (ov == bv && op < bp)) { bv = ov; bp = op; }
        }
        const double sv = __shfl(bv, (lane % RW) * LPR, 64);
        const uint32_t sp = (uint32_t)__shfl((int)bp, (lane % RW) * LPR, 64);
        if (lane < RW && sv > mxv) { mxv = sv; mxp = sp; }
      }
#pragma unroll
      for (int q = 0; q < PER; q++) va[0][q] = va[1][q];
      ms[0] = ms[1];
      gat(cq, ms[0], gv);                                      // round off + SEG
      ms[1] = ldc(off + 2 * SEG, va[1], cq);                   // round off + 2 SEG
      if (lane < RW && off < vlen) {
        const uint32_t m = min((uint32_t)SEG, vlen - off);
        if (m == SEG) {
          constexpr int U = SEG < 16 ? SEG : 16;
#pragma unroll
          for (int e0 = 0; e0 < SEG; e0 += U) {
            double u[U];
#pragma unroll
            for (int e = 0; e < U; e++) u[e] = buf[w][lane][e0 + e];
#pragma unroll
            for (int e = 0; e < U; e++) t += u[e];
          }
        } else {
          for (uint32_t e = 0; e < m; e++) t += buf[w][lane][e];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (own) {
      double v = (alpha == 0.0 || y == nullptr) ? beta * t : alpha * y[i] + beta * t;
      if (f) v = v * (f[i] ? 1.0 : 0.0);
      z[i] = v;
      if (AMX) amx[i] = mxp == 0xffffffffu ? ~0ull : k0 - lead + mxp;
    }
  }
}
template <int RW, bool AMX>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void k_spmv_tab(const uint64_t *ro, const uint32_t *col, const uint16_t *slot,
                                                  const double *a, uint32_t n, uint32_t TR, uint32_t ntiles,
                                                  const uint32_t *tnd, const uint64_t *toff, const uint32_t *tab,
                                                  const double *x, double *z, double alpha, const double *y,
                                                  double beta, const uint8_t *f, uint64_t *amx) {
  constexpr int PER = TabShape<RW>::PER, TMAX = TabShape<RW>::TMAX, SEG = 64 * PER / RW;
  __shared__ double xs[TMAX];
  __shared__ double buf[4][RW][SEG + 1];
  __shared__ uint64_t rk0[4][RW];
  __shared__ uint32_t rlen[4][RW];
  for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint32_t r0 = t * TR, r1 = min(n, r0 + TR), nd = tnd[t];
    if (nd > (uint32_t)TMAX)                   // TAB_DIRECT (and never past the LDS table)
      spmv_tab_rows<RW, PER, TMAX, false, AMX>(ro, col, slot, a, r0, r1, x, nullptr, 0, xs, z, alpha, y, beta, f,
                                               amx, buf, rk0, rlen);
    else {
      // the tile's table: every load of it in flight at once (nothing else is live
      // here), then LDS, then one barrier
      constexpr int TL = (TMAX + 255) / 256;
      const uint32_t *tb = tab + toff[t];
      uint32_t tc[TL];
      double tv[TL];
#pragma unroll
      for (int u = 0; u < TL; u++) {
        const uint32_t q = (uint32_t)u * 256 + threadIdx.x;
        tc[u] = tb[q < nd ? q : 0];
      }
#pragma unroll
      for (int u = 0; u < TL; u++) tv[u] = x[tc[u]];
#pragma unroll
      for (int u = 0; u < TL; u++) {
        const uint32_t q = (uint32_t)u * 256 + threadIdx.x;
        if (q < nd) xs[q] = tv[u];
      }
      __syncthreads();
      spmv_tab_rows<RW, PER, TMAX, true, AMX>(ro, col, slot, a, r0, r1, x, tb, nd, xs, z, alpha, y, beta, f, amx,
                                              buf, rk0, rlen);
    }
    __syncthreads();
  }
}
struct MvTab {
  const uint64_t *ro;
  uint32_t rn;
  uint64_t nnz;
  int rw;
  uint32_t TR, ntiles, ndirect;
  uint32_t *tnd;
  uint64_t *toff;
  uint32_t *tab;
  uint16_t *slot;
};
static std::vector<MvTab> g_mvtab;
static int g_mv_tab = -1;
extern "C" void amgd_spmv_set_tab(int on) { g_mv_tab = on; }
static bool mv_tab_on() {
  // off by default: per product 0.84x (level 1's R, 64 rows per wavefront) to 1.34x, and
  // no change end to end at 256^3 (SpMV 5.01 s per setup either way; profiles/r06/)
  if (g_mv_tab < 0) { const char *e = getenv("AMGD_MV_TAB"); g_mv_tab = e && *e ? atoi(e) : 0; }
  return g_mv_tab > 0;
}
static uint64_t g_tab_builds = 0, g_tab_tiles = 0, g_tab_direct = 0;
extern "C" void amgd_spmv_tab_stats(uint64_t *out3) { out3[0] = g_tab_builds; out3[1] = g_tab_tiles; out3[2] = g_tab_direct; }
static void mv_tab_free(MvTab &t) {
  amgd_free(t.tnd); amgd_free(t.toff); amgd_free(t.tab); amgd_free(t.slot);
}
// rows per wavefront of the tabled kernel, by the mean row: long rows (coarse levels) 4 per
// wavefront, so a tile can be 16 rows; short ones 64 (tiles of 256 rows)
static int tab_rw(uint64_t mean) { return mean >= 256 ? 4 : mean >= 96 ? 16 : 64; }
// Tables only for mean rows below TAB_MEAN_MAX: for the coarse levels' long rows (mean >=
// 256, 4 rows per wavefront) the tiled kernel measured 1.1-1.8x slower per product than
// k_spmv_pair (a tile of 16 rows per workgroup: one table load and barrier per 4 rows per
// wavefront; profiles/r06/mvlog_ab_r06g.txt)
#define TAB_MEAN_MAX 256
static void mv_tab_build(const dcsr *M) {
  if (!mv_tab_on() || M->rn == 0 || M->nnz < 32ull * M->rn || (int64_t)M->rn < sl_min_whole()) return;
  if (((uintptr_t)M->a & 15) || ((uintptr_t)M->col & 7)) return;
  for (const MvTab &e : g_mvtab)
    if (e.ro == M->ro && e.rn == M->rn && e.nnz == M->nnz) return;
  hipStream_t s = amgd_s();
  const uint64_t mean = M->nnz / M->rn;
  if (mean >= TAB_MEAN_MAX) return;
  MvTab t{};
  t.ro = M->ro; t.rn = M->rn; t.nnz = M->nnz;
  t.rw = tab_rw(mean);
  // tiles of ~12 K entries (3-6 K distinct columns at 256^3), at least one round of rows
  const uint32_t unit = 4u * (uint32_t)t.rw;
  uint64_t tr = 12288 / std::max<uint64_t>(mean, 1);
  tr = std::max<uint64_t>(unit, (tr / unit) * unit);
  t.TR = (uint32_t)tr;
  t.ntiles = (uint32_t)((M->rn + tr - 1) / tr);
  t.tnd = (uint32_t *)amgd_alloc(4ull * t.ntiles + 8);
  uint2 *span = (uint2 *)amgd_alloc(8ull * t.ntiles + 8);
  // the LDS table of the kernel that will read it (k_spmv_tab<rw>: xs[TMAX])
  const uint32_t tmax = t.rw == 4 ? TabShape<4>::TMAX : t.rw == 16 ? TabShape<16>::TMAX : TabShape<64>::TMAX;
  const int g = (int)std::min<uint32_t>(t.ntiles, 16384u);
  static bool attr = false;
  if (!attr) {
    HIPCK(hipFuncSetAttribute((const void *)k_tab_count, hipFuncAttributeMaxDynamicSharedMemorySize, 4 * TAB_BM_WORDS));
    HIPCK(hipFuncSetAttribute((const void *)k_tab_fill, hipFuncAttributeMaxDynamicSharedMemorySize, 6 * TAB_BM_WORDS));
    attr = true;
  }
  k_tab_count<<<g, 256, 4 * TAB_BM_WORDS, s>>>(M->ro, M->col, M->rn, t.TR, t.ntiles, tmax, t.tnd, span);
  KCHECK();
  t.toff = (uint64_t *)amgd_alloc(8ull * t.ntiles + 16);
  std::vector<uint32_t> hnd(t.ntiles);
  HIPCK(hipMemcpyAsync(hnd.data(), t.tnd, 4ull * t.ntiles, hipMemcpyDeviceToHost, s));
  HIPCK(hipStreamSynchronize(s));
  std::vector<uint64_t> hoff(t.ntiles + 1, 0);
  for (uint32_t q = 0; q < t.ntiles; q++) {
    const uint32_t nd = hnd[q];
    if (nd == TAB_DIRECT) t.ndirect++;
    hoff[q + 1] = hoff[q] + (nd == TAB_DIRECT ? 0 : nd);
  }
  amgd_h2d(t.toff, hoff.data(), 8ull * (t.ntiles + 1));
  t.tab = (uint32_t *)amgd_alloc(4 * hoff[t.ntiles] + 8);
  t.slot = (uint16_t *)amgd_alloc(2 * M->nnz + 16);
  k_tab_fill<<<g, 256, 6 * TAB_BM_WORDS, s>>>(M->ro, M->col, M->rn, t.TR, t.ntiles, t.tnd, span, t.toff, t.tab, t.slot);
  KCHECK();
  amgd_free(span);
  g_tab_builds++;
  g_tab_tiles += t.ntiles;
  g_tab_direct += t.ndirect;
  g_mvtab.push_back(t);
}
static const MvTab *mv_tab_find(const dcsr *M) {
  for (const MvTab &e : g_mvtab)
    if (e.ro == M->ro && e.rn == M->rn && e.nnz == M->nnz) return &e;
  return nullptr;
}
static void mv_tab_drop(const void *ro) {
  for (size_t q = 0; q < g_mvtab.size();)
    if ((const void *)g_mvtab[q].ro == ro) { MvTab t = g_mvtab[q]; g_mvtab.erase(g_mvtab.begin() + q); mv_tab_free(t); }
    else q++;
}
static void mv_tab_launch(const MvTab *tb, const dcsr *M, const double *x, double *z, double alpha,
                          const double *y, double beta, const uint8_t *f, uint64_t *amx) {
  const int g = (int)std::min<uint32_t>(tb->ntiles, 65536u);
#define TAB_L(RW, AMX_)                                                                             \
  k_spmv_tab<RW, AMX_><<<g, 256, 0, amgd_s()>>>(M->ro, M->col, tb->slot, M->a, M->rn, tb->TR, tb->ntiles, \
                                                tb->tnd, tb->toff, tb->tab, x, z, alpha, y, beta, f, amx)
  if (amx) {
    if (tb->rw == 64) TAB_L(64, true); else if (tb->rw == 16) TAB_L(16, true); else TAB_L(4, true);
  } else {
    if (tb->rw == 64) TAB_L(64, false); else if (tb->rw == 16) TAB_L(16, false); else TAB_L(4, false);
  }
#undef TAB_L
}
// Products with x take k_spmv_pair by default (round 5: long-row SpMV 5.02 -> 4.88 s per
// 256^3 setup, profiles/r05/pair/); AMGD_MV_PAIR=0 / amgd_spmv_set_pair(0) (tests, A/B):
// k_spmv_pipe.  Measured and dropped (profiles/r05/pair/): values one round ahead at 3
// wavefronts per SIMD (4.94 s), gathers two rounds ahead (5.01 / 5.08 s), 8 / 16 rows
// side by side in each load instead of one row's segment (5.51 / 5.98 s).  The lane
// kernels are bound by texture-address work: TA busy 87-96 % of the kernel's cycles, one
// TA cycle per distinct cache line, ~53 distinct lines per 64-lane x gather
// (profiles/r05/mvctr/)
static int g_mv_pair = -1;
extern "C" void amgd_spmv_set_pair(int on) { g_mv_pair = on < 0 ? -1 : on; }
static bool mv_pair(const dcsr *M) {
  if (g_mv_pair == -1) g_mv_pair = (int)sl_env("AMGD_MV_PAIR", 1);
  return g_mv_pair > 0 && ((uintptr_t)M->a & 15) == 0 && ((uintptr_t)M->col & 7) == 0;
}
// rows per wavefront of the lane kernel for n rows (>= ~2048 wavefronts in flight)
static int64_t g_rw_forced = -2;     // AMGD_SL_RW / amgd_spmv_set_rw (tests): 4, 16 or 64
extern "C" void amgd_spmv_set_rw(int rw) { g_rw_forced = rw < 0 ? -2 : rw; }
// row-count bounds of the 16 / 64-row shapes (log2; amgd_spmv_set_rw_bounds: A/B)
static int g_rw_lo = 16, g_rw_hi = 22;
extern "C" void amgd_spmv_set_rw_bounds(int lo, int hi) {
  g_rw_lo = lo > 0 ? lo : 16;
  g_rw_hi = hi > 0 ? hi : 22;
}
static int lane_rw(uint64_t n) {
  if (g_rw_forced == -2) g_rw_forced = sl_env("AMGD_SL_RW", 0);
  if (g_rw_forced == 4 || g_rw_forced == 16 || g_rw_forced == 64) return (int)g_rw_forced;
  return n >= (1ull << g_rw_hi) ? 64 : n >= (1ull << g_rw_lo) ? 16 : 4;
}
// Long-row products: k_spmv_pipe, 16 entries per lane per round (round 3: 256^3 SpMV
// 6.26 -> 5.46 s against the round-2 lane kernel; 8 per lane 5.64 s, 4: 6.98 s, 12:
// 7.95 s -- tools/ab_setup.py, r03m) -- except 8 for 4 rows per wavefront (round 4, per
// shape: RW=4 2041 -> 1580 ms and its list form 400 -> 309 ms per setup, half the
// registers, twice the wavefronts in flight on the coarse levels' few long rows; RW=16
// with 8 per lane: 2604 -> 2804 ms, RW=64 with 8: 723 -> 1132 ms, 8 rows x 8 in place of
// RW=16: 2639 -> 2727 ms; the RW 4 / 16 boundary at 2^16 rows stays: 2^18 / 2^20 /
// everywhere RW=4 measured slower, profiles/r04/ab_spmv_per).  The round-2
// lane kernel, the contiguous-chunk kernel, nontemporal loads and the fused selection /
// column-sum variants measured slower and were removed in round 4.
#define PAIR_LAUNCH(LIST, n_, list_, x_, z_, al, y_, be, f_, ml_)                             \
  do {                                                                                        \
    if (rw_ == 64)                                                                            \
      k_spmv_pair<LIST, 64, 16><<<gp_, 256, 0, amgd_s()>>>(M->ro, M->col, M->a, n_, list_, x_,  \
                                                    z_, al, y_, be, f_, ml_);                 \
    else if (rw_ == 16)                                                                       \
      k_spmv_pair<LIST, 16, 16><<<gp_, 256, 0, amgd_s()>>>(M->ro, M->col, M->a, n_, list_, x_,  \
                                                    z_, al, y_, be, f_, ml_);                 \
    else                                                                                      \
      k_spmv_pair<LIST, 4, 8><<<gp_, 256, 0, amgd_s()>>>(M->ro, M->col, M->a, n_, list_, x_,    \
                                                  z_, al, y_, be, f_, ml_);                   \
  } while (0)
#define LANE_LAUNCH(LIST, n_, list_, x_, z_, al, y_, be, f_, ml_)                             \
  do {                                                                                        \
    const int rw_ = lane_rw(n_);                                                              \
    amgd_route_hit(AMGD_R_SPMV_PIPE);                                                         \
    amgd_route_hit(rw_ == 64 ? AMGD_R_MV_RW64 : rw_ == 16 ? AMGD_R_MV_RW16 : AMGD_R_MV_RW4);   \
    const int gp_ = (int)std::min<uint64_t>(((uint64_t)(n_) + 4 * rw_ - 1) / (4 * rw_), 65536); \
    if ((x_) != nullptr && mv_pair(M)) {                                                      \
      amgd_route_hit(AMGD_R_MV_PAIR);                                                         \
      PAIR_LAUNCH(LIST, n_, list_, x_, z_, al, y_, be, f_, ml_);                               \
    } else if ((x_) != nullptr) {                                                             \
      if (rw_ == 64)                                                                          \
        k_spmv_pipe<LIST, 64, 16, true><<<gp_, 256, 0, amgd_s()>>>(M->ro, M->col, M->a, n_,     \
                                                 list_, x_, z_, al, y_, be, f_, ml_);           \
      else if (rw_ == 16)                                                                     \
        k_spmv_pipe<LIST, 16, 16, true><<<gp_, 256, 0, amgd_s()>>>(M->ro, M->col, M->a, n_,     \
                                                 list_, x_, z_, al, y_, be, f_, ml_);           \
      else                                                                                    \
        k_spmv_pipe<LIST, 4, 8, true><<<gp_, 256, 0, amgd_s()>>>(M->ro, M->col, M->a, n_,       \
                                                list_, x_, z_, al, y_, be, f_, ml_);            \
    } else {                                                                                  \
      if (rw_ == 64)                                                                          \
        k_spmv_pipe<LIST, 64, 16, false><<<gp_, 256, 0, amgd_s()>>>(M->ro, M->col, M->a, n_,    \
                                                  list_, x_, z_, al, y_, be, f_, ml_);          \
      else if (rw_ == 16)                                                                     \
        k_spmv_pipe<LIST, 16, 16, false><<<gp_, 256, 0, amgd_s()>>>(M->ro, M->col, M->a, n_,    \
                                                  list_, x_, z_, al, y_, be, f_, ml_);          \
      else                                                                                    \
        k_spmv_pipe<LIST, 4, 8, false><<<gp_, 256, 0, amgd_s()>>>(M->ro, M->col, M->a, n_,      \
                                                 list_, x_, z_, al, y_, be, f_, ml_);           \
    }                                                                                         \
  } while (0)
// ordered sums (x == nullptr) or products of the listed rows only (rows longer than
// maxlen are skipped: k_rows_exact does them)
__global__ __launch_bounds__(256) void k_spmv_wave_list(const uint64_t *ro, const uint32_t *col,
                                                        const double *a, const uint32_t *list,
                                                        uint32_t n, const double *x, double *z,
                                                        uint32_t maxlen) {
  __shared__ double buf[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint64_t r = (uint64_t)blockIdx.x * 4 + w; r < n; r += (uint64_t)gridDim.x * 4) {
    const uint32_t i = list[r];
    if (ro[i + 1] - ro[i] > maxlen) continue;
    const double t = wave_row_sum(col, a, x, ro[i], ro[i + 1], buf[w], lane);
    if (lane == 0) z[i] = t;
  }
}
// the listed rows longer than maxlen, appended to out (count in *cnt)
__global__ void k_list_long(const uint64_t *ro, const uint32_t *list, uint32_t n, uint32_t maxlen,
                            uint32_t *out, unsigned *cnt) {
  GRID_STRIDE(r, n) {
    const uint32_t i = list[r];
    if (ro[i + 1] - ro[i] > maxlen) out[atomicAdd(cnt, 1u)] = i;
  }
}
extern "C" void amgd_rows_exact(const uint64_t *ro, const uint32_t *col, const double *a,
                                const double *x, const uint32_t *list, const unsigned *nlist,
                                uint32_t nmax, uint64_t max_entries, double *z);
// Outlier rows (the orphan coarse point's column of find_support's R: 10^4 - 10^5
// entries among rows of ~10) take the grid-wide exact scan (amgd_rt.hip k_seg_*)
// instead of one lane / wave adding them one by one while the rest of the chip idles.
// By default a row is an outlier past max(SPMV_LONG, 16 x the matrix's mean row):
// where every row is long (coarse levels of a 3D Poisson hierarchy, means of 10^3 -
// 10^4) the lane kernels keep the whole chip busy and the per-row block walk of the
// segmented scan would be far slower.  AMGD_MV_LONG / amgd_spmv_set_long (tests) force
// an absolute threshold (0: never).
#define SPMV_LONG 4096
static int64_t g_mv_long = -1;    // -1: environment or automatic, -2: automatic
extern "C" void amgd_spmv_set_long(int64_t n) { g_mv_long = n; }
static uint32_t mv_long(const dcsr *M) {
  if (g_mv_long == -1) g_mv_long = sl_env("AMGD_MV_LONG", -2);
  if (g_mv_long == 0) return 0xffffffffu;
  if (g_mv_long > 0) return (uint32_t)g_mv_long;
  const uint64_t mean = M->rn ? M->nnz / M->rn : 0;
  return (uint32_t)std::min<uint64_t>(0xfffffffeu, std::max<uint64_t>(SPMV_LONG, 16 * mean));
}
extern "C" void amgd_spmv_rows(const dcsr *M, const uint32_t *list, uint32_t n, const double *x,
                               double *z) {
  if (!n) return;
  const uint32_t ml = mv_long(M);
  if (ml != 0xffffffffu && M->nnz > ml && amgd_max_row_len(M) > ml) {
    uint32_t *ll = (uint32_t *)amgd_alloc((size_t)n * 4 + 16);
    unsigned *cnt = (unsigned *)(ll + n);
    amgd_memset(cnt, 0, 4);
    amgd_route_hit(AMGD_R_MV_LONG);
    k_list_long<<<grid_for(n), 256, 0, amgd_s()>>>(M->ro, list, n, ml, ll, cnt);
    amgd_rows_exact(M->ro, M->col, M->a, x, ll, cnt, std::min<uint64_t>(n, M->nnz / (ml + 1) + 1),
                    M->nnz, z);
    amgd_free(ll);
  }
  if ((int64_t)n < sl_min_list()) {          // too few rows to fill the chip one row per lane
    int g = (int)std::min<uint64_t>(((uint64_t)n + 3) / 4, 65536);
    k_spmv_wave_list<<<g, 256, 0, amgd_s()>>>(M->ro, M->col, M->a, list, n, x, z, ml);
    KCHECK();
    return;
  }
  LANE_LAUNCH(true, n, list, x, z, 0.0, nullptr, 1.0, nullptr, ml);
  KCHECK();
}
// amgd_spmv_amax: z = M x plus, per row, the global entry index of its first largest product
// (find_support's selection, fused into the w = R' rs product of a full sweep).  Returns 1
// when the lane kernel produced them, 0 when the product took another kernel (short rows,
// few rows, a sharded product, an unaligned view): the caller selects the old way then.
static uint64_t *g_amx = nullptr;
static int g_amx_done = 0;
static void spmv_impl(const dcsr *M, const double *x, double *z, double alpha, const double *y,
                      double beta, const uint8_t *f);
extern "C" int amgd_spmv_amax(const dcsr *M, const double *x, double *z, uint64_t *amx) {
  g_amx = amx;
  g_amx_done = 0;
  amgd_spmv(M, x, z, 0.0, nullptr, 1.0, nullptr);
  g_amx = nullptr;
  KCHECK();
  return g_amx_done;
}
// algorithmic bytes of the event-timed (timer slot 1) lane-kernel products: each entry's
// column + value once, x gathered once per entry, row offsets, z (and y, f) once per row
// g_mv_bytes_strict: the same with x read once (8 B per column), the minimum any
// kernel must move -- the roofline's algorithmic bytes
static uint64_t g_mv_bytes = 0, g_mv_bytes_strict = 0, g_mv_launches = 0;
static uint64_t g_rw_bytes[3], g_rw_launches[3];      // per shape RW 4 / 16 / 64 (timer slots 2..4)
extern "C" void amgd_spmv_rw_counts(uint64_t *bytes, uint64_t *launches) {
  for (int i = 0; i < 3; i++) { bytes[i] = g_rw_bytes[i]; launches[i] = g_rw_launches[i]; }
}
extern "C" uint64_t amgd_spmv_bytes(void) { return g_mv_bytes; }
extern "C" uint64_t amgd_spmv_bytes_strict(void) { return g_mv_bytes_strict; }
extern "C" uint64_t amgd_spmv_launches(void) { return g_mv_launches; }
extern "C" void amgd_spmv_bytes_reset(void) {
  g_mv_bytes = g_mv_bytes_strict = g_mv_launches = 0;
  for (int i = 0; i < 3; i++) g_rw_bytes[i] = g_rw_launches[i] = 0;
}
// AMGD_MVLOG=1: one line per whole-matrix SpMV (rows, nnz, kernel, time, effective GB/s)
extern "C" void amgd_spmv(const dcsr *M, const double *x, double *z, double alpha, const double *y,
                          double beta, const uint8_t *f) {
  static int mvlog = -1;
  if (mvlog < 0) mvlog = getenv("AMGD_MVLOG") != nullptr;
  if (!mvlog) { spmv_impl(M, x, z, alpha, y, beta, f); return; }
  amgd_sync();
  const double t0 = amgd_wtime();
  spmv_impl(M, x, z, alpha, y, beta, f);
  amgd_sync();
  const double ms = (amgd_wtime() - t0) * 1e3;
  const int64_t slm = sl_min_whole();
  const char *k = M->nnz >= 32ull * M->rn ? ((int64_t)M->rn >= slm ? "lane" : "wave") : "stream";
  const MvTab *tb = x ? mv_tab_find(M) : nullptr;
  if (tb) fprintf(stderr, "spmvtab rw %d tr %u tiles %u direct %u\n", tb->rw, tb->TR, tb->ntiles, tb->ndirect);
  fprintf(stderr, "spmv %u x %u nnz %lu %s x%d %.3f ms %.0f GB/s\n", M->rn, M->cn,
          (unsigned long)M->nnz, k, x ? 1 : 0, ms,
          (12.0 * M->nnz + 16.0 * M->rn + (x ? 8.0 * M->nnz : 0.0)) / (ms * 1e6));
}
// Multi-GPU: a whole-matrix long-row product of >= MV_SHARD_MIN entries is split into
// contiguous row ranges of equal nnz (the row offsets are the work prefix); each rank
// runs the lane kernel on its rows (same per-row ordered sums, so the same bits) and
// one in-place allgatherv of z (8 B per row, >= 32 entries per row were read for it)
// completes the vector on every rank.  find_support's sweeps re-multiply the same
// pattern hundreds of times (removed entries are zeroed in place), so the split of a
// (row offsets, rows, nnz) triple is cached: no host sync beyond the allgatherv.  An
// entry is dropped when its row-offset buffer is freed (amgd_free), so a hit is always
// the same live matrix: every rank, running the same sequence of matrices, hits and
// misses alike and uses the same split (each rank's arena addresses differ, so a
// stale address match could otherwise differ between ranks and mismatch the
// allgatherv ranges).
#define MV_SHARD_MIN (1ull << 24)
struct MvSplit { const uint64_t *ro; uint32_t rn; uint64_t nnz; std::vector<uint32_t> split; std::vector<uint64_t> pre; };
static std::vector<MvSplit> g_mv_split;
// Longest row of a matrix whose pattern a caller holds fixed over a loop (find_support's
// R and R': hundreds of sweeps change values only): amgd_rowmax_pin computes it once,
// amgd_rowmax_unpin drops it (and so does freeing the row-offset buffer).  The long-row
// (outlier) paths -- a pick kernel plus the grid-wide scan, up to five launches per call
// -- are skipped when no row of a pinned matrix is long.  An unpinned matrix reports
// UINT32_MAX: the long-row paths run as before.
struct RowMax { const uint64_t *ro; uint32_t rn; uint64_t nnz; uint32_t mx; };
static std::vector<RowMax> g_rowmax;
__global__ void k_row_max(const uint64_t *ro, uint32_t rn, unsigned *mx) {
  unsigned m = 0;
  GRID_STRIDE(i, rn) m = max(m, (unsigned)(ro[i + 1] - ro[i]));
  for (int o = 32; o; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o, 64));
  if ((threadIdx.x & 63) == 0 && m) atomicMax(mx, m);
}
// AMGD_MVSTAT=1 (analysis): for a pinned long-row matrix, the x locality of its products --
// per block of B consecutive rows, the distinct columns and distinct 128-B lines of x they
// gather, against the entries (a sample of the blocks); and per 64-entry chunk of a row (one
// gather instruction of the lane kernels) the distinct lines.  Host-side, stderr.
#include <algorithm>
static void mv_pattern_stats(const dcsr *M) {
  static int on = -1;
  if (on < 0) { const char *e = getenv("AMGD_MVSTAT"); on = e && *e ? atoi(e) : 0; }
  if (!on || M->rn == 0 || M->nnz < 32ull * M->rn) return;
  amgd_sync();
  std::vector<uint64_t> ro(M->rn + 1);
  std::vector<uint32_t> col(M->nnz);
  HIPCK(hipMemcpy(ro.data(), M->ro, (M->rn + 1) * 8, hipMemcpyDeviceToHost));
  HIPCK(hipMemcpy(col.data(), M->col, M->nnz * 4, hipMemcpyDeviceToHost));
  double chunk_lines = 0, chunks = 0;
  for (uint32_t i = 0; i < M->rn; i += 61) {
    for (uint64_t k = ro[i]; k < ro[i + 1]; k += 64) {
      const uint64_t e = std::min(ro[i + 1], k + 64);
      uint32_t last = 0xffffffffu, d = 0;
      for (uint64_t q = k; q < e; q++) { const uint32_t l = col[q] >> 4; if (l != last) { d++; last = l; } }
      chunk_lines += d; chunks++;
    }
  }
  fprintf(stderr, "mvstat rn %u cn %u nnz %lu mean %.1f | lines per 64-entry chunk %.1f", M->rn, M->cn,
          (unsigned long)M->nnz, (double)M->nnz / M->rn, chunks ? chunk_lines / chunks : 0.0);
  std::vector<uint32_t> tmp;
  for (uint32_t B : {16u, 64u, 256u, 1024u}) {
    double ent = 0, dist = 0, lines = 0, blocks = 0, span = 0;
    const uint32_t nb = (M->rn + B - 1) / B, step = std::max<uint32_t>(1, nb / 400);
    for (uint32_t b = 0; b < nb; b += step) {
      const uint32_t r0 = b * B, r1 = std::min(M->rn, r0 + B);
      tmp.assign(col.begin() + ro[r0], col.begin() + ro[r1]);
      if (tmp.empty()) continue;
      std::sort(tmp.begin(), tmp.end());
      uint32_t d = 0, l = 0, lastc = 0xffffffffu, lastl = 0xffffffffu;
      for (uint32_t c : tmp) { if (c != lastc) { d++; lastc = c; } if ((c >> 4) != lastl) { l++; lastl = c >> 4; } }
      ent += tmp.size(); dist += d; lines += l; blocks++; span += tmp.back() - tmp.front();
    }
    if (blocks)
      fprintf(stderr, " | B%u: ent %.0f distinct %.0f (%.2f/ent) lines %.0f span %.0f", B, ent / blocks, dist / blocks,
              dist / ent, lines / blocks, span / blocks);
  }
  fprintf(stderr, "\n");
}
extern "C" void amgd_rowmax_pin(const dcsr *M) {
  for (const RowMax &e : g_rowmax)
    if (e.ro == M->ro && e.rn == M->rn && e.nnz == M->nnz) return;
  mv_pattern_stats(M);
  mv_tab_build(M);
  unsigned h = 0;
  if (M->rn) {
    unsigned *d = (unsigned *)amgd_alloc(4);
    amgd_memset(d, 0, 4);
    k_row_max<<<grid_for(M->rn), 256, 0, amgd_s()>>>(M->ro, M->rn, d);
    amgd_d2h(&h, d, 4);
    amgd_free(d);
  }
  g_rowmax.push_back({M->ro, M->rn, M->nnz, h});
}
extern "C" void amgd_rowmax_unpin(const dcsr *M) {
  mv_tab_drop(M->ro);
  for (size_t q = 0; q < g_rowmax.size();)
    if (g_rowmax[q].ro == M->ro) g_rowmax.erase(g_rowmax.begin() + q);
    else q++;
}
extern "C" uint32_t amgd_max_row_len(const dcsr *M) {
  for (const RowMax &e : g_rowmax)
    if (e.ro == M->ro && e.rn == M->rn && e.nnz == M->nnz) return e.mx;
  return 0xffffffffu;
}
void amgd_spmv_split_forget(const void *ro) {
  if (!g_mvtab.empty()) mv_tab_drop(ro);
  for (size_t q = 0; q < g_rowmax.size();)
    if ((const void *)g_rowmax[q].ro == ro) g_rowmax.erase(g_rowmax.begin() + q);
    else q++;
  if (g_mv_split.empty()) return;
  for (size_t q = 0; q < g_mv_split.size();)
    if ((const void *)g_mv_split[q].ro == ro) g_mv_split.erase(g_mv_split.begin() + q);
    else q++;
}
void amgd_spmv_split_clear(void) {
  g_mv_split.clear();
  g_rowmax.clear();
  while (!g_mvtab.empty()) mv_tab_drop(g_mvtab.back().ro);
}
static uint64_t g_mv_shard_calls = 0;
extern "C" uint64_t amgd_spmv_shard_calls(void) { return g_mv_shard_calls; }   // (test API)
static bool spmv_sharded(const dcsr *M0, const double *x, double *z, double alpha, const double *y,
                         double beta, const uint8_t *f) {
  const int N = amgd_nshards();
  if (N <= 1 || M0->rn < 64u * (uint32_t)N || !amgd_shard_worth(M0->nnz, MV_SHARD_MIN)) return false;
  const MvSplit *sp = nullptr;
  for (const MvSplit &e : g_mv_split)
    if (e.ro == M0->ro && e.rn == M0->rn && e.nnz == M0->nnz && (int)e.split.size() == N + 1) sp = &e;
  if (!sp) {
    MvSplit e{M0->ro, M0->rn, M0->nnz, std::vector<uint32_t>(N + 1), std::vector<uint64_t>(N + 1)};
    amgd_shard_split(M0->ro, M0->rn, e.split.data());
    amgd_gather_u64_at(M0->ro, e.split.data(), N + 1, e.pre.data());
    if (g_mv_split.size() >= 16) g_mv_split.erase(g_mv_split.begin());
    g_mv_split.push_back(std::move(e));
    sp = &g_mv_split.back();
  }
  g_mv_shard_calls++;
  int fs, ls;
  amgd_my_shards(&fs, &ls);
  amgd_timer_start(1);
  for (int q = fs; q < ls; q++) {
    const uint32_t r0 = sp->split[q], n = sp->split[q + 1] - r0;
    if (!n) continue;
    dcsr Ms = *M0;
    Ms.ro = M0->ro + r0;                       // absolute offsets: rows r0 .. r0+n
    const dcsr *M = &Ms;
    LANE_LAUNCH(false, n, (const uint32_t *)nullptr, x, z + r0, alpha, y ? y + r0 : nullptr, beta,
                f ? f + r0 : nullptr, 0xffffffffu);
    const uint64_t rest = 16ull * n + 8 + (y && alpha != 0.0 ? 8ull * n : 0) + (f ? (uint64_t)n : 0);
    g_mv_bytes += 12 * (sp->pre[q + 1] - sp->pre[q]) + (x ? 8 * (sp->pre[q + 1] - sp->pre[q]) : 0) + rest;
    g_mv_bytes_strict += 12 * (sp->pre[q + 1] - sp->pre[q]) + (x ? 8ull * M0->cn : 0) + rest;
    g_mv_launches++;
  }
  amgd_timer_stop(1);
  KCHECK();
  std::vector<uint64_t> off(N + 1);
  for (int s = 0; s <= N; s++) off[s] = 8ull * sp->split[s];
  void *b = z;
  amgd_allgatherv(1, &b, off.data());
  return true;
}
static void spmv_impl(const dcsr *M, const double *x, double *z, double alpha, const double *y,
                      double beta, const uint8_t *f) {
  if (M->rn == 0) return;
  if (M->nnz >= 32ull * M->rn && spmv_sharded(M, x, z, alpha, y, beta, f)) return;
  const int64_t sl_min = sl_min_whole();
  if (M->nnz >= 32ull * M->rn && (int64_t)M->rn >= sl_min) {
    const int rwi = lane_rw(M->rn) == 64 ? 2 : lane_rw(M->rn) == 16 ? 1 : 0;
    amgd_timer_start2(1, 2 + rwi);             // roofline: whole-matrix long-row products,
    const MvTab *tb = x ? mv_tab_find(M) : nullptr;
    if (tb) {                                  // tabled gathers (pinned pattern)
      const bool amx = g_amx && alpha == 0.0 && beta == 1.0 && !f;
      amgd_route_hit(AMGD_R_SPMV_PIPE);
      amgd_route_hit(AMGD_R_MV_TAB);
      amgd_route_hit(rwi == 2 ? AMGD_R_MV_RW64 : rwi == 1 ? AMGD_R_MV_RW16 : AMGD_R_MV_RW4);
      mv_tab_launch(tb, M, x, z, alpha, y, beta, f, amx ? g_amx : nullptr);
      if (amx) g_amx_done = 1;
    } else if (g_amx && x && alpha == 0.0 && beta == 1.0 && !f && mv_pair(M)) {
      const int rw_ = lane_rw(M->rn);          // + each row's first largest product
      const int gp_ = (int)std::min<uint64_t>(((uint64_t)M->rn + 4 * rw_ - 1) / (4 * rw_), 65536);
      amgd_route_hit(AMGD_R_SPMV_PIPE);
      amgd_route_hit(AMGD_R_MV_PAIR);
      amgd_route_hit(rw_ == 64 ? AMGD_R_MV_RW64 : rw_ == 16 ? AMGD_R_MV_RW16 : AMGD_R_MV_RW4);
      if (rw_ == 64)
        k_spmv_pair_amx<64, 16><<<gp_, 256, 0, amgd_s()>>>(M->ro, M->col, M->a, M->rn, x, z, g_amx);
      else if (rw_ == 16)
        k_spmv_pair_amx<16, 16><<<gp_, 256, 0, amgd_s()>>>(M->ro, M->col, M->a, M->rn, x, z, g_amx);
      else
        k_spmv_pair_amx<4, 8><<<gp_, 256, 0, amgd_s()>>>(M->ro, M->col, M->a, M->rn, x, z, g_amx);
      g_amx_done = 1;
    } else {
      LANE_LAUNCH(false, M->rn, (const uint32_t *)nullptr, x, z, alpha, y, beta, f, 0xffffffffu);
    }
    amgd_timer_stop2(1, 2 + rwi);              // all shapes and per shape (RW 4 / 16 / 64)
    const uint64_t rest = 16ull * M->rn + 8 + (y && alpha != 0.0 ? 8ull * M->rn : 0) + (f ? (uint64_t)M->rn : 0);
    g_mv_bytes += 12 * M->nnz + (x ? 8 * M->nnz : 0) + rest;
    g_mv_bytes_strict += 12 * M->nnz + (x ? 8ull * M->cn : 0) + rest;
    g_mv_launches++;
    g_rw_bytes[rwi] += 12 * M->nnz + (x ? 8ull * M->cn : 0) + rest;
    g_rw_launches[rwi]++;
  } else if (M->nnz >= 32ull * M->rn) {
    int g = (int)std::min<uint64_t>((M->rn + 3) / 4, 65536);
    k_spmv_wave<<<g, 256, 0, amgd_s()>>>(M->ro, M->col, M->a, M->rn, x, z, alpha, y, beta, f);
  } else {
    int g = (int)std::min<uint64_t>((M->rn + SPMV_ROWS - 1) / SPMV_ROWS, 16384);
    k_spmv<<<g, 256, 0, amgd_s()>>>(M->ro, M->col, M->a, M->rn, x, z, alpha, y, beta, f);
  }
  KCHECK();
}
// rows-filtered SpMV (k_spmv arithmetic at any row length): z_i = (M x)_i * f_i on
// the 256-row blocks holding a row i with fs[i] - fb <= fr
extern "C" void amgd_spmv_filt(const dcsr *M, const double *x, double *z, const uint8_t *f,
                               const uint32_t *fs, uint32_t fb, uint32_t fr) {
  if (M->rn == 0) return;
  int g = (int)std::min<uint64_t>((M->rn + SPMV_ROWS - 1) / SPMV_ROWS, 16384);
  k_spmv<<<g, 256, 0, amgd_s()>>>(M->ro, M->col, M->a, M->rn, x, z, 0.0, nullptr, 1.0, f, fs, fb,
                                  fr);
  KCHECK();
}
// z = M^T x: rows of Mt are columns of M with rows ascending -> ordered gather
extern "C" void amgd_spmvt(const dcsr *Mt, const double *x, double *z) {
  amgd_spmv(Mt, x, z, 0.0, nullptr, 1.0, nullptr);
}
__global__ void k_rowsum(const uint64_t *ro, const double *a, uint32_t rn, double *z) {
  GRID_STRIDE(i, rn) {
    double t = 0.0;
    for (uint64_t k = ro[i]; k < ro[i + 1]; k++) t += a[k];
    z[i] = t;
  }
}
extern "C" void amgd_colsum(const dcsr *Mt, double *z) {
  amgd_spmv(Mt, nullptr, z, 0.0, nullptr, 1.0, nullptr);   // t = sum of a, row order
}

// ---------------------------------------------------------------------------
// diagonal helpers (amg_setup.c:3363, 3389)
// ---------------------------------------------------------------------------
__global__ void k_diag(const uint64_t *ro, const uint32_t *col, const double *a, uint32_t rn,
                       double *D) {
  GRID_STRIDE(i, rn) {
    double d = 0.0;
    for (uint64_t k = ro[i]; k < ro[i + 1]; k++)
      if (col[k] == i) { d = a[k]; break; }
    D[i] = d;
  }
}
// long rows (coarse levels, 10^2 - 10^4 entries): one wavefront per row, the first
// entry with col == i found 64 entries at a time by ballot (same first match)
__global__ void k_diag_wave(const uint64_t *ro, const uint32_t *col, const double *a, uint32_t rn,
                            double *D) {
  const int lane = threadIdx.x & 63;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < rn;
       i += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
    const uint64_t k1 = ro[i + 1];
    double d = 0.0;
    for (uint64_t k0 = ro[i]; k0 < k1; k0 += 64) {
      const uint64_t k = k0 + lane;
      const unsigned long long m = __ballot(k < k1 && col[k] == (uint32_t)i);
      if (m) { d = a[k0 + __ffsll((long long)m) - 1]; break; }
    }
    if (lane == 0) D[i] = d;
  }
}
extern "C" void amgd_diag(const dcsr *A, double *D) {
  if (A->rn && A->nnz >= 16ull * A->rn)
    k_diag_wave<<<grid_for((uint64_t)A->rn * 64, 256, 16384), 256, 0, amgd_s()>>>(A->ro, A->col, A->a,
                                                                                 A->rn, D);
  else if (A->rn)
    k_diag<<<grid_for(A->rn), 256, 0, amgd_s()>>>(A->ro, A->col, A->a, A->rn, D);
  KCHECK();
}
__global__ void k_diag_op(const uint64_t *ro, const uint32_t *col, double *a, uint32_t rn,
                          const double *D, int op) {
  GRID_STRIDE(i, rn) {
    for (uint64_t k = ro[i]; k < ro[i + 1]; k++) {
      if (op == AMGD_DPLUS) { if (col[k] == i) { a[k] = a[k] + D[i]; break; } }
      else if (op == AMGD_DMINUS) { if (col[k] == i) { a[k] = a[k] - D[i]; break; } }
      else if (op == AMGD_DMULT) a[k] = a[k] * D[i];
      else a[k] = a[k] * D[col[k]];
    }
  }
}
// G lanes per row (coalesced on long rows).  op: DPLUS / DMINUS touch the first
// diagonal entry only (diagcsr_op, amg_setup.c:3389); DMULT a*=Dl[i]; MULTD a*=Dl[col];
// SCALE2 a = (a*Dl[i])*Dr[col]; SCALE_ABS a = |a*Dl[i]|*Dr[col]; SCALE2_ABS a = |(a*Dl[i])*Dr[col]|
// -- each the reference's sequence of separate passes, fused
template <int G>
__global__ __launch_bounds__(256) void k_diag_op_g(const uint64_t *ro, const uint32_t *col,
                                                   double *a, uint32_t rn, const double *Dl,
                                                   const double *Dr, int op) {
  const uint32_t sub = threadIdx.x & (G - 1);
  const uint64_t g0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) / G;
  const uint64_t gs = (uint64_t)gridDim.x * (256 / G);
  for (uint64_t i = g0; i < rn; i += gs) {
    const uint64_t k0 = ro[i], k1 = ro[i + 1];
    if (op == AMGD_DPLUS || op == AMGD_DMINUS) {
      uint64_t first = ~0ull;
      for (uint64_t k = k0 + sub; k < k1; k += G)
        if (col[k] == i) { first = k; break; }
#pragma unroll
      for (int o = G / 2; o > 0; o >>= 1) {
        unsigned long long u = __shfl_xor((unsigned long long)first, o, 64);
        first = u < first ? u : first;
      }
      if (sub == 0 && first != ~0ull)
        a[first] = op == AMGD_DPLUS ? a[first] + Dl[i] : a[first] - Dl[i];
      continue;
    }
    const double di = op == AMGD_SCALE_ABS_T ? 0.0 : Dl[i];   // (_T: Dl is per column)
    for (uint64_t k = k0 + sub; k < k1; k += G) {
      double v = a[k];
      switch (op) {
        case AMGD_DMULT: v = v * di; break;
        case AMGD_MULTD: v = v * Dl[col[k]]; break;
        case AMGD_SCALE2: v = (v * di) * Dr[col[k]]; break;
        case AMGD_SCALE_ABS: v = fabs(v * di) * Dr[col[k]]; break;
        case AMGD_SCALE_ABS_T: v = fabs(v * Dl[col[k]]) * Dr[i]; break;
        default: v = fabs((v * di) * Dr[col[k]]); break;
      }
      a[k] = v;
    }
  }
}
static int row_lanes(uint64_t nnz, uint64_t rn) {
  uint64_t avg = rn ? (nnz + rn - 1) / rn : 1;
  int G = 4;
  while (G < 64 && (uint64_t)G * 2 <= avg) G <<= 1;
  return G;
}
extern "C" void amgd_diag_op2(dcsr *A, const double *Dl, const double *Dr, int op) {
  if (!A->rn) return;
  const int G = row_lanes(A->nnz, A->rn);
  const int gb = grid_for((uint64_t)A->rn * G, 256, 65536);
  switch (G) {
    case 4: k_diag_op_g<4><<<gb, 256, 0, amgd_s()>>>(A->ro, A->col, A->a, A->rn, Dl, Dr, op); break;
    case 8: k_diag_op_g<8><<<gb, 256, 0, amgd_s()>>>(A->ro, A->col, A->a, A->rn, Dl, Dr, op); break;
    case 16: k_diag_op_g<16><<<gb, 256, 0, amgd_s()>>>(A->ro, A->col, A->a, A->rn, Dl, Dr, op); break;
    case 32: k_diag_op_g<32><<<gb, 256, 0, amgd_s()>>>(A->ro, A->col, A->a, A->rn, Dl, Dr, op); break;
    default: k_diag_op_g<64><<<gb, 256, 0, amgd_s()>>>(A->ro, A->col, A->a, A->rn, Dl, Dr, op); break;
  }
  KCHECK();
}
extern "C" void amgd_diag_op(dcsr *A, const double *D, int op) { amgd_diag_op2(A, D, nullptr, op); }
__global__ void k_vals(double *a, uint64_t n, int op, double s) {
  GRID_STRIDE(k, n) {
    double v = a[k];
    if (op == 0) v = fabs(v);
    else if (op == 1) v = v * v;
    else v = v * s;
    a[k] = v;
  }
}
extern "C" void amgd_vals_abs(dcsr *A) { if (A->nnz) k_vals<<<grid_for(A->nnz), 256, 0, amgd_s()>>>(A->a, A->nnz, 0, 0); }
extern "C" void amgd_vals_sqr(dcsr *A) { if (A->nnz) k_vals<<<grid_for(A->nnz), 256, 0, amgd_s()>>>(A->a, A->nnz, 1, 0); }
extern "C" void amgd_vals_scale(dcsr *A, double s) { if (A->nnz) k_vals<<<grid_for(A->nnz), 256, 0, amgd_s()>>>(A->a, A->nnz, 2, s); }

// s_i = 1 / sum_j (a_ij*a_ij), left to right (amg_setup.c:200-220)
__global__ void k_rowsum_sq_inv(const uint64_t *ro, const double *a, uint32_t rn, double *s) {
  GRID_STRIDE(i, rn) {
    double t = 0.0;
    for (uint64_t k = ro[i]; k < ro[i + 1]; k++) t += a[k] * a[k];
    s[i] = 1. / t;
  }
}
extern "C" void amgd_rowsum_sq_inv(const dcsr *A, double *s) {
  if (A->rn) k_rowsum_sq_inv<<<grid_for(A->rn), 256, 0, amgd_s()>>>(A->ro, A->a, A->rn, s);
  KCHECK();
}

// ---------------------------------------------------------------------------
// mpm (amg_setup.c:1684): X = alpha*A + beta*B, sorted merge per row; an
// entry present in both whose sum is exactly 0 is dropped.
// mxmpoint (amg_setup.c:1807): X = A.*B on the intersection (zeros kept).
// Count pass + scan + fill pass, one thread per row.
// ---------------------------------------------------------------------------
#define MPM_LONG 64   // rows with na + nb >= MPM_LONG and no repeated column: k_mpm_wave
template <bool FILL>
__global__ void k_mpm(const uint64_t *aro, const uint32_t *acol, const double *aa,
                      const uint64_t *bro, const uint32_t *bcol, const double *ba, uint32_t rn,
                      double alpha, double beta, uint64_t *cnt, const uint64_t *xro,
                      uint32_t *xcol, double *xa, const uint8_t *longrow = nullptr) {
  GRID_STRIDE(i, rn) {
    if (longrow && longrow[i]) continue;
    uint64_t ja = aro[i], ea = aro[i + 1], jb = bro[i], eb = bro[i + 1];
    uint64_t o = FILL ? xro[i] : 0, c = 0;
    while (ja < ea || jb < eb) {
      uint32_t col;
      double v;
      bool emit = true;
      if (ja < ea && jb < eb) {
        uint32_t ca = acol[ja], cb = bcol[jb];
        if (ca == cb) {
          col = ca;
          v = FILL ? alpha * aa[ja] + beta * ba[jb] : 0.0;
          if (FILL) emit = v != 0.0;
          else emit = (alpha * aa[ja] + beta * ba[jb]) != 0.0;
          ja++; jb++;
        } else if (ca < cb) {
          col = ca; v = FILL ? alpha * aa[ja] : 0.0; ja++;
        } else {
          col = cb; v = FILL ? beta * ba[jb] : 0.0; jb++;
        }
      } else if (ja == ea) {
        col = bcol[jb]; v = FILL ? beta * ba[jb] : 0.0; jb++;
      } else {
        col = acol[ja]; v = FILL ? alpha * aa[ja] : 0.0; ja++;
      }
      if (emit) {
        if (FILL) { xcol[o] = col; xa[o] = v; o++; }
        c++;
      }
    }
    if (!FILL) cnt[i] = c;
  }
}
// Long rows: one wavefront per row, every entry placed by rank instead of a
// sequential merge.  With strictly increasing columns in both rows, A entry p
// (column c) lands at p + #B<c - #matched<c - #dropped<c and an unmatched B entry
// q at q + #A<c - (same two counts); #B<c / #A<c come from a binary search in
// the other row, the matched / dropped counts from wave prefix sums over the
// row's own entries (a matched pair is dropped when alpha*a + beta*b == 0, the
// sequential merge's test).  Values are the merge's own expressions.  A row with
// a repeated column is flagged and left to the sequential merge.
__device__ __forceinline__ uint32_t lower_bound_u32(const uint32_t *c, uint32_t n, uint32_t key) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (c[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}
__global__ __launch_bounds__(256) void k_mpm_flag(const uint64_t *aro, const uint32_t *acol,
                                                  const uint64_t *bro, const uint32_t *bcol,
                                                  uint32_t rn, uint8_t *longrow) {
  const int lane = threadIdx.x & 63;
  for (uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6; i < rn;
       i += (uint64_t)gridDim.x * 4) {
    const uint64_t ka = aro[i], na = aro[i + 1] - ka, kb = bro[i], nb = bro[i + 1] - kb;
    if (na + nb < MPM_LONG) {
      if (lane == 0) longrow[i] = 0;
      continue;
    }
    bool dup = false;
    for (uint64_t p = lane; p + 1 < na; p += 64) dup |= acol[ka + p] >= acol[ka + p + 1];
    for (uint64_t q = lane; q + 1 < nb; q += 64) dup |= bcol[kb + q] >= bcol[kb + q + 1];
    const bool anyd = __ballot(dup) != 0;
    if (lane == 0) longrow[i] = anyd ? 0 : 1;
  }
}
// The other row's columns are staged in LDS when they fit (MPM_LDS per wavefront): the
// binary searches then read LDS instead of issuing ~log2(n) dependent global loads each.
#define MPM_LDS 2048
template <bool FILL>
__global__ __launch_bounds__(256) void k_mpm_wave(const uint64_t *aro, const uint32_t *acol,
                                                  const double *aa, const uint64_t *bro,
                                                  const uint32_t *bcol, const double *ba,
                                                  uint32_t rn, double alpha, double beta,
                                                  const uint8_t *longrow, uint64_t *cnt,
                                                  const uint64_t *xro, uint32_t *xcol,
                                                  double *xa) {
  __shared__ uint32_t stage[4][MPM_LDS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  // the columns of a row [k, k + n) where the searches read them: LDS if they fit
  auto stage_cols = [&](const uint32_t *colv, uint64_t k, uint32_t n) -> const uint32_t * {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (n > MPM_LDS) return colv + k;
    for (uint32_t e = lane; e < n; e += 64) stage[w][e] = colv[k + e];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return stage[w];
  };
  for (uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6; i < rn;
       i += (uint64_t)gridDim.x * 4) {
    if (!longrow[i]) continue;
    const uint64_t ka = aro[i], kb = bro[i];
    const uint32_t na = (uint32_t)(aro[i + 1] - ka), nb = (uint32_t)(bro[i + 1] - kb);
    const uint64_t o = FILL ? xro[i] : 0;
    const uint32_t *sb = stage_cols(bcol, kb, nb);
    uint32_t cm = 0, cd = 0;                      // matched / dropped so far (A side)
    for (uint32_t p0 = 0; p0 < na; p0 += 64) {
      const uint32_t p = p0 + lane;
      bool has = p < na, m = false, d = false;
      uint32_t c = 0, bs = 0;
      double v = 0.0;
      if (has) {
        c = acol[ka + p];
        bs = lower_bound_u32(sb, nb, c);
        m = bs < nb && sb[bs] == c;
        if (m) {
          v = alpha * aa[ka + p] + beta * ba[kb + bs];
          d = !(v != 0.0);
        } else if (FILL) {
          v = alpha * aa[ka + p];
        }
      }
      const uint64_t bm = __ballot(m), bd = __ballot(d);
      if (FILL && has && !d) {
        const uint64_t pos = (uint64_t)p + bs - (cm + __popcll(bm & lt)) - (cd + __popcll(bd & lt));
        xcol[o + pos] = c;
        xa[o + pos] = v;
      }
      cm += __popcll(bm);
      cd += __popcll(bd);
    }
    if (!FILL) {
      if (lane == 0) cnt[i] = (uint64_t)na + nb - cm - cd;
      continue;
    }
    const uint32_t *sa = stage_cols(acol, ka, na);
    uint32_t bmc = 0, bdc = 0;                    // matched / dropped so far (B side)
    for (uint32_t q0 = 0; q0 < nb; q0 += 64) {
      const uint32_t q = q0 + lane;
      bool has = q < nb, m = false, d = false;
      uint32_t c = 0, as = 0;
      if (has) {
        c = bcol[kb + q];
        as = lower_bound_u32(sa, na, c);
        m = as < na && sa[as] == c;
        if (m) d = !((alpha * aa[ka + as] + beta * ba[kb + q]) != 0.0);
      }
      const uint64_t bm = __ballot(m), bd = __ballot(d);
      if (has && !m) {
        const uint64_t pos =
            (uint64_t)q + as - (bmc + __popcll(bm & lt)) - (bdc + __popcll(bd & lt));
        xcol[o + pos] = c;
        xa[o + pos] = beta * ba[kb + q];
      }
      bmc += __popcll(bm);
      bdc += __popcll(bd);
    }
  }
}
extern "C" dcsr *amgd_mpm(double alpha, const dcsr *A, double beta, const dcsr *B) {
  if (A->rn != B->rn || A->cn != B->cn) {
    fprintf(stderr, "omp_amg_amd: mpm dimension mismatch (%u x %u vs %u x %u)\n", A->rn, A->cn,
            B->rn, B->cn);
    abort();
  }
  hipStream_t s = amgd_s();
  // the wave kernel pays for rows averaging >= MPM_LONG / 4 entries
  const bool use_w = A->rn && (A->nnz + B->nnz) >= (uint64_t)A->rn * (MPM_LONG / 4);
  uint8_t *lr = nullptr;
  const int gw = (int)std::min<uint64_t>(((uint64_t)A->rn + 3) / 4, 65536);
  uint64_t *cnt = (uint64_t *)amgd_alloc(((size_t)A->rn + 1) * 8);
  if (use_w) {
    lr = (uint8_t *)amgd_alloc((size_t)A->rn + 1);
    k_mpm_flag<<<gw, 256, 0, s>>>(A->ro, A->col, B->ro, B->col, A->rn, lr);
    k_mpm_wave<false><<<gw, 256, 0, s>>>(A->ro, A->col, A->a, B->ro, B->col, B->a, A->rn, alpha,
                                         beta, lr, cnt, nullptr, nullptr, nullptr);
  }
  if (A->rn)
    k_mpm<false><<<grid_for(A->rn), 256, 0, s>>>(A->ro, A->col, A->a, B->ro, B->col, B->a, A->rn,
                                                  alpha, beta, cnt, nullptr, nullptr, nullptr, lr);
  KCHECK();
  uint64_t nz = amgd_scan_u64(cnt, A->rn);
  dcsr *X = (dcsr *)malloc(sizeof(dcsr));
  X->rn = A->rn; X->cn = A->cn; X->nnz = nz; X->ro = cnt;
  X->col = (uint32_t *)amgd_alloc(nz * 4 + 4);
  X->a = (double *)amgd_alloc_f64(nz * 8 + 8);
  if (use_w)
    k_mpm_wave<true><<<gw, 256, 0, s>>>(A->ro, A->col, A->a, B->ro, B->col, B->a, A->rn, alpha,
                                        beta, lr, nullptr, X->ro, X->col, X->a);
  if (A->rn)
    k_mpm<true><<<grid_for(A->rn), 256, 0, s>>>(A->ro, A->col, A->a, B->ro, B->col, B->a, A->rn,
                                                 alpha, beta, nullptr, X->ro, X->col, X->a, lr);
  KCHECK();
  if (lr) amgd_free(lr);
  return X;
}

template <bool FILL>
__global__ void k_pointwise(const uint64_t *aro, const uint32_t *acol, const double *aa,
                            const uint64_t *bro, const uint32_t *bcol, const double *ba,
                            uint32_t rn, uint64_t *cnt, const uint64_t *xro, uint32_t *xcol,
                            double *xa) {
  GRID_STRIDE(i, rn) {
    uint64_t ja = aro[i], ea = aro[i + 1], jb = bro[i], eb = bro[i + 1];
    uint64_t o = FILL ? xro[i] : 0, c = 0;
    while (ja < ea && jb < eb) {
      uint32_t ca = acol[ja], cb = bcol[jb];
      if (ca == cb) {
        if (FILL) { xcol[o] = ca; xa[o] = aa[ja] * ba[jb]; o++; }
        c++; ja++; jb++;
      } else if (ca < cb) ja++;
      else jb++;
    }
    if (!FILL) cnt[i] = c;
  }
}
// long rows (R0 .* W_skel on coarse levels: rows of 10^2 - 10^4 entries): one
// wavefront per row.  When both rows are strictly increasing (checked first, by the
// whole wave) the merge's output is the intersection in A's column order, so each
// lane locates a 64-entry chunk of A's row in B's row by bisection and the matches
// are placed by ballot prefix counts; otherwise lane 0 runs the sequential merge.
template <bool FILL>
__global__ void k_pointwise_wave(const uint64_t *aro, const uint32_t *acol, const double *aa,
                                 const uint64_t *bro, const uint32_t *bcol, const double *ba,
                                 uint32_t rn, uint64_t *cnt, const uint64_t *xro, uint32_t *xcol,
                                 double *xa) {
  const int lane = threadIdx.x & 63;
  const unsigned long long below = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < rn;
       i += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
    const uint64_t a0 = aro[i], a1 = aro[i + 1], b0 = bro[i], b1 = bro[i + 1];
    bool mono = true;
    for (uint64_t k = a0 + 1 + lane; k < a1; k += 64) mono = mono && acol[k] > acol[k - 1];
    for (uint64_t k = b0 + 1 + lane; k < b1; k += 64) mono = mono && bcol[k] > bcol[k - 1];
    mono = __ballot(!mono) == 0ull;
    uint64_t o = FILL ? xro[i] : 0, c = 0;
    if (!mono) {
      if (lane == 0) {
        uint64_t ja = a0, jb = b0;
        while (ja < a1 && jb < b1) {
          const uint32_t ca = acol[ja], cb = bcol[jb];
          if (ca == cb) {
            if (FILL) { xcol[o] = ca; xa[o] = aa[ja] * ba[jb]; o++; }
            c++; ja++; jb++;
          } else if (ca < cb) ja++;
          else jb++;
        }
        if (!FILL) cnt[i] = c;
      }
      continue;
    }
    for (uint64_t k0 = a0; k0 < a1; k0 += 64) {
      const uint64_t k = k0 + lane;
      bool hit = false;
      uint64_t jb = 0;
      if (k < a1 && b0 < b1) {
        const uint32_t ca = acol[k];
        uint64_t lo = b0, hi = b1;
        while (lo < hi) {
          const uint64_t mid = (lo + hi) >> 1;
          if (bcol[mid] < ca) lo = mid + 1;
          else hi = mid;
        }
        hit = lo < b1 && bcol[lo] == ca;
        jb = lo;
      }
      const unsigned long long m = __ballot(hit);
      if (FILL && hit) {
        const uint64_t q = o + __popcll(m & below);
        xcol[q] = acol[k];
        xa[q] = aa[k] * ba[jb];
      }
      o += __popcll(m);
      c += __popcll(m);
    }
    if (!FILL && lane == 0) cnt[i] = c;
  }
}
extern "C" dcsr *amgd_mxmpoint(const dcsr *A, const dcsr *B) {
  if (A->rn != B->rn || A->cn != B->cn) {
    fprintf(stderr, "omp_amg_amd: mxmpoint dimension mismatch\n");
    abort();
  }
  hipStream_t s = amgd_s();
  uint64_t *cnt = (uint64_t *)amgd_alloc(((size_t)A->rn + 1) * 8);
  const bool wave = A->nnz + B->nnz >= 32ull * A->rn;
  const int gw = grid_for((uint64_t)A->rn * 64, 256, 16384);
  if (A->rn && wave)
    k_pointwise_wave<false><<<gw, 256, 0, s>>>(A->ro, A->col, A->a, B->ro, B->col, B->a, A->rn, cnt,
                                               nullptr, nullptr, nullptr);
  else if (A->rn)
    k_pointwise<false><<<grid_for(A->rn), 256, 0, s>>>(A->ro, A->col, A->a, B->ro, B->col, B->a,
                                                        A->rn, cnt, nullptr, nullptr, nullptr);
  uint64_t nz = amgd_scan_u64(cnt, A->rn);
  dcsr *X = (dcsr *)malloc(sizeof(dcsr));
  X->rn = A->rn; X->cn = A->cn; X->nnz = nz; X->ro = cnt;
  X->col = (uint32_t *)amgd_alloc(nz * 4 + 4);
  X->a = (double *)amgd_alloc_f64(nz * 8 + 8);
  if (A->rn && wave)
    k_pointwise_wave<true><<<gw, 256, 0, s>>>(A->ro, A->col, A->a, B->ro, B->col, B->a, A->rn,
                                              nullptr, X->ro, X->col, X->a);
  else if (A->rn)
    k_pointwise<true><<<grid_for(A->rn), 256, 0, s>>>(A->ro, A->col, A->a, B->ro, B->col, B->a,
                                                       A->rn, nullptr, X->ro, X->col, X->a);
  KCHECK();
  return X;
}

// ---------------------------------------------------------------------------
// SpGEMM X = A*B with the reference's arithmetic (mxm, amg_setup.c:1894):
//   X[i][j] = (((+0 + b_k0j*a_ik0) + b_k1j*a_ik1) + ...), k ascending,
//   exact zeros dropped, columns ascending; duplicate columns in a row of A:
//   the last one wins (the reference scatters A's row into a dense x).
//
// One row per work-group (a single wavefront, or 256 threads for big rows).
// The products of a row are enumerated flat: a window of NT consecutive A
// entries is loaded, their B-row lengths prefix-summed, and every lane takes
// one product (so a lane never idles on short B rows).  Keys go into an
// open-addressing hash in LDS; the numeric pass then applies the values layer
// by layer in ascending k (a B row has distinct columns, so the lanes of one
// layer never collide) -- every slot sees its additions in the reference's
// order.  Occupied slots are compacted in place, bitonic-sorted by column
// and written out.  Rows are binned: symbolic by product upper bound,
// numeric by the distinct count the symbolic pass found; rows with more than
// 4096 distinct columns use the dense-slab kernel.
// ---------------------------------------------------------------------------
#define EMPTY_KEY 0xffffffffu
#define LONG_BLOCKS 512         // resident long-row blocks (dense slabs)
#define OVERFLOW_MARK 0xffffffffffffffffull

__global__ void k_spgemm_ub(const uint64_t *aro, const uint32_t *acol, uint32_t rn,
                            const uint64_t *bro, uint64_t *ub) {
  GRID_STRIDE(i, rn) {
    uint64_t s = 0;
    for (uint64_t k = aro[i]; k < aro[i + 1]; k++) {
      if (k + 1 < aro[i + 1] && acol[k + 1] == acol[k]) continue;
      uint32_t c = acol[k];
      s += bro[c + 1] - bro[c];
    }
    ub[i] = s;
  }
}

// bin rows by v[i] (u64) against ascending thresholds lim[0..nb-2]; the last
// bin takes the rest.  skip0: rows with v == 0 go nowhere.
#define SG_MAXBIN 6
struct SgBins { uint64_t lim[SG_MAXBIN]; };
// sk (optional): rows with sk[i] <= sk_le are left out (the tiny rows of k_sg_tiny)
__global__ void k_bin_rows(const uint64_t *v, uint32_t rn, SgBins b, int nb, int skip0,
                           uint32_t *lists, unsigned *counts, const uint64_t *sk = nullptr,
                           uint64_t sk_le = 0) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t iters = (rn + stride - 1) / stride;
  for (uint64_t it = 0; it < iters; it++) {   // every lane iterates alike (wave_append)
    uint64_t i = i0 + it * stride;
    bool ok = i < rn;
    uint64_t x = ok ? v[i] : 0;
    if (skip0 && x == 0) ok = false;
    if (ok && sk && sk[i] <= sk_le) ok = false;
    int bin = nb - 1;
    for (int q = nb - 2; q >= 0; q--)
      if (x <= b.lim[q]) bin = q;
    for (int q = 0; q < nb; q++) {
      unsigned p = wave_append(&counts[q], ok && bin == q);
      if (ok && bin == q) lists[(uint64_t)q * ((uint64_t)rn + 1) + p] = (uint32_t)i;
    }
  }
}

__device__ __forceinline__ uint32_t sg_hash(uint32_t j, int lg) { return (j * 2654435761u) >> (32 - lg); }

// Emit a finished row from the LDS hash: occupied nonzero slots are compacted to
// the front (order kept), bitonic-sorted by column and written at xro[i].
template <int NT, uint32_t S>
__device__ __forceinline__ void sg_emit(uint32_t *hk, double *hv, uint32_t *wtot, uint32_t *scr,
                                        int t, uint64_t ob, uint32_t *xcol, double *xa,
                                        uint64_t *cnt_i) {
  uint32_t base = 0;
  for (uint32_t c0 = 0; c0 < S; c0 += NT) {
    uint32_t s = c0 + t;
    uint32_t key = hk[s];
    double val = hv[s];
    bool take = key != EMPTY_KEY && val != 0.0;
    uint32_t inc = block_incl_scan<NT>(take ? 1u : 0u, wtot);
    uint32_t tot = __shfl(inc, 63, 64);
    if (NT > 64) {
      if (t == NT - 1) scr[0] = inc;
      __syncthreads();
      tot = scr[0];
    }
    __syncthreads();
    if (take) {
      hk[base + inc - 1] = key;
      hv[base + inc - 1] = val;
    }
    base += tot;
    __syncthreads();
  }
  const uint32_t n = base;
  // Column order by rank: when the row's column span fits a bitmap in the free tail
  // of hk (and its word prefix in the free tail of hv), each key's rank is the
  // number of set bits below it -- O(n + span/32) instead of a bitonic sort.
  __shared__ uint32_t s_mm[2];
  if (t == 0) { s_mm[0] = 0xffffffffu; s_mm[1] = 0; }
  __syncthreads();
  {
    uint32_t mn = 0xffffffffu, mx = 0;
    for (uint32_t s = t; s < n; s += NT) { mn = min(mn, hk[s]); mx = max(mx, hk[s]); }
    if (mn != 0xffffffffu) { atomicMin(&s_mm[0], mn); atomicMax(&s_mm[1], mx); }
  }
  __syncthreads();
  const uint32_t cmin = s_mm[0], cmax = s_mm[1];
  const uint32_t words = n ? ((cmax - cmin) >> 5) + 1 : 0;
  if (n && words + 1 <= S - n) {
    uint32_t *bm = hk + n;
    uint32_t *pre = (uint32_t *)(hv + n);          // 2*(S-n) words free
    for (uint32_t w = t; w < words; w += NT) bm[w] = 0;
    __syncthreads();
    for (uint32_t s = t; s < n; s += NT) {
      const uint32_t d = hk[s] - cmin;
      atomicOr(&bm[d >> 5], 1u << (d & 31));
    }
    __syncthreads();
    const uint32_t per = (words + NT - 1) / NT, w0 = t * per, w1 = min(words, w0 + per);
    uint32_t loc = 0;
    for (uint32_t w = w0; w < w1; w++) loc += __popc(bm[w]);
    const uint32_t incl = block_incl_scan<NT>(loc, wtot);
    uint32_t run = incl - loc;
    for (uint32_t w = w0; w < w1; w++) { pre[w] = run; run += __popc(bm[w]); }
    __syncthreads();
    for (uint32_t s = t; s < n; s += NT) {
      const uint32_t k = hk[s], d = k - cmin, w = d >> 5;
      const uint32_t rank = pre[w] + __popc(bm[w] & ((1u << (d & 31)) - 1u));
      xcol[ob + rank] = k;
      xa[ob + rank] = hv[s];
    }
    if (t == 0) *cnt_i = n;
    __syncthreads();
    return;
  }
  uint32_t P = 1;
  while (P < n) P <<= 1;
  for (uint32_t s = n + t; s < P; s += NT) hk[s] = EMPTY_KEY;
  __syncthreads();
  for (uint32_t size = 2; size <= P; size <<= 1)
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t tt = t; tt < P / 2; tt += NT) {
        uint32_t lo = 2 * tt - (tt & (stride - 1));
        uint32_t hi = lo + stride;
        bool up = (lo & size) == 0;
        uint32_t kl = hk[lo], kh = hk[hi];
        if ((kl > kh) == up) {
          hk[lo] = kh; hk[hi] = kl;
          double x = hv[lo]; hv[lo] = hv[hi]; hv[hi] = x;
        }
      }
      __syncthreads();
    }
  for (uint32_t s = t; s < n; s += NT) { xcol[ob + s] = hk[s]; xa[ob + s] = hv[s]; }
  if (t == 0) *cnt_i = n;
  __syncthreads();
}

// insert key j into the open-addressing LDS hash (linear probing); returns the slot,
// counts newly filled slots in *nfill
// (at most S probes: a full table -- only possible in a symbolic pass past its
// capacity -- returns EMPTY_KEY instead of spinning)
template <int LG>
__device__ __forceinline__ uint32_t sg_insert(uint32_t *hk, uint32_t j, unsigned *nfill, bool count) {
  constexpr uint32_t S = 1u << LG;
  uint32_t sl = sg_hash(j, LG);
  for (uint32_t probe = 0; probe < S; probe++) {
    uint32_t old = atomicCAS(&hk[sl], EMPTY_KEY, j);
    if (old == EMPTY_KEY) {
      if (count) atomicAdd(nfill, 1u);
      return sl;
    }
    if (old == j) return sl;
    sl = (sl + 1) & (S - 1);
  }
  return EMPTY_KEY;
}

#define SG_U 4   // sub-chunks whose product loads are issued together
// MODE 0: count distinct columns (cap: overflow -> OVERFLOW_MARK)
// MODE 1: numeric, write nonzeros sorted at xro[i], count to cnt[i]
// RAP 1: the same kernel instantiated separately for the Galerkin products, so
// profiles list the RAP launches (the bench's roofline kernels) on their own
template <int NT, int LG, int MODE, int RAP = 0>
__global__ __launch_bounds__(NT) void k_sg_row(const uint32_t *rows, uint32_t nrows,
                                               const uint64_t *aro, const uint32_t *acol,
                                               const double *aa, const uint64_t *bro,
                                               const uint32_t *bcol, const double *ba, uint32_t cap,
                                               uint64_t *cnt, const uint64_t *xro, uint32_t *xcol,
                                               double *xa) {
  constexpr uint32_t S = 1u << LG;
  __shared__ uint32_t hk[S];
  __shared__ double hv[MODE ? S : 1];
  __shared__ uint32_t wend[NT];
  __shared__ uint64_t wbst[NT];
  __shared__ double wav[NT];
  __shared__ uint32_t wtot[NT / 64];
  __shared__ unsigned nfill;
  __shared__ int ovf;
  const int t = threadIdx.x;
  for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    const uint32_t i = rows[r];
    for (uint32_t s = t; s < S; s += NT) {
      hk[s] = EMPTY_KEY;
      if (MODE) hv[s] = 0.0;
    }
    if (t == 0) { nfill = 0; ovf = 0; }
    __syncthreads();
    const uint64_t a0 = aro[i], a1 = aro[i + 1];
    for (uint64_t wb = a0; wb < a1; wb += NT) {
      uint64_t ka = wb + t;
      uint32_t len = 0;
      uint64_t bs = 0;
      double av = 0.0;
      if (ka < a1) {
        uint32_t k = acol[ka];
        if (!(ka + 1 < a1 && acol[ka + 1] == k)) {
          bs = bro[k];
          len = (uint32_t)(bro[k + 1] - bs);
          av = aa[ka];
        }
      }
      uint32_t inc = block_incl_scan<NT>(len, wtot);
      wend[t] = inc;
      wbst[t] = bs;
      wav[t] = av;
      __syncthreads();
      const uint32_t T = wend[NT - 1];
      for (uint32_t q0 = 0; q0 < T; q0 += NT * SG_U) {
        // fetch the (column, product) of SG_U sub-chunks first: their loads are
        // independent, so one latency round serves SG_U sub-chunks
        int lq[SG_U];
        uint32_t jq[SG_U];
        double pq[SG_U];
#pragma unroll
        for (int u = 0; u < SG_U; u++) {
          const uint32_t q = q0 + u * NT + t;
          lq[u] = -1;
          jq[u] = 0;
          pq[u] = 0.0;
          if (q < T) {
            int lo = 0, hi = NT - 1;
            while (lo < hi) {
              int mid = (lo + hi) >> 1;
              if (wend[mid] > q) hi = mid;
              else lo = mid + 1;
            }
            const uint32_t st = lo ? wend[lo - 1] : 0u;
            const uint64_t kb = wbst[lo] + (q - st);
            jq[u] = bcol[kb];
            if (MODE == 1) pq[u] = ba[kb] * wav[lo];
            lq[u] = lo;
          }
        }
        // then insert and add sub-chunk by sub-chunk, in product order
#pragma unroll
        for (int u = 0; u < SG_U; u++) {
          const uint32_t qs = q0 + u * NT;
          if (qs >= T) break;              // uniform over the block
          const bool v = lq[u] >= 0;
          uint32_t sl = 0;
          if (v) {
            const uint32_t j = jq[u];
            sl = sg_hash(j, LG);
            while (true) {
              uint32_t old = atomicCAS(&hk[sl], EMPTY_KEY, j);
              if (old == EMPTY_KEY) {
                if (MODE == 0 && atomicAdd(&nfill, 1u) >= cap) ovf = 1;
                break;
              }
              if (old == j) break;
              sl = (sl + 1) & (S - 1);
            }
          }
          if (MODE == 1) {
            // layers of this sub-chunk: A-entries [lf, ll] (uniform bounds)
            uint32_t qa = qs, qb = min(qs + NT, T) - 1;
            int lf = 0, ll = 0;
            {
              int lo = 0, hi = NT - 1;
              while (lo < hi) { int mid = (lo + hi) >> 1; if (wend[mid] > qa) hi = mid; else lo = mid + 1; }
              lf = lo;
              lo = lf; hi = NT - 1;
              while (lo < hi) { int mid = (lo + hi) >> 1; if (wend[mid] > qb) hi = mid; else lo = mid + 1; }
              ll = lo;
            }
            if (lf == ll) {                // one B row: distinct columns, no collision
              if (v) hv[sl] = hv[sl] + pq[u];
            } else {
              for (int lay = lf; lay <= ll; lay++) {
                if (v && lq[u] == lay) hv[sl] = hv[sl] + pq[u];
                __syncthreads();
              }
            }
          } else if (MODE == 2) {          // pattern only: any order, a nonzero mark
            if (v) hv[sl] = 1.0;
          }
          __syncthreads();
        }
        if (MODE == 0 && ovf) break;
      }
      __syncthreads();
      if (MODE == 0 && ovf) break;
    }
    if (MODE == 0) {
      if (t == 0) cnt[i] = ovf ? OVERFLOW_MARK : (uint64_t)nfill;
      __syncthreads();
      continue;
    }
    sg_emit<NT, S>(hk, hv, wtot, wend, t, xro[i], xcol, xa, &cnt[i]);
  }
}

// k-sequential SpGEMM row kernel for long B rows (the avg B row spans the block):
// one row per work-group; the A entries are taken one at a time in ascending k and
// all NT threads cover that B row (coalesced, every product is a distinct column),
// then a barrier orders layer k before layer k+1 -- the reference's order with no
// per-product layer search.  MODE 0 counts distinct columns (no ordering needed),
// MODE 1 accumulates and emits like k_sg_row.
template <int NT, int LG, int MODE, int RAP = 0>
__global__ __launch_bounds__(NT) void k_sg_kseq(const uint32_t *rows, uint32_t nrows,
                                                const uint64_t *aro, const uint32_t *acol,
                                                const double *aa, const uint64_t *bro,
                                                const uint32_t *bcol, const double *ba,
                                                uint32_t cap, uint64_t *cnt, const uint64_t *xro,
                                                uint32_t *xcol, double *xa) {
  constexpr uint32_t S = 1u << LG;
  __shared__ uint32_t hk[S];
  __shared__ double hv[MODE ? S : 1];
  __shared__ uint64_t wbs[NT];
  __shared__ uint32_t wlen[NT];
  __shared__ double wav[NT];
  __shared__ uint32_t wtot[NT / 64 + 1];
  __shared__ unsigned nfill;
  __shared__ int ovf;
  const int t = threadIdx.x;
  for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    const uint32_t i = rows[r];
    for (uint32_t s = t; s < S; s += NT) {
      hk[s] = EMPTY_KEY;
      if (MODE) hv[s] = 0.0;
    }
    if (t == 0) { nfill = 0; ovf = 0; }
    __syncthreads();
    const uint64_t a0 = aro[i], a1 = aro[i + 1];
    for (uint64_t wb = a0; wb < a1; wb += NT) {
      const uint64_t ka = wb + t;
      uint32_t len = 0;
      uint64_t bs = 0;
      double av = 0.0;
      if (ka < a1) {
        const uint32_t k = acol[ka];
        if (!(ka + 1 < a1 && acol[ka + 1] == k)) {   // duplicate columns: the last one wins
          bs = bro[k];
          len = (uint32_t)(bro[k + 1] - bs);
          av = aa[ka];
        }
      }
      wbs[t] = bs;
      wlen[t] = len;
      wav[t] = av;
      __syncthreads();
      const int ne = (int)min((uint64_t)NT, a1 - wb);
      // chunks (layer e, offset j0) of up to 2*NT products, empty layers skipped; the
      // (column, value) loads of the next KD chunks are in flight while the current
      // chunk is inserted, so the HBM latency of the coming layers overlaps the LDS
      // work and barriers of this one (a row is a chain of dependent layer steps)
      constexpr int KD = 3;
      int ce[KD];
      uint32_t cj[KD], ca[KD], cb[KD];
      double pa[KD], pb[KD];
      bool va[KD], vb[KD];
      int fe = 0;
      uint32_t fj = 0;
      while (fe < ne && wlen[fe] == 0) fe++;
      auto fetch = [&](int ee, uint32_t jj, uint32_t &xa_, uint32_t &xb_, double &ya, double &yb,
                       bool &fa, bool &fb) {
        fa = fb = false;
        if (ee >= ne) return;
        const uint32_t L = wlen[ee];
        const uint64_t b0 = wbs[ee];
        const uint32_t ja = jj + t, jb = jj + NT + t;
        fa = ja < L;
        fb = jb < L;
        if (fa) { xa_ = bcol[b0 + ja]; if (MODE == 1) ya = ba[b0 + ja]; }
        if (fb) { xb_ = bcol[b0 + jb]; if (MODE == 1) yb = ba[b0 + jb]; }
      };
      auto step = [&]() {                           // the chunk after (fe, fj)
        if (fe >= ne) return;
        fj += 2 * NT;
        if (fj >= wlen[fe]) {
          fe++;
          fj = 0;
          while (fe < ne && wlen[fe] == 0) fe++;
        }
      };
#pragma unroll
      for (int d = 0; d < KD; d++) {
        ce[d] = fe;
        cj[d] = fj;
        ca[d] = cb[d] = 0;
        pa[d] = pb[d] = 0.0;
        fetch(fe, fj, ca[d], cb[d], pa[d], pb[d], va[d], vb[d]);
        step();
      }
      // raw B values are carried; the product is formed at insert time
      while (ce[0] < ne) {
        const double a = MODE ? wav[ce[0]] : 0.0;
        if (va[0]) {
          const uint32_t sl = sg_insert<LG>(hk, ca[0], &nfill, MODE == 0);
          if (MODE == 1) hv[sl] = hv[sl] + pa[0] * a;
          else if (MODE == 2) hv[sl] = 1.0;          // pattern only: a nonzero mark
          else if (sl == EMPTY_KEY) ovf = 1;
        }
        if (vb[0]) {
          const uint32_t sl = sg_insert<LG>(hk, cb[0], &nfill, MODE == 0);
          if (MODE == 1) hv[sl] = hv[sl] + pb[0] * a;
          else if (MODE == 2) hv[sl] = 1.0;
          else if (sl == EMPTY_KEY) ovf = 1;
        }
        if (MODE == 0 && (ovf || nfill > cap)) break;   // racy LDS read: early exit only
        if (MODE == 1 && ce[1] != ce[0]) __syncthreads();   // layer k before layer k+1
#pragma unroll
        for (int d = 0; d + 1 < KD; d++) {
          ce[d] = ce[d + 1]; cj[d] = cj[d + 1]; ca[d] = ca[d + 1]; cb[d] = cb[d + 1];
          pa[d] = pa[d + 1]; pb[d] = pb[d + 1]; va[d] = va[d + 1]; vb[d] = vb[d + 1];
        }
        ce[KD - 1] = fe;
        cj[KD - 1] = fj;
        fetch(fe, fj, ca[KD - 1], cb[KD - 1], pa[KD - 1], pb[KD - 1], va[KD - 1], vb[KD - 1]);
        step();
      }
      __syncthreads();
      if (MODE == 0 && (ovf || nfill > cap)) break;
    }
    if (MODE == 0) {
      __syncthreads();
      if (t == 0) cnt[i] = (ovf || nfill > cap) ? OVERFLOW_MARK : (uint64_t)nfill;
      __syncthreads();
      continue;
    }
    sg_emit<NT, S>(hk, hv, wtot, wlen, t, xro[i], xcol, xa, &cnt[i]);
  }
}

// long rows: block per row, dense slab acc[cn] + stamp[cn] per resident block
template <int MODE, int RAP = 0>
__global__ __launch_bounds__(256) void k_spgemm_long(
    const uint32_t *rows, uint32_t nrows, const uint64_t *aro, const uint32_t *acol,
    const double *aa, const uint64_t *bro, const uint32_t *bcol, const double *ba, uint32_t cn,
    double *slab_v, uint32_t *slab_s, uint64_t *cnt, const uint64_t *xro, uint32_t *xcol,
    double *xa) {
  double *acc = slab_v + (size_t)blockIdx.x * cn;
  uint32_t *stamp = slab_s + (size_t)blockIdx.x * cn;
  __shared__ uint32_t lo_s, hi_s;
  __shared__ unsigned long long tot;
  for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    uint32_t i = rows[r];
    if (MODE == 0 && cnt[i] != OVERFLOW_MARK) continue;   // exact count already (wide bin)
    uint32_t tag = r + 1;  // stamps are unique per (block, row) visit
    if (threadIdx.x == 0) { lo_s = 0xffffffffu; hi_s = 0; tot = 0; }
    __syncthreads();
    uint64_t a0 = aro[i], a1 = aro[i + 1];
    uint32_t lo = 0xffffffffu, hi = 0;
    for (uint64_t ka = a0; ka < a1; ka++) {
      uint32_t k = acol[ka];
      if (ka + 1 < a1 && acol[ka + 1] == k) continue;
      double av = aa[ka];
      for (uint64_t kb = bro[k] + threadIdx.x; kb < bro[k + 1]; kb += blockDim.x) {
        uint32_t j = bcol[kb];
        if (stamp[j] != tag) { stamp[j] = tag; acc[j] = 0.0; }
        if (MODE == 1) acc[j] = acc[j] + ba[kb] * av;
        lo = min(lo, j);
        hi = max(hi, j);
      }
      __syncthreads();   // order: all adds of step k before any add of step k+1
    }
    atomicMin(&lo_s, lo);
    atomicMax(&hi_s, hi);
    __syncthreads();
    uint32_t L = lo_s, H = hi_s;
    // ordered emission by block-wide scan over [L, H]
    uint64_t base = MODE == 1 ? xro[i] : 0;
    __shared__ unsigned wsum[256];
    unsigned long long running = 0;
    if (L <= H) {
      for (uint64_t c0 = L; c0 <= H; c0 += blockDim.x) {
        uint64_t c = c0 + threadIdx.x;
        bool take = c <= H && stamp[c] == tag && (MODE == 0 || acc[c] != 0.0);
        wsum[threadIdx.x] = take ? 1u : 0u;
        __syncthreads();
        // inclusive scan (Hillis-Steele) over 256 flags
        for (int o = 1; o < 256; o <<= 1) {
          unsigned v = threadIdx.x >= (unsigned)o ? wsum[threadIdx.x - o] : 0u;
          __syncthreads();
          wsum[threadIdx.x] += v;
          __syncthreads();
        }
        if (take && MODE == 1) {
          uint64_t p = base + running + wsum[threadIdx.x] - 1;
          xcol[p] = (uint32_t)c;
          xa[p] = acc[c];
        }
        running += wsum[255];
        __syncthreads();
      }
    }
    if (threadIdx.x == 0) cnt[i] = running;
    __syncthreads();
  }
}

void amgd_compact_rows(const uint64_t *sro, const uint32_t *scol, const double *sa,
                       const uint64_t *dro, uint32_t rn, uint32_t *dcol, double *da);
// Dense rows (past the hash bins' capacity) by sorting, one row at a time (round 6).
// k_spgemm_long gives such a row one work-group: its layers (A entries) run one after the
// other with a barrier each, then a block scan walks the row's whole column span to emit
// -- on the anisotropic grids' orphan rows (10^4 - 10^5 layers, spans of millions of
// columns) 58 ms a call, 1.7 s of configs[4].  Here every product of the row is written in
// layer order (A entries ascending, the last of duplicate columns, each B row ascending),
// a stable radix sort by column keeps that order within every column, and each column's
// run is summed from +0.0 left to right by one thread: the same sums as the layer walk
// (`acc[j] = acc[j] + b * a` in ascending k), exact zeros dropped, columns ascending.
__global__ void k_dr_len(const uint64_t *aro, const uint32_t *acol, const uint64_t *bro, uint32_t i,
                         uint64_t *len) {
  const uint64_t a0 = aro[i], n = aro[i + 1] - a0;
  GRID_STRIDE(e, n) {
    const uint32_t k = acol[a0 + e];
    len[e] = (e + 1 < n && acol[a0 + e + 1] == k) ? 0 : bro[k + 1] - bro[k];
  }
}
template <int MODE>
__global__ void k_dr_gen(const uint64_t *aro, const uint32_t *acol, const double *aa, const uint64_t *bro,
                         const uint32_t *bcol, const double *ba, uint32_t i, const uint64_t *off, uint32_t *key,
                         double *val) {
  const uint64_t a0 = aro[i], n = aro[i + 1] - a0;
  const int lane = threadIdx.x & 63;
  for (uint64_t e = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; e < n;
       e += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
    const uint32_t k = acol[a0 + e];
    if (e + 1 < n && acol[a0 + e + 1] == k) continue;        // duplicate column: the last one wins
    const double av = MODE == 1 ? aa[a0 + e] : 0.0;
    const uint64_t b0 = bro[k], b1 = bro[k + 1], o = off[e] - b0;
    for (uint64_t kb = b0 + lane; kb < b1; kb += 64) {
      key[o + kb] = bcol[kb];
      if (MODE == 1) val[o + kb] = ba[kb] * av;
    }
  }
}
__global__ void k_dr_heads(const uint32_t *key, uint64_t n, uint64_t *flag) {
  GRID_STRIDE(p, n) flag[p] = (p == 0 || key[p] != key[p - 1]) ? 1 : 0;
}
__global__ void k_dr_headpos(const uint32_t *key, uint64_t n, const uint64_t *run, uint64_t *head) {
  GRID_STRIDE(p, n) if (p == 0 || key[p] != key[p - 1]) head[run[p]] = p;
  if (blockIdx.x == 0 && threadIdx.x == 0) head[run[n]] = n;     // run[n] = number of runs
}
__global__ void k_dr_sum(const double *val, const uint64_t *head, uint64_t nruns, double *sum, uint64_t *nzf) {
  GRID_STRIDE(r, nruns) {
    double acc = 0.0;
    for (uint64_t p = head[r]; p < head[r + 1]; p++) acc = acc + val[p];
    sum[r] = acc;
    nzf[r] = acc != 0.0 ? 1 : 0;
  }
}
__global__ void k_dr_emit(const uint32_t *key, const uint64_t *head, const double *sum, const uint64_t *pos,
                          uint64_t nruns, const uint64_t *xro, uint32_t i, uint32_t *xcol, double *xa,
                          uint64_t *cnt) {
  const uint64_t base = xro[i];
  GRID_STRIDE(r, nruns) if (pos[r + 1] != pos[r]) {
    xcol[base + pos[r]] = key[head[r]];
    xa[base + pos[r]] = sum[r];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) cnt[i] = pos[nruns];
}
__global__ void k_dr_count(const uint64_t *run, uint64_t n, uint32_t i, uint64_t *cnt) { cnt[i] = run[n]; }
#define DR_MAX_PRODUCTS (1ull << 28)
// rows[0..nrows) (device list) by sorting; false (nothing done) when a row's products pass
// DR_MAX_PRODUCTS -- the caller then takes the block kernel.  MODE 0: cnt[i] := distinct
// columns (only for rows marked OVERFLOW_MARK); MODE 1: nonzero sums at xro[i], cnt[i] := count.
// the rows to process (MODE 0: only those whose count overflowed) with their A-row bounds,
// gathered on the device: one readback instead of one per row
__global__ void k_dr_pick(const uint32_t *rows, unsigned nrows, const uint64_t *cnt, int mode, const uint64_t *aro,
                          uint32_t *prow, uint64_t *pab, unsigned *np) {
  GRID_STRIDE(r, nrows) {
    const uint32_t i = rows[r];
    if (mode == 0 && cnt[i] != OVERFLOW_MARK) continue;
    const unsigned q = atomicAdd(np, 1u);
    prow[q] = i;
    pab[2 * q] = aro[i];
    pab[2 * q + 1] = aro[i + 1];
  }
}
static bool dense_rows_sorted(int mode, const uint32_t *rows, unsigned nrows_all, const dcsr *A, const dcsr *B,
                              uint64_t *cnt, const uint64_t *xro, uint32_t *xcol, double *xa) {
  hipStream_t s = amgd_s();
  unsigned nrows = 0;
  std::vector<uint32_t> hr;
  std::vector<uint64_t> ne;
  {
    uint32_t *prow = (uint32_t *)amgd_alloc((size_t)nrows_all * 4 + 4);
    uint64_t *pab = (uint64_t *)amgd_alloc((size_t)nrows_all * 16 + 16);
    unsigned *np = (unsigned *)amgd_alloc(16);
    amgd_memset(np, 0, 4);
    k_dr_pick<<<grid_for(nrows_all), 256, 0, s>>>(rows, nrows_all, cnt, mode, A->ro, prow, pab, np);
    KCHECK();
    amgd_d2h(&nrows, np, 4);
    hr.resize(nrows);
    ne.resize(nrows);
    if (nrows) {
      std::vector<uint64_t> ab(2 * (size_t)nrows);
      amgd_d2h(hr.data(), prow, (size_t)nrows * 4);
      amgd_d2h(ab.data(), pab, (size_t)nrows * 16);
      for (unsigned q = 0; q < nrows; q++) ne[q] = ab[2 * q + 1] - ab[2 * q];
    }
    amgd_free(prow); amgd_free(pab); amgd_free(np);
  }
  std::vector<uint64_t *> offs(nrows, nullptr);
  std::vector<uint64_t> np(nrows, 0);
  bool ok = true;
  for (unsigned q = 0; q < nrows && ok; q++) {
    offs[q] = (uint64_t *)amgd_alloc((ne[q] + 1) * 8);
    if (ne[q]) k_dr_len<<<grid_for(ne[q]), 256, 0, s>>>(A->ro, A->col, B->ro, hr[q], offs[q]);
    np[q] = amgd_scan_u64(offs[q], ne[q]);
    if (np[q] > DR_MAX_PRODUCTS) ok = false;
  }
  if (ok) {
    for (unsigned q = 0; q < nrows; q++) {
      if (!offs[q]) continue;
      const uint32_t i = hr[q];
      const uint64_t n = np[q];
      uint32_t *k1 = (uint32_t *)amgd_alloc(n * 4 + 4), *k2 = (uint32_t *)amgd_alloc(n * 4 + 4);
      double *v1 = mode ? (double *)amgd_alloc_f64(n * 8 + 8) : nullptr;
      double *v2 = mode ? (double *)amgd_alloc_f64(n * 8 + 8) : nullptr;
      if (ne[q]) {
        if (mode)
          k_dr_gen<1><<<grid_for(ne[q] * 64, 256, 16384), 256, 0, s>>>(A->ro, A->col, A->a, B->ro, B->col, B->a,
                                                                        i, offs[q], k1, v1);
        else
          k_dr_gen<0><<<grid_for(ne[q] * 64, 256, 16384), 256, 0, s>>>(A->ro, A->col, A->a, B->ro, B->col, B->a,
                                                                        i, offs[q], k1, nullptr);
      }
      KCHECK();
      size_t tb = 0;
      const int eb = bits_for(B->cn);
      void *tmp;
      if (mode) {
        HIPCK(rocprim::radix_sort_pairs(nullptr, tb, k1, k2, v1, v2, (size_t)n, 0, eb, s));
        tmp = amgd_alloc(tb + 16);
        HIPCK(rocprim::radix_sort_pairs(tmp, tb, k1, k2, v1, v2, (size_t)n, 0, eb, s));
      } else {
        HIPCK(rocprim::radix_sort_keys(nullptr, tb, k1, k2, (size_t)n, 0, eb, s));
        tmp = amgd_alloc(tb + 16);
        HIPCK(rocprim::radix_sort_keys(tmp, tb, k1, k2, (size_t)n, 0, eb, s));
      }
      amgd_free(tmp);
      uint64_t *run = (uint64_t *)amgd_alloc((n + 1) * 8);
      if (n) k_dr_heads<<<grid_for(n), 256, 0, s>>>(k2, n, run);
      const uint64_t nruns = amgd_scan_u64(run, n);
      if (mode == 0) {
        k_dr_count<<<1, 1, 0, s>>>(run, n, i, cnt);
      } else {
        uint64_t *head = (uint64_t *)amgd_alloc((nruns + 1) * 8);
        k_dr_headpos<<<grid_for(n ? n : 1), 256, 0, s>>>(k2, n, run, head);
        double *sum = (double *)amgd_alloc_f64(nruns * 8 + 8);
        uint64_t *pos = (uint64_t *)amgd_alloc((nruns + 1) * 8);
        if (nruns) k_dr_sum<<<grid_for(nruns), 256, 0, s>>>(v2, head, nruns, sum, pos);
        amgd_scan_u64(pos, nruns);
        k_dr_emit<<<grid_for(nruns ? nruns : 1), 256, 0, s>>>(k2, head, sum, pos, nruns, xro, i, xcol, xa, cnt);
        KCHECK();
        amgd_free(head); amgd_free(sum); amgd_free(pos);
      }
      KCHECK();
      amgd_free(run); amgd_free(k1); amgd_free(k2);
      if (v1) { amgd_free(v1); amgd_free(v2); }
    }
  }
  for (unsigned q = 0; q < nrows; q++) amgd_free(offs[q]);
  return ok;
}
static int g_dr_sort = -1;        // AMGD_DR_SORT=0 / amgd_spgemm_set_dr_sort(0): dense rows by the block kernel
static bool dr_sort_on() {
  if (g_dr_sort < 0) { const char *e = getenv("AMGD_DR_SORT"); g_dr_sort = e && *e ? atoi(e) : 1; }
  return g_dr_sort != 0;
}
extern "C" void amgd_spgemm_set_dr_sort(int on) { g_dr_sort = on < 0 ? -1 : on; }


// event timing of the numeric SpGEMM kernels (the RAP products) + algorithmic bytes:
// A (12 B/nnz + 8 B/row), B (12 B/nnz + 8 B/row) and X (12 B/nnz + 8 B/row) once each.
#define KSEQ_MIN 64
static int g_sg_flat = -1;      // AMGD_SG_FLAT=1 / amgd_spgemm_force_flat(1): flat kernels only
static bool sg_force_flat() {
  if (g_sg_flat < 0) { const char *e = getenv("AMGD_SG_FLAT"); g_sg_flat = (e && *e && *e != '0') ? 1 : 0; }
  return g_sg_flat == 1;
}
extern "C" void amgd_spgemm_force_flat(int on) { g_sg_flat = on ? 1 : 0; }
static int g_sg_win_forced = 0; // tests: the window applies whatever the column count
static int g_sg_win = -1;       // AMGD_SG_WIN: window of the dense-accumulator kernel (0: off)
static int sg_win() {
  if (g_sg_win < 0) {
    const char *e = getenv("AMGD_SG_WIN");
    g_sg_win = e ? atoi(e) : 2048;
    if (g_sg_win != 0 && g_sg_win != 1024 && g_sg_win != 2048 && g_sg_win != 4096 && g_sg_win != 8192 && g_sg_win != 16384) g_sg_win = 2048;
  }
  return g_sg_win;
}
extern "C" void amgd_spgemm_set_win(int w) {
  g_sg_win = w < 0 ? -1 : w;
  g_sg_win_forced = w > 0;
}
static uint32_t sg_win_p0() {
  static long v = -1;
  if (v < 0) { const char *e = getenv("AMGD_SG_WIN_P0"); v = e ? atol(e) : 48; }
  return (uint32_t)v;
}
static int g_sg_slot = -1;
static uint64_t g_sg_bytes = 0, g_sg_launches = 0;
extern "C" uint64_t amgd_spgemm_launches(void) { return g_sg_launches; }
static int g_sg_pattern = 0;    // amgd_spgemm_pattern: hash-bin rows emit the pattern only
extern "C" void amgd_spgemm_set_timer(int slot) { g_sg_slot = slot; }
extern "C" void amgd_sparse_reset_state(void) {
  g_sg_slot = -1;
  g_sg_pattern = 0;
}
static void sym_forget(void);
extern "C" void amgd_reset_call_state(void) {
  sym_forget();
  amgd_spat_forget();
  amgd_sparse_reset_state();
  amgd_interp_reset_state();
}
extern "C" void amgd_spgemm_bytes_reset(void) { g_sg_bytes = 0; g_sg_launches = 0; }
extern "C" uint64_t amgd_spgemm_bytes(void) { return g_sg_bytes; }

// Tiny rows (at most SG_TINY products: the fine levels' near-diagonal products, 10^6 -
// 10^7 rows of 1-8 products) take one thread each, the row's distinct columns kept
// sorted in registers (fixed-size arrays, every index compile-time): one work-group per
// row spent most of its time clearing a 4096-slot LDS table.  Products are visited in
// the hash kernels' order -- A entries ascending (the last of duplicate columns, as
// everywhere), each B row ascending -- and every column's sum starts from +0.0 and adds
// its products in that order: the same bits.  MODE 0 writes the distinct count, MODE 1
// the nonzero sums in column order at xro[i] and their count.
#define SG_TINY 32
__global__ void k_tiny_list(const uint64_t *ub, uint32_t rn, uint32_t *list, unsigned *cnt) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t iters = (rn + stride - 1) / stride;
  for (uint64_t it = 0; it < iters; it++) {   // uniform trip count (wave_append)
    const uint64_t i = i0 + it * stride;
    const bool take = i < rn && ub[i] <= SG_TINY;
    const unsigned p = wave_append(cnt, take);
    if (take) list[p] = (uint32_t)i;
  }
}
template <int MODE>
__global__ __launch_bounds__(256) void k_sg_tiny(const uint32_t *rows, uint32_t nrows,
                                                 const uint64_t *aro, const uint32_t *acol,
                                                 const double *aa, const uint64_t *bro,
                                                 const uint32_t *bcol, const double *ba,
                                                 uint64_t *cnt, const uint64_t *xro, uint32_t *xcol,
                                                 double *xa) {
  constexpr uint32_t T = SG_TINY, EMPTY = 0xffffffffu;
  GRID_STRIDE(r, nrows) {
    const uint32_t i = rows[r];
    uint32_t K[T];
    double V[T];
#pragma unroll
    for (uint32_t q = 0; q < T; q++) { K[q] = EMPTY; V[q] = 0.0; }
    const uint64_t a0 = aro[i], a1 = aro[i + 1];
    for (uint64_t ka = a0; ka < a1; ka++) {
      const uint32_t k = acol[ka];
      if (ka + 1 < a1 && acol[ka + 1] == k) continue;
      const double av = MODE ? aa[ka] : 0.0;
      const uint64_t b1 = bro[k + 1];
      for (uint64_t kb = bro[k]; kb < b1; kb++) {
        const uint32_t j = bcol[kb];
        const double p = MODE ? ba[kb] * av : 0.0;
        bool found = false;
#pragma unroll
        for (uint32_t q = 0; q < T; q++)
          if (K[q] == j) { if (MODE) V[q] = V[q] + p; found = true; }
        if (!found) {                        // sorted insert (EMPTY sorts last)
#pragma unroll
          for (uint32_t q = T - 1; q > 0; q--) {
            if (K[q - 1] > j) { K[q] = K[q - 1]; V[q] = V[q - 1]; }
            else if (K[q] > j) { K[q] = j; V[q] = 0.0 + p; }
          }
          if (K[0] > j) { K[0] = j; V[0] = 0.0 + p; }
        }
      }
    }
    uint32_t n = 0;
    if (MODE == 0) {
#pragma unroll
      for (uint32_t q = 0; q < T; q++) n += K[q] != EMPTY ? 1u : 0u;
    } else {
      const uint64_t ob = xro[i];
#pragma unroll
      for (uint32_t q = 0; q < T; q++)
        if (K[q] != EMPTY && V[q] != 0.0) { xcol[ob + n] = K[q]; xa[ob + n] = V[q]; n++; }
    }
    cnt[i] = n;
  }
}

// SGLOG: rows with >= 1024 outputs binned by column span (<=4K, 8K, 16K, 32K, 64K, more)
__global__ void k_span_hist(const uint64_t *ro, const uint32_t *col, uint32_t rn,
                            unsigned long long *h) {
  GRID_STRIDE(i, rn) {
    const uint64_t a = ro[i], b = ro[i + 1];
    if (b - a < 1024) continue;
    const uint32_t sp = col[b - 1] - col[a] + 1;
    int q = 0;
    while (q < 5 && sp > (4096u << q)) q++;
    atomicAdd(&h[q], 1ull);
  }
}
// Wave-private windowed SpGEMM (round 3).  k_sg_win shares one window accumulator
// among the 256 threads of a work-group, so every layer (A entry k) costs a barrier
// while typically only a few dozen of its B-row entries fall into the window.  Here
// every WAVEFRONT owns a row and a private LDS window: the 64 lanes of one wavefront
// execute a layer's additions in one instruction stream and LDS operations of one
// wavefront complete in issue order, so layer k's additions precede layer k+1's with
// no barrier at all.  Lane e holds the state of layer e of the current 64-layer chunk
// (B-row start, length, cursor, A value, next column); the in-window layers are taken
// in ascending k from a ballot mask, the next D layers' column / value loads in flight
// while the current one is added (wave-uniform parameters by readlane).  Windows
// start at the smallest pending column (empty column ranges are skipped); rows of
// more than 64 layers keep their cursors in global scratch indexed by the A entry.
// Every output is the sum, from +0 in ascending k, of its products -- mxm's order
// (amg_setup.c:1894-1960) -- and the window is emitted in column order, coalesced.
// MODE 2: distinct columns per row (a bit map: W columns in W / 8 bytes); MODE 1: values
// (W doubles).
__device__ __forceinline__ uint32_t rl32(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
  return ((uint64_t)rl32((uint32_t)(v >> 32), l) << 32) | rl32((uint32_t)v, l);
}
__device__ __forceinline__ double rld(double v, int l) {
  return __longlong_as_double((long long)rl64((uint64_t)__double_as_longlong(v), l));
}
template <int W, int MODE, int RAP = 0>
__global__ __launch_bounds__(256) void k_sg_wwin(const uint32_t *rows, uint32_t nrows,
                                                 const uint64_t *aro, const uint32_t *acol,
                                                 const double *aa, const uint64_t *bro,
                                                 const uint32_t *bcol, const double *ba,
                                                 uint64_t *cnt, const uint64_t *xro,
                                                 uint32_t *xcol, double *xa, uint32_t *curs) {
  constexpr int NWV = 4, D = 4;
  static_assert(MODE == 1 || MODE == 2, "k_sg_wwin: MODE 1 (values) or 2 (bit-map counts)");
  constexpr bool NUM = MODE == 1;
  constexpr int WB = NUM ? W * 8 : W / 8;           // LDS bytes per wavefront
  constexpr uint32_t NONE = 0xffffffffu;
  __shared__ __attribute__((aligned(16))) uint8_t lds[NWV * WB];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double *acc = (double *)(lds + wv * WB);
  uint8_t *mp = lds + wv * WB;
  uint32_t *mp32 = (uint32_t *)mp;
  const uint64_t ltm = lane ? (~0ull >> (64 - lane)) : 0ull;
  // curs holds nnz(A) cursors from A's first entry: a row-range view of a larger matrix
  // (sharded products) keeps absolute row offsets
  const uint64_t cbase = aro[0];
  for (uint32_t r = blockIdx.x * NWV + wv; r < nrows; r += gridDim.x * NWV) {
    const uint32_t i = rows[r];
    const uint64_t a0 = aro[i];
    const uint32_t nl = (uint32_t)(aro[i + 1] - a0);
    uint32_t mn = NONE, mx = 0;
    for (uint32_t e = lane; e < nl; e += 64) {        // the row's column range
      const uint32_t k = acol[a0 + e];
      if (e + 1 < nl && acol[a0 + e + 1] == k) continue;
      const uint64_t b0 = bro[k], b1 = bro[k + 1];
      if (b0 < b1) {
        mn = min(mn, bcol[b0]);
        mx = max(mx, bcol[b1 - 1]);
      }
    }
    for (int o = 32; o; o >>= 1) {
      mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
      mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
    }
    const bool single = nl <= 64;
    uint64_t lb0 = 0;
    uint32_t llen = 0, lcur = 0, lpk = NONE;
    double lav = 0.0;
    auto load_layer = [&](uint32_t c0, bool first) {
      const uint32_t e = c0 + (uint32_t)lane;
      lb0 = 0; llen = 0; lcur = 0; lpk = NONE; lav = 0.0;
      if (e < nl) {
        const uint32_t k = acol[a0 + e];
        if (!(e + 1 < nl && acol[a0 + e + 1] == k)) {   // duplicate columns: the last one wins
          lb0 = bro[k];
          llen = (uint32_t)(bro[k + 1] - lb0);
          if (NUM) lav = aa[a0 + e];
          if (!first) lcur = curs[a0 - cbase + e];
          if (lcur < llen) lpk = bcol[lb0 + lcur];
        }
      }
    };
    if (single) load_layer(0, true);
    const uint64_t ob = NUM ? xro[i] : 0;
    uint64_t nout = 0;
    bool first = true;
    uint32_t wb = mn;
    while (mn <= mx) {
      const uint32_t we = (uint32_t)min((uint64_t)mx, (uint64_t)wb + W - 1);   // inclusive
      if (NUM) {
        for (int q = lane; q < W; q += 64) acc[q] = 0.0;
      } else {
        for (int q = lane; q < WB / 4; q += 64) mp32[q] = 0u;
      }
      uint32_t nmin = NONE;
      for (uint32_t c0 = 0; c0 < nl; c0 += 64) {
        if (!single) load_layer(c0, first);
        uint64_t act = __ballot(lpk <= we);
        int qe[D];
        uint32_t qc[D];
        double qv[D];
        auto issue = [&](int s) {
          qe[s] = -1;
          qc[s] = NONE;
          qv[s] = 0.0;
          if (act) {
            const int e = __ffsll((long long)act) - 1;
            act &= act - 1;
            const uint64_t b0 = rl64(lb0, e);
            const uint32_t ln = rl32(llen, e), j = rl32(lcur, e) + (uint32_t)lane;
            qe[s] = e;
            if (j < ln) {
              qc[s] = bcol[b0 + j];
              if (NUM) qv[s] = ba[b0 + j];
            }
          }
        };
#pragma unroll
        for (int s = 0; s < D; s++) issue(s);
        while (qe[0] >= 0) {
          const int e = qe[0];
          uint32_t col = qc[0];
          double val = qv[0];
#pragma unroll
          for (int s = 0; s + 1 < D; s++) { qe[s] = qe[s + 1]; qc[s] = qc[s + 1]; qv[s] = qv[s + 1]; }
          issue(D - 1);
          const double av = NUM ? rld(lav, e) : 0.0;
          uint32_t cu = rl32(lcur, e);
          for (;;) {
            const bool in = col <= we;                 // a prefix of the lanes (sorted row)
            if (NUM) {
              if (in) {
                double *p = acc + (col - wb);
                *p = *p + val * av;
              }
            } else if (in) {
              atomicOr(&mp32[(col - wb) >> 5], 1u << ((col - wb) & 31));
            }
            const uint32_t n = (uint32_t)__popcll(__ballot(in));
            if (n < 64) {
              const uint32_t pk = (uint32_t)__shfl((int)col, (int)n, 64);   // first column past
              cu += n;
              if (lane == e) { lcur = cu; lpk = pk; }
              break;
            }
            cu += 64;                                  // more of this layer in the window
            const uint64_t b0 = rl64(lb0, e);
            const uint32_t ln = rl32(llen, e), j = cu + (uint32_t)lane;
            col = NONE;
            if (j < ln) {
              col = bcol[b0 + j];
              if (NUM) val = ba[b0 + j];
            }
          }
        }
        uint32_t m = lpk;
        for (int o = 32; o; o >>= 1) m = min(m, (uint32_t)__shfl_xor((int)m, o, 64));
        nmin = min(nmin, m);
        if (!single && c0 + lane < nl) curs[a0 - cbase + c0 + lane] = lcur;
      }
      if (NUM) {                                      // emit in column order
        for (int q = 0; q < W; q += 64) {
          const double v = acc[q + lane];
          const bool nz = v != 0.0;
          const uint64_t bm = __ballot(nz);
          if (nz) {
            const uint64_t o = ob + nout + (uint64_t)__popcll(bm & ltm);
            xcol[o] = wb + (uint32_t)(q + lane);
            xa[o] = v;
          }
          nout += (uint64_t)__popcll(bm);
        }
      } else {
        uint32_t c = 0;
        for (int q = lane; q < WB / 4; q += 64) c += (uint32_t)__popc(mp32[q]);
        for (int o = 32; o; o >>= 1) c += (uint32_t)__shfl_xor((int)c, o, 64);
        nout += c;
      }
      first = false;
      if (nmin > mx) break;
      wb = nmin;
    }
    if (lane == 0) cnt[i] = nout;
  }
}

// wide rows -> windowed (dense accumulator) or hash kernels.  The windowed kernel
// pays a barrier per layer per window: it is chosen when a layer brings enough
// products into a window, i.e. products * min(W, span) / (layers * span) >= p0,
// span = the row's output column range (from the first/last column of its B rows).
__global__ void k_win_split(const uint32_t *list, uint32_t n, const uint64_t *aro,
                            const uint32_t *acol, const uint64_t *bro, const uint32_t *bcol,
                            const uint64_t *ub, uint32_t W, uint32_t p0, uint32_t *wl,
                            uint32_t *hl, unsigned *cnt) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t c0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t iters = (n + stride - 1) / stride;
  for (uint64_t it = 0; it < iters; it++) {   // uniform trip count (wave_append)
    const uint64_t r = c0 + it * stride;
    const bool valid = r < n;
    bool w = false;
    uint32_t i = 0;
    if (valid) {
      i = list[r];
      const uint64_t a0 = aro[i], a1 = aro[i + 1];
      uint32_t mn = 0xffffffffu, mx = 0;
      for (uint64_t ka = a0; ka < a1; ka++) {
        const uint32_t k = acol[ka];
        const uint64_t b0 = bro[k], b1 = bro[k + 1];
        if (b0 < b1) {
          mn = min(mn, bcol[b0]);
          mx = max(mx, bcol[b1 - 1]);
        }
      }
      if (mn <= mx) {
        const double span = (double)(mx - mn) + 1.0;
        const double ppwl = (double)ub[i] * fmin((double)W, span) / ((double)(a1 - a0) * span);
        w = ppwl >= (double)p0;
      }
    }
    const unsigned p = wave_append(&cnt[0], valid && w);
    if (valid && w) wl[p] = i;
    const unsigned q = wave_append(&cnt[1], valid && !w);
    if (valid && !w) hl[q] = i;
  }
}
// Row lists in ascending row order.  The binning appends a wavefront's rows as one run,
// the runs in whatever order the wavefronts finished, so the rows in flight at once were
// spread over the whole matrix; sorted, the work-groups in flight (and each XCD's share of
// them) cover a narrow band of rows, whose products read mostly the same B rows.  Rows
// are independent: the order changes no value.  256^3 (profiles/r04/ab_sg_sort): symbolic
// windows 913 -> 813 ms, numeric windows 989 -> 803 and 505 -> 411 ms (RAP), the 8192-slot
// hash bins 364 -> 349 and 221 -> 211 ms; sorting the cheap bins as well changed nothing,
// nor did the same for the Q-factor / Q-application / interp_lmop lists (net -14 ms).
static void sort_list(uint32_t *list, unsigned n, uint32_t rn) {
  if (n < 2048) return;
  hipStream_t s = amgd_s();
  uint32_t *tmpk = (uint32_t *)amgd_alloc((size_t)n * 4 + 4);
  size_t tb = 0;
  const int eb = bits_for(rn);
  HIPCK(rocprim::radix_sort_keys(nullptr, tb, list, tmpk, (size_t)n, 0, eb, s));
  void *tmp = amgd_alloc(tb + 16);
  HIPCK(rocprim::radix_sort_keys(tmp, tb, list, tmpk, (size_t)n, 0, eb, s));
  HIPCK(hipMemcpyAsync(list, tmpk, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
  amgd_free(tmp);
  amgd_free(tmpk);
}
// The symbolic phase of a product (upper bounds, row bins, distinct counts, the distinct
// layout's offsets, the window split) depends only on the operands' patterns.  The
// interpolation loop's last Af*W (amgd_setup.c interpolation) and the Galerkin product's
// Af*W (the final weights on the same skeleton) share both patterns, so the first keeps
// its symbolic state and the second takes it over: only the numeric kernels run again.
// A kept state is taken only when a hash of both patterns (row offsets and columns) and
// the shapes match; otherwise the product runs in full.
struct SgSym {
  uint32_t rn, acn, bcn;
  uint64_t annz, bnnz, hash;
  uint64_t *ub, *cnt;               // per-row upper bounds; distinct layout offsets (scanned)
  uint32_t *lists, *wlists;         // row bins (numeric bins, sorted, window-split)
  unsigned hc[SG_MAXBIN], hn[SG_MAXBIN], wn[4];
  uint64_t dist;
  bool kseq, wide;
  int win, nlb;
};
static SgSym *g_sym_kept = nullptr;
static int g_sym_mode = 0;          // the next local product: 1 keeps its symbolic state, 2 may take the kept one
static uint64_t g_sym_reused = 0, g_sym_kept_n = 0;
static void sym_free(SgSym *y) {
  if (!y) return;
  amgd_free(y->ub); amgd_free(y->cnt); amgd_free(y->lists);
  if (y->wlists) amgd_free(y->wlists);
  free(y);
}
extern "C" void amgd_spgemm_sym_next(int mode) { g_sym_mode = mode; }
extern "C" void amgd_spgemm_sym_drop(void) { sym_free(g_sym_kept); g_sym_kept = nullptr; g_sym_mode = 0; }
extern "C" void amgd_spgemm_sym_stats(uint64_t *kept, uint64_t *reused) { *kept = g_sym_kept_n; *reused = g_sym_reused; }
// after an unwound setup the kept blocks were released by the rollback: forget them
static void sym_forget(void) { if (g_sym_kept) free(g_sym_kept); g_sym_kept = nullptr; g_sym_mode = 0; }
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
// order-independent hash of a pattern: wrapping sum of mixed (position, value) keys over
// the row offsets and then the columns
__global__ void k_pat_hash(const uint64_t *ro, uint32_t rn, const uint32_t *col, uint64_t nnz, uint64_t salt,
                           unsigned long long *out) {
  const uint64_t n = (uint64_t)rn + 1 + nnz;
  uint64_t h = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t v = i <= rn ? ro[i] : (uint64_t)col[i - rn - 1];
    h += mix64(salt + i * 0x2545f4914f6cdd1dull + (v << 1));
  }
  atomicAdd(out, (unsigned long long)h);
}
static uint64_t pat_hash2(const dcsr *A, const dcsr *B) {
  unsigned long long *d = (unsigned long long *)amgd_alloc(16);
  amgd_memset(d, 0, 16);
  hipStream_t s = amgd_s();
  k_pat_hash<<<grid_for((uint64_t)A->rn + A->nnz + 1, 256, 4096), 256, 0, s>>>(A->ro, A->rn, A->col, A->nnz,
                                                                                0x5a17ull, d);
  k_pat_hash<<<grid_for((uint64_t)B->rn + B->nnz + 1, 256, 4096), 256, 0, s>>>(B->ro, B->rn, B->col, B->nnz,
                                                                                0xb0b5ull, d + 1);
  KCHECK();
  unsigned long long h[2];
  amgd_d2h(h, d, 16);
  amgd_free(d);
  return (uint64_t)h[0] * 0x100000001b3ull ^ (uint64_t)h[1];
}

// symbolic phase: bins, distinct counts and their offsets, the window split
static SgSym *sg_symbolic(const dcsr *A, const dcsr *B) {
  hipStream_t s = amgd_s();
  SgSym *y = (SgSym *)calloc(1, sizeof(SgSym));
  const uint32_t rn = A->rn;
  const uint64_t L = (uint64_t)rn + 1;
  y->rn = rn; y->acn = A->cn; y->bcn = B->cn; y->annz = A->nnz; y->bnnz = B->nnz;
  uint64_t *ub = y->ub = (uint64_t *)amgd_alloc(L * 8);
  uint32_t *lists = y->lists = (uint32_t *)amgd_alloc((size_t)SG_MAXBIN * L * 4);
  unsigned *counts = (unsigned *)amgd_alloc(64);
  uint64_t *cnt = y->cnt = (uint64_t *)amgd_alloc(L * 8);
  HIPCK(hipMemsetAsync(counts, 0, 64, s));
  HIPCK(hipMemsetAsync(cnt, 0, L * 8, s));
  unsigned *hc = y->hc;
  // tiny rows (<= SG_TINY products): their own list (bin slot 5) and kernel, left out
  // of every other bin (AMGD_SG_TINY=0: off)
  static int tiny_on = -1;
  if (tiny_on < 0) { const char *e = getenv("AMGD_SG_TINY"); tiny_on = e && *e ? atoi(e) : 1; }
  uint32_t *tlist = lists + 5 * L;
  const uint64_t *tsk = tiny_on ? ub : nullptr;
  if (rn) {
    k_spgemm_ub<<<grid_for(rn), 256, 0, s>>>(A->ro, A->col, rn, B->ro, ub);
    SgBins b;
    b.lim[0] = 2048;
    k_bin_rows<<<grid_for(rn), 256, 0, s>>>(ub, rn, b, 2, 0, lists, counts, tsk, SG_TINY);
    if (tiny_on) k_tiny_list<<<grid_for(rn), 256, 0, s>>>(ub, rn, tlist, counts + 5);
    KCHECK();
    amgd_d2h(hc, counts, 24);
    sort_list(lists + L, hc[1], rn);           // the wide rows (cheap ones: no gain measured)
  }
  const unsigned ntiny = hc[5];
  if (ntiny)
    k_sg_tiny<0><<<grid_for(ntiny, 256, 16384), 256, 0, s>>>(tlist, ntiny, A->ro, A->col, A->a, B->ro,
                                                            B->col, B->a, cnt, nullptr, nullptr, nullptr);
  // symbolic: distinct count per row (row order in the lists is arbitrary; rows are independent)
  // long B rows (mean >= KSEQ_MIN): the k-sequential kernels; short ones: flat enumeration
  const uint64_t avgB = B->rn ? B->nnz / B->rn : 0;
  const bool kseq = y->kseq = avgB >= KSEQ_MIN && !sg_force_flat();
  y->wide = avgB >= 256;
  if (hc[0]) {
    if (kseq)
      k_sg_kseq<64, 12, 0><<<(int)std::min<unsigned>(hc[0], 65536u), 64, 0, s>>>(
          lists, hc[0], A->ro, A->col, A->a, B->ro, B->col, B->a, 2048, cnt, nullptr, nullptr, nullptr);
    else
      k_sg_row<64, 12, 0><<<(int)std::min<unsigned>(hc[0], 65536u), 64, 0, s>>>(
          lists, hc[0], A->ro, A->col, A->a, B->ro, B->col, B->a, 2048, cnt, nullptr, nullptr, nullptr);
  }
  // wide symbolic rows of long-B-row products: wave-private bit-map windows (k_sg_wwin
  // MODE 2); their cursors live in `curs` (one per A entry, scratch of each kernel)
  if (hc[1]) {
    if (kseq) {
      amgd_route_hit(AMGD_R_SG_WWIN_SYM);
      uint32_t *curs = (uint32_t *)amgd_alloc(A->nnz * 4 + 4);
      // bit-map windows of 32768 columns in 4 KB (round 4; the 4096-column byte maps
      // took 1239 against 909 ms per 256^3 setup, profiles/r04/ab_sym_ww)
      k_sg_wwin<32768, 2><<<(int)std::min<unsigned>((hc[1] + 3) / 4, 16384u), 256, 0, s>>>(
          lists + L, hc[1], A->ro, A->col, nullptr, B->ro, B->col, nullptr, cnt, nullptr, nullptr,
          nullptr, curs);
      KCHECK();
      amgd_free(curs);
    } else {
      k_sg_row<256, 14, 0><<<(int)std::min<unsigned>(hc[1], 8192u), 256, 0, s>>>(
          lists + L, hc[1], A->ro, A->col, A->a, B->ro, B->col, B->a, 8192, cnt, nullptr, nullptr,
          nullptr);
    }
  }
  KCHECK();
  // numeric bins by distinct count: wave/512, wave/2048, wave/4096, block/8192 slots, dense slab
  unsigned *hn = y->hn;
  if (rn) {
    HIPCK(hipMemsetAsync(counts, 0, 64, s));
    SgBins b;
    // (k-sequential kernels take the 8192-slot table up to 75% load)
    b.lim[0] = 256; b.lim[1] = 1024; b.lim[2] = 2048; b.lim[3] = kseq ? 6144 : 4096;
    k_bin_rows<<<grid_for(rn), 256, 0, s>>>(cnt, rn, b, 5, 1, lists, counts, tsk, SG_TINY);
    KCHECK();
    amgd_d2h(hn, counts, 20);
    for (int q = 1; q < 5; q++) sort_list(lists + q * L, hn[q], rn);
  }
  y->nlb = (int)std::min<unsigned>(hn[4], LONG_BLOCKS);
  if (hn[4] && dr_sort_on() && dense_rows_sorted(0, lists + 4 * L, hn[4], A, B, cnt, nullptr, nullptr, nullptr)) {
    amgd_route_hit(AMGD_R_SG_DRSORT);
  } else if (hn[4]) {             // recount (rows past the hash capacity carry OVERFLOW_MARK)
    double *slab_v = (double *)amgd_alloc_f64((size_t)y->nlb * B->cn * 8 + 8);
    uint32_t *slab_s = (uint32_t *)amgd_alloc((size_t)y->nlb * B->cn * 4 + 4);
    HIPCK(hipMemsetAsync(slab_s, 0, (size_t)y->nlb * B->cn * 4, s));
    k_spgemm_long<0><<<y->nlb, 256, 0, s>>>(lists + 4 * L, hn[4], A->ro, A->col, A->a, B->ro, B->col, B->a,
                                             B->cn, slab_v, slab_s, cnt, nullptr, nullptr, nullptr);
    KCHECK();
    amgd_free(slab_v);
    amgd_free(slab_s);
  }
  y->dist = amgd_scan_u64(cnt, rn);   // cnt := offsets of the distinct layout
  const int win = y->win = kseq ? sg_win() : 0;
  // wide bins (3: block hash, 4: dense slab) split into windowed / hash rows
  unsigned *wn = y->wn;
  if (win && (hn[3] || hn[4])) {
    uint32_t *wlists = y->wlists = (uint32_t *)amgd_alloc(2 * L * 4 + 16);
    unsigned *wc = (unsigned *)amgd_alloc(32);
    HIPCK(hipMemsetAsync(wc, 0, 32, s));
    const uint32_t p0 = g_sg_win_forced ? 0u : sg_win_p0();
    for (int q = 0; q < 2; q++) {
      const unsigned nb = hn[3 + q];
      if (!nb) continue;
      uint32_t *src = lists + (3 + q) * L;
      // windowed rows -> wlists[q]; hash rows compacted into the (copied) bin list
      uint32_t *tmp = (uint32_t *)amgd_alloc((size_t)nb * 4 + 4);
      HIPCK(hipMemcpyAsync(tmp, src, (size_t)nb * 4, hipMemcpyDeviceToDevice, s));
      k_win_split<<<grid_for(nb), 256, 0, s>>>(tmp, nb, A->ro, A->col, B->ro, B->col, ub,
                                               (uint32_t)win, p0, wlists + q * L, src, wc + 2 * q);
      KCHECK();
      amgd_free(tmp);
    }
    amgd_d2h(wn, wc, 16);
    sort_list(wlists, wn[0], rn);
    sort_list(wlists + L, wn[2], rn);
    sort_list(lists + 3 * L, wn[1], rn);
    sort_list(lists + 4 * L, wn[3], rn);
    amgd_free(wc);
    hn[3] = wn[1];
    hn[4] = wn[3];
    y->nlb = (int)std::min<unsigned>(hn[4], LONG_BLOCKS);
  }
  amgd_free(counts);
  return y;
}

// numeric phase on a symbolic state: every output the ordered sum of its products
static dcsr *sg_numeric(const dcsr *A, const dcsr *B, const SgSym *y) {
  hipStream_t s = amgd_s();
  const uint32_t rn = A->rn;
  const uint64_t L = (uint64_t)rn + 1;
  const uint32_t *lists = y->lists, *wlists = y->wlists, *tlist = lists + 5 * L;
  const unsigned *hn = y->hn, *wn = y->wn;
  const unsigned ntiny = y->hc[5];
  if (ntiny) amgd_route_hit(AMGD_R_SG_TINY);
  const bool kseq = y->kseq, wide = y->wide;
  const int win = y->win, nlb = y->nlb;
  const uint64_t *cnt = y->cnt;
  const uint64_t dist = y->dist;
  uint32_t *tcol = (uint32_t *)amgd_alloc(dist * 4 + 4);
  double *ta = (double *)amgd_alloc_f64(dist * 8 + 8);
  uint64_t *cnt2 = (uint64_t *)amgd_alloc(L * 8);
  HIPCK(hipMemsetAsync(cnt2, 0, L * 8, s));
  const uint32_t *densel = lists + 4 * L;
  double *slab_v = nullptr;
  uint32_t *slab_s = nullptr;
  const bool drs = hn[4] && dr_sort_on();
  if (hn[4] && !drs) {
    slab_v = (double *)amgd_alloc_f64((size_t)nlb * B->cn * 8 + 8);
    slab_s = (uint32_t *)amgd_alloc((size_t)nlb * B->cn * 4 + 4);
    HIPCK(hipMemsetAsync(slab_s, 0, (size_t)nlb * B->cn * 4, s));
  }
  uint32_t *curs = nullptr;
  if (win && (wn[0] || wn[2])) curs = (uint32_t *)amgd_alloc(A->nnz * 4 + 4);
  if (g_sg_slot >= 0) amgd_timer_start(g_sg_slot);
#define SG_NUM(KER, NT, LG, bin, gmax)                                                          \
  if (hn[bin]) {                                                                                \
    if (pat)                                                                                    \
      KER<NT, LG, 2, 0><<<(int)std::min<unsigned>(hn[bin], gmax), NT, 0, s>>>(                 \
          lists + (bin) * L, hn[bin], A->ro, A->col, A->a, B->ro, B->col, B->a, 0, cnt2, cnt, tcol, ta); \
    else if (rap)                                                                               \
      KER<NT, LG, 1, 1><<<(int)std::min<unsigned>(hn[bin], gmax), NT, 0, s>>>(                 \
          lists + (bin) * L, hn[bin], A->ro, A->col, A->a, B->ro, B->col, B->a, 0, cnt2, cnt, tcol, ta); \
    else                                                                                        \
      KER<NT, LG, 1, 0><<<(int)std::min<unsigned>(hn[bin], gmax), NT, 0, s>>>(                 \
          lists + (bin) * L, hn[bin], A->ro, A->col, A->a, B->ro, B->col, B->a, 0, cnt2, cnt, tcol, ta); \
  }
  const bool rap = g_sg_slot >= 0;
  const bool pat = g_sg_pattern != 0;
  if (ntiny)
    k_sg_tiny<1><<<grid_for(ntiny, 256, 16384), 256, 0, s>>>(tlist, ntiny, A->ro, A->col, A->a, B->ro,
                                                            B->col, B->a, cnt2, cnt, tcol, ta);
#define SG_WW(W_, rows_, nrw)                                                                   \
  do {                                                                                          \
    const int gw = (int)std::min<unsigned>((nrw + 3) / 4, 16384u);                              \
    if (rap)                                                                                    \
      k_sg_wwin<W_, 1, 1><<<gw, 256, 0, s>>>(rows_, nrw, A->ro, A->col, A->a, B->ro, B->col,     \
                                             B->a, cnt2, cnt, tcol, ta, curs);                  \
    else                                                                                        \
      k_sg_wwin<W_, 1, 0><<<gw, 256, 0, s>>>(rows_, nrw, A->ro, A->col, A->a, B->ro, B->col,     \
                                             B->a, cnt2, cnt, tcol, ta, curs);                  \
  } while (0)
  // threads per row of the 4096- / 8192-slot k-sequential kernels: 512 / 1024 -- one row per
  // work-group walks its layers one dependent step at a time, so more wavefronts per table
  // keep more of each layer's loads in flight (256^3: RAP kernels 1876 -> 1619 ms with 1024
  // threads on the 8192-slot bin; 256 threads on both measured slower, round 2)
  if (hn[0] || hn[1] || hn[2] || hn[3]) amgd_route_hit(kseq ? AMGD_R_SG_KSEQ : AMGD_R_SG_ROW);
  if (win && (wn[0] || wn[2])) amgd_route_hit(AMGD_R_SG_WWIN);
  if (hn[4]) amgd_route_hit(AMGD_R_SG_LONG);
  if (kseq && wide) {
    SG_NUM(k_sg_kseq, 256, 9, 0, 16384u)
    SG_NUM(k_sg_kseq, 256, 11, 1, 16384u)
    SG_NUM(k_sg_kseq, 512, 12, 2, 16384u)
    SG_NUM(k_sg_kseq, 1024, 13, 3, 8192u)
  } else if (kseq) {
    SG_NUM(k_sg_kseq, 64, 9, 0, 65536u)
    SG_NUM(k_sg_kseq, 64, 11, 1, 65536u)
    SG_NUM(k_sg_kseq, 512, 12, 2, 16384u)
    SG_NUM(k_sg_kseq, 1024, 13, 3, 8192u)
  } else {
    SG_NUM(k_sg_row, 64, 9, 0, 65536u)
    SG_NUM(k_sg_row, 64, 11, 1, 65536u)
    SG_NUM(k_sg_row, 64, 12, 2, 65536u)
    SG_NUM(k_sg_row, 256, 13, 3, 8192u)
  }
#undef SG_NUM
  // windowed rows: wave-private 1024-column windows (k_sg_wwin, round 3)
  // (1024 doubles per wavefront: 512 and 2048 measured slower at 256^3 -- 1081 / 1235
  // against 987 ms for the interpolation's windowed products, profiles/r04/ab_sym_ww)
  if (win && wn[0]) SG_WW(1024, wlists, wn[0]);
  if (win && wn[2]) SG_WW(1024, wlists + L, wn[2]);
  bool dr_done = false;
  if (drs) {
    dr_done = dense_rows_sorted(1, densel, hn[4], A, B, cnt2, cnt, tcol, ta);
    if (dr_done) amgd_route_hit(AMGD_R_SG_DRSORT);
    else {                        // a row past DR_MAX_PRODUCTS: the block kernel for all
      slab_v = (double *)amgd_alloc_f64((size_t)nlb * B->cn * 8 + 8);
      slab_s = (uint32_t *)amgd_alloc((size_t)nlb * B->cn * 4 + 4);
      HIPCK(hipMemsetAsync(slab_s, 0, (size_t)nlb * B->cn * 4, s));
    }
  }
  if (hn[4] && !dr_done) {
    if (rap)
      k_spgemm_long<1, 1><<<nlb, 256, 0, s>>>(densel, hn[4], A->ro, A->col, A->a, B->ro, B->col,
                                               B->a, B->cn, slab_v, slab_s, cnt2, cnt, tcol, ta);
    else
      k_spgemm_long<1, 0><<<nlb, 256, 0, s>>>(densel, hn[4], A->ro, A->col, A->a, B->ro, B->col,
                                               B->a, B->cn, slab_v, slab_s, cnt2, cnt, tcol, ta);
  }
#undef SG_WW
  KCHECK();
  if (g_sg_slot >= 0) amgd_timer_stop(g_sg_slot);
  uint64_t nz = amgd_scan_u64(cnt2, rn);
  if (g_sg_slot >= 0) {
    g_sg_bytes += 12 * (A->nnz + B->nnz + nz) + 8 * ((uint64_t)A->rn + B->rn + rn + 3);
    // launches of the RAP-instantiated numeric kernels (the rocprof regex of tools/gpurun_pmc.sh)
    for (int q = 0; q < 4; q++) g_sg_launches += hn[q] ? 1 : 0;
    g_sg_launches += (hn[4] ? 1 : 0) + (win ? (wn[0] ? 1 : 0) + (wn[2] ? 1 : 0) : 0);
  }
  dcsr *X = (dcsr *)malloc(sizeof(dcsr));
  X->rn = rn; X->cn = B->cn; X->nnz = nz;
  X->ro = cnt2;
  if (nz == dist) {               // no cancellation: the distinct layout is final
    X->col = tcol; X->a = ta;
  } else {                        // compact away exact-zero sums
    X->col = (uint32_t *)amgd_alloc(nz * 4 + 4);
    X->a = (double *)amgd_alloc_f64(nz * 8 + 8);
    amgd_compact_rows(cnt, tcol, ta, cnt2, rn, X->col, X->a);
    amgd_free(tcol); amgd_free(ta);
  }
  if (curs) amgd_free(curs);
  if (slab_v) { amgd_free(slab_v); amgd_free(slab_s); }
  return X;
}

static dcsr *spgemm_local(const dcsr *A, const dcsr *B) {
  if (A->cn != B->rn) {
    fprintf(stderr, "omp_amg_amd: spgemm inner dimension mismatch (%u vs %u)\n", A->cn, B->rn);
    abort();
  }
  hipStream_t s = amgd_s();
  static int sglog = -1;
  if (sglog < 0) sglog = getenv("AMGD_SGLOG") != nullptr;
  double t_start = 0;
  if (sglog) { amgd_sync(); t_start = amgd_wtime(); }
  const uint32_t rn = A->rn;
  const int mode = g_sym_mode;
  g_sym_mode = 0;
  SgSym *y = nullptr;
  const uint64_t h = mode ? pat_hash2(A, B) : 0;
  if (mode == 2 && g_sym_kept) {
    const SgSym *k = g_sym_kept;
    const bool kseq = B->rn && B->nnz / B->rn >= KSEQ_MIN && !sg_force_flat();
    if (k->hash == h && k->rn == rn && k->acn == A->cn && k->bcn == B->cn && k->annz == A->nnz &&
        k->bnnz == B->nnz && k->kseq == kseq && k->win == (kseq ? sg_win() : 0)) {
      y = g_sym_kept;
      g_sym_kept = nullptr;
      g_sym_reused++;
      amgd_route_hit(AMGD_R_SG_SYMREUSE);
    }
  }
  const bool reused = y != nullptr;
  if (!y) y = sg_symbolic(A, B);
  dcsr *X = sg_numeric(A, B, y);
  const SgSym info = *y;                    // bin counts for the log
  if (mode == 1) {                          // kept for the next product on these patterns
    amgd_spgemm_sym_drop();
    y->hash = h;
    g_sym_kept = y;
    g_sym_kept_n++;
  } else {
    sym_free(y);
    if (mode == 2) amgd_spgemm_sym_drop();  // one taker only
  }
  if (sglog) {
    uint64_t prods = 0;
    if (rn) {   // products = sum of the per-row upper bounds
      uint64_t *u2 = (uint64_t *)amgd_alloc(((size_t)rn + 1) * 8);
      k_spgemm_ub<<<grid_for(rn), 256, 0, s>>>(A->ro, A->col, rn, B->ro, u2);
      prods = amgd_scan_u64(u2, rn);
      amgd_free(u2);
    }
    amgd_sync();
    double ms = (amgd_wtime() - t_start) * 1e3;
    if (rn) {
      unsigned long long *hd = (unsigned long long *)amgd_alloc(64), hh[6];
      amgd_memset(hd, 0, 48);
      k_span_hist<<<grid_for(rn), 256, 0, s>>>(X->ro, X->col, rn, hd);
      amgd_d2h(hh, hd, 48);
      amgd_free(hd);
      fprintf(stderr, "spgemm span hist (rows >= 1024 out): %llu %llu %llu %llu %llu %llu\n", hh[0],
              hh[1], hh[2], hh[3], hh[4], hh[5]);
    }
    const char *kind = info.kseq ? (info.wide ? (info.win ? "kseq-w+win" : "kseq-w") : (info.win ? "kseq+win" : "kseq"))
                                 : "flat";
    fprintf(stderr, "spgemm %u x %u x %u  nnzA %lu nnzB %lu -> %lu  prods %lu (%.1f G/s)  %s  sym %u/%u num %u/%u/%u/%u dense %u win %u%s  %.2f ms\n",
            rn, A->cn, B->cn, (unsigned long)A->nnz, (unsigned long)B->nnz, (unsigned long)X->nnz,
            (unsigned long)prods, prods / (ms * 1e6), kind, info.hc[0], info.hc[1], info.hn[0], info.hn[1],
            info.hn[2], info.hn[3], info.hn[4], info.wn[0] + info.wn[2],
            mode == 1 ? " kept" : reused ? " symbolic-reused" : "", ms);
  }
  return X;
}

// ---------------------------------------------------------------------------
// Row-sharded SpGEMM (amgd_comm.hip): rows of A split into contiguous ranges of
// equal product count, each rank multiplies its ranges (a row view of A: the
// kernels only read ro[i]..ro[i+1], so no copy), the shard results are laid
// into the global CSR at their offsets and completed by one allgatherv of
// (ro, col, a).  Same kernels on the same rows: bit-identical to one GPU.
// ---------------------------------------------------------------------------
__global__ void k_ro_shift(const uint64_t *src, uint32_t n, uint64_t base, uint64_t *dst) {
  GRID_STRIDE(i, n) dst[i] = src[i] + base;
}
#define SG_SHARD_MIN (1ull << 22)   // products below which one GPU does the whole product
extern "C" dcsr *amgd_spgemm(const dcsr *A, const dcsr *B) {
  const int N = amgd_nshards();
  if (N <= 1 || A->rn < (uint32_t)N || A->cn != B->rn) return spgemm_local(A, B);
  const uint32_t rn = A->rn;
  uint64_t *ub = (uint64_t *)amgd_alloc(((size_t)rn + 1) * 8);
  k_spgemm_ub<<<grid_for(rn), 256, 0, amgd_s()>>>(A->ro, A->col, rn, B->ro, ub);
  KCHECK();
  const uint64_t prods = amgd_scan_u64(ub, rn);
  if (!amgd_shard_worth(prods, SG_SHARD_MIN)) {
    amgd_free(ub);
    return spgemm_local(A, B);
  }
  std::vector<uint32_t> split(N + 1);
  amgd_shard_split(ub, rn, split.data());
  amgd_free(ub);
  std::vector<uint64_t> aro(N + 1), nzs(N + 1, 0);
  amgd_gather_u64_at(A->ro, split.data(), N + 1, aro.data());
  int f, l;
  amgd_my_shards(&f, &l);
  std::vector<dcsr *> xs(N, nullptr);
  for (int q = f; q < l; q++) {
    dcsr v = *A;
    v.rn = split[q + 1] - split[q];
    v.ro = A->ro + split[q];
    v.nnz = aro[q + 1] - aro[q];
    xs[q] = spgemm_local(&v, B);
    nzs[q] = xs[q]->nnz;
  }
  amgd_allgather_u64(nzs.data());
  std::vector<uint64_t> base(N + 1, 0);
  for (int q = 0; q < N; q++) base[q + 1] = base[q] + nzs[q];
  const uint64_t nz = base[N];
  dcsr *X = (dcsr *)malloc(sizeof(dcsr));
  X->rn = rn;
  X->cn = B->cn;
  X->nnz = nz;
  X->ro = (uint64_t *)amgd_alloc(((size_t)rn + 1) * 8);
  X->col = (uint32_t *)amgd_alloc(nz * 4 + 4);
  X->a = (double *)amgd_alloc_f64(nz * 8 + 8);
  hipStream_t s = amgd_s();
  HIPCK(hipMemsetAsync(X->ro, 0, 8, s));
  for (int q = f; q < l; q++) {
    const uint32_t n = split[q + 1] - split[q];
    if (n) k_ro_shift<<<grid_for(n), 256, 0, s>>>(xs[q]->ro + 1, n, base[q], X->ro + split[q] + 1);
    if (nzs[q]) {
      HIPCK(hipMemcpyAsync(X->col + base[q], xs[q]->col, nzs[q] * 4, hipMemcpyDeviceToDevice, s));
      HIPCK(hipMemcpyAsync(X->a + base[q], xs[q]->a, nzs[q] * 8, hipMemcpyDeviceToDevice, s));
    }
    dcsr_free(&xs[q]);
  }
  KCHECK();
  std::vector<uint64_t> off(3 * (N + 1));
  for (int q = 0; q <= N; q++) {
    off[q] = ((uint64_t)split[q] + 1) * 8;   // ro entries split[q]+1 .. split[q+1]
    off[(N + 1) + q] = base[q] * 4;
    off[2 * (N + 1) + q] = base[q] * 8;
  }
  void *bufs[3] = {X->ro, X->col, X->a};
  amgd_allgatherv(3, bufs, off.data());
  return X;
}

// Pattern of A*B with the values left unspecified (every stored value is nonzero; the
// caller overwrites them): for operands whose stored values are all > 0 no sum can
// cancel, so the exact-zero drop of the reference's mxm removes nothing and the
// structural pattern IS the product's pattern.  The hash-bin rows then need no
// ordered numeric pass: keys are inserted in any order (no per-layer barrier, no value
// loads) and emitted sorted.  Falls back to amgd_spgemm when a value is not > 0.
__global__ void k_allpos(const double *a, uint64_t n, unsigned *bad) {
  GRID_STRIDE(k, n) if (!(a[k] > 0.0)) *bad = 1u;
}
static int g_sg_pat_on = 1;     // amgd_spgemm_set_pattern(0): full products (A/B runs)
extern "C" void amgd_spgemm_set_pattern(int on) { g_sg_pat_on = on < 0 ? 1 : on; }
extern "C" dcsr *amgd_spgemm_pattern(const dcsr *A, const dcsr *B) {
  if (!g_sg_pat_on) return amgd_spgemm(A, B);
  unsigned *bad = (unsigned *)amgd_alloc(16);
  amgd_memset(bad, 0, 4);
  if (A->nnz) k_allpos<<<grid_for(A->nnz), 256, 0, amgd_s()>>>(A->a, A->nnz, bad);
  if (B->nnz) k_allpos<<<grid_for(B->nnz), 256, 0, amgd_s()>>>(B->a, B->nnz, bad);
  KCHECK();
  unsigned hb = 0;
  amgd_d2h(&hb, bad, 4);
  amgd_free(bad);
  if (hb) return amgd_spgemm(A, B);
  g_sg_pattern = 1;
  dcsr *X = amgd_spgemm(A, B);
  g_sg_pattern = 0;
  return X;
}
__global__ void k_compact_rows(const uint64_t *sro, const uint32_t *scol, const double *sa,
                               const uint64_t *dro, uint32_t rn, uint32_t *dcol, double *da) {
  GRID_STRIDE(i, rn) {
    uint64_t s0 = sro[i], d0 = dro[i], n = dro[i + 1] - d0;
    for (uint64_t t = 0; t < n; t++) { dcol[d0 + t] = scol[s0 + t]; da[d0 + t] = sa[s0 + t]; }
  }
}
// long rows: one wavefront per row, coalesced copies
__global__ __launch_bounds__(256) void k_compact_rows_wave(const uint64_t *sro, const uint32_t *scol,
                                                          const double *sa, const uint64_t *dro,
                                                          uint32_t rn, uint32_t *dcol, double *da) {
  const int lane = threadIdx.x & 63;
  for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; i < rn;
       i += ((uint64_t)gridDim.x * blockDim.x) >> 6) {
    const uint64_t s0 = sro[i], d0 = dro[i], n = dro[i + 1] - d0;
    for (uint64_t t = lane; t < n; t += 64) { dcol[d0 + t] = scol[s0 + t]; da[d0 + t] = sa[s0 + t]; }
  }
}
void amgd_compact_rows(const uint64_t *sro, const uint32_t *scol, const double *sa,
                       const uint64_t *dro, uint32_t rn, uint32_t *dcol, double *da) {
  if (!rn) return;
  uint64_t nz = 0;
  HIPCK(hipMemcpyAsync(&nz, dro + rn, 8, hipMemcpyDeviceToHost, amgd_s()));
  HIPCK(hipStreamSynchronize(amgd_s()));
  if (nz >= 16ull * rn)
    k_compact_rows_wave<<<grid_for((uint64_t)rn * 64, 256, 65536), 256, 0, amgd_s()>>>(
        sro, scol, sa, dro, rn, dcol, da);
  else
    k_compact_rows<<<grid_for(rn), 256, 0, amgd_s()>>>(sro, scol, sa, dro, rn, dcol, da);
  KCHECK();
}

// ---------------------------------------------------------------------------
// device CSR -> host arrays with gslib's `uint` (unsigned long) indices
// ---------------------------------------------------------------------------
__global__ void k_widen(const uint32_t *c, uint64_t n, uint64_t *o) { GRID_STRIDE(k, n) o[k] = c[k]; }
extern "C" uint64_t amgd_to_host_cols(const dcsr *A, unsigned long *h_ro, unsigned long *h_col,
                                      double *h_a) {
  static_assert(sizeof(unsigned long) == 8, "LP64 expected");
  amgd_d2h(h_ro, A->ro, ((size_t)A->rn + 1) * 8);
  if (A->nnz) {
    uint64_t *w = (uint64_t *)amgd_alloc(A->nnz * 8);
    k_widen<<<grid_for(A->nnz), 256, 0, amgd_s()>>>(A->col, A->nnz, w);
    amgd_d2h(h_col, w, A->nnz * 8);
    amgd_free(w);
    amgd_d2h(h_a, A->a, A->nnz * 8);
  }
  return A->nnz;
}

// ---------------------------------------------------------------------------
// SpMV micro-benchmark matrices (test API only): rn rows of len0..len1 entries,
// columns start(i) + k*gap (sorted, distinct, start spread over the column range)
// ---------------------------------------------------------------------------
__global__ void k_bench_rowlen(uint32_t rn, uint32_t len0, uint32_t len1, uint64_t *cnt) {
  GRID_STRIDE(i, rn) {
    uint64_t h = (i * 0x9E3779B97F4A7C15ull) >> 33;
    cnt[i] = len0 + (len1 > len0 ? h % (len1 - len0 + 1) : 0);
  }
}
__global__ void k_bench_fill(const uint64_t *ro, uint32_t rn, uint32_t cn, uint32_t gap,
                             uint32_t *col, double *a) {
  GRID_STRIDE(i, rn) {
    const uint64_t k0 = ro[i], len = ro[i + 1] - k0;
    const uint64_t span = len ? (len - 1) * gap + 1 : 0;
    uint64_t start = (uint64_t)i * cn / rn;
    start = start > span / 2 ? start - span / 2 : 0;
    if (start + span > cn) start = cn > span ? cn - span : 0;
    for (uint64_t k = 0; k < len; k++) {
      col[k0 + k] = (uint32_t)(start + k * gap);
      a[k0 + k] = 1.0 + (double)((k0 + k) % 7) * 0.125;
    }
  }
}
extern "C" dcsr *amgd_bench_matrix(uint32_t rn, uint32_t cn, uint32_t len0, uint32_t len1,
                                   uint32_t gap) {
  hipStream_t s = amgd_s();
  uint64_t *ro = (uint64_t *)amgd_alloc(((size_t)rn + 1) * 8);
  k_bench_rowlen<<<grid_for(rn), 256, 0, s>>>(rn, len0, len1, ro);
  const uint64_t nnz = amgd_scan_u64(ro, rn);
  dcsr *A = (dcsr *)malloc(sizeof(dcsr));
  A->rn = rn; A->cn = cn; A->nnz = nnz; A->ro = ro;
  A->col = (uint32_t *)amgd_alloc(nnz * 4 + 4);
  A->a = (double *)amgd_alloc_f64(nnz * 8 + 8);
  k_bench_fill<<<grid_for(rn), 256, 0, s>>>(ro, rn, cn, gap, A->col, A->a);
  KCHECK();
  return A;
}
