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
  double *v2 = (double *)amgd_alloc(nz * 8 + 8);
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
  A->a = (double *)amgd_alloc(kept * 8 + 8);
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
extern "C" dcsr *amgd_sub_mat(const dcsr *A, const uint8_t *vr, const uint8_t *vc) {
  hipStream_t s = amgd_s();
  uint32_t *rmap = (uint32_t *)amgd_alloc(((size_t)A->rn + 1) * 4);
  uint32_t *cmap = (uint32_t *)amgd_alloc(((size_t)A->cn + 1) * 4);
  uint32_t srn = amgd_mask_rank(vr, A->rn, rmap);
  uint32_t scn = amgd_mask_rank(vc, A->cn, cmap);
  uint64_t *cnt = (uint64_t *)amgd_alloc(((size_t)srn + 1) * 8);
  if (A->rn) k_sub_count<<<grid_for(A->rn), 256, 0, s>>>(A->ro, A->col, A->rn, vr, vc, rmap, cnt);
  KCHECK();
  uint64_t nz = amgd_scan_u64(cnt, srn);
  dcsr *S = (dcsr *)malloc(sizeof(dcsr));
  S->rn = srn; S->cn = scn; S->nnz = nz; S->ro = cnt;
  S->col = (uint32_t *)amgd_alloc(nz * 4 + 4);
  S->a = (double *)amgd_alloc(nz * 8 + 8);
  if (A->rn)
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
__global__ void k_col_count(const uint32_t *col, uint64_t nz, uint64_t *cnt) {
  GRID_STRIDE(k, nz) atomicAdd((unsigned long long *)&cnt[col[k]], 1ull);
}
__global__ void k_tr_fill(const uint64_t *perm, const uint32_t *row, const double *a, uint64_t nz,
                          uint32_t *tcol, double *ta) {
  GRID_STRIDE(t, nz) {
    uint64_t p = perm[t];
    tcol[t] = row[p];
    ta[t] = a[p];
  }
}
extern "C" dcsr *amgd_transpose(const dcsr *A, uint64_t **perm_out) {
  hipStream_t s = amgd_s();
  uint64_t nz = A->nnz;
  uint64_t *cnt = (uint64_t *)amgd_alloc(((size_t)A->cn + 1) * 8);
  HIPCK(hipMemsetAsync(cnt, 0, ((size_t)A->cn + 1) * 8, s));
  uint64_t *perm = (uint64_t *)amgd_alloc(nz * 8 + 8);
  if (nz) {
    k_col_count<<<grid_for(nz), 256, 0, s>>>(A->col, nz, cnt);
    uint64_t *iota = (uint64_t *)amgd_alloc(nz * 8 + 8);
    uint32_t *kout = (uint32_t *)amgd_alloc(nz * 4 + 4);
    k_iota_u64<<<grid_for(nz), 256, 0, s>>>(iota, nz);
    size_t tb = 0;
    int eb = bits_for(A->cn);
    HIPCK(rocprim::radix_sort_pairs(nullptr, tb, A->col, kout, iota, perm, (size_t)nz, 0, eb, s));
    void *tmp = amgd_alloc(tb + 16);
    HIPCK(rocprim::radix_sort_pairs(tmp, tb, A->col, kout, iota, perm, (size_t)nz, 0, eb, s));
    amgd_free(tmp); amgd_free(iota); amgd_free(kout);
  }
  amgd_scan_u64(cnt, A->cn);
  dcsr *T = (dcsr *)malloc(sizeof(dcsr));
  T->rn = A->cn; T->cn = A->rn; T->nnz = nz; T->ro = cnt;
  T->col = (uint32_t *)amgd_alloc(nz * 4 + 4);
  T->a = (double *)amgd_alloc(nz * 8 + 8);
  if (nz) {
    uint32_t *row = (uint32_t *)amgd_alloc(nz * 4 + 4);
    k_row_of_entry<<<grid_for(A->rn), 256, 0, s>>>(A->ro, A->rn, row);
    k_tr_fill<<<grid_for(nz), 256, 0, s>>>(perm, row, A->a, nz, T->col, T->a);
    KCHECK();
    amgd_free(row);
  }
  if (perm_out) *perm_out = perm;
  else amgd_free(perm);
  return T;
}

// ---------------------------------------------------------------------------
// SpMV: t_i = sum_j a_ij x_col(j), left to right from +0.0 (apply_M).
// CSR-stream: a 256-thread block owns 256 consecutive rows, stages their
// (col, a) range through LDS with coalesced loads when it fits, then each
// thread sums its own row in order.  Long-row blocks read rows directly.
// ---------------------------------------------------------------------------
#define SPMV_ROWS 256
#define SPMV_LDS 2048
__global__ __launch_bounds__(256) void k_spmv(const uint64_t *ro, const uint32_t *col,
                                              const double *a, uint32_t rn, const double *x,
                                              double *z, double alpha, const double *y,
                                              double beta, const uint8_t *f) {
  __shared__ uint32_t sc[SPMV_LDS];
  __shared__ double sa[SPMV_LDS];
  for (uint64_t r0 = (uint64_t)blockIdx.x * SPMV_ROWS; r0 < rn;
       r0 += (uint64_t)gridDim.x * SPMV_ROWS) {
    uint64_t r1 = min((uint64_t)rn, r0 + SPMV_ROWS);
    uint64_t b0 = ro[r0], b1 = ro[r1];
    uint64_t i = r0 + threadIdx.x;
    double t = 0;
    if (b1 - b0 <= SPMV_LDS) {
      for (uint64_t k = b0 + threadIdx.x; k < b1; k += blockDim.x) {
        sc[k - b0] = col[k];
        sa[k - b0] = a[k];
      }
      __syncthreads();
      if (i < r1)
        for (uint64_t k = ro[i]; k < ro[i + 1]; k++) t += x ? sa[k - b0] * x[sc[k - b0]] : sa[k - b0];
      __syncthreads();
    } else if (i < r1) {
      for (uint64_t k = ro[i]; k < ro[i + 1]; k++) t += x ? a[k] * x[col[k]] : a[k];
    }
    if (i < r1) {
      double v = (alpha == 0.0 || y == nullptr) ? beta * t : alpha * y[i] + beta * t;
      if (f) v = v * (f[i] ? 1.0 : 0.0);
      z[i] = v;
    }
  }
}
// long rows: one wavefront per row; the 64 lanes load and multiply a chunk
// (coalesced) into LDS, lane 0 adds the chunk in order -- same sum, same order.
__global__ __launch_bounds__(256) void k_spmv_wave(const uint64_t *ro, const uint32_t *col,
                                                   const double *a, uint32_t rn, const double *x,
                                                   double *z, double alpha, const double *y,
                                                   double beta, const uint8_t *f) {
  __shared__ double buf[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + w; i < rn; i += (uint64_t)gridDim.x * 4) {
    uint64_t k0 = ro[i], k1 = ro[i + 1];
    double t = 0;
    for (uint64_t c0 = k0; c0 < k1; c0 += 64) {
      uint64_t k = c0 + lane;
      if (k < k1) buf[w][lane] = x ? a[k] * x[col[k]] : a[k];
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      if (lane == 0) {
        int m = (int)min((uint64_t)64, k1 - c0);
        int q = 0;
        for (; q + 8 <= m; q += 8) {
          double v0 = buf[w][q], v1 = buf[w][q + 1], v2 = buf[w][q + 2], v3 = buf[w][q + 3];
          double v4 = buf[w][q + 4], v5 = buf[w][q + 5], v6 = buf[w][q + 6], v7 = buf[w][q + 7];
          t += v0; t += v1; t += v2; t += v3; t += v4; t += v5; t += v6; t += v7;
        }
        for (; q < m; q++) t += buf[w][q];
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    if (lane == 0) {
      double v = (alpha == 0.0 || y == nullptr) ? beta * t : alpha * y[i] + beta * t;
      if (f) v = v * (f[i] ? 1.0 : 0.0);
      z[i] = v;
    }
  }
}
extern "C" void amgd_spmv(const dcsr *M, const double *x, double *z, double alpha, const double *y,
                          double beta, const uint8_t *f) {
  if (M->rn == 0) return;
  if (M->nnz >= 32ull * M->rn) {
    int g = (int)std::min<uint64_t>((M->rn + 3) / 4, 65536);
    k_spmv_wave<<<g, 256, 0, amgd_s()>>>(M->ro, M->col, M->a, M->rn, x, z, alpha, y, beta, f);
  } else {
    int g = (int)std::min<uint64_t>((M->rn + SPMV_ROWS - 1) / SPMV_ROWS, 16384);
    k_spmv<<<g, 256, 0, amgd_s()>>>(M->ro, M->col, M->a, M->rn, x, z, alpha, y, beta, f);
  }
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
extern "C" void amgd_diag(const dcsr *A, double *D) {
  if (A->rn) k_diag<<<grid_for(A->rn), 256, 0, amgd_s()>>>(A->ro, A->col, A->a, A->rn, D);
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
extern "C" void amgd_diag_op(dcsr *A, const double *D, int op) {
  if (A->rn) k_diag_op<<<grid_for(A->rn), 256, 0, amgd_s()>>>(A->ro, A->col, A->a, A->rn, D, op);
  KCHECK();
}
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
template <bool FILL>
__global__ void k_mpm(const uint64_t *aro, const uint32_t *acol, const double *aa,
                      const uint64_t *bro, const uint32_t *bcol, const double *ba, uint32_t rn,
                      double alpha, double beta, uint64_t *cnt, const uint64_t *xro,
                      uint32_t *xcol, double *xa) {
  GRID_STRIDE(i, rn) {
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
extern "C" dcsr *amgd_mpm(double alpha, const dcsr *A, double beta, const dcsr *B) {
  if (A->rn != B->rn || A->cn != B->cn) {
    fprintf(stderr, "omp_amg_amd: mpm dimension mismatch (%u x %u vs %u x %u)\n", A->rn, A->cn,
            B->rn, B->cn);
    abort();
  }
  hipStream_t s = amgd_s();
  uint64_t *cnt = (uint64_t *)amgd_alloc(((size_t)A->rn + 1) * 8);
  if (A->rn)
    k_mpm<false><<<grid_for(A->rn), 256, 0, s>>>(A->ro, A->col, A->a, B->ro, B->col, B->a, A->rn,
                                                  alpha, beta, cnt, nullptr, nullptr, nullptr);
  KCHECK();
  uint64_t nz = amgd_scan_u64(cnt, A->rn);
  dcsr *X = (dcsr *)malloc(sizeof(dcsr));
  X->rn = A->rn; X->cn = A->cn; X->nnz = nz; X->ro = cnt;
  X->col = (uint32_t *)amgd_alloc(nz * 4 + 4);
  X->a = (double *)amgd_alloc(nz * 8 + 8);
  if (A->rn)
    k_mpm<true><<<grid_for(A->rn), 256, 0, s>>>(A->ro, A->col, A->a, B->ro, B->col, B->a, A->rn,
                                                 alpha, beta, nullptr, X->ro, X->col, X->a);
  KCHECK();
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
extern "C" dcsr *amgd_mxmpoint(const dcsr *A, const dcsr *B) {
  if (A->rn != B->rn || A->cn != B->cn) {
    fprintf(stderr, "omp_amg_amd: mxmpoint dimension mismatch\n");
    abort();
  }
  hipStream_t s = amgd_s();
  uint64_t *cnt = (uint64_t *)amgd_alloc(((size_t)A->rn + 1) * 8);
  if (A->rn)
    k_pointwise<false><<<grid_for(A->rn), 256, 0, s>>>(A->ro, A->col, A->a, B->ro, B->col, B->a,
                                                        A->rn, cnt, nullptr, nullptr, nullptr);
  uint64_t nz = amgd_scan_u64(cnt, A->rn);
  dcsr *X = (dcsr *)malloc(sizeof(dcsr));
  X->rn = A->rn; X->cn = A->cn; X->nnz = nz; X->ro = cnt;
  X->col = (uint32_t *)amgd_alloc(nz * 4 + 4);
  X->a = (double *)amgd_alloc(nz * 8 + 8);
  if (A->rn)
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
// Symbolic pass counts distinct columns, numeric pass accumulates.  Rows are
// binned by their product upper bound:
//   short rows : one wavefront per row, open-addressing hash in LDS.  Steps
//                over k are sequential; within a step the 64 lanes take
//                distinct columns of B's row k, so every slot sees its
//                additions in ascending k -- bit-exact Gustavson.
//   long rows  : one 256-thread block per row, dense accumulator in a global
//                scratch slab (one per resident block), block barrier per k,
//                emitted in column order by a sweep over the touched range.
// ---------------------------------------------------------------------------
#define HS_SLOTS 2048           // LDS hash slots per wavefront row
#define SHORT_UB 1024           // products upper bound for the LDS path
#define EMPTY_KEY 0xffffffffu
#define LONG_BLOCKS 512         // resident long-row blocks (dense slabs)

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
__global__ void k_split_rows(const uint64_t *ub, uint32_t rn, uint32_t *shortl, uint32_t *longl,
                             unsigned *counts) {
  // every lane of a wave iterates the same number of times (wave_append needs the whole wave)
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t iters = (rn + stride - 1) / stride;
  for (uint64_t it = 0; it < iters; it++) {
    uint64_t i = i0 + it * stride;
    bool v = i < rn;
    bool sh = v && ub[i] <= SHORT_UB;
    unsigned ps = wave_append(&counts[0], sh);
    unsigned pl = wave_append(&counts[1], v && !sh);
    if (sh) shortl[ps] = (uint32_t)i;
    else if (v) longl[pl] = (uint32_t)i;
  }
}

__device__ inline uint32_t hslot(uint32_t j) { return (j * 2654435761u) >> (32 - 11); }

// MODE 0: count distinct; MODE 1: numeric -> write sorted nonzeros at xro[i], count in cnt[i]
template <int MODE>
__global__ __launch_bounds__(64) void k_spgemm_short(
    const uint32_t *rows, uint32_t nrows, const uint64_t *aro, const uint32_t *acol,
    const double *aa, const uint64_t *bro, const uint32_t *bcol, const double *ba, uint64_t *cnt,
    const uint64_t *xro, uint32_t *xcol, double *xa) {
  __shared__ uint32_t hk[HS_SLOTS];
  __shared__ double hv[HS_SLOTS];
  __shared__ uint32_t ok[SHORT_UB];
  __shared__ double ov[SHORT_UB];
  const int lane = threadIdx.x;
  for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    uint32_t i = rows[r];
    for (int s = lane; s < HS_SLOTS; s += 64) { hk[s] = EMPTY_KEY; hv[s] = 0.0; }
    __syncthreads();
    uint64_t a0 = aro[i], a1 = aro[i + 1];
    for (uint64_t ka = a0; ka < a1; ka++) {
      uint32_t k = acol[ka];
      if (ka + 1 < a1 && acol[ka + 1] == k) continue;
      double av = aa[ka];
      uint64_t b0 = bro[k], b1 = bro[k + 1];
      uint64_t nch = (b1 - b0 + 63) / 64;
      for (uint64_t ch = 0; ch < nch; ch++) {
        uint64_t kb = b0 + ch * 64 + lane;
        if (kb < b1) {
          uint32_t j = bcol[kb];
          uint32_t sl = hslot(j);
          while (true) {
            uint32_t old = atomicCAS(&hk[sl], EMPTY_KEY, j);
            if (old == EMPTY_KEY || old == j) break;
            sl = (sl + 1) & (HS_SLOTS - 1);
          }
          if (MODE == 1) hv[sl] = hv[sl] + ba[kb] * av;
        }
        __syncthreads();   // slot updates of chunk/step t land before step t+1
      }
    }
    // gather occupied slots (numeric: nonzero only) into ok/ov, then rank-sort
    __shared__ unsigned nout;
    if (lane == 0) nout = 0;
    __syncthreads();
    for (int s = lane; s < HS_SLOTS; s += 64) {
      uint32_t key = hk[s];
      bool take = key != EMPTY_KEY && (MODE == 0 || hv[s] != 0.0);
      if (take) {
        unsigned p = atomicAdd(&nout, 1u);
        ok[p] = key;
        if (MODE == 1) ov[p] = hv[s];
      }
    }
    __syncthreads();
    unsigned n = nout;
    if (MODE == 0) {
      if (lane == 0) cnt[i] = n;
    } else {
      uint64_t base = xro[i];
      for (unsigned e = lane; e < n; e += 64) {
        uint32_t key = ok[e];
        unsigned rank = 0;
        for (unsigned f = 0; f < n; f++) rank += ok[f] < key;
        xcol[base + rank] = key;
        xa[base + rank] = ov[e];
      }
      if (lane == 0) cnt[i] = n;
    }
    __syncthreads();
  }
}

// long rows: block per row, dense slab acc[cn] + stamp[cn] per resident block
template <int MODE>
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

// mid rows (more than SHORT_UB products): one 256-thread block per row, an
// 8192-slot open-addressing hash in LDS, a block barrier per k step (so every
// slot sees its additions in ascending k), and a bitonic sort of the (column,
// value) pairs for the ordered write.  Rows with more than MID_CAP distinct
// columns overflow to the dense-slab kernel above.
#define MID_SLOTS 8192
#define MID_CAP 4096
#define OVERFLOW_MARK 0xffffffffffffffffull
__device__ inline uint32_t hslot13(uint32_t j) { return (j * 2654435761u) >> (32 - 13); }

template <int MODE>
__global__ __launch_bounds__(256) void k_spgemm_mid(const uint32_t *rows, uint32_t nrows,
                                                    const uint64_t *aro, const uint32_t *acol,
                                                    const double *aa, const uint64_t *bro,
                                                    const uint32_t *bcol, const double *ba,
                                                    uint64_t *cnt, const uint64_t *xro,
                                                    uint32_t *xcol, double *xa) {
  __shared__ uint32_t hk[MID_SLOTS];
  __shared__ double hv[MID_SLOTS];
  __shared__ uint32_t sk[MODE == 1 ? MID_CAP : 1];
  __shared__ double sv[MODE == 1 ? MID_CAP : 1];
  __shared__ unsigned nfill, nout;
  __shared__ int ovf;
  const int tid = threadIdx.x;
  for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    uint32_t i = rows[r];
    for (int q = tid; q < MID_SLOTS; q += 256) { hk[q] = EMPTY_KEY; hv[q] = 0.0; }
    if (tid == 0) { nfill = 0; nout = 0; ovf = 0; }
    __syncthreads();
    uint64_t a0 = aro[i], a1 = aro[i + 1];
    for (uint64_t ka = a0; ka < a1 && !ovf; ka++) {
      uint32_t k = acol[ka];
      if (ka + 1 < a1 && acol[ka + 1] == k) continue;
      double av = aa[ka];
      uint64_t b0 = bro[k], b1 = bro[k + 1];
      for (uint64_t c0 = b0; c0 < b1; c0 += 256) {
        uint64_t kb = c0 + tid;
        if (kb < b1 && !ovf) {
          uint32_t j = bcol[kb];
          uint32_t sl = hslot13(j);
          bool ok = true;
          while (true) {
            uint32_t old = atomicCAS(&hk[sl], EMPTY_KEY, j);
            if (old == EMPTY_KEY) {
              if (atomicAdd(&nfill, 1u) >= MID_CAP) { ovf = 1; ok = false; }
              break;
            }
            if (old == j) break;
            sl = (sl + 1) & (MID_SLOTS - 1);
          }
          if (MODE == 1 && ok) hv[sl] = hv[sl] + ba[kb] * av;
        }
        __syncthreads();
      }
    }
    __syncthreads();
    if (ovf) {                    // symbolic only (numeric rows were routed by count)
      if (tid == 0) cnt[i] = OVERFLOW_MARK;
      __syncthreads();
      continue;
    }
    if (MODE == 0) {
      if (tid == 0) cnt[i] = nfill;
      __syncthreads();
      continue;
    }
    for (int q = tid; q < MID_SLOTS; q += 256) {
      uint32_t key = hk[q];
      if (key != EMPTY_KEY && hv[q] != 0.0) {
        unsigned p = atomicAdd(&nout, 1u);
        sk[p] = key;
        sv[p] = hv[q];
      }
    }
    __syncthreads();
    unsigned n = nout, P = 1;
    while (P < n) P <<= 1;
    for (unsigned q = n + tid; q < P; q += 256) { sk[q] = EMPTY_KEY; sv[q] = 0.0; }
    __syncthreads();
    for (unsigned size = 2; size <= P; size <<= 1)
      for (unsigned stride = size >> 1; stride > 0; stride >>= 1) {
        for (unsigned t = tid; t < P / 2; t += 256) {
          unsigned lo = 2 * t - (t & (stride - 1));
          unsigned hi = lo + stride;
          bool up = ((lo & size) == 0);
          uint32_t kl = sk[lo], kh = sk[hi];
          if ((kl > kh) == up) {
            sk[lo] = kh; sk[hi] = kl;
            double v = sv[lo]; sv[lo] = sv[hi]; sv[hi] = v;
          }
        }
        __syncthreads();
      }
    uint64_t base = xro[i];
    for (unsigned q = tid; q < n; q += 256) { xcol[base + q] = sk[q]; xa[base + q] = sv[q]; }
    if (tid == 0) cnt[i] = n;
    __syncthreads();
  }
}
__global__ void k_route_overflow(const uint32_t *midl, uint32_t nmid, const uint64_t *cnt,
                                 uint32_t *midok, uint32_t *dense, unsigned *counts) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t r0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t iters = (nmid + stride - 1) / stride;
  for (uint64_t it = 0; it < iters; it++) {
    uint64_t r = r0 + it * stride;
    bool v = r < nmid;
    uint32_t i = v ? midl[r] : 0;
    bool o = v && cnt[i] == OVERFLOW_MARK;
    unsigned p0 = wave_append(&counts[0], v && !o);
    unsigned p1 = wave_append(&counts[1], o);
    if (v && !o) midok[p0] = i;
    if (o) dense[p1] = i;
  }
}

void amgd_compact_rows(const uint64_t *sro, const uint32_t *scol, const double *sa,
                       const uint64_t *dro, uint32_t rn, uint32_t *dcol, double *da);

// event timing of the numeric SpGEMM kernels (the RAP products) + algorithmic bytes:
// A (12 B/nnz + 8 B/row), B (12 B/nnz + 8 B/row) and X (12 B/nnz + 8 B/row) once each.
static int g_sg_slot = -1;
static uint64_t g_sg_bytes = 0;
extern "C" void amgd_spgemm_set_timer(int slot) { g_sg_slot = slot; }
extern "C" void amgd_spgemm_bytes_reset(void) { g_sg_bytes = 0; }
extern "C" uint64_t amgd_spgemm_bytes(void) { return g_sg_bytes; }

extern "C" dcsr *amgd_spgemm(const dcsr *A, const dcsr *B) {
  if (A->cn != B->rn) {
    fprintf(stderr, "omp_amg_amd: spgemm inner dimension mismatch (%u vs %u)\n", A->cn, B->rn);
    abort();
  }
  hipStream_t s = amgd_s();
  uint32_t rn = A->rn;
  uint64_t *ub = (uint64_t *)amgd_alloc(((size_t)rn + 1) * 8);
  uint32_t *shortl = (uint32_t *)amgd_alloc(((size_t)rn + 1) * 4);
  uint32_t *longl = (uint32_t *)amgd_alloc(((size_t)rn + 1) * 4);
  unsigned *counts = (unsigned *)amgd_alloc(8);
  HIPCK(hipMemsetAsync(counts, 0, 8, s));
  if (rn) {
    k_spgemm_ub<<<grid_for(rn), 256, 0, s>>>(A->ro, A->col, rn, B->ro, ub);
    k_split_rows<<<grid_for(rn), 256, 0, s>>>(ub, rn, shortl, longl, counts);
    KCHECK();
  }
  unsigned hc[2];
  amgd_d2h(hc, counts, 8);
  // the row lists come out of atomics in arbitrary order; rows are independent
  // so order does not affect results
  uint64_t *cnt = (uint64_t *)amgd_alloc(((size_t)rn + 1) * 8);
  HIPCK(hipMemsetAsync(cnt, 0, ((size_t)rn + 1) * 8, s));
  double *slab_v = nullptr;
  uint32_t *slab_s = nullptr;
  int gs = (int)std::min<unsigned>(std::max(hc[0], 1u), 65536u);
  // symbolic: short rows (wave hash), mid rows (block hash, may overflow)
  if (hc[0])
    k_spgemm_short<0><<<gs, 64, 0, s>>>(shortl, hc[0], A->ro, A->col, A->a, B->ro, B->col, B->a,
                                        cnt, nullptr, nullptr, nullptr);
  if (hc[1])
    k_spgemm_mid<0><<<(int)std::min<unsigned>(hc[1], 16384u), 256, 0, s>>>(
        longl, hc[1], A->ro, A->col, A->a, B->ro, B->col, B->a, cnt, nullptr, nullptr, nullptr);
  KCHECK();
  uint32_t *midok = nullptr, *densel = nullptr;
  unsigned hr[2] = {0, 0};
  if (hc[1]) {
    midok = (uint32_t *)amgd_alloc((size_t)hc[1] * 4 + 4);
    densel = (uint32_t *)amgd_alloc((size_t)hc[1] * 4 + 4);
    unsigned *rc = (unsigned *)amgd_alloc(8);
    HIPCK(hipMemsetAsync(rc, 0, 8, s));
    k_route_overflow<<<grid_for(hc[1]), 256, 0, s>>>(longl, hc[1], cnt, midok, densel, rc);
    amgd_d2h(hr, rc, 8);
    amgd_free(rc);
  }
  int nlb = (int)std::min<unsigned>(hr[1], LONG_BLOCKS);
  if (hr[1]) {
    slab_v = (double *)amgd_alloc((size_t)nlb * B->cn * 8 + 8);
    slab_s = (uint32_t *)amgd_alloc((size_t)nlb * B->cn * 4 + 4);
    HIPCK(hipMemsetAsync(slab_s, 0, (size_t)nlb * B->cn * 4, s));
    k_spgemm_long<0><<<nlb, 256, 0, s>>>(densel, hr[1], A->ro, A->col, A->a, B->ro, B->col, B->a,
                                          B->cn, slab_v, slab_s, cnt, nullptr, nullptr, nullptr);
    KCHECK();
  }
  uint64_t dist = amgd_scan_u64(cnt, rn);   // cnt := offsets of the distinct layout
  uint32_t *tcol = (uint32_t *)amgd_alloc(dist * 4 + 4);
  double *ta = (double *)amgd_alloc(dist * 8 + 8);
  uint64_t *cnt2 = (uint64_t *)amgd_alloc(((size_t)rn + 1) * 8);
  HIPCK(hipMemsetAsync(cnt2, 0, ((size_t)rn + 1) * 8, s));
  if (hr[1]) HIPCK(hipMemsetAsync(slab_s, 0, (size_t)nlb * B->cn * 4, s));
  if (g_sg_slot >= 0) amgd_timer_start(g_sg_slot);
  if (hc[0])
    k_spgemm_short<1><<<gs, 64, 0, s>>>(shortl, hc[0], A->ro, A->col, A->a, B->ro, B->col, B->a,
                                        cnt2, cnt, tcol, ta);
  if (hr[0])
    k_spgemm_mid<1><<<(int)std::min<unsigned>(hr[0], 16384u), 256, 0, s>>>(
        midok, hr[0], A->ro, A->col, A->a, B->ro, B->col, B->a, cnt2, cnt, tcol, ta);
  if (hr[1])
    k_spgemm_long<1><<<nlb, 256, 0, s>>>(densel, hr[1], A->ro, A->col, A->a, B->ro, B->col, B->a,
                                          B->cn, slab_v, slab_s, cnt2, cnt, tcol, ta);
  KCHECK();
  if (g_sg_slot >= 0) amgd_timer_stop(g_sg_slot);
  if (midok) { amgd_free(midok); amgd_free(densel); }
  uint64_t nz = amgd_scan_u64(cnt2, rn);
  if (g_sg_slot >= 0)
    g_sg_bytes += 12 * (A->nnz + B->nnz + nz) + 8 * ((uint64_t)A->rn + B->rn + rn + 3);
  dcsr *X = (dcsr *)malloc(sizeof(dcsr));
  X->rn = rn; X->cn = B->cn; X->nnz = nz;
  if (nz == dist) {               // no cancellation: the distinct layout is final
    X->ro = cnt2; X->col = tcol; X->a = ta;
    amgd_free(cnt);
  } else {                        // compact away exact-zero sums
    X->ro = cnt2;
    X->col = (uint32_t *)amgd_alloc(nz * 4 + 4);
    X->a = (double *)amgd_alloc(nz * 8 + 8);
    amgd_compact_rows(cnt, tcol, ta, cnt2, rn, X->col, X->a);
    amgd_free(cnt); amgd_free(tcol); amgd_free(ta);
  }
  amgd_free(ub); amgd_free(shortl); amgd_free(longl); amgd_free(counts);
  if (slab_v) { amgd_free(slab_v); amgd_free(slab_s); }
  return X;
}

__global__ void k_compact_rows(const uint64_t *sro, const uint32_t *scol, const double *sa,
                               const uint64_t *dro, uint32_t rn, uint32_t *dcol, double *da) {
  GRID_STRIDE(i, rn) {
    uint64_t s0 = sro[i], d0 = dro[i], n = dro[i + 1] - d0;
    for (uint64_t t = 0; t < n; t++) { dcol[d0 + t] = scol[s0 + t]; da[d0 + t] = sa[s0 + t]; }
  }
}
void amgd_compact_rows(const uint64_t *sro, const uint32_t *scol, const double *sa,
                       const uint64_t *dro, uint32_t rn, uint32_t *dcol, double *da) {
  if (rn) k_compact_rows<<<grid_for(rn), 256, 0, amgd_s()>>>(sro, scol, sa, dro, rn, dcol, da);
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
