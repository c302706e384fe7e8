/*
 * oracle/amg_oracle.h -- TEST INFRASTRUCTURE, NOT THE PRODUCT.
 *
 * CPU restatement of the reference AMG setup (amg_setup.c / amg_tools.c of
 * nicooff/omp_amg).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and only as a checker/baseline.
 *
 * Parity pinned: tests/test_oracle_vs_ref.py checks this restatement
 * bit-for-bit (C/F sets, sparsity patterns AND every double) against the
 * reference itself compiled from /root/reference (oracle/_ref/libref_amg.so)
 * and against the committed fixtures in tests/golden/.
 *
 * It exports the same C ABI as the reference (amg_setup.h:5,8; amg_tools.h),
 * so one ctypes reader (omp_amg_amd/abi.py) reads all three implementations.
 */
#ifndef AMG_ORACLE_H
#define AMG_ORACLE_H

typedef unsigned long amg_uint;       /* gslib uint under -DUSE_LONG */

struct csr_mat { amg_uint rn, cn, *row_off, *col; double *a; };

struct amg_setup_data {
  double tolc, gamma;
  double *n, *nnz, *nnzf, *nnzfp, *m, *rho;
  struct csr_mat **A;
  amg_uint *id, **idc, **idf;
  double **C, **F, **D;
  struct csr_mat **Af, **W, **AfP;
  amg_uint nlevels, nullspace;
};

void amg_setup(amg_uint n, const amg_uint *Ai, const amg_uint *Aj,
               const double *Av, struct amg_setup_data *data);
void amg_export(struct amg_setup_data *data);
void free_data(struct amg_setup_data **data);

#endif
