/*
 * amg_setup.h -- drop-in C ABI of the MI355X AMG setup (libomp_amg_amd.so).
 *
 * Replaces, with the same names, argument meaning and data layout:
 *   amg_setup()  -- reference amg_setup.h:5  / amg_setup.c:60
 *   amg_export() -- reference amg_setup.h:8  / amg_setup.c:405 (writes amg.dat,
 *                   amg_W.dat, amg_AfP.dat, amg_Aff.dat in the cwd)
 *   free_data()  -- reference amg_setup.h:248 / amg_setup.c:3487
 *   struct csr_mat, struct amg_setup_data -- reference amg_tools.h:5-8, 25-50
 * with gslib's `uint` = unsigned long (the reference Makefile builds -DUSE_LONG).
 *
 * Every array in the returned struct is host memory obtained with malloc(), as
 * in the reference, so free_data() (or the caller's own free()) releases it.
 * The setup itself runs on the GPU (HIP, gfx950); if no HIP device is usable,
 * amg_setup() prints the reason to stderr and aborts -- there is no CPU
 * fallback in this library.
 */
#ifndef OMP_AMG_AMD_AMG_SETUP_H
#define OMP_AMG_AMD_AMG_SETUP_H

#ifdef __cplusplus
extern "C" {
#endif

typedef unsigned long amg_uint;   /* gslib `uint` under -DUSE_LONG (types.h:66-68) */

struct csr_mat {                  /* amg_tools.h:5-8 */
  amg_uint rn, cn, *row_off, *col;
  double *a;
};

struct amg_setup_data {           /* amg_tools.h:25-50 */
  double tolc;
  double gamma;
  double *n;
  double *nnz;
  double *nnzf;
  double *nnzfp;
  double *m;
  double *rho;
  struct csr_mat **A;
  amg_uint *id;
  amg_uint **idc;
  amg_uint **idf;
  double **C;
  double **F;
  double **D;
  struct csr_mat **Af;
  struct csr_mat **W;
  struct csr_mat **AfP;
  amg_uint nlevels;
  amg_uint nullspace;
};

/* reference amg_setup.h:5 -- COO input, 0-based, entries with value 0 dropped */
void amg_setup(amg_uint n, const amg_uint *Ai, const amg_uint *Aj, const double *Av,
               struct amg_setup_data *data);
/* reference amg_setup.h:8 */
void amg_export(struct amg_setup_data *data);
/* reference amg_setup.h:248 */
void free_data(struct amg_setup_data **data);

#ifdef __cplusplus
}
#endif
#endif
