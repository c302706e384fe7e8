/* oracle/ref_asan_driver.c -- TEST INFRASTRUCTURE.
 * Reads a COO case written by tests/golden/make_golden.py (u64 nz, u64 Ai[nz],
 * u64 Aj[nz], f64 Av[nz]) and runs the reference amg_setup on it.  Linked
 * against the reference sources with -fsanitize=address (oracle/Makefile) to
 * decide whether the reference is well-defined on the case. */
#include <stdio.h>
#include <stdlib.h>
typedef unsigned long amg_uint;
struct amg_setup_data;
void amg_setup(amg_uint n, const amg_uint *Ai, const amg_uint *Aj, const double *Av,
               struct amg_setup_data *data);
int main(int argc, char **argv) {
  if (argc < 2) return 2;
  FILE *f = fopen(argv[1], "rb");
  if (!f) return 2;
  amg_uint nz;
  if (fread(&nz, sizeof nz, 1, f) != 1) return 2;
  amg_uint *I = malloc(nz * sizeof *I), *J = malloc(nz * sizeof *J);
  double *V = malloc(nz * sizeof *V);
  if (fread(I, sizeof *I, nz, f) != nz || fread(J, sizeof *J, nz, f) != nz ||
      fread(V, sizeof *V, nz, f) != nz) return 2;
  fclose(f);
  void *data = calloc(1, 4096);
  amg_setup(nz, I, J, V, data);
  return 0;
}
