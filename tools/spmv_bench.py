"""SpMV micro-benchmark on generated matrices shaped like the 256^3 setup's
(rows, cols, mean row length from AMGD_MVLOG): every long-row kernel, with the x
gather and without (ordered row sums), contiguous and spread columns.
Prints effective GB/s at 12 B per entry (col + value) [+ 8 B gather]."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import omp_amg_amd as oa  # noqa: E402

oa.init()
L = oa.lib()
L.amgd_test_spmv_bench.argtypes = [C.c_uint32] * 5 + [C.c_int, C.c_int, C.POINTER(C.c_uint64)]
L.amgd_test_spmv_bench.restype = C.c_double
shapes = [(187960, 508253, 2070), (696213, 1847299, 715), (10661, 37121, 8442),
          (47782, 140178, 4751), (5842783, 5842783, 130), (1692, 8969, 6501)]
kernels = [("wave", 1 << 40, -1), ("rw4", 0, 4), ("rw16", 0, 16), ("rw64", 0, 64)]
for rn, cn, mean in shapes:
    for gapname in ("contig", "spread"):
        gap = 1 if gapname == "contig" else max(1, (cn // 2) // mean)
        for with_x in (1, 0):
            cells = []
            for kname, slm, rw in kernels:
                oa.spmv_sl_min(slm)
                oa.spmv_rw(rw)
                nnz = C.c_uint64()
                ms = L.amgd_test_spmv_bench(rn, cn, mean // 2, mean * 3 // 2, gap, with_x, 5, C.byref(nnz))
                gbs = nnz.value * (12 + 8 * with_x) / (ms * 1e6)
                cells.append(f"{kname} {ms:7.3f} ms {gbs:5.0f} GB/s")
            print(f"{rn:8d} x {cn:8d} mean {mean:5d} {gapname:6s} x={with_x} nnz {nnz.value/1e6:6.0f}M | "
                  + " | ".join(cells), flush=True)
oa.spmv_sl_min(-1)
oa.spmv_rw(-1)
