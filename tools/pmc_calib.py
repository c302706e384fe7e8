"""Calibration of the PMC byte counters for the lane SpMV's own access pattern
(MI355X_MICROARCH.md: FETCH_SIZE is calibrated only for 16-B-per-lane streaming reads;
"calibrate on a known byte count in your own access pattern").  Runs the default long-row SpMV (k_spmv_pipe; k_spmv_lane before round 3) on a
generated matrix far larger than the 256 MiB Infinity Cache, ordered row sums (x = NULL:
no gather), so the bytes read are known exactly: 12 B per entry + 8 B per row offset;
written: 8 B per row.  Run under rocprofv3 --pmc FETCH_SIZE (or WRITE_SIZE) with
--kernel-include-regex 'k_spmv_(lane|pipe)'; prints the known byte counts as JSON.
usage: python tools/pmc_calib.py [rows] [mean_row] [reps]"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import omp_amg_amd as oa  # noqa: E402

rn = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
mean = int(sys.argv[2]) if len(sys.argv) > 2 else 200
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
oa.init()
L = oa.lib()
L.amgd_test_spmv_bench.argtypes = [C.c_uint32] * 5 + [C.c_int, C.c_int, C.POINTER(C.c_uint64)]
L.amgd_test_spmv_bench.restype = C.c_double
oa.spmv_sl_min(0)
oa.spmv_rw(16)
nnz = C.c_uint64()
ms = L.amgd_test_spmv_bench(rn, rn, mean // 2, mean * 3 // 2, 1, 0, reps, C.byref(nnz))
print(json.dumps({"rows": rn, "nnz": nnz.value, "reps": reps, "ms_per_product": ms,
                  "read_bytes_per_product": 8 * nnz.value + 8 * (rn + 1),
                  "write_bytes_per_product": 8 * rn}))
