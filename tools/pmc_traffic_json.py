"""Per-setup HBM traffic of the two roofline kernels from rocprofv3 PMC passes
(tools/gpurun_pmc.sh: gpurun_out/<dir>/traffic_{spmv,rap}_{FETCH_SIZE,WRITE_SIZE}/, one
counter per pass, one 256^3 setup each, tools/probe_scale.py 256), in the format
bench.py's pmc_traffic() reads:

  python tools/pmc_traffic_json.py <gpurun_out/dir> <tag> > profiles/r03/traffic_<tag>.json

Correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are reported in
KB; FETCH_SIZE counts half the bytes of 16-B-per-lane streaming reads and other access
widths are uncalibrated, so the factor is measured on the lane SpMV's own access pattern
(tools/pmc_calib.py: a 2.4 GB streaming product with a known byte count, passes
calib_{FETCH_SIZE,WRITE_SIZE}) and applied to both kernels' counts."""
import csv
import glob
import json
import sys

d0, tag = sys.argv[1], sys.argv[2]


def counter(path, c):
    rows = list(csv.DictReader(open(glob.glob(f"{path}/**/*counter_collection.csv", recursive=True)[0])))
    vals = [float(r["Counter_Value"]) for r in rows if r["Counter_Name"] == c]
    return sum(vals), len(vals)


cal = json.loads(open(f"{d0}/calib.json").read().strip().splitlines()[-1])
fk, fn = counter(f"{d0}/calib_FETCH_SIZE", "FETCH_SIZE")
wk, wn = counter(f"{d0}/calib_WRITE_SIZE", "WRITE_SIZE")
f_fetch = cal["read_bytes_per_product"] / (fk * 1024 / fn)
f_write = cal["write_bytes_per_product"] / (wk * 1024 / wn)
names = {"spmv": "k_spmv_pair<false,RW,PER,...> + k_spmv_pipe<false,RW,PER,false> (roofline kernels)",
         "rap": "RAP SpGEMM numeric kernels (rap_roofline)"}
out = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one counter per pass (tools/gpurun_pmc.sh), "
                 f"one 256^3 setup (tools/probe_scale.py 256), tree of {tag}",
       "workload": {"m": 256, "stencil": 7, "world": 1},
       "units": "bytes per setup",
       "calibration": {"kernel": "k_spmv_pipe<false,16,16>, ordered row sums of a generated matrix "
                                 "(tools/pmc_calib.py)", **cal,
                       "FETCH_SIZE_KB_per_product": fk / fn, "WRITE_SIZE_KB_per_product": wk / wn,
                       "fetch_factor": f_fetch, "write_factor": f_write,
                       "note": "bytes = counter_KB * 1024 * factor; the guide's x2 holds for 16-B "
                               "streaming reads, this measures the factor for 4/8-B lane loads"}}
for k in ("spmv", "rap"):
    d = {"kernel": names[k]}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        v, n = counter(f"{d0}/traffic_{k}_{c}", c)
        d[c + "_raw_KB"] = v
        d["dispatches"] = n
    # L2->fabric bytes (MALL hits included: an upper bound on HBM bytes); the key keeps its
    # round-2 name for the files already committed
    d["hbm_bytes"] = (f_fetch * d["FETCH_SIZE_raw_KB"] + f_write * d["WRITE_SIZE_raw_KB"]) * 1024
    d["bytes_are"] = "L2->fabric (FETCH_SIZE/WRITE_SIZE, calibrated): an upper bound on HBM bytes"
    out[k] = d
print(json.dumps(out, indent=1))
