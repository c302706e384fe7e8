"""Per-setup HBM traffic of the two roofline kernels from the four rocprofv3 PMC passes
of tools/gpurun_round.sh (gpurun_out/traffic_{spmv,rap}_{FETCH_SIZE,WRITE_SIZE}/), in
the format bench.py's pmc_traffic() reads:

  python tools/pmc_traffic_json.py <tag> > profiles/r02/traffic_<tag>.json

gfx950 correction (MI355X_MICROARCH.md): FETCH_SIZE is in KB and counts half of wide
streaming reads (x2); WRITE_SIZE in KB as is.  One setup per pass (probe_scale.py 256)."""
import csv
import json
import sys

tag = sys.argv[1]
names = {"spmv": "k_spmv_lane<false,RW> (roofline kernel)",
         "rap": "RAP SpGEMM numeric kernels (rap_roofline)"}
out = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one counter per pass (tools/gpurun_round.sh), "
                 f"one 256^3 setup (tools/probe_scale.py 256), tree of bench line {tag}",
       "units": "bytes per setup",
       "gfx950_correction": "FETCH_SIZE counted in KB and doubled (MI355X_MICROARCH.md: gfx950 reports 1/2 "
                            "of wide streaming reads); WRITE_SIZE in KB as is"}
for k in ("spmv", "rap"):
    d = {"kernel": names[k]}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = list(csv.DictReader(open(f"gpurun_out/traffic_{k}_{c}/run_counter_collection.csv")))
        d[c + "_raw_KB"] = sum(float(r["Counter_Value"]) for r in rows if r["Counter_Name"] == c)
        d["dispatches"] = len({r.get("Dispatch_Id", r.get("Correlation_Id", i)) for i, r in enumerate(rows)})
    d["hbm_bytes"] = (2 * d["FETCH_SIZE_raw_KB"] + d["WRITE_SIZE_raw_KB"]) * 1024
    out[k] = d
print(json.dumps(out, indent=1))
