"""Sum the RAP SpGEMM numeric kernels (k_sg_row / k_sg_kseq / k_sg_wwin / k_spgemm_long,
instantiated with RAP=1; k_sg_win before round 4) in a rocprofv3 --stats kernel_stats.csv,
to cross-check bench.py's event-timed rap_roofline.kernel_ms_per_setup.

usage: python tools/rap_from_prof.py <kernel_stats.csv> <setups in the profiled run>
The summary covers every setup the profiled command ran; the per-setup figure divides by
the given count (no default: a missing count used to label a multi-setup sum "per setup")."""
import csv
import re
import sys

if len(sys.argv) != 3:
    sys.exit(__doc__)
rows = list(csv.DictReader(open(sys.argv[1])))
setups = int(sys.argv[2])
pat = re.compile(r"k_sg_(row|kseq)<\d+, \d+, 1, 1>|k_sg_win<\d+, 1>|k_sg_wwin<\d+, 1, 1>|k_spgemm_long<1, 1>")
tot, calls = 0.0, 0
for r in rows:
    if pat.search(r["Name"]):
        tot += float(r["TotalDurationNs"])
        calls += int(r["Calls"])
        print(f"{float(r['TotalDurationNs']) / 1e6:10.2f} ms {int(r['Calls']):6d} calls  {r['Name'][:70]}")
print(f"RAP numeric SpGEMM kernels: {tot / 1e6:.2f} ms over {calls} launches in {setups} setup(s) = "
      f"{tot / 1e6 / setups:.2f} ms per setup")
