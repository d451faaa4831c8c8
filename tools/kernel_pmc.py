"""Per-kernel PMC averages from a tools/row_profile.sh row directory:
python tools/kernel_pmc.py gpurun_out/<tag>/<row> [name-substring ...]
Prints, per kernel, every counter's mean per dispatch (the p1..p4 passes),
with the derived VALU-busy / wait fractions and HBM bytes (FETCH_SIZE KiB x
1024, WRITE_SIZE x 64 B on gfx950 as tools/pmc_summary.py counts them)."""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
subs = sys.argv[2:]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if subs and not any(s in n for s in subs):
            continue
        acc[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, cs in acc.items():
    m = {k: sum(v) / len(v) for k, v in cs.items()}
    print(n[:90])
    for k in sorted(m):
        print(f"   {k:24s} {m[k]:16.0f}")
    if "SQ_BUSY_CYCLES" in m and "SQ_ACTIVE_INST_VALU" in m and "SQ_WAVE_CYCLES" in m:
        print(f"   valu/wave_cycles {m['SQ_ACTIVE_INST_VALU'] / m['SQ_WAVE_CYCLES']:.3f}  "
              f"wait_any/wave_cycles {m.get('SQ_WAIT_ANY', 0) / m['SQ_WAVE_CYCLES']:.3f}")
