"""Sum scripts/pmc_probe.sh's counter passes per kernel (kernels whose name
contains argv[2]); prints per-dispatch means and the mean duration."""
import csv
import glob
import sys
from collections import defaultdict

out, match = sys.argv[1], sys.argv[2]
vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for fn in sorted(glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(fn)):
        k = r["Kernel_Name"]
        if match not in k:
            continue
        k = k.split("(")[0] + "<" + k.split("<", 1)[1].split(">")[0] + ">" if "<" in k else k.split("(")[0]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if r["Counter_Name"] == next(iter(vals[k])):
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, cs in vals.items():
    print(k, f"dispatches~{len(dur[k])} mean dur {sum(dur[k]) / max(1, len(dur[k])):.1f} us")
    for c, v in sorted(cs.items()):
        print(f"  {c:40s} {sum(v) / len(v):16.1f}")
