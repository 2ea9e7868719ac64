"""Gaps between consecutive launches of one kernel in a rocprofv3 kernel
trace (CSV), and what else ran in each gap.
python scripts/kernel_gaps.py run_kernel_trace.csv --match '0, 15, 15, false' --skip 20 --count 200"""
import argparse
import csv
import statistics

p = argparse.ArgumentParser()
p.add_argument("trace")
p.add_argument("--match", required=True)
p.add_argument("--skip", type=int, default=0, help="launches to skip first (warmup)")
p.add_argument("--count", type=int, default=100)
a = p.parse_args()
allk = []
with open(a.trace) as f:
    for r in csv.DictReader(f):
        allk.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "")))
allk.sort()
mine = [k for k in allk if a.match in k[2]][a.skip:a.skip + a.count]
gaps, durs, others = [], [], {}
for i in range(1, len(mine)):
    g0, g1 = mine[i - 1][1], mine[i][0]
    gaps.append((g1 - g0) / 1e3)
    durs.append((mine[i][1] - mine[i][0]) / 1e3)
    for s, e, n, q in allk:
        if s < g1 and e > g0 and a.match not in n:
            short = n.split("(")[0].split("<")[0][-40:]
            others[short] = others.get(short, 0) + 1
print(f"{len(mine)} launches: duration median {statistics.median(durs):.1f} us, gap to the next median "
      f"{statistics.median(gaps):.1f} us (min {min(gaps):.1f}, max {max(gaps):.1f}); period "
      f"{(mine[-1][0] - mine[0][0]) / 1e3 / (len(mine) - 1):.1f} us")
print("kernels overlapping the gaps:", others)
