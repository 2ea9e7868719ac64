"""Concurrency of a kernel trace (rocprofv3 --kernel-trace CSV): over the
window of the last N launches of the named kernels, the summed kernel time
over the wall span — above 1 means launches ran side by side.
python scripts/kernel_overlap.py run_kernel_trace.csv --match k_wf_ --last 400"""
import argparse
import csv

p = argparse.ArgumentParser()
p.add_argument("trace")
p.add_argument("--match", default="k_wf_")
p.add_argument("--last", type=int, default=400)
a = p.parse_args()
rows = []
with open(a.trace) as f:
    for r in csv.DictReader(f):
        if a.match in r["Kernel_Name"]:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:60],
                         r.get("Queue_Id", "")))
rows.sort()
rows = rows[-a.last:]
t0, t1 = rows[0][0], max(r[1] for r in rows)
busy = sum(r[1] - r[0] for r in rows)
# time with at least one of them running (union of intervals)
union, cur_s, cur_e = 0, None, None
for s, e, _, _ in rows:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            union += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
union += cur_e - cur_s
queues = sorted({r[3] for r in rows})
print(f"{len(rows)} launches of *{a.match}* over {(t1 - t0) / 1e3:.1f} us: kernel time {busy / 1e3:.1f} us, "
      f"covered {union / 1e3:.1f} us; concurrency (kernel time / covered) {busy / union:.2f}; queues {queues}")
