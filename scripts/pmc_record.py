#!/usr/bin/env python3
"""profiles/r02/pmc_<config>.json from rocprofv3 --pmc passes over
scripts/render_loop.py (one pass per counter group, as MI355X_MICROARCH.md
prescribes), read by bench.py's roofline when its build id equals the loaded
library's.

  pmc_record.py --config c2 --size 1920 1080 --dir gpurun_out/<tag>/pmc [--kernel k_render_tiles]

Per-launch averages over the matching dispatches of each pass:
  valu_insts_per_launch = SQ_INSTS_VALU (wave-instructions), salu = SQ_INSTS_SALU,
  hbm_bytes_per_launch  = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes; FETCH_SIZE
                          doubled per the gfx950 note), plus every other counter
                          found (SQ_WAVE_CYCLES, SQ_WAIT_INST_ANY, TCC_HIT/MISS, ...).
"""
import argparse
import collections
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "chaos-ray-tracing-course-2025_amd"))


def frames_of(ids: list, names: dict, frame_end: str) -> list:
    """Dispatch ids grouped into frames: a frame ends with (includes) a dispatch
    whose kernel name contains frame_end; dispatches after the last end are dropped."""
    frames, cur = [], []
    for i in ids:
        cur.append(i)
        if frame_end in names[i]:
            frames.append(cur)
            cur = []
    return frames


def averages(root: Path, kernel: str, last: int = 0, frame_end: str = "") -> tuple[dict, int]:
    """Per-dispatch averages of each counter over the kernel's dispatches of
    each pass; last > 0 keeps only the pass's `last` latest dispatches (the
    timed frames, after the plan tuning's trial frames).  With frame_end, a
    "launch" is one whole frame of several kernels (C3: every wavefront level,
    compose and pixel kernel up to and including the frame_end kernel): the
    counters are summed over each frame's dispatches and averaged over the
    last `last` frames."""
    out, ndisp = {}, 0
    for f in sorted(root.rglob("*counter_collection.csv")):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        names = {}
        for r in csv.DictReader(open(f)):
            if not any(k in r["Kernel_Name"] for k in kernel.split("|")):   # "a|b": any of them
                continue
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
            names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
        ids = sorted(per)
        if frame_end:
            frames = frames_of(ids, names, frame_end)
            if last > 0:
                frames = frames[-last:]
            if frames:
                ndisp = max(ndisp, len(frames))
                agg = collections.defaultdict(float)
                for fr in frames:
                    for i in fr:
                        for k, v in per[i].items():
                            agg[k] += v
                out.update({k: v / len(frames) for k, v in agg.items()})
            continue
        if last > 0:
            ids = ids[-last:]
        if ids:
            ndisp = max(ndisp, len(ids))
            agg = collections.defaultdict(float)
            for i in ids:
                for k, v in per[i].items():
                    agg[k] += v
            out.update({k: v / len(ids) for k, v in agg.items()})
    return out, ndisp


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", required=True)
    p.add_argument("--size", type=int, nargs=2, required=True)
    p.add_argument("--dir", required=True)
    p.add_argument("--kernel", default="k_render_tiles")
    p.add_argument("--out", default=None)
    p.add_argument("--command", default="")
    p.add_argument("--last", type=int, default=0, help="average only the latest N dispatches of each pass")
    p.add_argument("--frame-end", default="", help="per-frame sums: a frame ends with this kernel (C3: k_wf_pixels)")
    a = p.parse_args()
    from crt_amd import native as N
    c, n = averages(Path(a.dir), a.kernel, a.last, a.frame_end)
    rec = {"config": a.config, "size": a.size, "kernel": a.kernel, "build_id": N.build_id(),
           ("frames" if a.frame_end else "dispatches"): n,
           "counters_per_launch": c, "command": a.command,
           "method": "rocprofv3 --pmc, one pass per counter group; "
                     + (f"per-frame sums over every '{a.kernel}' dispatch of a frame (ending with {a.frame_end}), "
                        f"averaged over each pass's last {a.last} frames" if a.frame_end else
                        "per-dispatch averages of the kernel"
                        + (f" over each pass's last {a.last} dispatches (the timed frames)" if a.last else ""))}
    if "SQ_INSTS_VALU" in c:
        rec["valu_insts_per_launch"] = c["SQ_INSTS_VALU"]
    if "SQ_INSTS_SALU" in c:
        rec["salu_insts_per_launch"] = c["SQ_INSTS_SALU"]
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        rec["hbm_bytes_per_launch"] = int(round(2 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024))
    if "SQ_THREAD_CYCLES_VALU" in c and "SQ_INSTS_VALU" in c and c["SQ_INSTS_VALU"]:
        rec["valu_lane_utilisation"] = c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_INSTS_VALU"])
    if "SQ_WAIT_INST_ANY" in c and "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
        rec["wait_inst_frac"] = c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]
    out = Path(a.out) if a.out else ROOT / "profiles" / "r03" / f"pmc_{a.config}.json"
    out.parent.mkdir(parents=True, exist_ok=True)
    out.write_text(json.dumps(rec, indent=1) + "\n")
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
