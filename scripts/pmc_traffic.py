#!/usr/bin/env python3
"""profiles/pmc_traffic.json from a gpu_round.sh PMC pass (FETCH_SIZE / WRITE_SIZE).

MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are in KiB per
dispatch; on gfx950 FETCH_SIZE counts half of the bytes of wide reads, so it is
doubled; WRITE_SIZE is exact for 16-B-per-lane stores (the image writes here
are 12-B pixel stores; uncalibrated).  The render kernel of the C2 workload is
the only k_render_tiles dispatch of the render_loop.py run.
"""
import collections
import csv
import json
import sys
from pathlib import Path


def per_dispatch(path: Path, counter: str) -> float:
    vals = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if "k_render_tiles" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return sum(vals.values()) / len(vals)


def main():
    src = Path(sys.argv[1])
    dst = Path(sys.argv[2]) if len(sys.argv) > 2 else Path(__file__).resolve().parents[1] / "profiles" / "pmc_traffic.json"
    fetch_kib = per_dispatch(next((src / "fetch").rglob("*counter_collection.csv")), "FETCH_SIZE")
    write_kib = per_dispatch(next((src / "write").rglob("*counter_collection.csv")), "WRITE_SIZE")
    out = {"workload": "14-01/scene1 1920x1080", "kernel": "k_render_tiles (C2 render)",
           "fetch_size_kib": fetch_kib, "write_size_kib": write_kib,
           "hbm_bytes_per_launch": int(round(2 * fetch_kib * 1024 + write_kib * 1024)),
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                     "scripts/render_loop.py --frames 3; FETCH_SIZE doubled per the gfx950 note",
           "source": str(src)}
    dst.write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
