#!/usr/bin/env python3
"""Per-shard render time of a config's frame on ONE GPU: what each rank of an
N-GPU tiles-mode run (bench.py --gpus N) spends rendering its bucket shard
(crt_hip_render_shard_compact), shard by shard, for N = 1, 2, 4, 8.  The
slowest shard bounds the frame rate of the sharded frame before any gather
cost; comparing it with N=1 shows how far rendering alone can scale.

  python3 scripts/shard_times.py [--config c2|c3|c4|c5] [--reps 20] [--opt NAME=V ...] [--out file.json]

imbalance = slowest / fastest shard (the shards are the reference's bucket
grid dealt round-robin, compact: only tiles with a live pixel).
"""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, os.environ.get("CRT_PKG") or str(ROOT / "chaos-ray-tracing-course-2025_amd"))
sys.path.insert(0, str(ROOT))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--counts", default="1,2,4,8")
    p.add_argument("--opt", action="append", default=[])
    p.add_argument("--out", default=None)
    p.add_argument("--config", default="c2")
    a = p.parse_args()
    import torch
    from crt_amd import native as N
    import bench
    cfg = bench.CONFIGS[a.config]
    W, H = cfg["size"]
    sc = bench.make_scene(cfg, W, H)
    g = N.HipScene(sc, events=0, calibrate=1)
    for kv in a.opt:
        k, v = kv.split("=")
        g.set_option(k, int(v))
    st = N.RendererSettings.default(**cfg["settings"])
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    frame = torch.empty(W * H * 3, dtype=torch.float32, device="cuda")
    g.render_device(st, frame.data_ptr(), sp)   # tunes the plan
    out = {"config": a.config, "size": [W, H], "plan": g.plan_info(), "opts": a.opt, "shards": {}}
    for n in [int(x) for x in a.counts.split(",")]:
        buf = torch.empty(max(1, g.compact_stride(n)), dtype=torch.float32, device="cuda")
        per = []
        for k in range(n):
            g.render_shard_compact(st, k, n, buf.data_ptr(), sp)
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                g.render_shard_compact(st, k, n, buf.data_ptr(), sp)
                e1.record(stream)
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            per.append(float(np.median(ts)))
        out["shards"][str(n)] = {"median_ms": per, "max_ms": max(per), "min_ms": min(per),
                                 "imbalance": max(per) / max(min(per), 1e-9), "speedup_vs_n1": None}
    t1 = out["shards"].get("1", {}).get("max_ms")
    for n, d in out["shards"].items():
        d["speedup_vs_n1"] = round(t1 / d["max_ms"], 3) if t1 else None
    js = json.dumps(out)
    if a.out:
        Path(a.out).write_text(js)
    print(js)


if __name__ == "__main__":
    main()
