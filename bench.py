#!/usr/bin/env python3
"""bench.py — Mrays/s + frame ms of the MI355X render path (BASELINE.json metric).

Workload (configs[1], "C2"): scenes/14-01-acceleration-tree/scene1 at 1920x1080,
default RendererSettings (depth 3), one frame per step.  At HEAD the reference
traces exactly one ray per pixel on this scene (its shadow-ray loop is dead code,
crt_renderer.cpp:29-44), so rays = traversals = 2,073,600 per frame; the count
is re-measured by the instrumented kernel, not assumed.

N=1: the frame is rendered into HBM (scene + image resident; no PCIe in the
timed region).  N>1 (one process per GPU, torchrun), two modes:

  --mode frames (default, weak scaling): every rank renders its own whole
      frame per step into its own HBM (frame-parallel rendering of a frame
      sequence: per-GPU work fixed, no data-path collective — pixels never need
      to meet); value = all ranks' rays / the slowest rank's time.
  --mode tiles (strong scaling, the north_star's image-tile sharding): the
      reference's bucket grid is dealt round-robin to ranks, each rank renders
      its buckets packed, the tiles are gathered to rank 0 over RCCL
      (torch.distributed "nccl") and unpacked there — one frame per step;
      frame k's gather runs on RCCL's stream while frame k+1 renders
      (double-buffered, FramePipeline).

Also reported: the roofline of the render kernel (algorithmic bytes per launch
÷ measured kernel time vs 8 TB/s HBM) and the CPU oracle (restatement of the
reference, same threads-over-buckets structure) timed on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "chaos-ray-tracing-course-2025_amd"))
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (import before libcrt_hip so both share torch's HIP runtime)
import torch.distributed as dist  # noqa: E402

from crt_amd import native as N  # noqa: E402
from crt_amd.distributed import FramePipeline  # noqa: E402
from crt_amd.scene_npz import load_npz  # noqa: E402

SCENES = ROOT / "tests" / "golden" / "scenes"
# BASELINE.json configs: c2 is the headline (metric) workload; the others are
# the remaining single-GPU-sized configs, for --config runs (N>1 as for c2)
CONFIGS = {
    "c2": {"scene": "14-01-acceleration-tree__scene1", "size": (1920, 1080), "settings": {}, "cpu_size": (1920, 1080),
           "label": "14-01-acceleration-tree/scene1", "note": "primary rays (HEAD traces no shadow rays)"},
    "c3": {"scene": "11-01-refractive__scene8", "size": (1920, 1080), "settings": {"max_ray_depth": 8},
           "cpu_size": (480, 270), "label": "11-01-refractive/scene8", "note": "depth-8 reflect/refract recursion"},
    "c4": {"scene": "15-01-conclusion__scene2", "size": (3840, 2160), "settings": {}, "cpu_size": (240, 135),
           "label": "15-01-conclusion/scene2", "note": "GI 4 rays, depth 3 (the CLI default scene)"},
    "c5": {"synthetic": 1_000_000, "size": (3840, 2160), "settings": {}, "cpu_size": (480, 270),
           "label": "synthetic 1M-triangle random mesh", "note": "deep KD-tree, HBM-resident scene"},
}
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
NODE_BYTES, TRI_BYTES, PIXEL_BYTES = 32, 52, 12   # SURVEY §8(d) algorithmic bytes


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", choices=sorted(CONFIGS), default="c2",
                   help="BASELINE config (c2 = the headline metric workload)")
    p.add_argument("--width", type=int, default=None, help="override the config's image width")
    p.add_argument("--height", type=int, default=None, help="override the config's image height")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample (wall s)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--backend", default="nccl", help="torch.distributed backend for N>1 (nccl = RCCL)")
    p.add_argument("--check", action="store_true", help="rank 0: compare the last frame with a 1-GPU render")
    p.add_argument("--mode", choices=["frames", "tiles"], default="frames",
                   help="N>1: frames = each GPU renders whole frames (weak scaling, default); "
                        "tiles = one frame sharded over the GPUs + RCCL gather (strong scaling)")
    p.add_argument("--event-every", type=int, default=5,
                   help="bracket every k-th render of the timed region with HIP events (kernel time sample; "
                        "an event pair between two renders costs ~7 us of a ~165 us C2 step)")
    p.add_argument("--traffic-json", default=str(ROOT / "profiles" / "pmc_traffic.json"),
                   help="per-launch HBM bytes measured by rocprofv3 --pmc (profiles/), if present")
    return p.parse_args()


def make_scene(cfg: dict, width: int, height: int):
    if "synthetic" in cfg:
        from crt_amd.synthetic import c5_scene
        return c5_scene(cfg["synthetic"], width=width, height=height)
    return load_npz(SCENES / f"{cfg['scene']}.npz").set_resolution(width, height)


def cpu_baseline(scene, settings, seconds: float, size_note: str = "") -> dict:
    from oracle import pyoracle
    from crt_amd.native import WorkCounts
    threads = min(16, os.cpu_count() or 1)
    orc = pyoracle.OracleScene(scene)
    frames, rays = 0, 0
    t0 = time.perf_counter()
    while True:
        wc = WorkCounts()
        orc.render(settings, nthreads=threads, counts=wc)
        frames += 1
        rays += wc.traversals
        el = time.perf_counter() - t0
        if el >= seconds or frames >= 200:
            break
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": rays / el / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{frames} full frames of the same workload{size_note}, oracle/crt_oracle.cpp render_image "
                      f"(bucket queue, {threads} threads, g++ -O3 no FMA) on {model or 'host CPU'}, "
                      f"{el:.1f} s wall"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % max(1, torch.cuda.device_count())   # more ranks than GPUs only in rehearsals (gloo)
    torch.cuda.set_device(local)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(a.backend)

    cfg = CONFIGS[a.config]
    W, H = a.width or cfg["size"][0], a.height or cfg["size"][1]
    scene = make_scene(cfg, W, H)
    settings = N.RendererSettings.default(**cfg["settings"])
    # the library's own start/stop events (crt_hip_last_kernel_ms) would sit inside
    # this script's timing events and add ~8 us per frame: timing here uses torch's
    gpu = N.HipScene(scene, device=local, events=0)
    # an explicit stream: the render kernel, the gather and the timing events
    # all go on it (handle 0 would mean "the scene's own stream" to the C-ABI)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream

    frame = torch.empty(W * H * 3, dtype=torch.float32, device="cuda")
    timing = {"events": None, "i": 0, "n": 0}

    def timed(launch):
        # HIP events on the launch stream around every k-th render of the timed region
        ev = timing["events"]
        rec = ev is not None and timing["n"] % a.event_every == 0
        timing["n"] += 1
        if rec:
            ev[timing["i"]][0].record(stream)
        launch()
        if rec:
            ev[timing["i"]][1].record(stream)
            timing["i"] += 1

    def render_full():
        timed(lambda: gpu.render_device(settings, frame.data_ptr(), sptr))

    def render_shard(packed):
        timed(lambda: gpu.render_shard(settings, rank, world, packed.data_ptr(), sptr))

    tiles = world > 1 and a.mode == "tiles"
    if tiles:
        # frame k's RCCL gather overlaps frame k+1's shard render (crt_amd.distributed.FramePipeline)
        pipe = FramePipeline(rank, world, gpu.shard_stride(world),
                             lambda n: torch.empty(n, dtype=torch.float32, device="cuda"), render_shard,
                             lambda flat: gpu.unpack_shards(world, flat.data_ptr(), frame.data_ptr(), sptr), dist)

    def step():
        if tiles:
            pipe.step()
        else:
            render_full()

    def drain():
        if tiles:
            pipe.drain()

    # work counters of one full frame (outside the timed region)
    counts = gpu.count_work(settings)
    rays_per_frame = counts["traversals"]

    for _ in range(a.warmup):
        step()
    drain()
    torch.cuda.synchronize()

    # kernel duration: event pairs around every k-th render launch of the timed region, on the launch stream
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
    timing["events"] = ev
    timing["n"] = 0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in ev[:timing["i"]]]))

    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device="cuda" if a.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])

    if a.check and rank == 0:
        want = gpu.render(settings)
        got = frame.view(H, W, 3).cpu().numpy()
        same = np.array_equal(got.view(np.uint32), want.view(np.uint32))
        print(f"check: last frame {'bit-identical to' if same else 'DIFFERS from'} the 1-GPU render", flush=True)
        if not same:
            raise SystemExit(1)

    ms_per_step = elapsed / a.steps * 1e3
    frames_per_step = world if (world > 1 and not tiles) else 1
    mrays = rays_per_frame * frames_per_step * a.steps / elapsed / 1e6

    # roofline of the render kernel: algorithmic bytes of one launch / its duration
    shard_frac = 1.0 / world if tiles else 1.0
    alg_bytes = (NODE_BYTES * counts["node_tests"] + TRI_BYTES * counts["triangle_tests"]
                 + PIXEL_BYTES * W * H) * shard_frac
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic = None
    try:
        tj = json.loads(Path(a.traffic_json).read_text())
        if a.config == "c2" and tj.get("workload") == f"14-01/scene1 {W}x{H}" and world == 1:
            traffic = tj.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass

    out = None
    if rank == 0:
        cpu = None
        if world == 1 and not a.no_cpu_baseline:
            cw, ch = cfg["cpu_size"] if (W, H) == cfg["size"] else (W, H)
            note = "" if (cw, ch) == (W, H) else f" at {cw}x{ch} (same scene and settings; Mrays/s is per-ray work, size-independent up to image content)"
            cpu = cpu_baseline(scene if (cw, ch) == (W, H) else make_scene(cfg, cw, ch), settings, a.cpu_seconds, note)
        out = {
            "metric": ("Mrays/sec + frame ms, 1920x1080 scene 14-01" if a.config == "c2"
                       else f"Mrays/sec + frame ms, {W}x{H} {cfg['label']}"),
            "value": round(mrays, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "strong" if tiles else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": (f"scene file scenes/{cfg['label']}.crtscene (parsed fixture tests/golden/scenes)" if "scene" in cfg
                     else "synthetic mesh (crt_amd.synthetic.c5_scene, SURVEY §8(d) C5 spec)"),
            "config": {"workload": f"{cfg['label']} {W}x{H}, RendererSettings defaults "
                                   f"(max_ray_depth {settings.max_ray_depth}), {cfg['note']}",
                       "config": a.config,
                       "rays_per_frame": rays_per_frame, "node_tests_per_frame": counts["node_tests"],
                       "triangle_tests_per_frame": counts["triangle_tests"],
                       "parallelism": (f"bucket-shard{world}+rccl-gather" if tiles else
                                       f"frame-parallel{world}" if world > 1 else "single-gpu"),
                       "frames_per_step": frames_per_step,
                       "frame_ms": round(ms_per_step, 5), "kernel_ms": round(kern_ms, 5)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
