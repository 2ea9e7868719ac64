#!/usr/bin/env python3
"""bench.py — Mrays/s + frame ms of the MI355X render path (BASELINE.json metric).

Workload (configs[1], "C2"): scenes/14-01-acceleration-tree/scene1 at 1920x1080,
default RendererSettings (depth 3), one frame per step.  At HEAD the reference
traces exactly one ray per pixel on this scene (its shadow-ray loop is dead code,
crt_renderer.cpp:29-44), so rays = traversals = 2,073,600 per frame; the count
is re-measured by the instrumented kernel, not assumed.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5]

N=1: the frame is rendered into HBM (scene + image resident; no PCIe in the
timed region).  The end-to-end figure of the reference's call (render_image
returns a host image, main.cpp:37-43: render + D2H into a pinned host buffer)
is reported beside it as config.e2e_ms.

N>1: one process per GPU.  Without torchrun's environment, `--gpus N` starts
the N rank processes itself (python -m torch.distributed.run, before this
process touches the GPU) and exits with their status.  The mode (`--mode
auto`, crt_amd.distributed.select_mode): a frame the library's GPU-count
policy keeps on one GPU (its one-GPU estimate under 2 ms: C2, C3) cannot
strong-scale, so every rank renders whole frames (`frames`, weak scaling);
longer frames (C4, C5) take `tiles` (strong scaling, the north_star's
image-tile sharding); the other mode is measured as `secondary`.  Tiles: the reference's bucket
grid (crt_renderer.cpp:160-174) is dealt bucket k -> rank k mod N, each rank
renders its buckets packed, the packed shards are gathered to rank 0 over RCCL
(torch.distributed "nccl") and unpacked there, one frame per step; frame k's
gather runs on RCCL's stream while frame k+1 renders (FramePipeline).
By default only the LIVE 8x8 tiles travel (`--shards compact`): tiles with a
pixel whose camera ray passes the reference's root-cell test — every other
pixel is a miss, i.e. the background, written by the unpack on rank 0
(lossless; 28% of C2's tiles are live).  `--payload u8` gathers write_ppm's
8-bit components instead (device quantise-and-pack, crt_image_ppm.cpp:9-23;
4x fewer bytes again, the PPM the CLI writes).

N=1, C2: `secondary` is BASELINE C2's "primary + shadow rays" leg — the
course's earlier renderer (option "shadows"), on which the reference's only
published number was taken — with its own roofline.

Also reported: the roofline of the render kernel (see roofline_block) and the
CPU baseline (oracle/crt_oracle.cpp, the from-scratch restatement of the
reference's render_image with its bucket queue and thread pool) timed on this
host in child processes that never touch the GPU: all cores of the affinity
mask, and one core pinned.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
PKG = Path(os.environ["CRT_PKG"]).resolve() if os.environ.get("CRT_PKG") else ROOT / "chaos-ray-tracing-course-2025_amd"   # CRT_PKG: A/B builds
for _p in (str(PKG), str(ROOT)):
    if _p not in sys.path:
        sys.path.insert(0, _p)

SCENES = ROOT / "tests" / "golden" / "scenes"
# BASELINE.json configs: c2 is the headline (metric) workload; the others are
# the remaining configs, for --config runs
CONFIGS = {
    "c2": {"scene": "14-01-acceleration-tree__scene1", "size": (1920, 1080), "settings": {}, "cpu_size": (1920, 1080),
           "label": "14-01-acceleration-tree/scene1", "note": "primary rays (HEAD traces no shadow rays)"},
    "c3": {"scene": "11-01-refractive__scene8", "size": (1920, 1080), "settings": {"max_ray_depth": 8},
           "cpu_size": (1920, 1080), "label": "11-01-refractive/scene8", "note": "depth-8 reflect/refract recursion"},
    "c4": {"scene": "15-01-conclusion__scene2", "size": (3840, 2160), "settings": {}, "cpu_size": (240, 135),
           "label": "15-01-conclusion/scene2", "note": "GI 4 rays, depth 3 (the CLI default scene)"},
    "c5": {"synthetic": 1_000_000, "size": (3840, 2160), "settings": {}, "cpu_size": (480, 270),
           "label": "synthetic 1M-triangle random mesh", "note": "deep KD-tree, HBM-resident scene"},
}

# Peaks (/opt/skills/guides/MI355X_MICROARCH.md): HBM3E 8 TB/s; L2 ~34.5 TB/s
# aggregate; VALU issue: a wave64 VALU instruction occupies a SIMD-32 for 2
# cycles -> 256 CUs x 4 SIMDs x 2.4 GHz / 2 wave-instructions/s.
HBM_PEAK_GBS = 8000.0
L2_PEAK_GBS = 34500.0
VALU_PEAK_GINST = 256 * 4 * 2.4 / 2.0
NODE_BYTES, TRI_BYTES, PIXEL_BYTES = 32, 52, 12      # SURVEY §8(d) algorithmic bytes
PNODE_BYTES, SLOT_BYTES = 64, 48                     # device records (crt_layout.h)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # a C2 frame is ~0.06 ms: 200 frames (12 ms) keep the pipeline's fill and
    # drain (the first frame runs alone) under 1 % of the timed region
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--config", choices=sorted(CONFIGS), default="c2",
                   help="BASELINE config (c2 = the headline metric workload)")
    p.add_argument("--width", type=int, default=None, help="override the config's image width")
    p.add_argument("--height", type=int, default=None, help="override the config's image height")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample, all cores (wall s)")
    p.add_argument("--cpu-single-seconds", type=float, default=6.0, help="bounded single-core CPU sample (wall s)")
    p.add_argument("--no-cpu-full", action="store_true",
                   help="skip the CPU baseline's full-size frame (configs whose sample is a reduced size: C4, C5)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (render + D2H) timing")
    p.add_argument("--backend", default="nccl", help="torch.distributed backend for N>1 (nccl = RCCL; gloo stages "
                                                    "shards through host memory, for rehearsals on one GPU)")
    p.add_argument("--no-check", dest="check", action="store_false",
                   help="skip rank 0's bit-comparison of the last timed frame (and of the last one-at-a-time frame) "
                        "with a blocking 1-GPU render (on by default)")
    p.add_argument("--check", dest="check", action="store_true", help=argparse.SUPPRESS)   # the default; old scripts
    p.set_defaults(check=True)
    p.add_argument("--mode", choices=["auto", "tiles", "frames"], default="auto",
                   help="N>1: tiles = one frame sharded over the GPUs + RCCL gather (strong scaling); frames = each "
                        "GPU renders whole frames (weak scaling); auto (default) = frames when the library's GPU-count "
                        "policy gives the frame one GPU (its one-GPU estimate is under 2 ms: C2, C3), else tiles "
                        "(C4, C5); the other mode is measured as `secondary`")
    p.add_argument("--payload", choices=["f32", "u8"], default="f32",
                   help="tiles mode: gather fp32 RGB (the render_image image) or write_ppm's 8-bit components")
    p.add_argument("--shards", choices=["compact", "full"], default="compact",
                   help="tiles mode: gather only the live tiles (camera ray passes the root-cell test; the rest is "
                        "background by construction — lossless) or every bucket")
    p.add_argument("--shadows", action="store_true",
                   help="trace the shadow rays (option \"shadows\": the course's earlier renderer, dead code at HEAD; "
                        "a separate report, never the HEAD-parity headline): rays = camera + shadow rays")
    p.add_argument("--set", action="append", default=[], metavar="OPTION=V",
                   help="A/B runs: crt_hip_scene_set_option on the benched scene (repeatable)")
    p.add_argument("--no-secondary", action="store_true", help="N>1: skip the secondary frames-mode measurement")
    p.add_argument("--camera-orbit", type=int, default=60, metavar="POSES",
                   help="N=1: also time frames with a new camera pose every frame (crt_hip_scene_set_camera; the pose "
                        "swings around the scene's centre over POSES frames), reported beside the fixed-camera line "
                        "as config.camera_orbit; 0 skips it")
    p.add_argument("--event-every", type=int, default=5,
                   help="bracket every k-th render of the timed region with HIP events (kernel time sample; "
                        "an event pair between two renders costs ~7 us of a ~165 us C2 step)")
    p.add_argument("--pmc-json", default=None,
                   help="PMC record of the render kernel (profiles/r05/pmc_<config>.json by default); used for "
                        "the issue roofline and measured HBM traffic when its build id equals the library's")
    p.add_argument("--selftest-launch", action="store_true",
                   help="launcher plumbing only: ranks join the process group and report; no GPU work")
    p.add_argument("--cpu-worker", default=None, help=argparse.SUPPRESS)
    p.add_argument("--shim-worker", default=None, help=argparse.SUPPRESS)
    return p.parse_args(argv)


# --------------------------------------------------------------------------
#  N>1 launcher (parent process: never touches the GPU)
# --------------------------------------------------------------------------
def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(nproc: int, argv: list[str]) -> int:
    """Start `nproc` rank processes of this script under torch.distributed.run
    (one per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in their environment) as
    children, and return their exit status.  Nothing here initialises HIP."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(Path(__file__).resolve()), *argv]
    print(f"bench: launching {nproc} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


# --------------------------------------------------------------------------
#  CPU baseline (child processes: oracle only, no GPU)
# --------------------------------------------------------------------------
def make_scene(cfg: dict, width: int, height: int):
    if "synthetic" in cfg:
        from crt_amd.synthetic import c5_scene
        return c5_scene(cfg["synthetic"], width=width, height=height)
    from crt_amd.scene_npz import load_npz
    return load_npz(SCENES / f"{cfg['scene']}.npz").set_resolution(width, height)


def cpu_worker(spec: dict) -> dict:
    """Times the oracle's render_image (bucket queue + thread pool, like
    crt_renderer.cpp:157-199) on whole frames: at least `min_frames`, until
    `seconds` of wall time.  Scene build stays outside the timer (main.cpp:37)."""
    if spec.get("pin") is not None:
        os.sched_setaffinity(0, {int(spec["pin"])})
    from crt_amd.native import RendererSettings, WorkCounts
    from oracle import pyoracle
    cfg = CONFIGS[spec["config"]]
    scene = make_scene(cfg, spec["w"], spec["h"])
    st = RendererSettings.default(**cfg["settings"])
    orc = pyoracle.OracleScene(scene).set_shadows(bool(spec.get("shadows")))
    wc = WorkCounts()
    if spec.get("once"):   # one timed frame (a full-size frame of minutes), its rays counted in it
        s = time.perf_counter()
        orc.render(st, nthreads=spec["threads"], counts=wc)
        el = time.perf_counter() - s
        return {"rays_per_frame": int(wc.traversals), "frames": 1, "best_s": el, "median_s": el, "wall_s": el}
    orc.render(st, nthreads=spec["threads"], counts=wc)      # warm-up frame, and the frame's ray count
    rays = int(wc.traversals)
    times = []
    t0 = time.perf_counter()
    while len(times) < spec["min_frames"] or (time.perf_counter() - t0 < spec["seconds"] and len(times) < 500):
        s = time.perf_counter()
        orc.render(st, nthreads=spec["threads"])
        times.append(time.perf_counter() - s)
    return {"rays_per_frame": rays, "frames": len(times), "best_s": min(times),
            "median_s": statistics.median(times), "wall_s": time.perf_counter() - t0}


def run_cpu_worker(spec: dict) -> dict:
    out = subprocess.run([sys.executable, str(Path(__file__).resolve()), "--cpu-worker", json.dumps(spec)],
                         capture_output=True, text=True, check=True)
    return json.loads(out.stdout.strip().splitlines()[-1])


def cpu_info() -> dict:
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None
    try:   # cgroup v2 CPU quota: "max 100000" or "<quota> <period>"
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"model": model or "host CPU", "affinity_cpus": len(os.sched_getaffinity(0)), "cgroup_cpu_quota": quota}


def cpu_baseline(config: str, w: int, h: int, seconds: float, single_seconds: float, size_note: str,
                 shadows: bool = False, full: tuple | None = None) -> dict:
    """Legs: hardware_concurrency() threads (the affinity mask, as
    crt_renderer.cpp:178 would spawn), threads = the cgroup CPU quota when it
    is smaller (what the box actually grants: `value` is the better of the
    two, `cores` its thread count, `effective_cpus` the quota), and one
    pinned core.  full = (W, H): the sample is a reduced size; one frame at
    the benched size on the quota's threads is timed too (`full_size`, with
    its per-ray rate against the sample's)."""
    info = cpu_info()
    affinity = info["affinity_cpus"]
    quota = info["cgroup_cpu_quota"]
    effective = min(affinity, int(round(quota))) if quota else affinity
    legs = {}
    for n in sorted({affinity, effective}):
        legs[n] = run_cpu_worker({"config": config, "w": w, "h": h, "threads": n, "pin": None,
                                  "seconds": seconds, "min_frames": 5, "shadows": shadows})
    pin = sorted(os.sched_getaffinity(0))[0]
    single = run_cpu_worker({"config": config, "w": w, "h": h, "threads": 1, "pin": pin,
                             "seconds": single_seconds, "min_frames": 2, "shadows": shadows})
    rays = legs[affinity]["rays_per_frame"]
    best_n = min(legs, key=lambda n: legs[n]["median_s"])
    multi = legs[best_n]
    full_leg = None
    if full:
        f = run_cpu_worker({"config": config, "w": full[0], "h": full[1], "threads": best_n, "pin": None,
                            "seconds": 0, "min_frames": 1, "shadows": shadows, "once": True})
        fv = f["rays_per_frame"] / f["median_s"] / 1e6
        full_leg = {"w": full[0], "h": full[1], "threads": best_n, "frames": 1, "rays": f["rays_per_frame"],
                    "frame_ms": round(f["median_s"] * 1e3, 1), "value": round(fv, 3), "unit": "Mrays/s",
                    "per_ray_vs_sample": round(fv / (rays / multi["median_s"] / 1e6), 4),
                    "note": "one whole frame at the benched size (no warm-up frame), the same oracle and threads"}
    return {
        "value": round(rays / multi["median_s"] / 1e6, 3), "unit": "Mrays/s", "cores": best_n, "kind": "port",
        "effective_cpus": effective, "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
        "best": round(rays / multi["best_s"] / 1e6, 3), "frame_ms_median": round(multi["median_s"] * 1e3, 3),
        "frame_ms_best": round(multi["best_s"] * 1e3, 3),
        "legs": {str(n): {"threads": n, "value": round(rays / l["median_s"] / 1e6, 3),
                          "frame_ms_median": round(l["median_s"] * 1e3, 3), "frames": l["frames"]}
                 for n, l in legs.items()},
        "single_core": {"value": round(single["rays_per_frame"] / single["median_s"] / 1e6, 3), "unit": "Mrays/s",
                        "frame_ms_median": round(single["median_s"] * 1e3, 3), "frames": single["frames"],
                        "pinned_cpu": pin},
        "cpu_model": info["model"],
        "full_size": full_leg,
        "sample": f"{multi['frames']} whole frames{size_note} of the same workload, oracle/crt_oracle.cpp "
                  f"render_image (24-px bucket queue, g++ -O3, no FMA) in a child process on {info['model']}: "
                  f"{best_n} threads (legs: {', '.join(f'{n} threads' for n in sorted(legs))}; the affinity mask "
                  f"is {affinity} CPUs inside a {quota} CPU cgroup quota); value = rays / median frame time; "
                  f"single_core = the same on one pinned CPU ({single['frames']} frames)",
    }


def cold_cli(cfg: dict, w: int, h: int, settings) -> dict | None:
    """The reference CLI's timed region on a fresh process (main.cpp:37-43):
    bin/crt_renderer on the config's scene written as a .crtscene of this
    size, on one GPU.  execution_ms is the "Execution time" it prints — the
    first crt_hip_render of a new scene: tile-plan calibration, GI / Fresnel
    tables, the render and the D2H copy; process_ms the whole process (HIP
    start, load, tree build, upload, render, PPM write)."""
    if "scene" not in cfg:
        return None
    import tempfile
    from crt_amd.scene_json import arrays_to_crtscene
    sc = make_scene(cfg, w, h)
    if any(t == 3 for t in sc.a["tex_i"]):   # bitmap textures would need their files next to the scene
        return None
    doc = arrays_to_crtscene(sc.a, {})
    doc["settings"]["image_settings"].update(width=w, height=h)
    exe = PKG / "bin" / "crt_renderer"
    with tempfile.TemporaryDirectory() as td:
        scene = Path(td) / "scene.crtscene"
        scene.write_text(json.dumps(doc))
        cmd = [str(exe), str(scene), str(Path(td) / "out.ppm"), "--gpus", "1",
               "--max-depth", str(settings.max_ray_depth), "--gi-rays", str(settings.diffuse_reflection_ray_count)]
        t0 = time.perf_counter()
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        wall = (time.perf_counter() - t0) * 1e3
    if r.returncode != 0 or not r.stdout.startswith("Execution time: "):
        return {"error": (r.stderr or r.stdout)[-300:]}
    secs = float(r.stdout.split("Execution time: ", 1)[1].split()[0])
    return {"execution_ms": round(secs * 1e3, 3), "process_ms": round(wall, 1),
            "command": "bin/crt_renderer scene.crtscene out.ppm --gpus 1 (fresh process)"}


REFTREES = {"c2": "14-01-acceleration-tree__scene1", "c3": "11-01-refractive__scene8", "c4": "15-01-conclusion__scene2"}


def shim_worker(spec: dict) -> dict:
    """The reference's main.cpp timed region with the crt::render_image shim
    linked (csrc/shim/crt_render_image_hip.cpp -> crt_hip_render_image_tree,
    csrc/shim/crt_shim_core.cpp), in a process that has not touched the GPU:
    the Scene the reference built (its vertex array and acceleration tree as
    its own compiled TUs produced them, tests/golden/reftree_*.npz) handed
    over as render_image hands it.  first = the first call (it creates the
    device scene: HIP start-up, upload, BVH, bins, inside the reference's
    timer); repeat = the median of the calls after it (the cached device scene,
    its content compared with the caller's while the frame renders)."""
    import ctypes as C
    import numpy as np
    from crt_amd import native as N
    cfg = CONFIGS[spec["config"]]
    name = REFTREES[spec["config"]]
    z = np.load(ROOT / "tests" / "golden" / f"reftree_{name}.npz")
    sc = make_scene(cfg, spec["w"], spec["h"])
    ts = N.TreeScene(sc, z["vertices"], z["bounds"], z["children"], z["leaf_offsets"], z["leaf_triangles"])
    st = N.RendererSettings.default(**cfg["settings"])
    L = N.lib()
    first_out = np.zeros((spec["h"], spec["w"], 3), np.float32)   # render_image's Image (crt_image.h:15-19)
    t0 = time.perf_counter()
    rc = L.crt_hip_render_image_tree(ts.tree_desc_ptr(), C.byref(st), first_out.ctypes.data)
    first = (time.perf_counter() - t0) * 1e3
    if rc != 0:
        return {"error": N.last_error()}
    out = np.zeros_like(first_out)
    ts_ms = []
    for _ in range(spec["frames"]):
        t0 = time.perf_counter()
        L.crt_hip_render_image_tree(ts.tree_desc_ptr(), C.byref(st), out.ctypes.data)
        ts_ms.append((time.perf_counter() - t0) * 1e3)
    same = bool(np.array_equal(out.view(np.uint32), first_out.view(np.uint32)))
    stats = N.render_image_tree_stats()
    return {"first_call_ms": round(first, 3), "repeat_ms": round(statistics.median(ts_ms), 4),
            "repeat_ms_min": round(min(ts_ms), 4), "repeats": len(ts_ms), "repeat_equals_first": same,
            "creates": stats["creates"], "reuses": stats["reuses"]}


def shim_timing(config: str, w: int, h: int, frames: int = 30) -> dict | None:
    if config not in REFTREES:
        return None
    try:
        out = subprocess.run([sys.executable, str(Path(__file__).resolve()), "--shim-worker",
                              json.dumps({"config": config, "w": w, "h": h, "frames": frames})],
                             capture_output=True, text=True, timeout=300)
        d = json.loads(out.stdout.strip().splitlines()[-1])
    except (subprocess.SubprocessError, ValueError, IndexError) as e:
        return {"error": str(e)[-300:]}
    d["scene"] = f"tests/golden/reftree_{REFTREES[config]}.npz (the reference's built Scene) at {w}x{h}"
    d["note"] = ("crt_hip_render_image_tree (the shim's body) in a fresh process; the reference's timer "
                 "(main.cpp:37-43) also holds render_image's zero-filled Image (crt_image.h:15-19) and the shim's "
                 "flatten of the Scene, both host work outside this call")
    return d


# --------------------------------------------------------------------------
#  roofline
# --------------------------------------------------------------------------
def roofline_block(kernel_ms: float, counts: dict, waves: dict, npx: int, pmc: dict | None,
                   build_id: str, shard_frac: float) -> dict:
    """Bounds of the dominant render kernel, per launch:
      s8d     — SURVEY §8(d) algorithmic bytes (32 B/node test + 52 B/triangle
                test + 12 B/pixel, the kernel's own pruned counts) / kernel time:
                a work rate; lanes share these records through the caches, so
                it is not an HBM occupancy (it can exceed the HBM peak).
      l2      — wave-unique record bytes (per wave step one 64-B node record,
                per triangle step one 48-B slot record; crt_hip_wave_counts)
                + 12 B/pixel, against the L2 bandwidth.
      hbm     — measured HBM bytes (rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE of
                this build) against the HBM peak.
      valu    — measured VALU wave-instructions (SQ_INSTS_VALU of this build)
                against the VALU issue rate.
    `bound` names the candidate with the largest fraction."""
    sec = kernel_ms * 1e-3
    s8d = (NODE_BYTES * counts["node_tests"] + TRI_BYTES * counts["triangle_tests"] + PIXEL_BYTES * npx) * shard_frac
    uniq = (PNODE_BYTES * waves.get("node_steps", 0) + SLOT_BYTES * waves.get("triangle_steps", 0)
            + PIXEL_BYTES * npx) * shard_frac
    cand = {}
    if waves.get("node_steps", 0) > 0:   # wave-unique records are counted by the packet walks only
        cand["l2"] = {"achieved": uniq / sec / 1e9, "peak": L2_PEAK_GBS, "unit": "GB/s",
                      "bytes_per_launch": int(uniq)}
    fresh = pmc is not None and pmc.get("build_id") == build_id
    traffic = None
    if fresh:
        traffic = pmc.get("hbm_bytes_per_launch")
        if traffic:
            traffic = traffic * shard_frac
            cand["hbm"] = {"achieved": traffic / sec / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "bytes_per_launch": int(traffic)}
        if pmc.get("valu_insts_per_launch"):
            v = pmc["valu_insts_per_launch"] * shard_frac
            cand["valu"] = {"achieved": v / sec / 1e9, "peak": VALU_PEAK_GINST, "unit": "Ginst/s",
                            "insts_per_launch": int(v), "salu_insts_per_launch": pmc.get("salu_insts_per_launch")}
    for c in cand.values():
        c["frac"] = round(c["achieved"] / c["peak"], 5)
        c["achieved"] = round(c["achieved"], 2)
    if not cand:   # no PMC of this build and no wave-step counts: no bound can be named
        b, bound = {"achieved": None, "peak": None, "unit": None, "frac": None}, None
    else:
        bound = max(cand, key=lambda k: cand[k]["frac"])
        b = cand[bound]
    return {"bound": {"valu": "valu_issue", "l2": "l2", "hbm": "hbm", None: None}[bound], "achieved": b["achieved"],
            "peak": b["peak"], "unit": b["unit"], "frac": b["frac"],
            "traffic": int(traffic) if traffic else None,
            "measured": bound is not None,
            "pmc": (f"{pmc.get('source', '?')} (build {build_id})" if fresh else
                    f"stale or absent (library build {build_id}); traffic/valu omitted"),
            "candidates": cand,
            "s8d_work_rate": {"achieved": round(s8d / sec / 1e9, 2), "unit": "GB/s", "bytes_per_launch": int(s8d),
                              "note": "SURVEY §8(d) algorithmic bytes / kernel time: lanes share records through "
                                      "the caches, so this is a work rate, not HBM occupancy"}}


def load_pmc(path: str | None, config: str, w: int, h: int) -> dict | None:
    p = Path(path) if path else ROOT / "profiles" / "r06" / f"pmc_{config}.json"
    try:
        d = json.loads(p.read_text())
    except (OSError, ValueError):
        return None
    if d.get("config") != config or d.get("size") != [w, h]:
        return None
    d["source"] = str(p.relative_to(ROOT)) if p.is_relative_to(ROOT) else str(p)
    return d


# --------------------------------------------------------------------------
#  ranks
# --------------------------------------------------------------------------
def policy_gpus(scene, settings, visible: int) -> int:
    """crt_auto_gpus: the GPUs the library's policy gives this frame out of
    `visible`; reads the scene description only (no GPU)."""
    import ctypes as C
    from crt_amd import native as N
    return int(N.lib().crt_auto_gpus(N._desc_ptr(scene), C.byref(settings), int(visible)))


def selftest_launch(a) -> None:
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        dist.init_process_group(a.backend if a.backend != "nccl" else "gloo")
        import torch
        t = torch.ones(1)
        dist.all_reduce(t)
        world = dist.get_world_size()
        ok = int(t.item()) == world
    else:
        ok = True
    if int(os.environ.get("RANK", "0")) == 0:
        from crt_amd import native as N
        from crt_amd.distributed import select_mode
        cfg = CONFIGS[a.config]
        st = N.RendererSettings.default(**cfg["settings"])
        mode = select_mode(a.mode, policy_gpus(make_scene(cfg, *cfg["size"]), st, max(world, a.gpus)))
        print(json.dumps({"selftest": "launch", "n_gpus": world, "requested": a.gpus, "all_reduce_ok": ok,
                          "mode": mode, "scaling": "strong" if mode == "tiles" else "weak"}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    argv = sys.argv[1:]
    a = parse(argv)
    if a.cpu_worker is not None:
        print(json.dumps(cpu_worker(json.loads(a.cpu_worker))), flush=True)
        return 0
    if a.shim_worker is not None:
        print(json.dumps(shim_worker(json.loads(a.shim_worker))), flush=True)
        return 0
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(a.gpus, argv)
    if a.selftest_launch:
        selftest_launch(a)
        return 0

    import numpy as np
    import torch  # import before libcrt_hip so both share torch's HIP runtime
    import torch.distributed as dist
    from crt_amd import native as N
    from crt_amd.distributed import FrameParallel, FramePipeline, select_mode

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(1, torch.cuda.device_count())
    if world > ndev and a.backend == "nccl":
        raise SystemExit(f"bench: {world} ranks need {world} GPUs for RCCL (found {ndev}); "
                         f"rehearse with --backend gloo")
    local = local % ndev                       # more ranks than GPUs only in gloo rehearsals
    torch.cuda.set_device(local)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(a.backend)
        world = dist.get_world_size()          # what the process group actually initialised
    dist_backend = dist.get_backend() if world > 1 else None
    host_staged = world > 1 and dist_backend != "nccl"

    cfg = CONFIGS[a.config]
    W, H = a.width or cfg["size"][0], a.height or cfg["size"][1]
    scene = make_scene(cfg, W, H)
    settings = N.RendererSettings.default(**cfg["settings"])
    # the library's own start/stop events (crt_hip_last_kernel_ms) would sit inside
    # this script's timing events and add ~8 us per frame: timing here uses torch's
    # calibrate 1: the measured tile plan with its split threshold tuned on the
    # first frame (a long-running renderer's steady state; one-shot callers
    # default to the fixed threshold, see cold_cli below)
    t_create = time.perf_counter()
    gpu = N.HipScene(scene, device=local, events=0, shadows=int(a.shadows), calibrate=1)
    for kv in a.set:   # A/B runs: options of the benched scene (crt_hip_scene_set_option)
        k, v = kv.split("=", 1)
        gpu.set_option(k, int(v))
    create_wall_ms = (time.perf_counter() - t_create) * 1e3
    build_id = N.build_id()
    # the same scene created again in this warm process (no runtime / code
    # object / host-table start-up): what a second scene costs
    t_create = time.perf_counter()
    g2 = N.HipScene(scene, device=local, events=0, shadows=int(a.shadows), calibrate=1)
    warm_create = {"wall": round((time.perf_counter() - t_create) * 1e3, 3),
                   **{k: round(v, 3) for k, v in g2.info().items()
                      if k in ("prep_ms", "tree_build_ms", "bvh_ms", "bins_ms", "upload_ms", "create_ms")}}
    del g2
    # an explicit stream: the render kernel, the gather and the timing events
    # all go on it (handle 0 would mean "the scene's own stream" to the C-ABI)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream

    npx = W * H
    frame = torch.empty(npx * 3, dtype=torch.float32, device="cuda")
    frame8 = torch.empty(npx * 3, dtype=torch.uint8, device="cuda")
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

    u8 = a.payload == "u8"
    compact = a.shards == "compact"
    stride = (gpu.compact_stride(world) if compact else gpu.shard_stride(world)) if world > 1 else npx * 3
    shard_f32 = torch.empty(stride, dtype=torch.float32, device="cuda")   # u8 payload / host staging scratch

    def render_shard(packed):
        # packed: this rank's slot of the gather (device, or host for gloo)
        dst = shard_f32 if (u8 or host_staged) else packed
        rs = gpu.render_shard_compact if compact else gpu.render_shard
        timed(lambda: rs(settings, rank, world, dst.data_ptr(), sptr))
        if u8:
            tgt = packed if not host_staged else shard_u8
            N.quantize_rgb8(shard_f32.data_ptr(), stride, tgt.data_ptr(), 255, sptr)
            if host_staged:
                packed.copy_(shard_u8)
        elif host_staged:
            packed.copy_(shard_f32)

    def unpack(flat):
        src = flat
        if host_staged:
            src = flat_dev_u8 if u8 else flat_dev
            src.copy_(flat)
        if u8:
            up = gpu.unpack_compact_rgb8 if compact else gpu.unpack_shards_rgb8
            up(world, src.data_ptr(), frame8.data_ptr(), sptr)
        else:
            up = gpu.unpack_compact if compact else gpu.unpack_shards
            up(world, src.data_ptr(), frame.data_ptr(), sptr)

    mode = select_mode(a.mode, policy_gpus(scene, settings, world)) if world > 1 else "single"
    other = {"tiles": "frames", "frames": "tiles"}.get(mode)
    if world > 1:
        dt = torch.uint8 if u8 else torch.float32
        shard_u8 = torch.empty(stride, dtype=torch.uint8, device="cuda")
        if host_staged and rank == 0:
            flat_dev = torch.empty(stride * world, dtype=torch.float32, device="cuda")
            flat_dev_u8 = torch.empty(stride * world, dtype=torch.uint8, device="cuda")
        dev = "cpu" if host_staged else "cuda"
        pipe = FramePipeline(rank, world, stride, lambda n: torch.empty(n, dtype=dt, device=dev), render_shard,
                             unpack, dist)

    fpar = FrameParallel(rank, world, lambda k: timed(lambda: gpu.render_device(settings, frame.data_ptr(), sptr)))

    def step(m):
        if m == "tiles":
            pipe.step()
        else:
            fpar.step()

    def drain(m):
        if m == "tiles":
            pipe.drain()

    # work counters of one full frame (outside the timed region)
    counts = gpu.count_work(settings)
    waves = gpu.wave_counts()
    rays_per_frame = counts["traversals"]

    def measure(m, steps):
        for _ in range(a.warmup):
            step(m)
        drain(m)
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        timing["events"], timing["n"], timing["i"] = ev, 0, 0
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step(m)
        drain(m)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        km = float(np.mean([s.elapsed_time(e) for s, e in ev[:timing["i"]]]))
        timing["events"] = None
        if world > 1:   # max over ranks
            t = torch.tensor([el, km], dtype=torch.float64, device="cuda" if dist_backend == "nccl" else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el, km = float(t[0]), float(t[1])
        return el, km

    elapsed, kern_ms = measure(mode, a.steps)
    # the last frame of the timed region, kept for the check below (the
    # measurements after this one write into the same buffers)
    timed_last = (frame8 if (mode == "tiles" and u8) else frame).clone() if (a.check and rank == 0) else None

    # camera bins (crt_bins.hip): the frames above keep one camera, so the
    # first binning's lists serve them all (option "bins_reuse", a frame whose
    # camera and plan are the last binning's); beside them the same frames
    # binning every one (bins_reuse 0: the next frames' binnings overlap frame
    # k's render) and with the bins off (every camera ray through the BVH
    # walk), each back to back and one at a time
    bins = None
    one_last = None
    if mode == "single" and not a.shadows:
        b_ms = gpu.bins_ms(50)
        if b_ms > 0.0:
            def back_to_back():
                for _ in range(a.warmup):
                    step(mode)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    step(mode)
                torch.cuda.synchronize()
                return (time.perf_counter() - t0) / a.steps * 1e3

            def one_at_a_time():
                # a host sync after each frame: the single-frame latency (HIP
                # events around the frame's launches on its stream)
                ser = []
                for _ in range(max(10, a.steps // 2)):
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    gpu.render_device(settings, frame.data_ptr(), sptr)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    ser.append(e0.elapsed_time(e1))
                return statistics.median(ser)

            one_ms = one_at_a_time()
            one_last = frame.clone() if a.check else None   # for the check below
            i0 = gpu.info()
            gpu.set_option("bins_reuse", 0)
            rebin_ms = back_to_back()
            rebin_one_ms = one_at_a_time()
            gpu.set_option("bins_reuse", 1)
            i1 = gpu.info()
            gpu.set_option("bins", 0)
            off_ms = back_to_back()
            off_one_ms = one_at_a_time()
            gpu.set_option("bins", 1)
            bins = {"lists_reused": True, "list_sets": 3, "bins_ms": round(b_ms, 5),
                    "frame_ms_one_at_a_time": round(one_ms, 5),
                    "rebinned_every_frame": {"ms_per_step": round(rebin_ms, 5),
                                             "value": round(rays_per_frame / (rebin_ms * 1e-3) / 1e6, 3),
                                             "frame_ms_one_at_a_time": round(rebin_one_ms, 5),
                                             "binnings": i1["bins_binnings"] - i0["bins_binnings"]},
                    "bins_off": {"ms_per_step": round(off_ms, 5),
                                 "value": round(rays_per_frame / (off_ms * 1e-3) / 1e6, 3),
                                 "frame_ms_one_at_a_time": round(off_one_ms, 5)},
                    "note": "ms_per_step frames keep the scene's camera: the first frame bins (k_bins_project [+ "
                            "k_bins_pairs] + k_bins_sort), the rest render its lists again (option bins_reuse; a "
                            "camera move bins again, see camera_orbit); rebinned_every_frame = bins_reuse 0, the "
                            "next frames' binnings overlapping frame k's render (3 sets of lists, "
                            "crt_kernel_common.h kBinSets); one_at_a_time = a host sync after every frame; bins_ms = "
                            "the binning alone (HIP events, 50 binnings); bins_off = the BVH walk for every camera ray"}

    # moving camera: a new pose before every frame, frames back to back
    # (the binning of each frame runs with its own pose; frames in flight keep
    # theirs), then the last orbit frame against a blocking render of its pose
    orbit = None
    if mode == "single" and a.camera_orbit > 0 and "scene" in cfg and not a.shadows:
        from crt_amd.camera import orbit_poses
        fov = float(scene.a["cam_fov"][0])
        cams = [N.CameraDesc(N.Vec3(*[float(v) for v in loc]), (N.C.c_float * 9)(*[float(v) for v in rot]), W, H, fov)
                for loc, rot in orbit_poses(scene.a, a.camera_orbit)]
        home = N.CameraDesc(N.Vec3(*[float(v) for v in scene.a["cam_loc"]]),
                            (N.C.c_float * 9)(*[float(v) for v in scene.a["cam_rot"]]), W, H, fov)
        moves0 = gpu.info()["view_rebuilds"]

        def orbit_step(k):
            gpu.set_camera_desc(cams[k % len(cams)])
            gpu.render_device(settings, frame.data_ptr(), sptr)

        for k in range(a.warmup):
            orbit_step(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(a.steps):
            orbit_step(k)
        torch.cuda.synchronize()
        o_el = time.perf_counter() - t0
        o_ms = o_el / a.steps * 1e3
        o_check = None
        if a.check:
            o_last = frame.clone()
            gpu.set_camera_desc(cams[(a.steps - 1) % len(cams)])
            o_want = gpu.render(settings)
            o_check = ("bit-identical" if np.array_equal(o_last.view(H, W, 3).cpu().numpy().view(np.uint32),
                                                         o_want.view(np.uint32)) else "DIFFERS")
        gpu.set_camera_desc(home)
        orbit = {"poses": len(cams), "frames": a.steps, "ms_per_step": round(o_ms, 5),
                 "value": round(npx / (o_ms * 1e-3) / 1e6, 3), "unit": "Mrays/s (camera rays: one per pixel)",
                 "vs_fixed_camera": round(o_ms / (elapsed / a.steps * 1e3), 4),
                 "vs_rebinned": (round(o_ms / bins["rebinned_every_frame"]["ms_per_step"], 4) if bins else None),
                 "view_rebuilds": gpu.info()["view_rebuilds"] - moves0, "check": o_check,
                 "note": "crt_hip_scene_set_camera before every frame (yaw 20 deg sin, pitch 6 deg cos around the "
                         "scene's centre), frames issued back to back into HBM; every frame bins its own pose "
                         "(vs_fixed_camera: against ms_per_step, whose frames reuse one binning; "
                         "vs_rebinned: against camera_bins.rebinned_every_frame)"}
        if o_check == "DIFFERS":
            print("check: orbit frame DIFFERS from the blocking render of its pose", flush=True)
            raise SystemExit(1)

    check = None
    if a.check and rank == 0:
        # the reference's blocking call (crt_hip_render, one frame with nothing
        # in flight; itself pinned to the oracle by the -m gpu suite) against
        # the last frame of the timed region and, for camera-bins frames, the
        # last one-at-a-time frame
        torch.cuda.synchronize()
        want = gpu.render(settings)
        if mode == "tiles" and u8:
            wd = torch.from_numpy(want).reshape(-1).to("cuda")
            w8 = torch.empty(npx * 3, dtype=torch.uint8, device="cuda")
            N.quantize_rgb8(wd.data_ptr(), npx * 3, w8.data_ptr(), 255, sptr)
            torch.cuda.synchronize()
            results = {"timed": torch.equal(w8, timed_last)}
        else:
            wb = want.view(np.uint32)
            results = {"timed": np.array_equal(timed_last.view(H, W, 3).cpu().numpy().view(np.uint32), wb)}
            if one_last is not None:
                results["one_at_a_time"] = np.array_equal(one_last.view(H, W, 3).cpu().numpy().view(np.uint32), wb)
        same = all(results.values())
        check = "bit-identical" if same else "DIFFERS"
        verdicts = ", ".join(f"{k} frame " + ("bit-identical" if v else "DIFFERS") for k, v in results.items())
        print(f"check: {verdicts} "
              f"against the blocking 1-GPU render (mode {mode}, payload {a.payload}, world {world}, "
              f"backend {dist_backend or 'none'}, {W}x{H})", flush=True)
        if not same:
            raise SystemExit(1)

    ms_per_step = elapsed / a.steps * 1e3
    frames_per_step = world if mode == "frames" else 1
    mrays = rays_per_frame * frames_per_step * a.steps / elapsed / 1e6

    secondary = None
    if world > 1 and not a.no_secondary:
        el2, km2 = measure(other, a.steps)
        fps2 = world if other == "frames" else 1
        secondary = {"mode": other, "scaling": "weak" if other == "frames" else "strong",
                     "value": round(rays_per_frame * fps2 * a.steps / el2 / 1e6, 3),
                     "unit": "Mrays/s", "ms_per_step": round(el2 / a.steps * 1e3, 5), "kernel_ms": round(km2, 5),
                     "frames_per_step": fps2}

    # BASELINE C2's "primary + shadow rays": the course's earlier renderer (the
    # reference's published 0.066962 s was taken at tag 14-01, which traced
    # shadow rays; at HEAD the loop is dead code, crt_renderer.cpp:29-44),
    # option "shadows" on the same scene: frames back to back and one at a
    # time, its rays counted, its last frame checked against a blocking render
    # (pinned to the oracle by tests/test_png_pins.py), its own roofline
    if world == 1 and not a.shadows and a.config == "c2" and secondary is None:
        gs = N.HipScene(scene, device=local, events=0, shadows=1, calibrate=1)
        cs = gs.count_work(settings)
        ws = gs.wave_counts()
        for _ in range(a.warmup):
            gs.render_device(settings, frame.data_ptr(), sptr)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            gs.render_device(settings, frame.data_ptr(), sptr)
        torch.cuda.synchronize()
        s_ms = (time.perf_counter() - t0) / a.steps * 1e3
        s_last = frame.clone()
        ser = []
        for _ in range(max(10, a.steps // 2)):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            gs.render_device(settings, frame.data_ptr(), sptr)
            e1.record(stream)
            torch.cuda.synchronize()
            ser.append(e0.elapsed_time(e1))
        s_one = statistics.median(ser)
        s_check = "bit-identical" if np.array_equal(s_last.view(H, W, 3).cpu().numpy().view(np.uint32),
                                                    gs.render(settings).view(np.uint32)) else "DIFFERS"
        s_roof = roofline_block(s_one, cs, ws, npx, load_pmc(None, "c2s", W, H), build_id, 1.0)
        s_roof["kernel_ms_basis"] = f"one frame at a time (HIP events around its launches, median): {s_one:.5f} ms"
        secondary = {"mode": "shadow_rays", "metric": "Mrays/sec + frame ms, 1920x1080 scene 14-01 (primary + shadow "
                                                      "rays)",
                     "value": round(cs["traversals"] / (s_ms * 1e-3) / 1e6, 3), "unit": "Mrays/s",
                     "ms_per_step": round(s_ms, 5), "frame_ms_one_at_a_time": round(s_one, 5),
                     "rays_per_frame": cs["traversals"], "node_tests_per_frame": cs["node_tests"],
                     "triangle_tests_per_frame": cs["triangle_tests"], "check": s_check, "roofline": s_roof,
                     "vs_reference_published_s": round(0.066962 / (s_ms * 1e-3), 1),
                     "note": "the course's earlier renderer (option shadows; the reference's published KD-tree time, "
                             "0.066962 s at src/README.md:11, was taken at tag 14-01, which traced shadow rays): camera "
                             "bins for the camera rays; one shadow ray per (diffuse hit, light), deferred: written by "
                             "the render kernel, traced one per lane by k_shadow_vis over the light's bins to its "
                             "first hit within the light (crt_bvh.h lbin_first_hit; the BVH where they do not "
                             "decide), the visible terms summed by k_shadow_compose; not HEAD parity"}
        del gs
        if s_check == "DIFFERS":
            print("check: shadow-ray frame DIFFERS from the blocking render", flush=True)
            raise SystemExit(1)

    # end-to-end frame time of the reference's call: render_image returns a
    # host image (crt_image.h:11-27), the CLI times the whole call (main.cpp:37-43)
    e2e = e2e_page = None
    if world == 1 and not a.no_e2e:
        host = torch.empty(npx * 3, dtype=torch.float32, pin_memory=True)
        page = np.zeros(npx * 3, np.float32)

        def e2e_of(ptr):
            for _ in range(3):
                gpu.render_host(settings, ptr)
            ts = []
            for _ in range(max(5, min(a.steps, 50))):
                s = time.perf_counter()
                gpu.render_host(settings, ptr)
                ts.append(time.perf_counter() - s)
            return statistics.median(ts) * 1e3

        e2e = e2e_of(host.data_ptr())
        e2e_page = e2e_of(page.ctypes.data)
    cold = shim = None
    if world == 1 and rank == 0 and not a.no_e2e:
        cold = cold_cli(cfg, W, H, settings)
        if not a.shadows:
            shim = shim_timing(a.config, W, H)

    shard_frac = 1.0 / world if mode == "tiles" else 1.0
    pmc = load_pmc(a.pmc_json, a.config, W, H)
    # the dominant kernel is the render; a camera-bins frame also runs the
    # binning launches before it (their time measured alone above)
    render_ms = bins["frame_ms_one_at_a_time"] if bins else kern_ms
    roof = roofline_block(render_ms, counts, waves, npx, pmc, build_id, shard_frac)
    if bins:
        roof["kernel_ms_basis"] = ("render kernel = a frame that renders the last binning's lists, one at a time "
                                   f"(HIP events around its launch, median): {bins['frame_ms_one_at_a_time']:.5f} ms")

    out = None
    if rank == 0:
        cpu = None
        if world == 1 and not a.no_cpu_baseline:
            cw, ch = cfg["cpu_size"] if (W, H) == cfg["size"] else (W, H)
            note = "" if (cw, ch) == (W, H) else f" at {cw}x{ch} (same scene and settings; Mrays/s is per-ray work)"
            cpu = cpu_baseline(a.config, cw, ch, a.cpu_seconds, a.cpu_single_seconds, note, a.shadows,
                               full=(W, H) if (cw, ch) != (W, H) and not a.no_cpu_full else None)
        parallel = {"single": "single-gpu", "tiles": f"bucket-shard{world}+{'rccl' if dist_backend == 'nccl' else dist_backend}"
                    f"-gather-{a.shards}-{a.payload}", "frames": f"frame-parallel{world}"}[mode]
        out = {
            "metric": ("Mrays/sec + frame ms, 1920x1080 scene 14-01" if a.config == "c2"
                       else f"Mrays/sec + frame ms, {W}x{H} {cfg['label']}")
                      + (" (primary + shadow rays)" if a.shadows else ""),
            "value": round(mrays, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True,
            "scaling": "strong" if mode == "tiles" else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": (f"scene file scenes/{cfg['label']}.crtscene (parsed fixture tests/golden/scenes)" if "scene" in cfg
                     else "synthetic mesh (crt_amd.synthetic.c5_scene, SURVEY §8(d) C5 spec)"),
            "config": {"workload": f"{cfg['label']} {W}x{H}, RendererSettings defaults "
                                   f"(max_ray_depth {settings.max_ray_depth}), "
                                   + ("shadow rays traced (option shadows; HEAD traces none)" if a.shadows else cfg["note"]),
                       "config": a.config,
                       "rays_per_frame": rays_per_frame, "node_tests_per_frame": counts["node_tests"],
                       "triangle_tests_per_frame": counts["triangle_tests"],
                       "parallelism": parallel, "world_size_initialised": world,
                       "dist_backend": dist_backend, "payload": a.payload if mode == "tiles" else None,
                       "shards": a.shards if mode == "tiles" else None,
                       "gather_bytes_per_rank": (stride * (1 if u8 else 4)) if mode == "tiles" else None,
                       "frames_per_step": frames_per_step,
                       "frame_ms": round(ms_per_step, 5), "kernel_ms": round(kern_ms, 5),
                       "e2e_ms": round(e2e, 4) if e2e is not None else None,
                       "e2e_pageable_ms": round(e2e_page, 4) if e2e_page is not None else None,
                       "e2e_note": ("crt_hip_render into a pinned (e2e_ms) / pageable (e2e_pageable_ms) host buffer, "
                                    "median of blocking calls: the render and the fp32 image in host memory, the "
                                    "reference's render_image call (main.cpp:37-43); the image copy is compact "
                                    "(crt_api.hip image_to_host: each row's non-background span over PCIe, the "
                                    "background written by host threads)") if e2e is not None else None,
                       "cold_cli": cold,
                       "shim": shim,
                       "check": check, "build_id": build_id,
                       "camera_bins": bins,
                       "camera_orbit": orbit,
                       "scene_create_ms": {"wall": round(create_wall_ms, 3),
                                           **{k: round(v, 3) for k, v in gpu.info().items()
                                              if k in ("prep_ms", "tree_build_ms", "bvh_ms", "bins_ms", "upload_ms",
                                                       "create_ms")}},
                       "scene_create_ms_second": warm_create,
                       "plan": gpu.plan_info()},
            "roofline": roof,
            "secondary": secondary,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
