"""Multi-GPU path on CPU: bucket sharding + the single gather, world_size 2
(and 3), gloo backend.  The per-shard render is injected (the CPU oracle
renders each rank's buckets) so the partition, packing, gather and unpack
logic of crt_amd.distributed is exercised without GPUs; tests/test_gpu_parity.py
covers the device-side shard kernel and unpack kernel."""
import os
import socket

import numpy as np
import pytest


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, W, H, out_path):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root / "chaos-ray-tracing-course-2025_amd"))
    sys.path.insert(0, str(root))
    import torch
    import torch.distributed as dist
    from crt_amd.distributed import FrameSharder, unpack_numpy
    from crt_amd.native import RendererSettings, shard_plan
    from crt_amd.scene_npz import load_npz
    from oracle import pyoracle

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    sc = load_npz(root / "tests/golden/scenes/14-01-acceleration-tree__scene1.npz").set_resolution(W, H)
    bucket = sc.desc().bucket_size
    stride = max(3 * int((p[:, 2] * p[:, 3]).sum()) for p in
                 (shard_plan(W, H, bucket, s, world) for s in range(world)))
    stride = (stride + 63) // 64 * 64
    fs = FrameSharder(W, H, bucket, rank, world, stride, lambda n: torch.zeros(n, dtype=torch.float32))
    orc = pyoracle.OracleScene(sc)
    st = RendererSettings.default()
    packed = fs.packed.numpy()
    for x, y, w, h, off, _ in fs.plan:           # this rank's buckets, packed row-major
        for row in range(h):
            px = orc.render_pixels(st, (y + row) * W + x, w)
            packed[3 * (off + row * w): 3 * (off + (row + 1) * w)] = px.reshape(-1)
    fs.gather(dist)
    if rank == 0:
        gathered = torch.cat(fs.gather_list).numpy()
        img = unpack_numpy(gathered, W, H, bucket, world, stride)
        np.save(out_path, img)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H", [(2, 200, 120), (3, 100, 75)])
def test_sharded_frame_equals_single_render(tmp_path, oracle, world, W, H):
    import torch.multiprocessing as mp
    from crt_amd.native import RendererSettings
    from conftest import bits, scene_npz
    out = tmp_path / "frame.npy"
    mp.spawn(_worker, args=(world, free_port(), W, H, str(out)), nprocs=world, join=True)
    got = np.load(out)
    want = oracle.OracleScene(scene_npz("14-01-acceleration-tree__scene1").set_resolution(W, H)).render(
        RendererSettings.default())
    assert np.array_equal(bits(got), bits(want))


def test_shard_plan_partitions_the_frame():
    from crt_amd.native import shard_plan
    for W, H, b, world in [(1920, 1080, 24, 8), (333, 200, 24, 3), (100, 60, 24, 5), (10, 10, 24, 2)]:
        cover = np.zeros((H, W), np.int32)
        for s in range(world):
            p = shard_plan(W, H, b, s, world)
            assert (p[:, 5] % world == s).all()                  # bucket k → shard k % world
            packed = 0
            for x, y, w, h, off, _ in p:
                assert off == packed
                packed += w * h
                cover[y:y + h, x:x + w] += 1
        nx, ny = int(W / b + 0.5), int(H / b + 0.5)              # crt_renderer.cpp:160-161
        assert (cover == (1 if nx and ny else 0)).all()


def _pipeline_worker(rank, world, port, W, H, frames, out_path):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root / "chaos-ray-tracing-course-2025_amd"))
    sys.path.insert(0, str(root))
    import torch
    import torch.distributed as dist
    from crt_amd.distributed import FramePipeline, unpack_numpy
    from crt_amd.native import RendererSettings, shard_plan
    from crt_amd.scene_npz import load_npz
    from oracle import pyoracle

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    sc = load_npz(root / "tests/golden/scenes/14-01-acceleration-tree__scene1.npz").set_resolution(W, H)
    bucket = sc.desc().bucket_size
    stride = max(3 * int((p[:, 2] * p[:, 3]).sum()) for p in
                 (shard_plan(W, H, bucket, s, world) for s in range(world)))
    orc = pyoracle.OracleScene(sc)
    st = RendererSettings.default()
    base = np.zeros(stride, np.float32)
    for x, y, w, h, off, _ in shard_plan(W, H, bucket, rank, world):
        for row in range(h):
            base[3 * (off + row * w): 3 * (off + (row + 1) * w)] = orc.render_pixels(st, (y + row) * W + x, w).reshape(-1)
    state = {"k": 0, "out": []}

    def render(packed):                  # frame k = oracle frame * (k + 1)
        packed.numpy()[:] = base * np.float32(state["k"] + 1)
        state["k"] += 1

    def unpack(flat):
        state["out"].append(unpack_numpy(flat.numpy(), W, H, bucket, world, stride))

    pipe = FramePipeline(rank, world, stride, lambda n: torch.zeros(n, dtype=torch.float32), render, unpack, dist)
    for _ in range(frames):
        pipe.step()
    pipe.drain()
    if rank == 0:
        np.save(out_path, np.stack(state["out"]))
    dist.barrier()
    dist.destroy_process_group()


def test_frame_pipeline_keeps_frames_apart(tmp_path, oracle):
    """Double-buffered frames (bench.py's N-GPU loop): every frame comes out
    whole and in order although frame k+1 renders before frame k is unpacked."""
    import torch.multiprocessing as mp
    from crt_amd.native import RendererSettings
    from conftest import bits, scene_npz
    W, H, frames, world = 120, 72, 5, 2
    out = tmp_path / "frames.npy"
    mp.spawn(_pipeline_worker, args=(world, free_port(), W, H, frames, str(out)), nprocs=world, join=True)
    got = np.load(out)
    want = oracle.OracleScene(scene_npz("14-01-acceleration-tree__scene1").set_resolution(W, H)).render(
        RendererSettings.default())
    assert got.shape == (frames, H, W, 3)
    for k in range(frames):
        assert np.array_equal(bits(got[k]), bits(want * np.float32(k + 1)))


def _compact_worker(rank, world, port, W, H, out_path):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root / "chaos-ray-tracing-course-2025_amd"))
    sys.path.insert(0, str(root))
    import torch
    import torch.distributed as dist
    from crt_amd.distributed import FramePipeline, unpack_compact_numpy
    from crt_amd.native import RendererSettings, shard_compact_plan
    from crt_amd.scene_npz import load_npz
    from oracle import pyoracle

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    sc = load_npz(root / "tests/golden/scenes/14-01-acceleration-tree__scene1.npz").set_resolution(W, H)
    d = sc.desc()
    bucket = d.bucket_size
    orc = pyoracle.OracleScene(sc)
    # any mask whose dead pixels are misses is lossless; on the GPU it is the
    # root-cell test (crt_hip_live_mask), here the oracle's own hit/miss
    ys, xs = np.mgrid[0:H, 0:W]
    hits, _, _ = orc.trace(orc.camera_rays(np.stack([xs.ravel(), ys.ravel()], 1)))
    mask = hits["hit"].reshape(H, W).astype(np.uint8)
    plans = [shard_compact_plan(W, H, bucket, s, world, mask) for s in range(world)]
    stride = max(64, max(3 * int((p[:, 2] * p[:, 3]).sum()) for p in plans))
    st = RendererSettings.default()

    def render(packed):
        a = packed.numpy()
        for x, y, w, h, off in plans[rank]:
            for row in range(h):
                a[3 * (off + row * w): 3 * (off + (row + 1) * w)] = orc.render_pixels(st, (y + row) * W + x, w).reshape(-1)

    out = []
    bg = (d.background_color.x, d.background_color.y, d.background_color.z)
    pipe = FramePipeline(rank, world, stride, lambda n: torch.zeros(n, dtype=torch.float32), render,
                         lambda flat: out.append(unpack_compact_numpy(flat.numpy(), W, H, bucket, world, stride, mask,
                                                                      bg)), dist)
    pipe.step()
    pipe.drain()
    if rank == 0:
        np.save(out_path, out[0])
    dist.barrier()
    dist.destroy_process_group()


def test_compact_sharded_frame_equals_single_render(tmp_path, oracle):
    """Compact shards over gloo (world 3): only live tiles are packed and
    gathered, the unpack fills the rest with the background — the frame equals
    the oracle's single render bit for bit, and the live plans partition the
    live part of every shard's buckets."""
    import torch.multiprocessing as mp
    from crt_amd.native import RendererSettings
    from conftest import bits, scene_npz
    W, H, world = 150, 90, 3
    out = tmp_path / "frame.npy"
    mp.spawn(_compact_worker, args=(world, free_port(), W, H, str(out)), nprocs=world, join=True)
    want = oracle.OracleScene(scene_npz("14-01-acceleration-tree__scene1").set_resolution(W, H)).render(
        RendererSettings.default())
    assert np.array_equal(bits(np.load(out)), bits(want))


def test_compact_plan_covers_live_pixels():
    from crt_amd.native import shard_compact_plan, shard_plan
    rng = np.random.default_rng(5)
    for W, H, b, world in [(333, 200, 24, 3), (100, 60, 20, 5), (64, 64, 24, 2)]:
        mask = (rng.random((H, W)) < 0.02).astype(np.uint8)
        cover = np.zeros((H, W), np.int32)
        for s in range(world):
            p = shard_compact_plan(W, H, b, s, world, mask)
            packed = 0
            for x, y, w, h, off in p:
                assert off == packed and w <= 8 and h <= 8 and mask[y:y + h, x:x + w].any()
                packed += w * h
                cover[y:y + h, x:x + w] += 1
            full = shard_compact_plan(W, H, b, s, world, None)          # no mask: every tile of the buckets
            assert int((full[:, 2] * full[:, 3]).sum()) == int((shard_plan(W, H, b, s, world)[:, 2:4].prod(1)).sum())
        assert (cover <= 1).all() and (cover[mask == 1] == 1).all()


def test_mode_rule_by_policy():
    """bench.py --gpus N picks whole frames per GPU when the library's policy
    gives the frame one GPU (C2, C3: a one-GPU frame under 2 ms cannot
    strong-scale) and sharded tiles when it gives it more (C4, C5)."""
    import ctypes as C
    from conftest import scene_npz
    from crt_amd import native as N
    from crt_amd.distributed import select_mode
    from crt_amd.synthetic import c5_scene
    os.environ.pop("CRT_HIP_GPUS", None)
    cases = [(scene_npz("14-01-acceleration-tree__scene1").set_resolution(1920, 1080), {}, "frames"),
             (scene_npz("11-01-refractive__scene8").set_resolution(1920, 1080), {"max_ray_depth": 8}, "frames"),
             (scene_npz("15-01-conclusion__scene2").set_resolution(3840, 2160), {}, "tiles"),
             (c5_scene(1_000_000), {}, "tiles")]
    for sc, over, want in cases:
        st = N.RendererSettings.default(**over)
        pol = N.lib().crt_auto_gpus(N._desc_ptr(sc), C.byref(st), 8)
        assert select_mode("auto", pol) == want
        assert select_mode("tiles", pol) == "tiles" and select_mode("frames", pol) == "frames"
    with pytest.raises(ValueError):
        select_mode("rows", 1)


def _frames_worker(rank, world, port, W, H, steps, out_path):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root / "chaos-ray-tracing-course-2025_amd"))
    sys.path.insert(0, str(root))
    import hashlib
    import torch.distributed as dist
    from crt_amd.camera import orbit_poses
    from crt_amd.distributed import FrameParallel
    from crt_amd.native import RendererSettings
    from crt_amd.scene_npz import load_npz
    from oracle import pyoracle

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    path = root / "tests/golden/scenes/14-01-acceleration-tree__scene1.npz"
    poses = orbit_poses(load_npz(path).a, steps * world)
    st = RendererSettings.default()

    def render(k):   # frame k: the k-th pose of an orbit, rendered whole on this rank
        sc = load_npz(path).set_resolution(W, H).set_camera(location=poses[k][0], rotation=poses[k][1])
        img = pyoracle.OracleScene(sc).render(st)
        return hashlib.sha256(img.tobytes()).hexdigest()

    fp = FrameParallel(rank, world, render)
    for _ in range(steps):
        fp.step()
    got = fp.collect(dist)
    if rank == 0:
        import json
        Path(out_path).write_text(json.dumps(got))
    dist.barrier()
    dist.destroy_process_group()


def test_frames_mode_accounts_every_frame(tmp_path, oracle):
    """Frames mode at world 2 (bench.py's default for C2 / C3 at N > 1):
    step s renders frame s * world + rank; every frame of the run is rendered
    exactly once, by its rank, and equals the frame rendered alone."""
    import hashlib
    import json
    import torch.multiprocessing as mp
    from crt_amd.camera import orbit_poses
    from crt_amd.native import RendererSettings
    from conftest import scene_npz
    W, H, steps, world = 96, 54, 3, 2
    out = tmp_path / "frames.json"
    mp.spawn(_frames_worker, args=(world, free_port(), W, H, steps, str(out)), nprocs=world, join=True)
    got = json.loads(out.read_text())
    assert [k for k, _ in got] == list(range(steps * world))
    poses = orbit_poses(scene_npz("14-01-acceleration-tree__scene1").a, steps * world)
    for k, digest in got:
        sc = scene_npz("14-01-acceleration-tree__scene1").set_resolution(W, H).set_camera(
            location=poses[k][0], rotation=poses[k][1])
        img = oracle.OracleScene(sc).render(RendererSettings.default())
        assert hashlib.sha256(img.tobytes()).hexdigest() == digest, f"frame {k}"


@pytest.mark.parametrize("config,mode", [("c2", "frames"), ("c4", "tiles")])
def test_bench_launcher_picks_mode(config, mode):
    """bench.py --gpus 2 without torchrun's environment starts two rank
    processes itself (python -m torch.distributed.run) and reports the mode
    its rule picks (--selftest-launch: ranks join a gloo group, no GPU work)."""
    import json
    import subprocess
    import sys
    from conftest import ROOT
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "CRT_HIP_GPUS")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--selftest-launch", "--config", config],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["all_reduce_ok"] and d["mode"] == mode
    assert d["scaling"] == ("weak" if mode == "frames" else "strong")
