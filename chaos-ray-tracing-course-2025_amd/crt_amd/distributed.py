"""Multi-GPU frame rendering: bucket shards + one gather to rank 0.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI).
The reference's bucket grid (crt_renderer.cpp:160-174) is dealt round-robin to
ranks — bucket k → rank k % world — which balances the centre-heavy scenes
without any exchange: pixels are independent (per-pixel PCG seed, read-only
scene, crt_renderer.cpp:147-155).  The single data-path collective is the final
gather of every rank's packed buckets to rank 0, which then scatters them into
the row-major frame (crt_hip_unpack_shards).  Output is bit-identical for any
world size.

Compact shards (crt_hip_*_compact, the bench default) cut each bucket into
8x8 tiles and pack only the live ones — tiles with a pixel whose camera ray
passes the reference's root-cell test; every other pixel is a miss, i.e. the
background, written by the unpack on rank 0.  Lossless, and on 14-01/scene1
3.5x fewer bytes through rank 0's xGMI links.

The render and unpack steps are injected so the same orchestration runs on
GPUs (HipScene.render_shard / unpack_shards) and, in tests, under gloo on CPU.
"""
from __future__ import annotations

from typing import Callable

import numpy as np

from .native import shard_compact_plan, shard_plan


def select_mode(requested: str, policy_gpus: int) -> str:
    """The N-GPU mode of bench.py.  requested: "auto" | "tiles" |
    "frames"; policy_gpus: crt_auto_gpus of the frame for the N visible GPUs
    (the GPUs one frame pays for: 1 when its one-GPU estimate is under 2 ms).
    A frame that does not pay for a second GPU cannot strong-scale (C2: 1.08x,
    C3: 1.13x at 8 shards), so "auto" renders whole frames per GPU (weak
    scaling); frames that do (C4, C5) are sharded as tiles (strong scaling)."""
    if requested not in ("auto", "tiles", "frames"):
        raise ValueError(f"mode {requested!r}")
    if requested != "auto":
        return requested
    return "frames" if policy_gpus <= 1 else "tiles"


class FrameParallel:
    """Whole frames per rank (frames mode): step s renders frame
    s * world + rank on this rank, with no collective on the data path.
    `render(frame_index)` renders one frame (and returns an optional digest
    of it, kept with its index); `collect(dist)` hands every rank's
    (frame, digest) pairs to every rank, so rank 0 can account for each frame
    of the run exactly once."""

    def __init__(self, rank: int, world: int, render: Callable[[int], object]):
        self.rank, self.world, self.render = rank, world, render
        self.steps = 0
        self.done: list = []

    def step(self) -> None:
        k = self.steps * self.world + self.rank
        self.done.append((k, self.render(k)))
        self.steps += 1

    def collect(self, dist) -> list:
        out = [None] * self.world
        dist.all_gather_object(out, self.done)
        return sorted(x for part in out for x in part)


class FrameSharder:
    """Buffers + steps of one sharded frame for `rank` of `world`."""

    def __init__(self, width: int, height: int, bucket_size: int, rank: int, world: int,
                 stride: int, alloc: Callable[[int], object]):
        self.width, self.height, self.bucket = width, height, bucket_size
        self.rank, self.world, self.stride = rank, world, stride
        self.plan = shard_plan(width, height, bucket_size, rank, world)
        self.packed = alloc(stride)
        self.gather_list = [alloc(stride) for _ in range(world)] if rank == 0 else None

    def gather(self, dist, group=None) -> None:
        """The one collective: rank r's packed buckets → slot r on rank 0."""
        dist.gather(self.packed, self.gather_list, dst=0, group=group)


class FramePipeline:
    """Frames rendered back to back, each sharded over the ranks, with frame
    k's gather overlapping frame k+1's shard render (double-buffered).

    `render(packed)` fills this rank's packed buckets of the next frame,
    `unpack(gathered_flat)` (rank 0) scatters a gathered frame into the
    output.  With the "nccl" backend `Work.wait()` only orders the caller's
    current stream after the collective, so rank 0 issues
    render(k+1) → gather(k+1) → wait(gather k) → unpack(k) and the GPU runs
    the gather of frame k on RCCL's stream while frame k+1 renders.  A packed
    buffer is reused two frames later, after its gather was waited on.
    """

    def __init__(self, rank: int, world: int, stride: int, alloc: Callable[[int], object],
                 render: Callable[[object], None], unpack: Callable[[object], None], dist, group=None):
        self.rank, self.world, self.stride = rank, world, stride
        self.render, self.unpack, self.dist, self.group = render, unpack, dist, group
        self.packed = [alloc(stride), alloc(stride)]
        if rank == 0:
            self.flat = [alloc(stride * world), alloc(stride * world)]
            self.views = [[f[i * stride:(i + 1) * stride] for i in range(world)] for f in self.flat]
        else:
            self.flat = self.views = None
        self.pending = None
        self.frames = 0

    def step(self) -> None:
        b = self.frames % 2
        self.render(self.packed[b])
        work = self.dist.gather(self.packed[b], self.views[b] if self.rank == 0 else None, dst=0,
                                group=self.group, async_op=True)
        if self.pending is not None:
            self._finish(*self.pending)
        self.pending = (b, work)
        self.frames += 1

    def drain(self) -> None:
        if self.pending is not None:
            self._finish(*self.pending)
            self.pending = None

    def _finish(self, b: int, work) -> None:
        work.wait()
        if self.rank == 0:
            self.unpack(self.flat[b])


def unpack_numpy(gathered: np.ndarray, width: int, height: int, bucket_size: int, world: int,
                 stride: int) -> np.ndarray:
    """Host mirror of crt_hip_unpack_shards (used by CPU tests)."""
    out = np.zeros((height, width, 3), np.float32)
    for s in range(world):
        for x, y, w, h, off, _ in shard_plan(width, height, bucket_size, s, world):
            src = gathered[s * stride + 3 * off: s * stride + 3 * (off + w * h)]
            out[y:y + h, x:x + w] = src.reshape(h, w, 3)
    return out


def unpack_compact_numpy(gathered: np.ndarray, width: int, height: int, bucket_size: int, world: int, stride: int,
                         live_mask: np.ndarray | None, background) -> np.ndarray:
    """Host mirror of crt_hip_unpack_compact (used by CPU tests): live tiles
    from their shard's slot, the background everywhere else."""
    out = np.empty((height, width, 3), np.float32)
    out[:] = np.asarray(background, np.float32)
    for s in range(world):
        for x, y, w, h, off in shard_compact_plan(width, height, bucket_size, s, world, live_mask):
            src = gathered[s * stride + 3 * off: s * stride + 3 * (off + w * h)]
            out[y:y + h, x:x + w] = src.reshape(h, w, 3)
    return out
