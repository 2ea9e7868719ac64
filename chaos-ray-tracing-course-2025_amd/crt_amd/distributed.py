"""Multi-GPU frame rendering: bucket shards + one gather to rank 0.

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI).
The reference's bucket grid (crt_renderer.cpp:160-174) is dealt round-robin to
ranks — bucket k → rank k % world — which balances the centre-heavy scenes
without any exchange: pixels are independent (per-pixel PCG seed, read-only
scene, crt_renderer.cpp:147-155).  The single data-path collective is the final
gather of every rank's packed buckets to rank 0, which then scatters them into
the row-major frame (crt_hip_unpack_shards).  Output is bit-identical for any
world size.

The render and unpack steps are injected so the same orchestration runs on
GPUs (HipScene.render_shard / unpack_shards) and, in tests, under gloo on CPU.
"""
from __future__ import annotations

from typing import Callable

import numpy as np

from .native import shard_plan


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


def unpack_numpy(gathered: np.ndarray, width: int, height: int, bucket_size: int, world: int,
                 stride: int) -> np.ndarray:
    """Host mirror of crt_hip_unpack_shards (used by CPU tests)."""
    out = np.zeros((height, width, 3), np.float32)
    for s in range(world):
        for x, y, w, h, off, _ in shard_plan(width, height, bucket_size, s, world):
            src = gathered[s * stride + 3 * off: s * stride + 3 * (off + w * h)]
            out[y:y + h, x:x + w] = src.reshape(h, w, 3)
    return out
