#!/usr/bin/env python3
"""Diagnostic: cost of the wave-coherent light-bin walk (crt_walks.h
occluded_lbins_wave) on C2's shadow rays, from the host restatement
(tests/tools/prune_sim.cpp lbins_sim_steps): per 8x8 tile and light, the
candidates the wave walks = sum over its distinct cells of the longest walk of
a lane in that cell, next to the mean per lane.
  python3 scripts/lbins_wave_cost.py [--width 960 --height 540 --n 64 --emax 0.02]"""
import argparse
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tests"))

from conftest import scene_npz  # noqa: E402
import test_light_bins as T  # noqa: E402
import test_prune as P  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="14-01-acceleration-tree__scene1")
    ap.add_argument("--width", type=int, default=960)
    ap.add_argument("--height", type=int, default=540)
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--emax", type=float, default=0.02)
    a = ap.parse_args()
    import subprocess
    subprocess.run(["make", "-s", "-C", str(P.TOOLS)], check=True)
    sim = C.CDLL(str(P.SIM))
    from oracle import pyoracle
    from crt_amd.native import _desc_ptr, HostScene
    sc = scene_npz(a.scene).set_resolution(a.width, a.height)
    orc = pyoracle.OracleScene(sc)
    ys, xs = np.mgrid[0:a.height, 0:a.width]
    cam = orc.camera_rays(np.stack([xs.ravel(), ys.ravel()], 1))
    rs, rt, _, _, _ = T.bvh_run(sim, sc, cam)
    hit = rs >= 0
    tile = ((ys.ravel() // 8) * ((a.width + 7) // 8) + xs.ravel() // 8)[hit]
    p = (cam[hit, :3] + cam[hit, 3:] * rt[hit, None]).astype(np.float32)
    fn = HostScene(sc).face_normals().reshape(-1, 3)[rs[hit]].astype(np.float32)
    lights = T.scene_lights(sc)
    rays = T.shadow_rays(p, fn, lights, np.float32(1e-2), None)
    n = len(rays)
    cell, steps = np.zeros(n, np.int32), np.zeros(n, np.int32)
    sim.lbins_sim_steps.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_double, C.c_int, C.c_void_p, C.c_void_p]
    rc = sim.lbins_sim_steps(C.cast(_desc_ptr(sc), C.c_void_p), rays.ctypes.data, n, a.emax, a.n,
                             cell.ctypes.data, steps.ctypes.data)
    assert rc == 0
    nl = len(lights)
    tiles = np.tile(tile, nl)
    light = rays[:, 7].astype(np.int64)
    key = tiles * nl + light
    order = np.lexsort((cell, key))
    k, c, s = key[order], cell[order], steps[order]
    # per (tile, light, cell): max steps; per (tile, light): sum over cells, and cell count
    grp = np.flatnonzero(np.r_[True, (k[1:] != k[:-1]) | (c[1:] != c[:-1])])
    mx = np.maximum.reduceat(s, grp)
    kg = k[grp]
    wg = np.flatnonzero(np.r_[True, kg[1:] != kg[:-1]])
    wave = np.add.reduceat(mx, wg)
    cells = np.diff(np.r_[wg, len(kg)])
    ko = np.sort(key)
    so = steps[np.argsort(key, kind="stable")]
    lg = np.flatnonzero(np.r_[True, ko[1:] != ko[:-1]])
    lane_max = np.maximum.reduceat(so, lg)
    print(f"rays {n}  undecided {(cell == -2).mean():.4f}  lane steps mean {steps.mean():.2f} p99 {np.percentile(steps, 99):.0f} max {steps.max()}")
    print(f"waves {len(wave)}  wave steps mean {wave.mean():.1f} p90 {np.percentile(wave, 90):.0f} max {wave.max()}  cells/wave mean {cells.mean():.2f} max {cells.max()}")
    for cap in (16, 32, 48, 64):
        over = steps > cap
        print(f"cap {cap}: rays over {over.mean():.4f}, waves with one {np.maximum.reduceat(over[np.argsort(key, kind='stable')].astype(np.int8), lg).mean():.4f}")
    print(f"per-lane walk: wave = longest lane, mean {lane_max.mean():.1f} p90 {np.percentile(lane_max, 90):.0f} max {lane_max.max()}")


if __name__ == "__main__":
    main()
