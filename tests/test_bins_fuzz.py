"""Camera fuzz of the camera bins, the BVH walk and the proof (CPU, no GPU).

The camera bins rest on camera geometry (the 2-pixel margin against the fp32
ray generation, the "hull strictly in front of the camera" test with its
everywhere cap, the dmin bound; crt_bins.h).  This fuzz moves the camera: random
poses — camera inside the mesh, looking exactly along an axis, far away
(beyond the hull margins' origin bound) — fields of view 5-170 degrees, aspect
ratios 1:8 to 8:1 and odd sizes, on course meshes and random meshes (one with a
floor that reaches behind the camera: everywhere hulls).  On every camera ray
(>= 10^7 per run, seeded), tests/tools/prune_sim.cpp bins_fuzz checks

  * bins walk == BVH walk: the same t bits and tie flag, and the same triangle
    without a tie (the proof / fallback then see the same inputs);
  * the product's answer (bins or BVH, then proof or exact kd fallback) == the
    reference-order walk: the same triangle and t bits (a triangle's copies
    in several leaves are one record, crt_acceleration_tree.cpp:44-58);

and on a sample of each case's pixels the product's (triangle, t) equals the
CPU oracle's trace (oracle/crt_oracle.cpp, pinned to the compiled reference).
How often each special path fires is recorded in profiles/r04/bins_fuzz.json
when the environment variable CRT_FUZZ_RECORD is set.
"""
import ctypes as C
import json
import os
import time
from pathlib import Path

import numpy as np
import pytest

from conftest import scene_npz
from test_prune import sim  # noqa: F401  (builds tests/tools/_build/libprune_sim.so)

_P = C.c_void_p
ROOT = Path(__file__).resolve().parents[1]

MESHES = ["14-01-acceleration-tree__scene1", "09-02-diffuse-smooth-shading__scene3", "12-01-textures__scene4",
          "11-01-refractive__scene8", "15-01-conclusion__scene2", "13-01-optimizations__scene0"]
RAYS_TARGET = 10_000_000


def rotation(rng, axis_aligned: bool):
    if axis_aligned:   # an exact axis permutation with signs: camera looking along +-x, +-y or +-z
        p = rng.permutation(3)
        m = np.zeros((3, 3))
        m[np.arange(3), p] = rng.choice([-1.0, 1.0], 3)
        if np.linalg.det(m) < 0:
            m[0] = -m[0]
        return m
    a, b, c = rng.uniform(-np.pi, np.pi, 3)
    rz = np.array([[np.cos(c), np.sin(c), 0], [-np.sin(c), np.cos(c), 0], [0, 0, 1]])
    ry = np.array([[np.cos(b), 0, -np.sin(b)], [0, 1, 0], [np.sin(b), 0, np.cos(b)]])
    rx = np.array([[1, 0, 0], [0, np.cos(a), np.sin(a)], [0, -np.sin(a), np.cos(a)]])
    return rz @ ry @ rx


def size(rng, pixels: int):
    aspect = float(np.exp(rng.uniform(np.log(1 / 8), np.log(8))))
    w = max(1, int(round(np.sqrt(pixels * aspect)))) | 1            # odd sizes
    h = max(1, int(round(pixels / w))) | 1
    return w, h


def mesh_bounds(sc):
    a = sc.a
    pos = np.concatenate([a[f"m{i}_pos"].reshape(-1, 3) for i in range(int(a["mesh_count"][0]))], 0)
    return pos.min(0), pos.max(0)


def cases(seed: int = 2024):
    from crt_amd import native as N
    rng = np.random.default_rng(seed)
    out = []
    for k in range(40):
        kind = k % 8
        pixels = int(rng.integers(170_000, 370_000))
        w, h = size(rng, pixels)
        fov = float(rng.uniform(5, 170))
        rot = rotation(rng, axis_aligned=kind in (1, 5))
        if kind in (0, 1, 2, 3, 4):   # a course mesh; the camera around it, inside it, or far out
            sc = scene_npz(MESHES[k % len(MESHES)])
            lo, hi = mesh_bounds(sc)
            c, ext = (lo + hi) / 2, (hi - lo)
            if kind == 2:
                loc = c + rng.uniform(-0.3, 0.3, 3) * ext                      # inside the mesh's box
            elif kind == 3:
                loc = c + rng.normal(size=3) * 1e4 * (1 + np.abs(ext).max())   # beyond the margins' origin bound
            else:
                d = rng.normal(size=3)
                loc = c + d / np.linalg.norm(d) * np.abs(ext).max() * rng.uniform(0.6, 3.0)
                # look at the mesh: the camera's -z axis (row 2 of R) towards the centre
                fwd = (c - loc) / np.linalg.norm(c - loc)
                if kind != 1:
                    up = rng.normal(size=3)
                    x = np.cross(up, -fwd)
                    x /= np.linalg.norm(x)
                    y = np.cross(-fwd, x)
                    rot = np.stack([x, y, -fwd])
            sc.set_camera(loc, rot, fov).set_resolution(w, h)
        elif kind == 5:   # random triangle soup, camera inside it looking along an axis
            n = int(rng.integers(200, 4000))
            cen = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
            v = (cen[:, None, :] + rng.uniform(-0.08, 0.08, (n, 3, 3))).astype(np.float32).reshape(-1, 3)
            sc = N.SyntheticScene(v, np.arange(len(v), dtype=np.int32), width=w, height=h,
                                  camera_location=tuple(rng.uniform(-0.5, 0.5, 3)),
                                  camera_rotation=tuple(rot.ravel()), fov_degrees=fov)
        else:             # soup above a floor reaching behind the camera (everywhere hulls)
            n = int(rng.integers(200, 3000))
            cen = rng.uniform([-3, -0.8, -8], [3, 2, -1.5], (n, 3)).astype(np.float32)
            v = (cen[:, None, :] + rng.uniform(-0.2, 0.2, (n, 3, 3))).astype(np.float32).reshape(-1, 3)
            fl = np.array([[-60, -1, 60], [60, -1, 60], [60, -1, -60], [-60, -1, -60]], np.float32)
            b = len(v)
            idx = np.concatenate([np.arange(b, dtype=np.int32), np.array([b, b + 1, b + 2, b, b + 2, b + 3], np.int32)])
            yaw = rng.uniform(-0.5, 0.5)
            r = np.array([[np.cos(yaw), 0, -np.sin(yaw)], [0, 1, 0], [np.sin(yaw), 0, np.cos(yaw)]])
            sc = N.SyntheticScene(np.concatenate([v, fl], 0), idx, width=w, height=h,
                                  camera_location=(float(rng.uniform(-1, 1)), 0.3, 0.0),
                                  camera_rotation=tuple(r.ravel()), fov_degrees=fov)
        out.append((f"case{k}-kind{kind}-{w}x{h}-fov{fov:.0f}", sc))
    return out


def test_camera_fuzz_bins_bvh_proof(sim, oracle):  # noqa: F811
    from crt_amd.native import _desc_ptr
    sim.bins_fuzz.argtypes = [_P, C.c_int, _P, _P, C.c_int64, _P]
    sim.bins_fuzz.restype = C.c_int
    rng = np.random.default_rng(7)
    nth = max(1, min(16, len(os.sched_getaffinity(0))))
    totals = np.zeros(11, np.uint64)
    per_case = []
    sampled = 0
    t0 = time.perf_counter()
    for name, sc in cases():
        info_w, info_h = sc.desc().camera.width, sc.desc().camera.height
        npx = info_w * info_h
        sample = np.unique(rng.integers(0, npx, 1500)).astype(np.int64)
        got = np.zeros((len(sample), 2), np.int64)
        out = np.zeros(11, np.uint64)
        assert sim.bins_fuzz(C.cast(_desc_ptr(sc), _P), nth, out.ctypes.data, sample.ctypes.data, len(sample),
                             got.ctypes.data) == 0, name
        assert out[0] == npx
        assert out[1] == 0, f"{name}: {int(out[1])} camera rays: bins walk != BVH walk"
        assert out[2] == 0, f"{name}: {int(out[2])} camera rays: product != reference-order walk"
        orc = oracle.OracleScene(sc)
        rays = orc.camera_rays(np.stack([sample % info_w, sample // info_w], 1))
        hits, _, _ = orc.trace(rays)
        want_tri = np.where(hits["hit"] != 0, hits["triangle_index"], -1)
        want_t = np.where(hits["hit"] != 0, hits["distance"].view(np.uint32).astype(np.int64), 0)
        assert np.array_equal(got[:, 0], want_tri), f"{name}: triangle differs from the oracle"
        assert np.array_equal(got[:, 1], want_t), f"{name}: t differs from the oracle"
        totals += out
        sampled += len(sample)
        per_case.append({"case": name, "rays": int(out[0]), "bins_built": int(out[3]), "over_cap_rays": int(out[4]),
                         "ties": int(out[5]), "kd_fallbacks": int(out[6]), "everywhere_hulls": int(out[7]),
                         "hits": int(out[8]), "records": int(out[9]), "camera_beyond_origin_bound": int(out[10])})
    wall = time.perf_counter() - t0
    assert totals[0] >= RAYS_TARGET
    # the special paths all fired somewhere
    assert any(c["bins_built"] == 0 for c in per_case) and any(c["everywhere_hulls"] > 0 and c["bins_built"]
                                                               for c in per_case)
    assert any(c["camera_beyond_origin_bound"] for c in per_case)
    if os.environ.get("CRT_FUZZ_RECORD"):
        rec = {"rays": int(totals[0]), "differ_bins_vs_bvh": int(totals[1]), "differ_product_vs_reference": int(totals[2]),
               "cases": len(per_case), "cases_with_bins": sum(c["bins_built"] for c in per_case),
               "rays_in_cells_over_cap": int(totals[4]), "ties": int(totals[5]), "kd_fallbacks": int(totals[6]),
               "cases_with_everywhere_hulls": sum(c["everywhere_hulls"] > 0 for c in per_case),
               "cases_everywhere_over_cap": sum(c["everywhere_hulls"] > 64 for c in per_case),
               "cases_camera_beyond_origin_bound": sum(c["camera_beyond_origin_bound"] for c in per_case),
               "oracle_sampled_rays": sampled, "threads": nth, "wall_s": round(wall, 1), "per_case": per_case}
        path = ROOT / "profiles" / "r04" / "bins_fuzz.json"
        path.parent.mkdir(parents=True, exist_ok=True)
        path.write_text(json.dumps(rec, indent=1))
