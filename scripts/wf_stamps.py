"""Diagnostic: where a wavefront level's time goes.  With a CRT_WF_STAMPS build
(scripts/make_variant.sh stamps WF_FLAGS=-DCRT_WF_STAMPS HOST_AB_FLAGS=-DCRT_WF_STAMPS)
every wave of k_wf_level stamps s_memrealtime (100 MHz) at its start and end;
this renders C3 (11-01-refractive/scene8, 1920x1080, depth 8) a few times,
dumps one frame's stamps and prints per level: waves, the level's span, and
the spread of wave durations and end times (is a level a tail of long rays or
a wall of uniform work?)."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
PKG = Path(os.environ.get("CRT_PKG", ROOT / "abtest" / "stamps")).resolve()
sys.path.insert(0, str(PKG))
sys.path.insert(0, str(ROOT))
from crt_amd import native as N  # noqa: E402
from crt_amd.scene_npz import load_npz  # noqa: E402

scene = os.environ.get("SCENE", "11-01-refractive__scene8")
w, h = (int(v) for v in os.environ.get("SIZE", "1920x1080").split("x"))
depth = int(os.environ.get("DEPTH", "8"))
out = Path(os.environ.get("OUT", "gpurun_out/stamps"))
out.mkdir(parents=True, exist_ok=True)
print("lib", N.LIB_PATH, N.build_id(), flush=True)
sc = load_npz(ROOT / "tests" / "golden" / "scenes" / f"{scene}.npz").set_resolution(w, h)
st = N.RendererSettings.default(max_ray_depth=depth)
g = N.HipScene(sc)
for kv in os.environ.get("OPTS", "").split(","):
    if kv:
        k, v = kv.split("=")
        g.set_option(k, int(v))
for _ in range(4):
    g.render(st)
fn = out / f"{scene}.txt"
os.environ["CRT_WF_STAMPS_FILE"] = str(fn)
if os.environ.get("COUNT"):   # a counting frame: per-wave sum / max of its lanes' node + triangle tests
    g.count_work(st)
else:
    g.render(st)
del os.environ["CRT_WF_STAMPS_FILE"]
a = np.loadtxt(fn, dtype=np.int64).reshape(-1, 9)   # level wave start walk trace end fallback_lanes steps_sum steps_max
a = a[a[:, 5] > 0]   # waves wholly past the queue return before their end stamp
t0 = a[:, 2].min()
print(f"frame span {(a[:, 5].max() - t0) / 100:.1f} us, {len(a)} waves")
print("lvl waves   span | wave p50/p90/max (us) | walk p50/p90 | proof+fb p50/p90 | shade p50 | fb lanes/wave mean, waves with fb, p50/p90 dur of fb waves")
for L in np.unique(a[:, 0]):
    b = a[a[:, 0] == L]
    s, wk, tr, e, fb = b[:, 2], b[:, 3], b[:, 4], b[:, 5], b[:, 6]
    ok = wk > 0
    d = (e - s) / 100
    walk = (wk[ok] - s[ok]) / 100
    proof = (tr[ok] - wk[ok]) / 100
    shade = (e - tr) / 100
    p = lambda x, q: float(np.percentile(x, q)) if len(x) else float("nan")
    hasfb = fb > 0
    print(f"{L:3d} {len(b):6d} {(e.max() - s.min()) / 100:6.1f} | {p(d, 50):5.1f}/{p(d, 90):5.1f}/{d.max():5.1f} | "
          f"{p(walk, 50):5.1f}/{p(walk, 90):5.1f} | {p(proof, 50):5.1f}/{p(proof, 90):5.1f} | {p(shade, 50):5.1f} | "
          f"{fb.mean():5.2f} {hasfb.sum():5d} {p(d[hasfb], 50):5.1f}/{p(d[hasfb], 90):5.1f} vs {p(d[~hasfb], 50):5.1f}")
    if os.environ.get("COUNT"):
        lanes = np.minimum(64, 64)
        eff = b[:, 7] / np.maximum(1, 64 * b[:, 8])
        print(f"      steps/lane mean {b[:, 7].sum() / (64 * len(b)):6.1f}  wave max p50/p90 {p(b[:, 8], 50):6.0f}/{p(b[:, 8], 90):6.0f}"
              f"  lane use (sum / 64 max) {b[:, 7].sum() / max(1, 64 * b[:, 8].sum()):.2f}"
              f"  us per max-step {np.median(d / np.maximum(1, b[:, 8])) * 1000:.0f} ns")
