set -u
OUT=gpurun_out/r03l; mkdir -p $OUT
timeout -k 10 200 python3 scripts/render_loop.py --frames 20 --opt traversal=8,14 > $OUT/rl_default.json 2>&1 && tail -1 $OUT/rl_default.json | cut -c1-400
timeout -k 10 200 python3 scripts/render_loop.py --frames 20 --opt calibrate=0,1,2 --ab CRT_DUMMY=1 > /dev/null 2>&1
for c in 0 1; do timeout -k 10 200 python3 - <<PY > $OUT/rl_cal$c.json 2>&1
import sys, json, numpy as np; sys.path.insert(0,'chaos-ray-tracing-course-2025_amd')
from crt_amd import native as N; from crt_amd.scene_npz import load_npz
sc = load_npz('tests/golden/scenes/14-01-acceleration-tree__scene1.npz')
st = N.RendererSettings.default()
out = {}
for t in (8, 14):
    g = N.HipScene(sc, traversal=t, calibrate=$c)
    g.render(st)
    ts = []
    for _ in range(20):
        _, s = g.render(st, with_stats=True); ts.append(s["kernel_ms"])
    out[f"traversal={t} calibrate=$c"] = [float(np.median(ts)), float(np.min(ts)), g.plan_info()]
print(json.dumps(out))
PY
tail -1 $OUT/rl_cal$c.json; done
timeout -k 10 200 python3 scripts/shard_times.py --config c2 --reps 20 --opt traversal=14 --out $OUT/shards_c2_t14.json > $OUT/sh.log 2>&1 && tail -1 $OUT/shards_c2_t14.json | python3 -c "import json,sys; d=json.load(sys.stdin); print({k:(round(v['max_ms'],4), v['speedup_vs_n1']) for k,v in d['shards'].items()})"
timeout -k 10 200 python3 scripts/wave_timeline.py --opt traversal=14 --out $OUT/timeline_c2_t14.json > $OUT/tl.log 2>&1; tail -3 $OUT/tl.log | cut -c1-600
