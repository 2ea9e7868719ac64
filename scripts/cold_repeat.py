"""The CLI's cold render (bench.py cold_cli) repeated: fresh processes, one
GPU, to see the spread of the single sample the bench line carries.
python scripts/cold_repeat.py --config c2 --reps 6"""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
from crt_amd import native as N  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--config", default="c2")
p.add_argument("--reps", type=int, default=6)
a = p.parse_args()
cfg = bench.CONFIGS[a.config]
w, h = cfg["size"]
st = N.RendererSettings.default(**cfg.get("settings", {}))
out = [bench.cold_cli(cfg, w, h, st) for _ in range(a.reps)]
print(json.dumps({"config": a.config, "execution_ms": [o["execution_ms"] for o in out],
                  "process_ms": [o["process_ms"] for o in out]}))
