#!/usr/bin/env python3
"""Summarise render_loop.py JSON lines: one line per file, 'variant median min'.
  python3 scripts/ab_summary.py file.json [...]"""
import json
import sys

for path in sys.argv[1:]:
    lines = [l for l in open(path).read().splitlines() if l.startswith("{")]
    if not lines:
        print(path, "no result")
        continue
    d = json.loads(lines[-1])
    parts = []
    for name, k in d["kernel"].items():
        parts.append("%s %.4f %.4f" % (name.split("=")[-1], k["median_ms"], k["min_ms"]))
    print(path.rsplit("/", 1)[-1], " | ".join(parts))
