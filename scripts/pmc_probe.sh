#!/bin/bash
# Counter passes (one rocprofv3 --pmc run each) over one command, summed per
# kernel by scripts/pmc_probe_sum.py for kernels matching MATCH.
#   TAG=x MATCH='k_wf_level<14, false' CMD="scripts/render_loop.py ..." bash scripts/pmc_probe.sh "C1 C2" "C3 C4" ...
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-probe}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- python3 $CMD > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($grp) failed"; tail -3 "$OUT/p$i.log"; exit 1; }
done
python3 scripts/pmc_probe_sum.py "$OUT" "$MATCH"
