#!/bin/bash
# Round evidence session: GPU tests, graft smoke, bench line, rocprofv3 kernel
# trace of the bench command, PMC passes (SQ issue/stall, instruction mix,
# HBM FETCH_SIZE / WRITE_SIZE) on the C2 render kernel.  Each GPU step has its
# own time limit; a fault / abort / timeout ends the session.
#   TAG=r01 bash scripts/gpu_round.sh
set -u
cd "$(dirname "$0")/.."
TAG=${TAG:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT/pmc"
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-tests,smoke,bench,prof,pmc,rehearse}
[[ $STEPS == *tests* ]] && run pytest_gpu 900 python -m pytest tests -m gpu -q -rf
[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
[[ $STEPS == *bench* ]] && run bench 600 python bench.py
[[ $STEPS == *prof* ]] && run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline
if [[ $STEPS == *pmc* ]]; then
  run pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA -d "$OUT/pmc/sq" -o run --output-format csv -- python3 scripts/render_loop.py --frames 3
  run pmc_inst 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LEVEL_WAVES -d "$OUT/pmc/inst" -o run --output-format csv -- python3 scripts/render_loop.py --frames 3
  run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc/fetch" -o run --output-format csv -- python3 scripts/render_loop.py --frames 3
  run pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc/write" -o run --output-format csv -- python3 scripts/render_loop.py --frames 3
fi
# N=2 rehearsal on the one GPU (two ranks share cuda:0; gloo, so no RCCL duplicate-device refusal)
[[ $STEPS == *rehearse* ]] && run rehearse2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 3 --backend gloo
exit 0
