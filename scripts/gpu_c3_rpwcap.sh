set -u
OUT=gpurun_out/rpwcap; mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 300 python scripts/render_loop.py --scene 11-01-refractive__scene8 --depth 8 --frames 8 --opt wf_rpw=32,40,48,56,64 > $OUT/r$r.log 2>&1 || exit 1
  tail -1 $OUT/r$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['kernel']; [print($r, k, round(v['median_ms'],4)) for k,v in d.items()]"
done
