set -e
for v in 0 4 1; do
  DMX_RN_MB_KV=$v DMX_BENCH_BREAKDOWN=gpurun_out/bd_rn$v.json timeout -k 10 300 python bench.py --steps 50 --cpu-steps 0 --config4-steps 0 --config5-steps 0 --legs-steps 0 > gpurun_out/bench_rn$v.json 2>/dev/null
  python -c "import json;print($v, json.load(open('gpurun_out/bench_rn$v.json'))['value'])"
done
