#!/bin/bash
# RT_HEAVY sweep (k_trace heavy class threshold, quad_visit calls; 0 = off) on the GPU box:
#   tools/heavy_sweep.sh OUT.jsonl "0 4 8 16"   (extra bench args via BENCH_ARGS)
set -o pipefail
OUT=$1; shift
for h in $1; do
  RT_HEAVY=$h timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-stats --no-roofline-pass $BENCH_ARGS > /tmp/hs.json 2> /tmp/hs.err || { echo "RT_HEAVY=$h failed"; tail -5 /tmp/hs.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('/tmp/hs.json')); print(json.dumps({'RT_HEAVY': int(sys.argv[1]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'args': sys.argv[2]}))" "$h" "$BENCH_ARGS" | tee -a $OUT
done
