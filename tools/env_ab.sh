#!/bin/bash
# Bench one library under several environment settings: tools/env_ab.sh OUT.jsonl "ENV=1 ENV2=x" "ENV=2" ...
# ("-" = no extra env); extra bench args via BENCH_ARGS.
set -o pipefail
OUT=$1; shift
for e in "$@"; do
  [ "$e" = "-" ] && e=""
  env $e timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-stats --no-roofline-pass $BENCH_ARGS > /tmp/ea.json 2> /tmp/ea.err || { echo "setting '$e' failed"; tail -5 /tmp/ea.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('/tmp/ea.json')); print(json.dumps({'env': sys.argv[1], 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'args': sys.argv[2]}))" "$e" "$BENCH_ARGS" >> $OUT
done
