#!/bin/bash
# Bench a list of library builds (make variant V=name) on the GPU box, one line each:
#   tools/variant_bench.sh OUT.jsonl name1 name2 ...   ("default" = lib/librt_hip.so)
# extra bench args via BENCH_ARGS.
set -o pipefail
OUT=$1; shift
for v in "$@"; do
  if [ "$v" = default ]; then lib=""; else lib=sycl-ray-tracing_amd/lib/librt_hip_$v.so; fi
  RT_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-stats --no-roofline-pass $BENCH_ARGS > /tmp/vb.json 2> /tmp/vb.err || { echo "variant $v failed"; tail -5 /tmp/vb.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('/tmp/vb.json')); print(json.dumps({'variant': sys.argv[1], 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'args': sys.argv[2]}))" "$v" "$BENCH_ARGS" >> $OUT
done
