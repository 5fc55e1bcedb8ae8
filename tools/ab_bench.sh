#!/bin/bash
# A/B bench on the GPU box: each argument is "label:VAR=val,VAR=val" (env for that run; RT_HIP_LIB
# selects a library build). Runs them in the order given, one JSON line each, into OUT.jsonl.
#   tools/ab_bench.sh OUT.jsonl "head:RT_HIP_LIB=sycl-ray-tracing_amd/lib/librt_hip_head.so" "new:" ...
# extra bench args via BENCH_ARGS.
set -o pipefail
OUT=$1; shift
for spec in "$@"; do
  label=${spec%%:*}; envs=${spec#*:}
  ( IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
    timeout -k 10 300 python bench.py --steps ${STEPS:-8} --warmup 1 --no-cpu-baseline --no-stats --no-roofline-pass $BENCH_ARGS > /tmp/ab.json 2> /tmp/ab.err ) || { echo "$label failed"; tail -5 /tmp/ab.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('/tmp/ab.json')); print(json.dumps({'label': sys.argv[1], 'env': sys.argv[2], 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'args': sys.argv[3]}))" "$label" "$envs" "$BENCH_ARGS" | tee -a $OUT
done
