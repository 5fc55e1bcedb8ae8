#!/bin/bash
# Cooperative occlusion drain per launch (RT_COOP_LIVE: launches of at most that many live paths):
# parity with it always on, then cfg2 A/B and the cfg4 8-way shard over thresholds
set -o pipefail
mkdir -p gpurun_out
RT_COOP_LIVE=1073741824 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_coop.log 2>&1 || { tail -30 gpurun_out/pytest_coop.log; exit 1; }
tail -1 gpurun_out/pytest_coop.log
O=gpurun_out/ab_coop.jsonl
for i in 1 2; do
  for c in -1 65536 262144 1073741824; do
    RT_COOP_LIVE=$c BENCH_ARGS="" tools/variant_bench.sh $O default || exit 1
  done
done
cat $O
for c in -1 65536 262144 1073741824; do
  RT_COOP_LIVE=$c timeout -k 10 200 python tools/shard_probe.py --config cfg4 --worlds 8 --reps 2 > gpurun_out/probe_c.log 2>&1 || exit 1
  echo "cfg4w8 coop=$c $(tail -1 gpurun_out/probe_c.log)"
done
