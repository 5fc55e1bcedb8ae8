#!/bin/bash
# r03: k_tail entry threshold (RT_TAIL_ENTER scales the live count at which a lane enters the
# tail kernel) with the camera-ahead steps: cfg2 and the cfg4 8-way shard
set -o pipefail
SET=${SET:-"RT_TAIL_ENTER=1 RT_TAIL_ENTER=0.8 RT_TAIL_ENTER=0.6 RT_TAIL_ENTER=0.4"}
for i in 1 2; do
  for e in $SET; do
    env $e tools/variant_bench.sh gpurun_out/ab_tail.jsonl default || exit 1
    sed -i '$ s/"args": ""/"args": "'"$e"'"/' gpurun_out/ab_tail.jsonl
  done
done
cat gpurun_out/ab_tail.jsonl
for e in $SET; do
  env $e timeout -k 10 200 python tools/shard_probe.py --config cfg4 --worlds 8 --reps 2 > gpurun_out/probe_tail.log 2>&1 || exit 1
  echo "$e $(tail -1 gpurun_out/probe_tail.log)"
done
