#!/bin/bash
# r03: runtime knobs on the cfg4 8-way shard (rank 0 rows, one GPU): lanes, trace grid fills
set -o pipefail
for e in "X=0" "RT_LANES=2" "RT_LANES=4" "RT_TRACE_FILLS=0.5" "RT_TRACE_FILLS=2" "RT_LANES=4 RT_TRACE_FILLS=0.5"; do
  env $e timeout -k 10 200 python tools/shard_probe.py --config cfg4 --worlds 8 --reps 2 > gpurun_out/probe_k.log 2>&1 || exit 1
  echo "$e $(tail -1 gpurun_out/probe_k.log)" | tee -a gpurun_out/shard_knobs.txt
done
