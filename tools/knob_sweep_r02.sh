#!/bin/bash
# Runtime knobs re-swept at the current build (cfg2, alternating with the default)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/knobs.jsonl
for i in 1 2; do
  for e in "X=0" "RT_TRACE_FILLS=0.75" "RT_TRACE_FILLS=1.25" "RT_LANES=2" "RT_LANES=4" "RT_HEAVY=4" "RT_HEAVY=8"; do
    env $e tools/variant_bench.sh $O default || exit 1
    sed -i '$ s/"args": ""/"args": "'"$e"'"/' $O
  done
done
cat $O
