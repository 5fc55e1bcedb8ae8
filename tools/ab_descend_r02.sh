#!/bin/bash
# k_trace / k_tail inner trips per quad_visit call (RT_VISIT_DESCEND 1 / 2 default / 3) with paired occlusion trips: cfg2 A/B
set -o pipefail
mkdir -p gpurun_out
tools/ab.sh gpurun_out/ab_descend.jsonl 2 default d1 d3 || exit 1
cat gpurun_out/ab_descend.jsonl
