#!/bin/bash
# k_tail inner-node trips per quad_visit call (RT_TAIL_DESCEND 2 = default, 4, 8): cfg2 A/B and the cfg4 8-way shard
set -o pipefail
mkdir -p gpurun_out
tools/ab.sh gpurun_out/ab_td.jsonl 2 default td4 td8 || exit 1
cat gpurun_out/ab_td.jsonl
for v in default td4 td8; do
  lib=""; [ "$v" != default ] && lib=sycl-ray-tracing_amd/lib/librt_hip_$v.so
  RT_HIP_LIB=$lib timeout -k 10 200 python tools/shard_probe.py --config cfg4 --worlds 8 --reps 2 > gpurun_out/probe_$v.log 2>&1 || exit 1
  echo "cfg4w8 $v $(tail -1 gpurun_out/probe_$v.log)"
done
