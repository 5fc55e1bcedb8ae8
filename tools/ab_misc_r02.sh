#!/bin/bash
# k_step exact-walk roles out of line (xr), top-64 search-BVH nodes staged in LDS (top64) vs default: cfg2 A/B, cfg4 8-way shard
set -o pipefail
mkdir -p gpurun_out
tools/ab.sh gpurun_out/ab_misc.jsonl 2 default xr top64 || exit 1
cat gpurun_out/ab_misc.jsonl
for v in default xr top64; do
  lib=""; [ "$v" != default ] && lib=sycl-ray-tracing_amd/lib/librt_hip_$v.so
  RT_HIP_LIB=$lib timeout -k 10 200 python tools/shard_probe.py --config cfg4 --worlds 8 --reps 2 > gpurun_out/probe_$v.log 2>&1 || exit 1
  echo "cfg4w8 $v $(tail -1 gpurun_out/probe_$v.log)"
done
