#!/bin/bash
# RT_T2_WINDOW (relative window past the closest hit walked for the second-hit bound): 1e-3 (default), 1e-4 (w4),
# 1e-5 (w5): parity of each, traversal counters, cfg2 A/B, cfg4 8-way shard
set -o pipefail
mkdir -p gpurun_out
for v in w4 w5; do
  RT_HIP_LIB=sycl-ray-tracing_amd/lib/librt_hip_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1 || { tail -30 gpurun_out/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/pytest_$v.log)"
done
for v in default w4 w5; do
  lib=""; [ "$v" != default ] && lib=sycl-ray-tracing_amd/lib/librt_hip_$v.so
  RT_HIP_LIB=$lib timeout -k 10 200 python tools/window_stats.py > gpurun_out/wstats_$v.json 2> /dev/null || exit 1
  cat gpurun_out/wstats_$v.json
done
tools/ab.sh gpurun_out/ab_window.jsonl 2 default w4 w5 || exit 1
cat gpurun_out/ab_window.jsonl
for v in default w4 w5; do
  lib=""; [ "$v" != default ] && lib=sycl-ray-tracing_amd/lib/librt_hip_$v.so
  RT_HIP_LIB=$lib timeout -k 10 200 python tools/shard_probe.py --config cfg4 --worlds 8 --reps 2 > gpurun_out/probe_$v.log 2>&1 || exit 1
  echo "cfg4w8 $v $(tail -1 gpurun_out/probe_$v.log)"
done
