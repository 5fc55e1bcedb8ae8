#!/bin/bash
# Occlusion leaf trips pairing the stack-top leaf (lp) vs default: parity of both, cfg2 A/B, cfg4 8-way shard
set -o pipefail
mkdir -p gpurun_out
for v in default lp; do
  lib=""; [ "$v" != default ] && lib=sycl-ray-tracing_amd/lib/librt_hip_$v.so
  RT_HIP_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_brute.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1 || { tail -30 gpurun_out/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/pytest_$v.log)"
done
tools/ab.sh gpurun_out/ab_lp.jsonl 3 default lp || exit 1
cat gpurun_out/ab_lp.jsonl
for v in default lp; do
  lib=""; [ "$v" != default ] && lib=sycl-ray-tracing_amd/lib/librt_hip_$v.so
  RT_HIP_LIB=$lib timeout -k 10 200 python tools/shard_probe.py --config cfg4 --worlds 8 --reps 2 > gpurun_out/probelp_$v.log 2>&1 || exit 1
  echo "cfg4w8 $v $(tail -1 gpurun_out/probelp_$v.log)"
done
