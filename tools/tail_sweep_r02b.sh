#!/bin/bash
# k_tail with its path step out of line: parity, then entry threshold / occupancy sweeps (cfg2 frame, cfg4 8-way shard)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_ts.log 2>&1 || { tail -20 gpurun_out/pytest_gpu_ts.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_ts.log
O=gpurun_out/tail_sweep_b.jsonl
for i in 1 2; do
  tools/variant_bench.sh $O default o2 || exit 1
  RT_TAIL_ENTER=2 tools/variant_bench.sh $O default || exit 1
  RT_TAIL_ENTER=0.5 tools/variant_bench.sh $O default || exit 1
done
cat $O
for e in "" "RT_TAIL_ENTER=2" "RT_TAIL_ENTER=4" "RT_TAIL_LIB=o2"; do
  lib=""; [ "$e" = "RT_TAIL_LIB=o2" ] && lib=sycl-ray-tracing_amd/lib/librt_hip_o2.so && e=""
  env $e RT_HIP_LIB=$lib timeout -k 10 200 python tools/shard_probe.py --config cfg4 --worlds 8 --reps 2 > gpurun_out/probe_x.log 2>&1 || exit 1
  echo "cfg4w8 [$e] [$lib] $(tail -1 gpurun_out/probe_x.log)"
done
