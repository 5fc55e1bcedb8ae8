#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
L=sycl-ray-tracing_amd/lib
timeout -k 10 600 python -u tools/knob_probe.py --sets "-" "RT_DRAIN_ROWS=1" "RT_DRAIN_ROWS=3" "RT_TAIL_ENTER=2.8" --reps 2 --rounds 2 --out gpurun_out/r04j_probe.json > gpurun_out/r04j_probe.log 2>&1 || { tail -30 gpurun_out/r04j_probe.log; exit 1; }
grep round gpurun_out/r04j_probe.log
RT_HIP_LIB=$L/librt_hip_tocc4.so timeout -k 10 400 python -u tools/knob_probe.py --sets "-" "RT_TAIL_ENTER=2.8" "RT_TAIL_ENTER=4.2" --reps 2 --rounds 2 --out gpurun_out/r04j_tocc4.json > gpurun_out/r04j_tocc4.log 2>&1 || { tail -30 gpurun_out/r04j_tocc4.log; exit 1; }
grep round gpurun_out/r04j_tocc4.log
timeout -k 10 600 python -u tools/shard_probe.py --config cfg4 --worlds 1,2,4,8 --reps 1 --all-ranks > gpurun_out/r04j_scaling_cfg4.log 2>&1 || { tail -30 gpurun_out/r04j_scaling_cfg4.log; exit 1; }
tail -3 gpurun_out/r04j_scaling_cfg4.log
