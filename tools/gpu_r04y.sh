#!/bin/bash
# Fast lane with the default 4 hardware queues (its stream shares one with a lane).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/knob_probe.py --sets "-" "RT_FAST_K=96" "RT_FAST_K=192" --reps 2 --rounds 2 --out gpurun_out/r04y_fast.json > gpurun_out/r04y_fast.log 2>&1 || { tail -30 gpurun_out/r04y_fast.log; exit 1; }
grep round gpurun_out/r04y_fast.log
GPU_MAX_HW_QUEUES=8 timeout -k 10 600 python -u tools/knob_probe.py --sets "-" --reps 2 --rounds 1 --out gpurun_out/r04y_hwq8.json > gpurun_out/r04y_hwq8.log 2>&1 || { tail -30 gpurun_out/r04y_hwq8.log; exit 1; }
grep round gpurun_out/r04y_hwq8.log
