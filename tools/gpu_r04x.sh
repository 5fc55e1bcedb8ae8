#!/bin/bash
# Fast lane (RT_FAST_K): schedule parity (bitwise), then the shard / cfg2 A/B with 8 hardware queues.
set -o pipefail
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=8
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "schedules or goldens" > gpurun_out/r04x_pytest.log 2>&1 || { tail -40 gpurun_out/r04x_pytest.log; exit 1; }
tail -1 gpurun_out/r04x_pytest.log
timeout -k 10 1000 python -u tools/knob_probe.py --sets "-" "RT_FAST_K=192" "RT_FAST_K=384" "RT_FAST_K=192,RT_FAST_AT=0.1" "RT_FAST_K=96" --reps 2 --rounds 2 --out gpurun_out/r04x_fast.json > gpurun_out/r04x_fast.log 2>&1 || { tail -30 gpurun_out/r04x_fast.log; exit 1; }
grep round gpurun_out/r04x_fast.log
