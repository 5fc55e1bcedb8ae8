#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
RT_HEAVY_ROWS=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "schedules or goldens or parked or cfg2_full" > gpurun_out/r04f_parity_heavyrows.log 2>&1 || { tail -40 gpurun_out/r04f_parity_heavyrows.log; exit 1; }
tail -1 gpurun_out/r04f_parity_heavyrows.log
timeout -k 10 1000 python -u tools/knob_probe.py --sets "RT_HEAVY_ROWS=0" "RT_HEAVY_ROWS=1" "RT_HEAVY_ROWS=1,RT_HEAVY=10" "RT_HEAVY_ROWS=1,RT_HEAVY=16" "RT_HEAVY_ROWS=1,RT_HEAVY=4" --reps 2 --rounds 2 --out gpurun_out/r04f_heavyrows_probe.json > gpurun_out/r04f_heavyrows_probe.log 2>&1 || { tail -30 gpurun_out/r04f_heavyrows_probe.log; exit 1; }
grep round gpurun_out/r04f_heavyrows_probe.log
