#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "rows or schedules or goldens or parked or cfg2_full" > gpurun_out/r04g_parity.log 2>&1 || { tail -40 gpurun_out/r04g_parity.log; exit 1; }
tail -1 gpurun_out/r04g_parity.log
timeout -k 10 1000 python -u tools/knob_probe.py --sets "RT_DRAIN_ROWS=0" "RT_DRAIN_ROWS=4" "RT_DRAIN_ROWS=2" "RT_DRAIN_ROWS=1" --reps 2 --rounds 2 --out gpurun_out/r04g_drain_probe.json > gpurun_out/r04g_drain_probe.log 2>&1 || { tail -30 gpurun_out/r04g_drain_probe.log; exit 1; }
grep round gpurun_out/r04g_drain_probe.log
