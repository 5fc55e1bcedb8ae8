#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u tools/knob_probe.py --sets "RT_TAIL_ROWS=1,RT_TAIL_PATHS=1" "RT_TAIL_ROWS=1,RT_TAIL_PATHS=1,RT_TAIL_ENTER=2.8" "RT_TAIL_ROWS=1,RT_TAIL_PATHS=1,RT_TAIL_ENTER=0.7" "RT_TAIL_ROWS=1,RT_TAIL_PATHS=2,RT_TAIL_ENTER=2.8" "RT_TAIL_ROWS=1,RT_TAIL_PATHS=2,RT_TAIL_ENTER=0.7" "RT_TAIL_ROWS=1,RT_TAIL_PATHS=3,RT_TAIL_ENTER=1.4" "RT_TAIL_ROWS=0" --reps 2 --rounds 2 --out gpurun_out/r04d_tail_probe.json > gpurun_out/r04d_tail_probe.log 2>&1 || { tail -30 gpurun_out/r04d_tail_probe.log; exit 1; }
grep round gpurun_out/r04d_tail_probe.log
