#!/bin/bash
# Knob re-sweep at the current build (camera ahead off in the tail, octet exact walks).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u tools/knob_probe.py --sets "-" "RT_TAIL_ROWS=0" "RT_TAIL_ENTER=1.0" "RT_DRAIN_ROWS=4" "RT_HEAVY=4" "RT_HEAVY=10" --reps 2 --rounds 2 --out gpurun_out/r04w_knobs.json > gpurun_out/r04w_knobs.log 2>&1 || { tail -30 gpurun_out/r04w_knobs.log; exit 1; }
grep round gpurun_out/r04w_knobs.log
