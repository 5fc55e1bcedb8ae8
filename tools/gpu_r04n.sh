#!/bin/bash
# Exact-walk step budget with octet walks.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/knob_probe.py --sets "-" "RT_STEP_BUDGET=128" "RT_STEP_BUDGET=256" "RT_STEP_BUDGET=512" "RT_TAIL_ENTER=1.0" "RT_TAIL_ENTER=0.7" --reps 2 --rounds 2 --out gpurun_out/r04n_budget.json > gpurun_out/r04n_budget.log 2>&1 || { tail -30 gpurun_out/r04n_budget.log; exit 1; }
grep round gpurun_out/r04n_budget.log
