#!/bin/bash
# Where the cfg4 8-way shard's time goes at the round-4 build: per-iteration arrays (1 lane and
# lane 0 of 4), launch timeline, exact-walk step budget sweep.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/iter_profile.py --config cfg4 --world 8 --lanes 1 --raw --out gpurun_out/r04l_iter1 > gpurun_out/r04l_iter1.json 2> gpurun_out/r04l_iter1.err || { tail -20 gpurun_out/r04l_iter1.err; exit 1; }
timeout -k 10 300 python -u tools/iter_profile.py --config cfg4 --world 8 --lanes 4 --raw --out gpurun_out/r04l_iter4 > gpurun_out/r04l_iter4.json 2> gpurun_out/r04l_iter4.err || { tail -20 gpurun_out/r04l_iter4.err; exit 1; }
timeout -k 10 300 python -u tools/timeline.py --config cfg4 --world 8 --rank 1 --out gpurun_out/r04l_tl > gpurun_out/r04l_tl.json 2> gpurun_out/r04l_tl.err || { tail -20 gpurun_out/r04l_tl.err; exit 1; }
cat gpurun_out/r04l_tl.json | head -c 1500
timeout -k 10 600 python -u tools/knob_probe.py --sets "-" "RT_STEP_BUDGET=64" "RT_STEP_BUDGET=256" "RT_STEP_BUDGET=8192" --reps 2 --rounds 2 --out gpurun_out/r04l_budget.json > gpurun_out/r04l_budget.log 2>&1 || { tail -30 gpurun_out/r04l_budget.log; exit 1; }
grep round gpurun_out/r04l_budget.log
