#!/bin/bash
# k_trace's smallest grid (sparse launches) and k_step's.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/knob_probe.py --sets "-" "RT_TRACE_MIN_BLOCKS=256" "RT_TRACE_MIN_BLOCKS=64" "RT_TRACE_MIN_BLOCKS=2048" --reps 2 --rounds 2 --out gpurun_out/r04bb_minblocks.json > gpurun_out/r04bb_minblocks.log 2>&1 || { tail -30 gpurun_out/r04bb_minblocks.log; exit 1; }
grep round gpurun_out/r04bb_minblocks.log
