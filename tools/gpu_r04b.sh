#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04b_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r04b_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r04b_pytest_gpu.log
timeout -k 10 600 python -u tools/knob_probe.py --sets "RT_TILE_H=0" "RT_TILE_H=2" "RT_TILE_H=4" "RT_TILE_H=8" --reps 2 --rounds 2 --out gpurun_out/r04b_tile_probe.json > gpurun_out/r04b_tile_probe.log 2>&1 || { tail -30 gpurun_out/r04b_tile_probe.log; exit 1; }
tail -12 gpurun_out/r04b_tile_probe.log
