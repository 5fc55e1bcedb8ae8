#!/bin/bash
# Iteration floor: k_trace + k_step over 1 / 64 / 4096 paths (tail kernel off, one lane).
set -o pipefail
mkdir -p gpurun_out
for px in 1 8 64; do
timeout -k 10 300 python -u tools/floor_probe.py --px $px --spp 64 > gpurun_out/r04ii_floor_px$px.json 2> gpurun_out/r04ii_floor_px$px.err || { tail -20 gpurun_out/r04ii_floor_px$px.err; exit 1; }
cat gpurun_out/r04ii_floor_px$px.json
done
