#!/bin/bash
# Inner trips per row_visit call in the tail kernel (RT_TAIL_DESCEND, default 2).
set -o pipefail
mkdir -p gpurun_out
L=sycl-ray-tracing_amd/lib
for round in 1 2; do
timeout -k 10 300 python -u tools/knob_probe.py --sets "-" --reps 2 --rounds 1 --out gpurun_out/r04gg_base_$round.json > gpurun_out/r04gg_base_$round.log 2>&1 || exit 1
grep '"round"' gpurun_out/r04gg_base_$round.log
for d in 1 3 4; do
RT_HIP_LIB=$L/librt_hip_td$d.so timeout -k 10 300 python -u tools/knob_probe.py --sets "-" --reps 2 --rounds 1 --out gpurun_out/r04gg_td${d}_$round.json > gpurun_out/r04gg_td${d}_$round.log 2>&1 || exit 1
echo td$d; grep '"round"' gpurun_out/r04gg_td${d}_$round.log
done
done
