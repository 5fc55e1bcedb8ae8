#!/bin/bash
# drain rows (parity + probe), then the tail kernel at 4 waves/SIMD (variant library)
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_r04g.sh || exit 1
L=sycl-ray-tracing_amd/lib
for lib in librt_hip.so librt_hip_tocc4.so; do
  RT_HIP_LIB=$L/$lib timeout -k 10 600 python -u tools/knob_probe.py --sets "RT_TAIL_ENTER=1.4" "RT_TAIL_ENTER=2.8" "RT_TAIL_ENTER=4.2" --reps 2 --rounds 1 --out gpurun_out/r04h_tocc_$lib.json > gpurun_out/r04h_tocc_$lib.log 2>&1 || { tail -20 gpurun_out/r04h_tocc_$lib.log; exit 1; }
  echo $lib; grep round gpurun_out/r04h_tocc_$lib.log
done
