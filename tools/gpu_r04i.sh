#!/bin/bash
# drain rows (parity + probe); trace occupancy 7 / 8 and tail occupancy 4 (variant libraries)
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_r04g.sh || exit 1
L=sycl-ray-tracing_amd/lib
for lib in librt_hip.so librt_hip_trocc7.so librt_hip_trocc8.so librt_hip_tocc4.so librt_hip.so; do
  RT_HIP_LIB=$L/$lib timeout -k 10 300 python -u tools/knob_probe.py --sets "-" --reps 2 --rounds 1 --out gpurun_out/r04i_$lib.json > gpurun_out/r04i_$lib.log 2>&1 || { tail -20 gpurun_out/r04i_$lib.log; exit 1; }
  echo $lib $(grep round gpurun_out/r04i_$lib.log)
done
RT_HIP_LIB=$L/librt_hip_tocc4.so timeout -k 10 300 python -u tools/knob_probe.py --sets "RT_TAIL_ENTER=2.8" --reps 2 --rounds 1 --out gpurun_out/r04i_tocc4_e28.json > gpurun_out/r04i_tocc4_e28.log 2>&1 && echo tocc4_e28 $(grep round gpurun_out/r04i_tocc4_e28.log)
