#!/bin/bash
# drain rows + host polling (parity + probes); trace occupancy 7 / 8 and tail occupancy 4 (variant libraries)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "rows or schedules or goldens or parked or cfg2_full" > gpurun_out/r04i_parity.log 2>&1 || { tail -40 gpurun_out/r04i_parity.log; exit 1; }
tail -1 gpurun_out/r04i_parity.log
timeout -k 10 900 python -u tools/knob_probe.py --sets "RT_HOST_BLOCKING=1,RT_DRAIN_ROWS=0" "RT_DRAIN_ROWS=0" "RT_DRAIN_ROWS=4" "RT_DRAIN_ROWS=2" --reps 2 --rounds 2 --out gpurun_out/r04i_drain_probe.json > gpurun_out/r04i_drain_probe.log 2>&1 || { tail -30 gpurun_out/r04i_drain_probe.log; exit 1; }
grep round gpurun_out/r04i_drain_probe.log
L=sycl-ray-tracing_amd/lib
for lib in librt_hip_trocc7.so librt_hip_trocc8.so librt_hip_tocc4.so; do
  RT_HIP_LIB=$L/$lib timeout -k 10 300 python -u tools/knob_probe.py --sets "RT_DRAIN_ROWS=0" --reps 2 --rounds 1 --out gpurun_out/r04i_$lib.json > gpurun_out/r04i_$lib.log 2>&1 || { tail -20 gpurun_out/r04i_$lib.log; exit 1; }
  echo $lib $(grep round gpurun_out/r04i_$lib.log)
done
