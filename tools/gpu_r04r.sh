#!/bin/bash
# Camera-ahead modes: tail kernel off (now the default) / predictive, mode 2 in dense launches.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "goldens or schedules or cfg4_full or parked or cfg2_full" > gpurun_out/r04r_pytest.log 2>&1 || { tail -40 gpurun_out/r04r_pytest.log; exit 1; }
tail -2 gpurun_out/r04r_pytest.log
timeout -k 10 1000 python -u tools/knob_probe.py --sets "-" "RT_TAIL_SPEC_CAM=2" "RT_SPEC_CAM_DENSE=262144" "RT_SPEC_CAM_DENSE=65536" "RT_TAIL_SPEC_CAM=1" "RT_SPEC_CAM_SPARSE=16384" "RT_SPEC_CAM_SPARSE=65536" "RT_TAIL_ENTER=2.8" --reps 2 --rounds 2 --out gpurun_out/r04r_cam.json > gpurun_out/r04r_cam.log 2>&1 || { tail -30 gpurun_out/r04r_cam.log; exit 1; }
grep round gpurun_out/r04r_cam.log
