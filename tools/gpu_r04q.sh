#!/bin/bash
# Camera-ahead policies: off in the tail kernel (RT_TAIL_SPEC_CAM=0), only where the pixel's
# previous sample ended (RT_SPEC_CAM=2): parity (goldens + schedules) and the shard / cfg2 A/B;
# counters of one cfg2 / cfg4-shard render.
set -o pipefail
mkdir -p gpurun_out
RT_TAIL_SPEC_CAM=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "goldens or schedules or cfg4_full or parked" > gpurun_out/r04q_pytest.log 2>&1 || { tail -40 gpurun_out/r04q_pytest.log; exit 1; }
tail -2 gpurun_out/r04q_pytest.log
RT_SPEC_CAM=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "goldens or cfg4_full or cfg2_full" > gpurun_out/r04q_pytest2.log 2>&1 || { tail -40 gpurun_out/r04q_pytest2.log; exit 1; }
tail -2 gpurun_out/r04q_pytest2.log
timeout -k 10 300 python -u tools/stats_probe.py --config cfg2 > gpurun_out/r04q_stats_cfg2.json 2>&1 && timeout -k 10 300 python -u tools/stats_probe.py --config cfg4 --world 8 > gpurun_out/r04q_stats_cfg4w8.json 2>&1 || exit 1
tail -c 400 gpurun_out/r04q_stats_cfg2.json gpurun_out/r04q_stats_cfg4w8.json
timeout -k 10 1000 python -u tools/knob_probe.py --sets "-" "RT_TAIL_SPEC_CAM=0" "RT_SPEC_CAM=2" "RT_SPEC_CAM=2,RT_TAIL_SPEC_CAM=0" --reps 2 --rounds 2 --out gpurun_out/r04q_cam.json > gpurun_out/r04q_cam.log 2>&1 || { tail -30 gpurun_out/r04q_cam.log; exit 1; }
grep round gpurun_out/r04q_cam.log
