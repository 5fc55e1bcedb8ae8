#!/bin/bash
# Tail kernel: camera rays ahead that a round waits for only when the next step reads them.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "schedules or goldens or cfg4_full" > gpurun_out/r04cc_pytest.log 2>&1 || { tail -40 gpurun_out/r04cc_pytest.log; exit 1; }
tail -1 gpurun_out/r04cc_pytest.log
timeout -k 10 1000 python -u tools/knob_probe.py --sets "-" "RT_TAIL_SPEC_CAM=1,RT_TAIL_CAM_ASYNC=1" "RT_TAIL_SPEC_CAM=2,RT_TAIL_CAM_ASYNC=1" "RT_TAIL_SPEC_CAM=1" --reps 2 --rounds 2 --out gpurun_out/r04cc_camasync.json > gpurun_out/r04cc_camasync.log 2>&1 || { tail -30 gpurun_out/r04cc_camasync.log; exit 1; }
grep round gpurun_out/r04cc_camasync.log
