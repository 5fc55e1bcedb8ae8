#!/bin/bash
# Occlusion role by rows in k_trace launches below a live count (closest role stays on quads).
set -o pipefail
mkdir -p gpurun_out
RT_ROW_BELOW_ANY=1000000000 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "goldens or cfg4_full or cfg2_full" > gpurun_out/r04ff_pytest.log 2>&1 || { tail -40 gpurun_out/r04ff_pytest.log; exit 1; }
tail -1 gpurun_out/r04ff_pytest.log
timeout -k 10 1000 python -u tools/knob_probe.py --sets "-" "RT_ROW_BELOW_ANY=65536" "RT_ROW_BELOW_ANY=262144" "RT_ROW_BELOW_ANY=1000000000" "RT_ROW_BELOW_ANY=16384" --reps 2 --rounds 2 --out gpurun_out/r04ff_rowany.json > gpurun_out/r04ff_rowany.log 2>&1 || { tail -30 gpurun_out/r04ff_rowany.log; exit 1; }
grep round gpurun_out/r04ff_rowany.log
