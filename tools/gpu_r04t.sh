#!/bin/bash
# Issue priority for the latency-bound waves (RT_PRIO: bit 0 k_tail, bit 1 k_trace drains).
set -o pipefail
mkdir -p gpurun_out
RT_PRIO=3 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "goldens or schedules" > gpurun_out/r04t_pytest.log 2>&1 || { tail -40 gpurun_out/r04t_pytest.log; exit 1; }
tail -1 gpurun_out/r04t_pytest.log
timeout -k 10 1000 python -u tools/knob_probe.py --sets "-" "RT_PRIO=1" "RT_PRIO=2" "RT_PRIO=3" "LANES=4" --reps 2 --rounds 2 --out gpurun_out/r04t_prio.json > gpurun_out/r04t_prio.log 2>&1 || { tail -30 gpurun_out/r04t_prio.log; exit 1; }
grep round gpurun_out/r04t_prio.log
