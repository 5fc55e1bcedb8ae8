#!/bin/bash
# Wave walks (rt_coop.h): row-walk tests (+ wave modes), the schedule parity test, query bench,
# A/B of RT_COOP bits and of k_trace built without the coop code.
set -o pipefail
mkdir -p gpurun_out
L=sycl-ray-tracing_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04p_pytest.log 2>&1 || { tail -40 gpurun_out/r04p_pytest.log; exit 1; }
tail -2 gpurun_out/r04p_pytest.log
timeout -k 10 300 python -u tools/query_bench.py --modes 4,8,10,5,9,11 > gpurun_out/r04p_query.log 2>&1 || { tail -20 gpurun_out/r04p_query.log; exit 1; }
cat gpurun_out/r04p_query.log
timeout -k 10 900 python -u tools/knob_probe.py --sets "-" "RT_COOP=0" "RT_COOP=1" "RT_COOP=2" --reps 2 --rounds 2 --out gpurun_out/r04p_coop.json > gpurun_out/r04p_coop.log 2>&1 || { tail -30 gpurun_out/r04p_coop.log; exit 1; }
grep round gpurun_out/r04p_coop.log
RT_HIP_LIB=$L/librt_hip_nocooptr.so timeout -k 10 400 python -u tools/knob_probe.py --sets "RT_COOP=1" "RT_COOP=0" --reps 2 --rounds 2 --out gpurun_out/r04p_nocooptr.json > gpurun_out/r04p_nocooptr.log 2>&1 || { tail -30 gpurun_out/r04p_nocooptr.log; exit 1; }
grep round gpurun_out/r04p_nocooptr.log
