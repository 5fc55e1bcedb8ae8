#!/bin/bash
# k_trace box test with fused multiply-adds (variant fma) vs default: parity of the variant, then A/B on cfg2
set -o pipefail
mkdir -p gpurun_out
RT_HIP_LIB=sycl-ray-tracing_amd/lib/librt_hip_fma.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fma.log 2>&1 || { tail -20 gpurun_out/pytest_fma.log; exit 1; }
tail -1 gpurun_out/pytest_fma.log
tools/ab.sh gpurun_out/ab_fma.jsonl 3 default fma || exit 1
RT_TAIL_PATHS=4 tools/variant_bench.sh gpurun_out/ab_fma.jsonl default || exit 1
RT_TAIL_PATHS=6 tools/variant_bench.sh gpurun_out/ab_fma.jsonl default || exit 1
cat gpurun_out/ab_fma.jsonl
