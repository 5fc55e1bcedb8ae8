#!/bin/bash
# Octet exact walks (rt_octet.h): full GPU suite, A/B against the one-lane exact walks, iteration profile.
set -o pipefail
mkdir -p gpurun_out
L=sycl-ray-tracing_amd/lib
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04m_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r04m_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r04m_pytest_gpu.log
timeout -k 10 300 python -u tools/iter_profile.py --config cfg4 --world 8 --lanes 1 --raw --out gpurun_out/r04m_iter1 > gpurun_out/r04m_iter1.json 2> gpurun_out/r04m_iter1.err || { tail -20 gpurun_out/r04m_iter1.err; exit 1; }
timeout -k 10 400 python -u tools/knob_probe.py --sets "-" --reps 2 --rounds 2 --out gpurun_out/r04m_octet.json > gpurun_out/r04m_octet.log 2>&1 || { tail -30 gpurun_out/r04m_octet.log; exit 1; }
grep round gpurun_out/r04m_octet.log
RT_HIP_LIB=$L/librt_hip_exact1.so timeout -k 10 400 python -u tools/knob_probe.py --sets "-" --reps 2 --rounds 2 --out gpurun_out/r04m_exact1.json > gpurun_out/r04m_exact1.log 2>&1 || { tail -30 gpurun_out/r04m_exact1.log; exit 1; }
grep round gpurun_out/r04m_exact1.log
