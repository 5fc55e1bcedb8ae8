#!/bin/bash
# LLVM scheduling strategies for the whole kernel library (max-ILP, max-memory-clause) vs default.
set -o pipefail
mkdir -p gpurun_out
L=sycl-ray-tracing_amd/lib
for v in ilp mclause; do
RT_HIP_LIB=$L/librt_hip_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "goldens" > gpurun_out/r04aa_pytest_$v.log 2>&1 || { tail -30 gpurun_out/r04aa_pytest_$v.log; exit 1; }
tail -1 gpurun_out/r04aa_pytest_$v.log
done
for round in 1 2; do
timeout -k 10 300 python -u tools/knob_probe.py --sets "-" --reps 2 --rounds 1 --out gpurun_out/r04aa_base_$round.json > gpurun_out/r04aa_base_$round.log 2>&1 || exit 1
grep round gpurun_out/r04aa_base_$round.log
for v in ilp mclause; do
RT_HIP_LIB=$L/librt_hip_$v.so timeout -k 10 300 python -u tools/knob_probe.py --sets "-" --reps 2 --rounds 1 --out gpurun_out/r04aa_${v}_$round.json > gpurun_out/r04aa_${v}_$round.log 2>&1 || exit 1
echo $v; grep round gpurun_out/r04aa_${v}_$round.log
done
done
