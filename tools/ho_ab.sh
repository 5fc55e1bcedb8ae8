#!/bin/bash
# The exact-walk hand-over test per library build (make variant V=name): LIBS="default name ..." tools/ho_ab.sh
set -o pipefail
for v in $LIBS; do
  if [ "$v" = default ]; then lib=""; else lib=sycl-ray-tracing_amd/lib/librt_hip_$v.so; fi
  RT_HIP_LIB=$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k exact_handovers -x -q -s --timeout 150 --timeout-method thread > gpurun_out/ho_$v.log 2>&1
  echo "$v: $(grep -E '^hand-overs' gpurun_out/ho_$v.log | head -1) | $(tail -1 gpurun_out/ho_$v.log)"
done
