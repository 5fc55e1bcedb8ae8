#!/bin/bash
# A/B of library builds (make variant V=name) with tools/knob_probe.py: LIBS="default name1 ..." tools/lib_ab.sh
# (cfg4 8-way shard and cfg2 frame per build, builds alternating over 2 rounds; results in gpurun_out/libab/)
set -o pipefail
mkdir -p gpurun_out/libab
for r in 1 2; do
  for v in ${LIBS:-default}; do
    if [ "$v" = default ]; then lib=""; else lib=sycl-ray-tracing_amd/lib/librt_hip_$v.so; fi
    RT_HIP_LIB=$lib timeout -k 10 200 python -u tools/knob_probe.py --rounds 1 --reps 2 --sets - --out gpurun_out/libab/${v}_$r.json > gpurun_out/libab/${v}_$r.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/libab/${v}_$r.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/libab/${v}_$r.json'))['results']['-'];print('$v', d['cfg4_shard_ms'], d['cfg2_ms'])"
  done
done
