#!/bin/bash
# Closest-hit walks taking the stack top's node in the same trip (variant pair, RT_CLOSEST_PAIR=1): parity, counters, cfg2 A/B, cfg4 8-way shard
set -o pipefail
mkdir -p gpurun_out
L=sycl-ray-tracing_amd/lib/librt_hip_cpair.so
RT_HIP_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_brute.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_cpair.log 2>&1 || { tail -30 gpurun_out/pytest_cpair.log; exit 1; }
echo "cpair $(tail -1 gpurun_out/pytest_cpair.log)"
RT_HIP_LIB=$L timeout -k 10 200 python tools/window_stats.py > gpurun_out/wstats_cpair.json 2> /dev/null || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/wstats_cpair.json'))['stats']; print({k: d[k] for k in ('vol','tri','any_vol','verify','fallback','quad_visits','drain_slots','drain_visits','wave_slots')})"
tools/ab.sh gpurun_out/ab_cpair.jsonl 3 default cpair || exit 1
cat gpurun_out/ab_cpair.jsonl
for v in default cpair; do
  lib=""; [ "$v" != default ] && lib=$L
  RT_HIP_LIB=$lib timeout -k 10 200 python tools/shard_probe.py --config cfg4 --worlds 8 --reps 2 > gpurun_out/probec_$v.log 2>&1 || exit 1
  echo "cfg4w8 $v $(tail -1 gpurun_out/probec_$v.log)"
done
