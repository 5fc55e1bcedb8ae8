#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/qab
for r in 1 2 3; do
  for q in 0 1; do
    RT_QBVH=$q timeout -k 10 200 python -u tools/knob_probe.py --rounds 1 --reps 2 --sets - --out gpurun_out/qab/q${q}_$r.json > gpurun_out/qab/q${q}_$r.log 2>&1 || { echo "q=$q failed"; tail -5 gpurun_out/qab/q${q}_$r.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/qab/q${q}_$r.json'))['results']['-'];print('qbvh=$q', d['cfg4_shard_ms'], d['cfg2_ms'])"
  done
done
