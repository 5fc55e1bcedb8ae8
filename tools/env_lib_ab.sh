#!/bin/bash
# A/B of a setting read when the scene is uploaded (so once per process) with
# tools/knob_probe.py: VAR=RT_X VALUES="0 1" tools/env_lib_ab.sh — one process per value,
# values alternating over 3 rounds; cfg4 8-way shard and cfg2 frame ms per run; results in
# gpurun_out/envab/. (Settings read at every render: tools/knob_probe.py --sets in one process.)
set -o pipefail
VAR=${VAR:?set VAR}
mkdir -p gpurun_out/envab
for r in 1 2 3; do
  for v in ${VALUES:-0 1}; do
    env "$VAR=$v" timeout -k 10 200 python -u tools/knob_probe.py --rounds 1 --reps 2 --sets - --out gpurun_out/envab/${VAR}_${v}_$r.json > gpurun_out/envab/${VAR}_${v}_$r.log 2>&1 || { echo "$VAR=$v failed"; tail -5 gpurun_out/envab/${VAR}_${v}_$r.log; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/envab/${VAR}_${v}_$r.json'))['results']['-'];print('$VAR=$v', d['cfg4_shard_ms'], d['cfg2_ms'])"
  done
done
