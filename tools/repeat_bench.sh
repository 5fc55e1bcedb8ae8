#!/bin/bash
# The default bench line N times in a row on one box (run-to-run spread of the headline).
set -o pipefail
N=${1:-5}
mkdir -p gpurun_out
for i in $(seq $N); do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/rep_$i.json 2> gpurun_out/rep_$i.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['roofline']['frac'] if d.get('roofline') else None)" gpurun_out/rep_$i.json
done
