#!/bin/bash
# Measurement refresh (GPU box): tools/refresh.sh ROOFDIR. Roofline roofline profiles (trace, FETCH, WRITE, SQ/TCC counters),
# traffic.json, cfg2 / cfg3 bench lines, strong-scaling shard probes.
set -o pipefail
R=${1:-r02_roof_i}
mkdir -p gpurun_out
PMC_DETAIL=1 tools/profile_roofline.sh gpurun_out/$R --config cfg2 || exit 1
python3 tools/update_traffic.py gpurun_out/$R --build "$(cat BUILD_COMMIT 2>/dev/null)" || exit 1
cp profiles/traffic.json gpurun_out/traffic.json
timeout -k 10 300 python -u bench.py > gpurun_out/bench_cfg2.json 2> gpurun_out/bench_cfg2.err || exit 1
cat gpurun_out/bench_cfg2.json
timeout -k 10 300 python -u bench.py --config cfg3 > gpurun_out/bench_cfg3.json 2> gpurun_out/bench_cfg3.err || exit 1
for c in cfg2 cfg4 cfg5; do
  timeout -k 10 240 python -u tools/shard_probe.py --config $c --worlds 1,2,4,8 --reps 1 > gpurun_out/probe_$c.log 2>&1 || exit 1
  tail -1 gpurun_out/probe_$c.log
done
