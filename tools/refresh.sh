#!/bin/bash
# Measurement refresh (GPU box): tools/refresh.sh TAG. Roofline profiles of the cfg2 1-lane
# command (trace, FETCH, WRITE, SQ/TCC counters) into gpurun_out/TAG_roof, traffic.json,
# the cfg2 / cfg3 bench lines, and the strong-scaling shard probes (every rank).
set -o pipefail
T=${1:-r03}
mkdir -p gpurun_out
PMC_DETAIL=1 tools/profile_roofline.sh gpurun_out/${T}_roof --config cfg2 || exit 1
python3 tools/update_traffic.py gpurun_out/${T}_roof --build "$(cat BUILD_COMMIT 2>/dev/null)" --commit-dir profiles/${T}_roof || exit 1
cp profiles/traffic.json gpurun_out/traffic.json  # (then copy gpurun_out/${T}_roof to profiles/${T}_roof, the path it records)
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench_cfg2.json 2> gpurun_out/${T}_bench_cfg2.err || exit 1
cat gpurun_out/${T}_bench_cfg2.json
timeout -k 10 300 python -u bench.py --config cfg3 > gpurun_out/${T}_bench_cfg3.json 2> gpurun_out/${T}_bench_cfg3.err || exit 1
if [ -n "$PROBES" ]; then
  for c in cfg2 cfg4 cfg5; do
    timeout -k 10 600 python -u tools/shard_probe.py --config $c --worlds 1,2,4,8 --reps 1 --all-ranks > gpurun_out/${T}_probe_$c.log 2>&1 || exit 1
    tail -1 gpurun_out/${T}_probe_$c.log
  done
fi
