#!/bin/bash
# r03: the next sample's camera ray traced ahead (RT_SPEC_CAM) against the build before this
# round's changes ("pre"), cfg2 A/B, then the cfg4 8-way shard (rank 0); GPU suite first.
set -o pipefail
bash tools/check_gpu.sh || exit 1
for i in 1 2; do
  tools/variant_bench.sh gpurun_out/ab_spec.jsonl default pre || exit 1
  RT_SPEC_CAM=0 tools/variant_bench.sh gpurun_out/ab_spec.jsonl default || exit 1
  RT_TAIL_PATHS=4 tools/variant_bench.sh gpurun_out/ab_spec.jsonl default || exit 1
done
cat gpurun_out/ab_spec.jsonl
for e in "RT_SPEC_CAM=1" "RT_SPEC_CAM=0" "RT_TAIL_PATHS=4"; do
  env $e timeout -k 10 200 python tools/shard_probe.py --config cfg4 --worlds 1,8 --reps 1 > gpurun_out/probe_spec.log 2>&1 || exit 1
  echo "$e $(tail -1 gpurun_out/probe_spec.log)"
done
