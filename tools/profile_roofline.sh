#!/bin/bash
# The roofline command under rocprofv3 (GPU box): `bench.py --roofline-only` renders
# the frame once with the stats kernels (counter pass), then twice with ONE lane
# (warm + timed), so the k_trace<false, false> dispatches in these profiles are exactly
# the 1-lane launches whose mean duration bench.py's roofline line reports.
# Usage: tools/profile_roofline.sh OUTDIR [bench args...]
set -o pipefail
OUT=${1:-gpurun_out/roof}; shift
ARGS=${@:---config cfg2}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$name" -o "$name" -- python3 bench.py --roofline-only --no-cpu-baseline $ARGS > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"
  for db in $(find "$OUT/$name" -name "*.db"); do
    if [ "$name" = trace ]; then python3 tools/rocpd_summary.py trace "$db" > "$OUT/$name.summary.txt" 2>&1
    else python3 tools/rocpd_summary.py pmc "$db" > "$OUT/$name.summary.txt" 2>&1
         python3 tools/rocpd_summary.py pmcjson "$OUT/$name.json" "$db" > /dev/null 2>&1; fi
  done
  for f in $(find "$OUT/$name" -name "*kernel_stats.csv"); do cp "$f" "$OUT/$name.kernel_stats.csv"; done
  rm -rf "$OUT/$name"
  return $rc
}
run trace --kernel-trace --stats --output-format csv rocpd || exit 1
run pmc_fetch --pmc FETCH_SIZE || exit 1
run pmc_write --pmc WRITE_SIZE || exit 1
# occupancy / issue / wait counters of the same command (one pass each)
if [ -n "$PMC_DETAIL" ]; then
  run pmc_a --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU || exit 1
  run pmc_b --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_THREAD_CYCLES_VALU SQ_LEVEL_WAVES SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT || exit 1
  run pmc_c --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE TCP_PENDING_STALL_CYCLES_sum || exit 1
fi
