#!/bin/bash
# rocprofv3 passes over a bench run (GPU box). Usage: tools/profile_gpu.sh OUTDIR [bench args...]
# Pass 0: kernel trace + stats. Passes 1..: PMC counters, each in its own run
# (never combined with tracing domains; at most 8 SQ / 4 TCC counters per pass).
set -o pipefail
OUT=${1:-gpurun_out/prof}; shift
ARGS=${@:---config cfg2s --steps 1 --warmup 0 --no-cpu-baseline --no-stats}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() { # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$name" -o "$name" -- python3 bench.py $ARGS > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"
  # keep only text summaries (the sqlite files of long runs exceed what gpurun copies back)
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
run pmc1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU || exit 1
run pmc2 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_THREAD_CYCLES_VALU SQ_LEVEL_WAVES SQ_INSTS_VALU_FLOPS_FP64 SQ_LDS_BANK_CONFLICT || exit 1
run pmc3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE TCP_PENDING_STALL_CYCLES_sum || exit 1
run pmc4 --pmc FETCH_SIZE || exit 1
