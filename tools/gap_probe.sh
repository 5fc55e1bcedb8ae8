#!/bin/bash
# Launch gaps of the wavefront loop (GPU box): rocprofv3 kernel traces of tools/floor_probe.py
# (1 / 64 / 4096 pixels, one lane, no tail kernel), summarised per stream by
# tools/rocpd_summary.py gaps. Usage: tools/gap_probe.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/gaps}
mkdir -p "$OUT"
export TMPDIR=/tmp
for px in 1 8 64; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format rocpd -d "$OUT/px$px" -o px$px -- python3 tools/floor_probe.py --px $px > "$OUT/px$px.log" 2>&1 || exit 1
  for db in $(find "$OUT/px$px" -name "*.db"); do python3 tools/rocpd_summary.py gaps "$db" "$OUT/gaps_px$px.json" > /dev/null || exit 1; done
  rm -rf "$OUT/px$px"
  tail -1 "$OUT/px$px.log"
done
