#!/bin/bash
# Launch + short-walk latency: the query kernels on tiny batches (back-to-back launches).
set -o pipefail
mkdir -p gpurun_out
for n in 64 4096 65536; do
timeout -k 10 300 python -u tools/query_bench.py --n $n --reps 200 --modes 4,8,5,9 > gpurun_out/r04ee_query_n$n.log 2>&1 || { tail -20 gpurun_out/r04ee_query_n$n.log; exit 1; }
grep '"mode"' gpurun_out/r04ee_query_n$n.log
done
