#!/bin/bash
# rows (rt_row.h) on the GPU: correctness vs quads and the octree, the parity suite with
# rows everywhere, the query micro-benchmark, and the knob probe (cfg4 8-way shard, cfg2)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rows.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04c_rows.log 2>&1 || { tail -40 gpurun_out/r04c_rows.log; exit 1; }
tail -1 gpurun_out/r04c_rows.log
RT_ROW_BELOW=1000000000 RT_TAIL_ROWS=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_brute.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04c_parity_rows.log 2>&1 || { tail -40 gpurun_out/r04c_parity_rows.log; exit 1; }
tail -1 gpurun_out/r04c_parity_rows.log
timeout -k 10 300 python -u tools/query_bench.py --modes 4,8,5,9 --n 262144 --reps 3 > gpurun_out/r04c_query_bench.log 2>&1 || { tail -20 gpurun_out/r04c_query_bench.log; exit 1; }
cat gpurun_out/r04c_query_bench.log
timeout -k 10 900 python -u tools/knob_probe.py --sets "RT_TAIL_ROWS=0" "RT_TAIL_ROWS=1" "RT_TAIL_ROWS=1,RT_TAIL_PATHS=1" "RT_ROW_BELOW=32768" "RT_ROW_BELOW=131072" "RT_ROW_BELOW=131072,RT_TAIL_ROWS=1" --reps 2 --rounds 2 --out gpurun_out/r04c_row_probe.json > gpurun_out/r04c_row_probe.log 2>&1 || { tail -30 gpurun_out/r04c_row_probe.log; exit 1; }
grep round gpurun_out/r04c_row_probe.log
