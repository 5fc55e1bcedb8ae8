#!/bin/bash
# Full GPU suite + smoke on the current build, then a cfg2 bench line without the CPU leg
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_check.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_check.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_check.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
for i in 1 2; do tools/variant_bench.sh gpurun_out/check_bench.jsonl default || exit 1; done
cat gpurun_out/check_bench.jsonl
