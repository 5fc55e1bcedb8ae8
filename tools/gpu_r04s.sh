#!/bin/bash
# Round-4 lock-in at the current build: full GPU suite, smoke, measurement refresh with probes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04s_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r04s_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r04s_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04s_smoke.log 2>&1 || { tail -20 gpurun_out/r04s_smoke.log; exit 1; }
tail -1 gpurun_out/r04s_smoke.log
PROBES=1 tools/refresh.sh r04s
