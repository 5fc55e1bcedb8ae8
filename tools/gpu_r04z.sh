#!/bin/bash
# Final check at the round's last build: full GPU suite, smoke, cfg2 bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04z_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r04z_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r04z_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04z_smoke.log 2>&1 || { tail -20 gpurun_out/r04z_smoke.log; exit 1; }
tail -1 gpurun_out/r04z_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r04z_bench_cfg2.json 2> gpurun_out/r04z_bench_cfg2.err || { tail -20 gpurun_out/r04z_bench_cfg2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r04z_bench_cfg2.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], d['build'], r['frac'], r['traffic_source']['same_build'], d['parity'])"
