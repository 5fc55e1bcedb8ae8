#!/bin/bash
# Round-3 GPU check: the GPU suite, smoke, then the cfg5 replica sweep (one GPU: the
# N = 8 share and the whole sweep) and a two-rank torchrun rehearsal of the N > 1 line
# (gloo, both ranks on GPU 0) with its strong_cfg4 object. Results under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
if [ -n "$SWEEP" ]; then
  timeout -k 10 300 python -u bench.py --config cfg5sweep --sim-world 8 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/sweep_sim8.json 2> gpurun_out/sweep_sim8.err || { tail -20 gpurun_out/sweep_sim8.err; exit 1; }
  cat gpurun_out/sweep_sim8.json
  timeout -k 10 400 python -u bench.py --config cfg5sweep --steps 1 --warmup 0 > gpurun_out/sweep_1gpu.json 2> gpurun_out/sweep_1gpu.err || { tail -20 gpurun_out/sweep_1gpu.err; exit 1; }
  cat gpurun_out/sweep_1gpu.json
fi
if [ -n "$REHEARSE" ]; then
  RT_BENCH_DEVICE_MOD=1 RT_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 1 --no-stats --no-roofline-pass > gpurun_out/rehearse_n2.json 2> gpurun_out/rehearse_n2.err || { tail -30 gpurun_out/rehearse_n2.err; exit 1; }
  cat gpurun_out/rehearse_n2.json
fi
