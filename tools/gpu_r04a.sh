#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04a_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r04a_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r04a_pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/r04a_bench_cfg2.json 2> gpurun_out/r04a_bench_cfg2.err || { tail -30 gpurun_out/r04a_bench_cfg2.err; exit 1; }
cat gpurun_out/r04a_bench_cfg2.json
RT_BENCH_LOOPBACK=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 1 --warmup 1 --no-stats --no-roofline-pass > gpurun_out/r04a_rehearse_loopback_n2.json 2> gpurun_out/r04a_rehearse_loopback_n2.err || { tail -30 gpurun_out/r04a_rehearse_loopback_n2.err; exit 1; }
cat gpurun_out/r04a_rehearse_loopback_n2.json
RT_BENCH_DEVICE_MOD=1 RT_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 1 --no-stats --no-roofline-pass > gpurun_out/r04a_rehearse_torchrun_n2.json 2> gpurun_out/r04a_rehearse_torchrun_n2.err || { tail -30 gpurun_out/r04a_rehearse_torchrun_n2.err; exit 1; }
cat gpurun_out/r04a_rehearse_torchrun_n2.json
