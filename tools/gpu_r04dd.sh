#!/bin/bash
# N = 2 rehearsals on one GPU at the round's last build: the one-process driver over the loopback
# exchange, and two torchrun ranks (gloo) sharing the GPU.
set -o pipefail
mkdir -p gpurun_out
RT_BENCH_LOOPBACK=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 1 --warmup 1 --no-stats --no-roofline-pass > gpurun_out/r04dd_rehearse_loopback_n2.json 2> gpurun_out/r04dd_rehearse_loopback_n2.err || { tail -30 gpurun_out/r04dd_rehearse_loopback_n2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r04dd_rehearse_loopback_n2.json')); print(d['value'], d.get('parity'), d.get('strong_cfg4',{}).get('bitwise'), d['build'])"
RT_BENCH_DEVICE_MOD=1 RT_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 1 --no-stats --no-roofline-pass > gpurun_out/r04dd_rehearse_torchrun_n2.json 2> gpurun_out/r04dd_rehearse_torchrun_n2.err || { tail -30 gpurun_out/r04dd_rehearse_torchrun_n2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r04dd_rehearse_torchrun_n2.json')); print(d['value'], d.get('parity'), d.get('strong_cfg4',{}).get('bitwise'), d['build'])"
