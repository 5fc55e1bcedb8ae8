#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/iter_profile.py --config cfg4 --world 8 --lanes 1 --out gpurun_out/r04e_iter > gpurun_out/r04e_iter.json 2> gpurun_out/r04e_iter.err || { tail -20 gpurun_out/r04e_iter.err; exit 1; }
cat gpurun_out/r04e_iter.json
timeout -k 10 300 python -u tools/timeline.py --config cfg4 --world 8 --rank 1 --out gpurun_out/r04e_tl_cfg4w8 > gpurun_out/r04e_tl.json 2> gpurun_out/r04e_tl.err || { tail -20 gpurun_out/r04e_tl.err; exit 1; }
cat gpurun_out/r04e_tl.json
