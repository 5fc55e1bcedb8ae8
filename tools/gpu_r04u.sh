#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/iter_profile.py --config cfg4 --world 8 --lanes 1 --out gpurun_out/r04u_iter1 > gpurun_out/r04u_iter1.json 2> gpurun_out/r04u_iter1.err || { tail -20 gpurun_out/r04u_iter1.err; exit 1; }
timeout -k 10 300 python -u tools/iter_profile.py --config cfg4 --world 8 --lanes 4 --out gpurun_out/r04u_iter4 > gpurun_out/r04u_iter4.json 2> gpurun_out/r04u_iter4.err || { tail -20 gpurun_out/r04u_iter4.err; exit 1; }
grep -o '"frame_ms[^,]*\|"kernel_ms[^}]*}\|"tail_row.*' gpurun_out/r04u_iter1.json gpurun_out/r04u_iter4.json
