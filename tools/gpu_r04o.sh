#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
RT_COOP=0 timeout -k 10 300 python -u tools/iter_profile.py --config cfg4 --world 8 --lanes 1 --out gpurun_out/r04o_iter1 > gpurun_out/r04o_iter1.json 2> gpurun_out/r04o_iter1.err || { tail -20 gpurun_out/r04o_iter1.err; exit 1; }
RT_COOP=3 timeout -k 10 300 python -u tools/iter_profile.py --config cfg4 --world 8 --lanes 1 --out gpurun_out/r04o_iter1c > gpurun_out/r04o_iter1c.json 2> gpurun_out/r04o_iter1c.err || { tail -20 gpurun_out/r04o_iter1c.err; exit 1; }
RT_COOP=0 timeout -k 10 300 python -u tools/iter_profile.py --config cfg4 --world 8 --lanes 4 --out gpurun_out/r04o_iter4 > gpurun_out/r04o_iter4.json 2> gpurun_out/r04o_iter4.err || { tail -20 gpurun_out/r04o_iter4.err; exit 1; }
grep -o '"frame_ms[^,]*\|"tail_row.*' gpurun_out/r04o_iter1.json gpurun_out/r04o_iter1c.json gpurun_out/r04o_iter4.json
