#!/bin/bash
# Where a cfg2 frame's time goes at the round's last build (3 lanes, HIP events per launch).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/timeline.py --config cfg2 --out gpurun_out/r04hh_tl_cfg2 > gpurun_out/r04hh_tl_cfg2.json 2> gpurun_out/r04hh_tl_cfg2.err || { tail -20 gpurun_out/r04hh_tl_cfg2.err; exit 1; }
head -c 1200 gpurun_out/r04hh_tl_cfg2.json
timeout -k 10 300 python -u tools/iter_profile.py --config cfg2 --lanes 3 --out gpurun_out/r04hh_iter3 > gpurun_out/r04hh_iter3.json 2> gpurun_out/r04hh_iter3.err || { tail -20 gpurun_out/r04hh_iter3.err; exit 1; }
grep -o '"frame_ms[^,]*\|"bands.*' gpurun_out/r04hh_iter3.json | head -c 1500
