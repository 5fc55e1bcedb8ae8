#!/bin/bash
# Lane imbalance: which lane ends last, with the lanes on their streams as usual and reversed.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
timeout -k 10 300 python -u tools/timeline.py --config cfg4 --world 8 --rank 1 --out gpurun_out/r04v_tl_a$rep > gpurun_out/r04v_tl_a$rep.json 2> gpurun_out/r04v_tl_a$rep.err || { tail -20 gpurun_out/r04v_tl_a$rep.err; exit 1; }
RT_LANE_REV=1 timeout -k 10 300 python -u tools/timeline.py --config cfg4 --world 8 --rank 1 --out gpurun_out/r04v_tl_b$rep > gpurun_out/r04v_tl_b$rep.json 2> gpurun_out/r04v_tl_b$rep.err || { tail -20 gpurun_out/r04v_tl_b$rep.err; exit 1; }
done
for f in gpurun_out/r04v_tl_*.json; do python3 -c "
import json,sys; t=open('$f').read(); d=json.loads(t[:t.index('}]')+2]+'}') if False else None" 2>/dev/null; head -c 900 $f; echo; done
