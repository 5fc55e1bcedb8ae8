# k_tail sweep (GPU box): paths per wave 0 (off) / 4 / 8 at 1 GPU and a simulated 8-GPU shard
mkdir -p gpurun_out/tail
for tp in ${TPS:-0 4 8}; do
  RT_TAIL_PATHS=$tp timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-stats > gpurun_out/tail/n1_$tp.json 2> gpurun_out/tail/n1_$tp.err || exit 1
  RT_TAIL_PATHS=$tp timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-stats --sim-world 8 > gpurun_out/tail/n8_$tp.json 2> gpurun_out/tail/n8_$tp.err || exit 1
done
