# lanes sweep (GPU box): one vs two wavefront lanes per GPU, 1 GPU and a simulated 8-GPU shard
mkdir -p gpurun_out/lanes
for ln in ${LANES:-1 2}; do
  RT_LANES=$ln timeout -k 10 120 python -u bench.py --no-cpu-baseline > gpurun_out/lanes/n1_$ln.json 2> gpurun_out/lanes/n1_$ln.err || exit 1
  RT_LANES=$ln timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-stats --sim-world 8 > gpurun_out/lanes/n8_$ln.json 2> gpurun_out/lanes/n8_$ln.err || exit 1
done
