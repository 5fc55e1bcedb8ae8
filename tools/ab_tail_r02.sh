set -o pipefail
mkdir -p gpurun_out
tools/ab.sh gpurun_out/ab_tail.jsonl 2 base tx ts || exit 1
for v in base tx ts; do
  RT_HIP_LIB=sycl-ray-tracing_amd/lib/librt_hip_$v.so timeout -k 10 200 python tools/shard_probe.py --config cfg4 --worlds 8 --reps 2 > gpurun_out/probe_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/probe_$v.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('$v', d['runs'])"
done
cat gpurun_out/ab_tail.jsonl
