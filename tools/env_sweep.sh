# Environment sweep (GPU box). SWEEP="A=1,B=2 A=3" — each entry is one setting of
# comma-separated env vars; every setting runs bench at 1 GPU and/or a simulated
# N-GPU shard (NS="1 8"); BARGS: extra bench arguments (e.g. --steps 12). Results: gpurun_out/sweep/<tag>_n<N>.json
mkdir -p gpurun_out/sweep
for cfg in $SWEEP; do
  tag=$(echo "$cfg" | tr ',=/' '___')
  for n in ${NS:-1 8}; do
    sim=""; [ "$n" != 1 ] && sim="--sim-world $n"
    env $(echo "$cfg" | tr ',' ' ') timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-stats $BARGS $sim > gpurun_out/sweep/${tag}_n$n.json 2> gpurun_out/sweep/${tag}_n$n.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/sweep/${tag}_n$n.json'));print('$cfg n=$n',d['value'],d['ms_per_step'])"
  done
done
