# k_step occupancy sweep (GPU box): librt_hip.so (3 waves/SIMD) vs socc4 / socc5 builds
mkdir -p gpurun_out/socc
for v in "" _socc4 _socc5; do
  RT_HIP_LIB=sycl-ray-tracing_amd/lib/librt_hip$v.so timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-stats > gpurun_out/socc/n1$v.json 2> gpurun_out/socc/n1$v.err || exit 1
done
