# RT_T2_WINDOW sweep (GPU box): default 1e-3 vs 1e-4 / 1e-5 builds
mkdir -p gpurun_out/win
for v in "" _w1e4 _w1e5; do
  RT_HIP_LIB=sycl-ray-tracing_amd/lib/librt_hip$v.so timeout -k 10 120 python -u tools/query_bench.py --modes 4,5 > gpurun_out/win/qb$v.log 2>&1 || exit 1
  RT_HIP_LIB=sycl-ray-tracing_amd/lib/librt_hip$v.so timeout -k 10 120 python -u bench.py --no-cpu-baseline > gpurun_out/win/n1$v.json 2> gpurun_out/win/n1$v.err || exit 1
done
