mkdir -p gpurun_out/occ
for occ in 4 5 6 8; do
  RT_HIP_LIB=sycl-ray-tracing_amd/lib/librt_hip_occ$occ.so timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-stats > gpurun_out/occ/n1_$occ.json 2> gpurun_out/occ/n1_$occ.err || exit 1
  RT_HIP_LIB=sycl-ray-tracing_amd/lib/librt_hip_occ$occ.so timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-stats --sim-world 8 > gpurun_out/occ/n8_$occ.json 2> gpurun_out/occ/n8_$occ.err || exit 1
done
