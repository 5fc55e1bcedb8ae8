"""Resource usage (VGPRs, spills, occupancy, LDS) of the product's kernels from the compiler's
kernel-resource-usage remarks:  python tools/kernel_regs.py [rt_render.hip] [-- extra hipcc flags]"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def usage(src=None, extra=()):
    src = src or os.path.join(REPO, "sycl-ray-tracing_amd", "csrc", "rt_render.hip")
    cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
           "-fno-fast-math", "-fno-gpu-flush-denormals-to-zero", "-fhip-fp32-correctly-rounded-divide-sqrt",
           "-Wno-unused-function", "-Wno-unknown-pragmas", "-Rpass-analysis=kernel-resource-usage", *extra,
           "-c", src, "-o", "/tmp/kernel_regs.o"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = {}, None
    for line in out.splitlines():
        m = re.search(r"Name: (\S+)", line)
        if m:
            cur = m.group(1)
            rows[cur] = {}
            continue
        m = re.search(r"\s(VGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
        if m and cur:
            rows[cur][m.group(1).split(" [")[0]] = int(m.group(2))
    return {k: v for k, v in rows.items() if re.search(r"k_(trace|step|tail)", k)}


if __name__ == "__main__":
    args = sys.argv[1:]
    extra = args[args.index("--") + 1:] if "--" in args else []
    src = args[0] if args and args[0] != "--" else None
    for k, v in usage(src, extra).items():
        print(f"{k[:64]:64s} vgpr {v.get('VGPRs')} spill {v.get('VGPRs Spill')} sspill {v.get('SGPRs Spill')} "
              f"occ {v.get('Occupancy')} lds {v.get('LDS Size')}")
