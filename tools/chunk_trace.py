"""Analyse per-chunk records of a RT_CHUNK_TRACE build (librt_hip_trace.so).

Run on the GPU box, e.g.
  RT_HIP_LIB=sycl-ray-tracing_amd/lib/librt_hip_trace.so RT_CHUNK_TRACE_ITERS=20,100,300 \
  RT_CHUNK_TRACE_OUT=gpurun_out/ct python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-stats
  python tools/chunk_trace.py gpurun_out/ct.*
Record (8 x u32): start, end (100 MHz ticks), max / sum node visits of the
chunk's lanes, sum of triangle tests, role | xcc << 4, wave id, lanes.
"""
import sys

import numpy as np


def main(paths):
    for p in sorted(paths):
        r = np.fromfile(p, dtype=np.uint32).reshape(-1, 8).astype(np.int64)
        if r.size == 0:
            print(p, "empty")
            continue
        t0 = r[:, 0].min()
        st, en = r[:, 0] - t0, r[:, 1] - t0
        dur = (en - st) * 10e-3  # us
        vmax, vsum, tsum, lanes = r[:, 2], r[:, 3], r[:, 4], r[:, 7]
        role = r[:, 5] & 15
        span = (en.max() - st.min()) * 10e-3
        print(f"{p}: {len(r)} chunks, launch span {span:.1f} us, lanes {lanes.sum()}")
        for name, m in (("closest", role == 1), ("any", role == 2)):
            if not m.any():
                continue
            d, vm, vs = dur[m], vmax[m], vsum[m]
            simt = vs.sum() / max(1, (vm * 64).sum())
            per_visit = d.sum() / max(1, vm.sum())
            print(f"  {name:7s} chunks {m.sum():6d}  dur us p50 {np.median(d):6.1f} p90 {np.percentile(d, 90):6.1f} "
                  f"max {d.max():6.1f}  vmax p50 {np.median(vm):4.0f} p90 {np.percentile(vm, 90):4.0f} max {vm.max():4d}  "
                  f"mean visits/lane {vs.sum() / lanes[m].sum():5.2f}  SIMT {simt:.3f}  us per max-visit {per_visit:.2f}")
        # waves: busy time and end time
        w = r[:, 6]
        order = np.argsort(w)
        ws, idx = np.unique(w[order], return_index=True)
        busy = np.add.reduceat(dur[order], idx)
        last = np.maximum.reduceat(en[order], idx) * 10e-3
        first = np.minimum.reduceat(st[order], idx) * 10e-3
        print(f"  waves {len(ws)}: busy us p50 {np.median(busy):.1f} p90 {np.percentile(busy, 90):.1f} max {busy.max():.1f}; "
              f"first start p50 {np.median(first):.1f} max {first.max():.1f}; end p50 {np.median(last):.1f} "
              f"p99 {np.percentile(last, 99):.1f} max {last.max():.1f}")
        hist = np.histogram(st * 10e-3, bins=10, range=(0, span))[0]
        print("  chunk starts per tenth of the span:", hist.tolist())


if __name__ == "__main__":
    main(sys.argv[1:])
