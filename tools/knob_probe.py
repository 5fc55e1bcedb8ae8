"""Frame time of a cfg4 N-way shard and of the full cfg2 frame under several wavefront
schedules (rt_test_schedule keys), in one process.

  python tools/knob_probe.py --sets - "tail_paths=2,tail_enter=2" "lanes=3" \
      [--world 8 --rank 1] [--reps 3] [--rounds 2] [--out gpurun_out/knob_probe.json]

Settings alternate round by round (A B C A B C ...), min over reps per round; "-" is the
product's schedule.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "sycl-ray-tracing_amd"), os.path.join(REPO, "tools"), REPO):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", nargs="+", required=True)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=1)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--no-cfg2", action="store_true")
    ap.add_argument("--out", default="gpurun_out/knob_probe.json")
    args = ap.parse_args()
    import torch

    import bench
    import rt_amd
    from rt_amd.dist import ShardedFrame

    P, sky, cam17 = bench.build_inputs("cfg4")
    _, _, _, W4, H4, spp4, nb4, _ = bench.CONFIGS["cfg4"]
    _, _, _, W2, H2, spp2, nb2, _ = bench.CONFIGS["cfg2"]
    rk = rt_amd.RenderKernel(W4, H4, spp4, nb4, rt_amd.Image(1, 1), P.triangles, P.materials,
                             P.emissive_triangle_indices, P.material_indices, None, rt_amd.BVH(P.triangles),
                             rt_amd.Image.from_rgb(sky), None, device=0)
    rk.set_camera(rt_amd.Camera(cam17[:16], cam17[16]))
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def apply(s):
        # a set: "-" (the product's schedule) or "key=value,..." of rt_test_schedule keys
        # (lanes, tail_paths, tail_enter, tail_rows, drain_rows, heavy_calls, spec_cam, ...)
        rk.test_schedule(reset=1)
        if s != "-":
            rk.test_schedule(**{kv.split("=", 1)[0]: float(kv.split("=", 1)[1]) for kv in s.split(",")})

    def timed(cfg):
        if cfg == "cfg4":
            rk.width, rk.height, rk.render_samples = W4, H4, spp4
            fr = ShardedFrame(rk, args.rank, args.world, device=dev)
        else:
            rk.width, rk.height, rk.render_samples = W2, H2, spp2
            fr = ShardedFrame(rk, 0, 1, device=dev)
        fr.render(stream)
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            fr.render(stream)
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
        return min(ts) * 1e3, rk.last_iterations()

    res = {s: {"cfg4_shard_ms": [], "cfg2_ms": [], "iters": []} for s in args.sets}
    for rnd in range(args.rounds):
        for s in args.sets:
            apply(s)
            ms4, it4 = timed("cfg4")
            res[s]["cfg4_shard_ms"].append(round(ms4, 2))
            res[s]["iters"].append(it4)
            if not args.no_cfg2:
                ms2, _ = timed("cfg2")
                res[s]["cfg2_ms"].append(round(ms2, 2))
            print(json.dumps({"round": rnd, "set": s, **{k: v[-1] for k, v in res[s].items() if v}}), flush=True)
    apply("-")
    out = {"what": f"cfg4 rank {args.rank} of {args.world} shard and full cfg2 frame per schedule setting (rt_test_schedule), min of "
                   f"{args.reps} renders per round, settings alternating over {args.rounds} rounds (one MI355X)",
           "results": res}
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
