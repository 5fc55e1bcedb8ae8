"""bench.py — render throughput of the MI355X path tracer (BASELINE.json metric).

A "step" is one full render of the configured frame (RenderKernel::render,
render_kernel.cpp:189-211): every pixel, every sample, every bounce, then the
in-place tone-map, plus (N > 1) the RCCL gather of the HDR shards to rank 0.
Scene, BVH, env map and camera are resident in HBM before timing starts
(the reference times render() only, main.cpp:93-116).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2]
  N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints ONE JSON line. Extra objects:
  roofline      the render kernel's algorithmic bytes per launch (SURVEY.md
                §8(d) byte model x the kernel's own traversal counters, read
                from a stats-enabled render of the same workload) / its mean
                launch time from HIP events on the launch stream, vs 8 TB/s.
                `traffic` is the PMC-measured HBM bytes per launch from
                profiles/ (rocprofv3 --pmc pass of this command), or null.
  cpu_baseline  the pinned CPU restatement oracle (oracle/cpu_oracle.cpp,
                "port") on a bounded row subset of the same frame, on the
                host cores; its rows are also compared with the GPU's
                (parity, per-channel L-inf after tone-map).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(REPO, "sycl-ray-tracing_amd"), os.path.join(REPO, "tools"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

CONFIGS = {
    # name: (scene, sky, camera, W, H, spp, bounces, description)
    "cfg1": ("cornell12", "S", "cornell", 256, 256, 4, 3, "Cornell 12-tri 256x256x4spp x3"),
    "cfg2": ("dragon", "L", "dragon", 1920, 1080, 64, 8,
             "PBRT Dragon stand-in (1,000,002 tris) 1920x1080x64spp x8 bounces, SKY-L 2048x1024 env IS+MIS"),
    "cfg3": ("dragon", "L", "dragon", 1920, 1080, 256, 8,
             "PBRT Dragon stand-in 1920x1080x256spp x8 bounces, SKY-L env IS+MIS"),
    "cfg4": ("dragon", "L", "dragon", 3840, 2160, 256, 8, "PBRT Dragon stand-in 3840x2160x256spp x8 bounces"),
    # profiling-sized cfg2 (same scene / camera / ray mix, 1/16 of the pixels, 1/4 of the samples); not a bench line
    "cfg2s": ("dragon", "L", "dragon", 480, 270, 16, 8, "profiling-sized cfg2: dragon 480x270x16spp x8"),
}
HBM_PEAK_GBS = 8000.0  # /opt/skills/guides/MI355X_MICROARCH.md (spec)
# Algorithmic bytes per unit of work: the records a query
# must read. Search-BVH box test 32 B (half of a 64-B node), triangle test
# 48 B (a, e1, e2 as 3 x 16 B), octree verification slab test 64 B (one
# record), queue ray 32 B + result 8 B per query; step kernel: material
# 32 B, env texel 16 B, env-CDF fence load 64 B (16 keys; rt_trace.h fence_count). (SURVEY.md §8(d)'s model of the
# reference's own octree walk — 56 B per child volume, 36 B per triangle —
# is reported beside it as `ref_model_bytes_per_sample`.)
BYTES = {"box": 32, "tri": 48, "verify": 64, "ray": 40, "mat": 32, "env": 16, "cdf": 64}


def _query_bytes(g) -> float:
    return (BYTES["box"] * (g("vol") + g("any_vol")) + BYTES["tri"] * (g("tri") + g("any_tri")) +
            BYTES["verify"] * g("verify") + BYTES["ray"] * (g("rays") + g("any_rays")))


def _step_bytes(g) -> float:
    return BYTES["mat"] * g("mat") + BYTES["env"] * g("env") + BYTES["cdf"] * g("cdf")


def algo_bytes(st: dict, kernel: str) -> float:
    """Algorithmic bytes of one kernel class over the counted render. The
    counters are totals over every kernel, plus the tail kernel's share
    (tail_*): k_trace = query work minus the tail's, k_step = step work
    minus the tail's, "other" (k_tail) = its query and step work. k_trace's
    exact-walk role (st["fallback"] queries, ~1e-6 of them) shares the box /
    triangle counters, so those bytes are booked to it (< 0.1 %)."""
    tot = lambda k: st[k]  # noqa: E731
    tail = lambda k: st.get("tail_" + k, 0)  # noqa: E731
    rest = lambda k: st[k] - st.get("tail_" + k, 0)  # noqa: E731
    if kernel == "trace":
        return _query_bytes(rest)
    if kernel == "step":
        return _step_bytes(rest)
    if kernel == "other":
        return _query_bytes(tail) + _step_bytes(tail)
    return _query_bytes(tot) + _step_bytes(tot)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_inputs(cfg):
    import rt_amd
    import scenes
    scene, sky_kind, cam, W, H, spp, nb, _ = CONFIGS[cfg]
    P = rt_amd.parse_obj(scenes.scene_path(scene))
    sky = scenes.make_sky(sky_kind)
    cam17 = rt_amd.Camera.preset(cam).as17()
    return P, sky, cam17


def cpu_baseline(P, sky, cam17, cfg, gpu_frame, threads, row_step):
    """Oracle on every row_step-th row (full spp) of the same frame."""
    from oracle_bindings import OracleScene
    import golden_io as gio
    _, _, _, W, H, spp, nb, _ = CONFIGS[cfg]
    S = OracleScene(P.triangles, P.material_indices, P.materials, P.emissive_triangle_indices, env=sky)
    rows = np.arange(row_step // 2, H, row_step)
    xs, ys = np.meshgrid(np.arange(W), rows)
    px = np.stack([xs.ravel(), ys.ravel()], 1).astype(np.int32)
    res, sec = S.render(cam17, W, H, spp, nb, pixels=px, threads=threads)
    samples = px.shape[0] * spp
    par = gio.compare_rgb(gpu_frame[rows].reshape(-1, 4), res) if gpu_frame is not None else None
    return dict(value=samples / sec / 1e6, unit="Msamples/s", cores=threads, kind="port",
                sample=f"{rows.size} rows (every {row_step}th row, all {W} px, {spp} spp, {nb} bounces) = "
                       f"{samples / 1e6:.2f} Msamples in {sec:.2f} s, OpenMP dynamic over pixels"), par


def load_traffic(cfg, n_gpus):
    """PMC HBM bytes per launch from a committed rocprofv3 --pmc pass."""
    p = os.path.join(REPO, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None
    d = json.load(open(p))
    e = d.get(f"{cfg}_n{n_gpus}") or d.get(cfg)
    return None if e is None else e.get("bytes_per_launch")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stats", action="store_true", help="skip the counter pass (roofline.achieved = null)")
    ap.add_argument("--cpu-row-step", type=int, default=10)
    ap.add_argument("--sim-world", type=int, default=0,
                    help="diagnostic: render only rank 0's rows of an N-GPU run, on this one GPU (not a bench line)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    import rt_amd
    from rt_amd.dist import ShardedFrame
    scene, sky_kind, cam, W, H, spp, nb, desc = CONFIGS[args.config]

    t0 = time.time()
    if rank == 0:
        build_inputs(args.config)  # materialise the scene file once
    if world > 1:
        dist.barrier()
    P, sky, cam17 = build_inputs(args.config)
    rk = rt_amd.RenderKernel(W, H, spp, nb, rt_amd.Image(1, 1), P.triangles, P.materials,
                             P.emissive_triangle_indices, P.material_indices, None, rt_amd.BVH(P.triangles),
                             rt_amd.Image.from_rgb(sky), None, device=local)
    rk.set_camera(rt_amd.Camera(cam17[:16], cam17[16]))
    frame = ShardedFrame(rk, rank, args.sim_world or world, device=dev)
    info = rk.bvh_info()
    log(f"[rank {rank}] setup {time.time() - t0:.1f}s  bvh {info}")

    stream = torch.cuda.current_stream(dev).cuda_stream

    # counter pass (same workload, stats kernel variant) -> algorithmic bytes
    stats = None
    if not args.no_stats:
        rk.set_stats(True)
        frame.render(stream)
        torch.cuda.synchronize(dev)
        stats = rk.stats()
        rk.set_stats(False)
        log(f"[rank {rank}] counters {stats}  iterations {rk.last_iterations()}")

    for _ in range(args.warmup):
        frame.render(stream)
        if not args.sim_world:
            frame.gather()
    torch.cuda.synchronize(dev)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    rk.kernel_timing(1)  # HIP events around every kernel launch, on the launch stream
    kms = []
    t_start = time.perf_counter()
    for _ in range(args.steps):
        frame.render(stream)
        full = frame.gather() if not args.sim_world else frame.shard
        kms.append(rk.device_last_kernel_ms())
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    ktime = rk.kernel_timing(0)
    log(f"[rank {rank}] kernel time per class over {args.steps} steps: {ktime}")

    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    kernel_ms = float(np.mean(kms))

    samples_per_step = W * H * spp if not args.sim_world else frame.rows * W * spp
    value = samples_per_step * args.steps / elapsed / 1e6

    roofline = None
    if stats is not None:
        dom = max(("trace", "step"), key=lambda k: ktime[k][0])
        tot_ms, launches = ktime[dom]
        per_render = algo_bytes(stats, dom)          # the counter pass rendered one frame
        algo = per_render / max(launches / args.steps, 1)  # per launch
        avg_ms = tot_ms / max(launches, 1)
        achieved = algo / (avg_ms * 1e-3) / 1e9
        samples_rank = frame.rows * W * spp
        roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": load_traffic(args.config, world),
                    "algo_bytes_per_launch": round(algo), "avg_launch_ms": round(avg_ms, 4),
                    "launches_per_step": launches / args.steps,
                    "kernel_ms_per_step": {k: round(v[0] / args.steps, 2) for k, v in ktime.items()},
                    "bytes_per_sample_all_kernels": round(sum(algo_bytes(stats, k) for k in ktime) / samples_rank, 1),
                    "closest_rays_per_sample": round(stats["rays"] / samples_rank, 3),
                    "any_rays_per_sample": round(stats["any_rays"] / samples_rank, 3),
                    "render_ms": round(kernel_ms, 3),
                    # run_wave overlaps its lanes (streams), so a launch's HIP-event duration includes
                    # the other lanes' kernels running beside it; the frame-level figure is all
                    # kernels' algorithmic bytes over the render time
                    "frame_achieved_GBps": round(sum(algo_bytes(stats, k) for k in ktime) / (kernel_ms * 1e-3) / 1e9, 1)}

    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = int(os.environ.get("OMP_NUM_THREADS", 0)) or len(os.sched_getaffinity(0))
        threads = min(threads, len(os.sched_getaffinity(0)))
        gpu_frame = full.cpu().numpy()
        cpu, parity = cpu_baseline(P, sky, cam17, args.config, gpu_frame, threads, args.cpu_row_step)

    if world > 1:
        dist.barrier()
    if rank == 0:
        out = {
            "metric": "Msamples/sec (W×H×spp/s) at 1080p; per-channel L∞ vs CPU ref",
            "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: procedural 1,000,002-triangle stand-in for the absent pbrt_dragon.obj and a "
                    "synthetic 2048x1024 env map (SURVEY.md §8d)",
            "config": {"workload": f"{args.config}: {desc}", "W": W, "H": H, "spp": spp, "bounces": nb,
                       "parallelism": f"rows y%{world} per GPU + RCCL gather" if world > 1 else "1 GPU"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "parity": parity,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
