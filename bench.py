"""bench.py — render throughput of the MI355X path tracer (BASELINE.json metric).

A "step" is one full render of the configured frame (RenderKernel::render,
render_kernel.cpp:189-211): every pixel, every sample, every bounce, then the
in-place tone-map, plus (N > 1) the RCCL exchange of the HDR shards with the
root. Scene, BVH, env map and camera are resident in HBM before timing starts
(the reference times render() only, main.cpp:93-116).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2] [--scaling weak|strong]

N GPUs, two launch modes, the same JSON line:
  * one process (no launcher): one librt_hip context over devices 0..N-1
    (rt_create_multi: rows y -> device y mod N, ncclScatter / ncclGather of
    the frame through device 0). Exits non-zero if fewer than N devices answer.
  * torchrun --nproc-per-node N: one process per GPU, each renders rows
    y % WORLD_SIZE == RANK on LOCAL_RANK, torch.distributed (RCCL) gather to
    rank 0. --gpus must equal WORLD_SIZE.

Workload. N = 1 is the config's frame (cfg2: 1920x1080 x 64 spp x 8 bounces).
For N > 1, --scaling weak (default) renders a frame of N times the pixels at
the same 16:9 framing, spp and bounces (W, H scaled by sqrt(N): 4 GPUs =
3840x2160), so each GPU's work equals the 1-GPU line's and `value` (all
samples / max-over-ranks time) is whole-job throughput; --scaling strong
splits the config's own frame N ways.

Rank 0 prints ONE JSON line. Extra objects:
  roofline      k_trace (the traversal kernel): algorithmic bytes per launch
                (DESIGN.md §5 byte model x the kernel's own traversal counters,
                from a stats render of the same frame) / its mean launch
                duration, measured in a separate ONE-LANE render after the
                timed steps (one stream, so launches do not overlap: HIP
                events around each launch time that kernel alone), vs 8 TB/s.
                `traffic`: PMC FETCH_SIZE bytes per launch of the same 1-lane
                command from profiles/traffic.json, or null.
                `ref_model_*`: SURVEY.md §8(d)'s byte model of the REFERENCE's
                octree walk (56 B per non-empty child volume test, 36 B per
                triangle test) counted by the oracle on the cpu_baseline rows,
                and the rate it implies at `value`.
  cpu_baseline  the pinned CPU restatement oracle (oracle/cpu_oracle.cpp,
                "port") on a bounded row subset of the same frame, on the
                host cores (model named); its rows are also compared with the
                GPU's (parity, per-channel L-inf after tone-map).
"""
from __future__ import annotations

import argparse
import json
import math
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
    # one cfg5 material variant (metalness 1/3, roughness 0.25 on the dragon) at the cfg5 frame
    "cfg5": ("dragon", "L", "dragon", 1920, 1080, 1024, 8,
             "PBRT Dragon stand-in, cfg5 variant m=1/3 r=0.25, 1920x1080x1024spp x8 bounces"),
    # BASELINE config 5 as replicas: all 16 material variants (metalness x roughness on the dragon,
    # tools/gen_golden.py), each a 1920x1080x1024spp frame, variant v on GPU v mod N (rt_render_variants)
    "cfg5sweep": ("dragon", "L", "dragon", 1920, 1080, 1024, 8,
                  "PBRT Dragon stand-in, Cook-Torrance sweep: 16 material variants (metalness {0,1/3,2/3,1} x "
                  "roughness {0.05,0.25,0.5,1}) x 1920x1080x1024spp x8 bounces, variant v on GPU v mod N"),
    # profiling-sized cfg2 (same scene / camera / ray mix, 1/16 of the pixels, 1/4 of the samples); not a bench line
    "cfg2s": ("dragon", "L", "dragon", 480, 270, 16, 8, "profiling-sized cfg2: dragon 480x270x16spp x8"),
}
CFG5_VARIANT = (1, 1.0 / 3.0, 0.25)  # (material index, metalness, roughness) as tools/gen_golden.py writes them
CFG5_GRID = [(m, r) for m in range(4) for r in range(4)]  # variant v = (metalness index, roughness index)
CFG5_METAL = [0.0, 1.0 / 3.0, 2.0 / 3.0, 1.0]
CFG5_ROUGH = [0.05, 0.25, 0.5, 1.0]
# The sweep's static schedule: position p of this order renders on GPU p mod N. A variant's
# frame time follows its roughness (one MI355X, profiles/r03_sweep_variant_ms.json: r = 0.05 /
# 0.25 / 0.5 / 1.0 -> 2.65 / 2.54 / 2.17 / 1.81 s; metalness within 1.5 %), so the order pairs
# the slowest with the fastest: N = 8 -> {0.05, 1.0} or {0.25, 0.5} per GPU (max 4.71 s against
# the 4.58 s mean), N = 4 and 2 -> every roughness on every GPU. (v mod N in grid order would put
# two r = 0.05 frames on GPU 0: 5.31 s, 0.86.)
CFG5_ORDER = [0, 4, 8, 12, 1, 5, 9, 13, 3, 7, 11, 15, 2, 6, 10, 14]
HBM_PEAK_GBS = 8000.0  # /opt/skills/guides/MI355X_MICROARCH.md (spec)
# Algorithmic bytes per unit of work: the records a query
# must read. Search-BVH box test 48 B (one child record + its oriented slab, r05), triangle test
# 48 B (a, e1, e2 as 3 x 16 B), octree verification slab test 64 B (one
# record), queue ray 32 B + result 8 B per query; step kernel: material
# 32 B, env texel 16 B, env-CDF fence load 64 B (16 keys; rt_trace.h fence_count).
BYTES = {"box": 48, "tri": 48, "verify": 64, "ray": 40, "mat": 32, "env": 16, "cdf": 64}
# the reference's octree walk, 56 B per child-volume test, 36 B per triangle
REF_BYTES = {"vol": 56, "tri": 36}


def _query_bytes(g) -> float:
    return (BYTES["box"] * (g("vol") + g("any_vol")) + BYTES["tri"] * (g("tri") + g("any_tri")) +
            BYTES["verify"] * g("verify") + BYTES["ray"] * (g("rays") + g("any_rays")))


def _step_bytes(g) -> float:
    return BYTES["mat"] * g("mat") + BYTES["env"] * g("env") + BYTES["cdf"] * g("cdf")


# Wavefront step model: what a path step must read besides the scene
# records above. Per step (the `steps` counter): the slot's 4 state records (64 B), its
# continuation and camera-ahead results (16 B), live-list entry and wait count (8 B);
# per shaded bounce: the hit triangle (48 B) and the pending throughput (16 B); per
# occlusion query: its candidate (16 B) and answer (1 B); per sample: the fin record
# (16 B). Exact for scenes without emissive triangles (cfg2-cfg5: every material load
# is a shade).
SLOT_BYTES = {"step": 88, "shade": 64, "occ": 17, "sample": 16}


def step_model_bytes(st: dict, samples: float) -> dict:
    rest = lambda k: st[k] - st.get("tail_" + k, 0)  # noqa: E731
    scene = _step_bytes(rest)
    tail_frac = 1.0 - rest("rays") / max(st["rays"], 1)
    slot = (SLOT_BYTES["step"] * rest("steps") + SLOT_BYTES["shade"] * rest("mat") +
            SLOT_BYTES["occ"] * rest("any_rays") + SLOT_BYTES["sample"] * samples * (1.0 - tail_frac))
    return {"scene": scene, "slot": slot}


def algo_bytes(st: dict, kernel: str) -> float:
    """Algorithmic bytes of one kernel class over the counted render. The
    counters are totals over every kernel, plus the tail kernel's share
    (tail_*): k_trace = query work minus the tail's, k_step = step work
    minus the tail's, "other" (k_tail) = its query and step work. k_step's
    exact-walk roles (st["fallback"] queries, ~1e-6 of them) share the box /
    triangle counters, so those bytes are booked to k_trace (< 0.1 %)."""
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


def frame_dims(cfg: str, n: int, scaling: str):
    """(W, H) of the job: the config's frame, or for weak scaling N x its pixels at its aspect."""
    W, H = CONFIGS[cfg][3], CONFIGS[cfg][4]
    if n <= 1 or scaling == "strong":
        return W, H
    s = math.sqrt(n)
    return int(round(W * s)), int(round(H * s))


def cfg5_tables(P):
    """The 16 cfg5 material tables (material 1 = the dragon's, as tools/gen_golden.py overrides it)."""
    out = []
    for mi, ri in CFG5_GRID:
        m = P.materials.copy()
        m[1, 8] = np.float32(repr(CFG5_METAL[mi]))
        m[1, 9] = np.float32(repr(CFG5_ROUGH[ri]))
        out.append(m)
    return out


def build_inputs(cfg):
    import rt_amd
    import scenes
    scene, sky_kind, cam, W, H, spp, nb, _ = CONFIGS[cfg]
    P = rt_amd.parse_obj(scenes.scene_path(scene))
    if cfg == "cfg5":
        mi, m, r = CFG5_VARIANT
        P.materials[mi, 8] = np.float32(repr(m))
        P.materials[mi, 9] = np.float32(repr(r))
    sky = scenes.make_sky(sky_kind)
    cam17 = rt_amd.Camera.preset(cam).as17()
    return P, sky, cam17


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(P, sky, cam17, W, H, spp, nb, gpu_frame, threads, row_step):
    """Oracle on every row_step-th row (full spp) of the same frame, with the
    reference-walk counters (SURVEY.md §8(d) byte model)."""
    from oracle_bindings import OracleScene
    import golden_io as gio
    S = OracleScene(P.triangles, P.material_indices, P.materials, P.emissive_triangle_indices, env=sky)
    rows = np.arange(row_step // 2, H, row_step)
    xs, ys = np.meshgrid(np.arange(W), rows)
    px = np.stack([xs.ravel(), ys.ravel()], 1).astype(np.int32)
    res, sec, cnt = S.render(cam17, W, H, spp, nb, pixels=px, threads=threads, counters=True)
    samples = px.shape[0] * spp
    par = gio.compare_rgb(gpu_frame[rows].reshape(-1, 4), res) if gpu_frame is not None else None
    ref_b = (REF_BYTES["vol"] * float(cnt[1]) + REF_BYTES["tri"] * float(cnt[3])) / samples
    cpu = dict(value=samples / sec / 1e6, unit="Msamples/s", cores=threads, kind="port", cpu_model=cpu_model(),
               sample=f"{rows.size} rows (every {row_step}th row, all {W} px, {spp} spp, {nb} bounces) = "
                      f"{samples / 1e6:.2f} Msamples in {sec:.2f} s, OpenMP dynamic over pixels")
    ref = dict(ref_model_bytes_per_sample=round(ref_b, 1),
               ref_model_rays_per_sample=round(float(cnt[0]) / samples, 3),
               ref_model_vol_tests_per_ray=round(float(cnt[1]) / max(float(cnt[0]), 1.0), 2),
               ref_model_tri_tests_per_ray=round(float(cnt[3]) / max(float(cnt[0]), 1.0), 2))
    return cpu, par, ref


def load_traffic(key):
    """PMC HBM bytes per k_trace launch from a committed rocprofv3 --pmc pass."""
    p = os.path.join(REPO, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None
    e = json.load(open(p)).get(key)
    return None if e is None else e.get("bytes_per_launch")


def build_commit():
    """The build of the library this process loaded (its rt_build_id: the kernel sources' hash and
    any experiment flags, compiled in by `make`), prefixed with the commit BUILD_COMMIT names when
    that stamp is of the same sources."""
    try:
        from rt_amd import _capi
        lib_id = _capi.lib().rt_build_id().decode()
    except Exception:  # noqa: BLE001  (no library: no build to report)
        return None
    try:
        stamp = open(os.path.join(REPO, "BUILD_COMMIT")).read().split()
    except OSError:
        stamp = []
    src = lambda b: b.split("src=")[-1].split()[0] if b and "src=" in b else None  # noqa: E731
    if len(stamp) >= 2 and src(stamp[1]) == src(lib_id):
        return f"{stamp[0]} {lib_id}"
    return lib_id


def traffic_source(key):
    """Where the committed FETCH_SIZE figure comes from: its profile, the build it measured and
    whether that is the build running now (profiles/traffic.json, tools/update_traffic.py)."""
    p = os.path.join(REPO, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None
    e = json.load(open(p)).get(key)
    if e is None:
        return None
    now = build_commit()
    src = lambda b: b.split("src=")[-1].split()[0] if b and "src=" in b else None  # noqa: E731  (the kernel sources' hash)
    return {"profile": e.get("profile"), "build": e.get("build"), "running_build": now,
            "same_build": bool(src(now) and src(now) == src(e.get("build")))}


def load_traffic_class(key, cls):
    """PMC FETCH_SIZE bytes per launch of one kernel class from profiles/traffic.json."""
    p = os.path.join(REPO, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None
    e = json.load(open(p)).get(key)
    return None if e is None else e.get("per_class_bytes_per_launch", {}).get(cls)


def fail(msg: str, code: int = 2):
    log("bench.py: " + msg)
    sys.exit(code)


def sweep_parity(frames_by_variant, variants) -> dict:
    """Every golden pixel of the rendered cfg5 variants (tests/golden, written by the compiled
    reference) against the GPU's frame: per-channel L-inf and the bitwise-identical fraction."""
    import golden_io as gio
    got, want = [], []
    for v, fr in zip(variants, frames_by_variant):
        mi, ri = CFG5_GRID[v]
        g = np.load(os.path.join(gio.GOLDEN, f"render_cfg5_sweep_m{mi}_r{ri}.npz"))
        px = g["px"]
        got.append(fr[px[:, 1], px[:, 0]])
        want.append(g["rgba"])
    c = gio.compare_rgb(np.concatenate(got), np.concatenate(want))
    c["pixels"] = int(sum(w.shape[0] for w in want))
    c["against"] = "tests/golden/render_cfg5_sweep_m*_r*.npz (compiled reference, 48 px per variant)"
    return c


def run_sweep(args, rank, world, dev, single_process_multi, torch, dist):
    """--config cfg5sweep: BASELINE config 5 as replicas. A step renders all 16 material
    variants (1920x1080x1024spp x8 each); variant v runs on GPU v mod N with no exchange
    (rt_render_variants: one context over the N GPUs, or under torchrun one context per
    rank rendering v = rank mod N). Strong scaling: the 16 frames are the whole job.
    --sim-world K renders only rank 0's share of a K-GPU sweep on this one GPU."""
    import rt_amd
    _, _, _, W, H, spp, nb, desc = CONFIGS["cfg5sweep"]
    n_gpus = args.gpus
    t0 = time.time()
    P, sky, cam17 = build_inputs("cfg5sweep")
    tables = cfg5_tables(P)
    share = args.sim_world or world
    # (single process: every variant, position p on GPU p mod N; torchrun / sim: this rank's positions)
    me = args.sim_rank if args.sim_world else rank
    mine = [CFG5_ORDER[p] for p in range(len(tables)) if single_process_multi or p % share == me]
    devices = list(range(n_gpus)) if single_process_multi else dev.index
    rk = rt_amd.RenderKernel(W, H, spp, nb, rt_amd.Image(1, 1), P.triangles, P.materials,
                             P.emissive_triangle_indices, P.material_indices, None, rt_amd.BVH(P.triangles),
                             rt_amd.Image.from_rgb(sky), None, device=devices)
    rk.set_camera(rt_amd.Camera(cam17[:16], cam17[16]))
    ndev = n_gpus if single_process_multi else 1
    init = torch.zeros((H, W, 4), dtype=torch.float32)
    init[..., 3] = 1.0
    bufs = [init.to(torch.device("cuda", i % ndev if single_process_multi else dev.index)) for i in range(len(mine))]
    setup_s = time.time() - t0

    inits = {b.device: init.to(b.device) for b in bufs}

    def step():  # a fresh framebuffer per variant (the reference's Image is read-modify-write), then the sweep
        for b in bufs:
            b.copy_(inits[b.device])
        for d in inits:
            torch.cuda.synchronize(d)
        rk.render_variants([tables[v] for v in mine], device_ptrs=[b.data_ptr() for b in bufs])

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t_start = time.perf_counter()
    kms = []
    for _ in range(args.steps):
        step()
        kms.append(rk.last_kernel_ms())
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    cdev = dev if world == 1 or dist.get_backend() == "nccl" else "cpu"  # (gloo rehearsals: host tensors)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    n_frames = len(tables) if not args.sim_world else len(mine)
    value = n_frames * W * H * spp * args.steps / elapsed / 1e6
    frames = [b.cpu().numpy() for b in bufs]
    parity = sweep_parity(frames, mine)
    if world > 1:  # parity of every rank's variants, worst case on rank 0
        pt = torch.tensor([parity["linf"], 1.0 - parity["bitwise_fraction"]], dtype=torch.float64, device=cdev)
        dist.all_reduce(pt, op=dist.ReduceOp.MAX)
        parity["linf"], parity["bitwise_fraction"] = float(pt[0]), 1.0 - float(pt[1])
        parity["pixels"] *= world
    cpu = None
    if rank == 0 and world == 1 and n_gpus == 1 and not args.no_cpu_baseline:
        threads = int(os.environ.get("OMP_NUM_THREADS", 0)) or len(os.sched_getaffinity(0))
        threads = min(threads, len(os.sched_getaffinity(0)))
        Pv = rt_amd.parse_obj(__import__("scenes").scene_path("dragon"))
        Pv.materials = tables[mine[0]]
        cpu, cpar, _ = cpu_baseline(Pv, sky, cam17, W, H, spp, nb, frames[0], threads, 540)
        cpu["sample"] = f"variant {mine[0]}: " + cpu["sample"]
        cpu["parity_rows"] = cpar
    if rank == 0:
        if single_process_multi:
            par = f"one process, rt_render_variants over {n_gpus} GPUs: variant v on GPU v mod {n_gpus}, no exchange"
        elif world > 1:
            par = f"{world} processes (torchrun): rank r renders variants v % {world} == r, no exchange"
        else:
            par = "1 GPU" + (f" (sim: rank {args.sim_rank}'s share of a {args.sim_world}-GPU sweep)"
                             if args.sim_world else "")
        out = {
            "metric": "Msamples/sec (W×H×spp/s) at 1080p; per-channel L∞ vs CPU ref",
            "value": round(value, 3), "unit": "Msamples/s", "n_gpus": n_gpus, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: procedural 1,000,002-triangle stand-in for the absent pbrt_dragon.obj and a "
                    "synthetic 2048x1024 env map (SURVEY.md §8d)",
            "config": {"workload": f"cfg5sweep: {desc}", "W": W, "H": H, "spp": spp, "bounces": nb,
                       "variants": n_frames, "variants_this_rank": [int(v) for v in mine], "parallelism": par},
            "setup_s": round(setup_s, 2),
            "device_ms_per_step": round(float(np.mean(kms)), 2),
            "roofline": None,  # (the kernels are cfg2's; their roofline is the cfg2 line's: bench.py --config cfg2)
            "cpu_baseline": cpu,
            "parity": parity,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if rank == 0 and parity["bitwise_fraction"] < 1.0:
        fail(f"PARITY FAILURE: cfg5 sweep pixels differ from the reference's goldens ({parity})", code=3)


def frame_compare(a, b, torch) -> dict:
    """Two frames of the same pixels (device tensors [..., 4] f32): the fraction of pixels whose
    four channels are bit-identical (NaN bits included), per-channel L-inf on RGB with NaN ==
    NaN, and ok = every pixel bit-identical (the multi-GPU partition must not change a bit)."""
    a = a.reshape(-1, 4).contiguous()
    b = b.reshape(-1, 4).contiguous()
    same = (a.view(torch.int32) == b.view(torch.int32)).all(dim=1)
    na, nb = torch.isnan(a[:, :3]), torch.isnan(b[:, :3])
    both = ~(na | nb)
    diff = torch.where(both, (a[:, :3] - b[:, :3]).abs(), torch.zeros_like(a[:, :3]))
    nan_mismatch = int((na != nb).sum())
    n = a.shape[0]
    frac = float(same.float().mean()) if n else 1.0
    return {"pixels": n, "bitwise_fraction": frac, "linf": float("inf") if nan_mismatch else
            (float(diff.max()) if n else 0.0), "nan_mismatch": nan_mismatch, "ok": bool(n == 0 or bool(same.all()))}


def solo_kernel(rk, P, sky, cam17, dev, single_process_multi):
    """A single-device RenderKernel on this rank's GPU: rk itself (torchrun: one device per
    process), or a new one when rk spans several devices (one-process multi-device context)."""
    if not single_process_multi:
        return rk
    import rt_amd
    k = rt_amd.RenderKernel(rk.width, rk.height, rk.render_samples, rk.max_bounces, rt_amd.Image(1, 1), P.triangles,
                            P.materials, P.emissive_triangle_indices, P.material_indices, None, rt_amd.BVH(P.triangles),
                            rt_amd.Image.from_rgb(sky), None, device=dev.index)
    k.set_camera(rt_amd.Camera(cam17[:16], cam17[16]))
    return k


def multi_parity(full, solo, dev, torch, rows_every=61, first=7) -> dict:
    """N > 1: rows first, first + rows_every, ... of the gathered N-GPU frame against the same
    rows rendered by ONE device alone (render_kernel.cpp:189-211 writes the whole Image&, so a
    gather that drops or permutes rows must show here). Bitwise."""
    from rt_amd.dist import ShardedFrame
    dev = torch.device(dev)
    sub = ShardedFrame(solo, first, rows_every, device=dev)
    sub.render(torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else None)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    c = frame_compare(full[first::rows_every], sub.shard[: sub.rows], torch)
    c["against"] = (f"rows {first}::{rows_every} ({sub.rows} rows x {solo.width} px) rendered by one device alone "
                    f"(a single-device context on {dev})")
    return c


def strong_cfg4(args, rk, P, sky, cam17, rank, world, dev, single_process_multi, torch, dist) -> dict:
    """N > 1: the north star's 8-GPU target config (cfg4: 3840x2160x256spp x8, BASELINE
    configs[3]) as a STRONG split over the same N GPUs (the line's own partition: rows
    y % N, RCCL exchange to the root), and the same frame on one GPU alone, one timed
    render each after a warm-up: efficiency = T_1 / (N * T_N). The line's `value` stays
    the weak-scaling cfg2 job; this object carries the fixed-size figure."""
    import rt_amd
    from rt_amd.dist import ShardedFrame
    _, _, _, W4, H4, spp4, nb4, desc4 = CONFIGS["cfg4"]
    n = args.gpus
    saved = (rk.width, rk.height, rk.render_samples, rk.max_bounces)
    rk.width, rk.height, rk.render_samples, rk.max_bounces = W4, H4, spp4, nb4
    stream = torch.cuda.current_stream(dev).cuda_stream

    def timed(frame, gather, reps=1):
        frame.render(stream)  # warm (and the wave buffers of this size)
        if gather:
            frame.gather()
        torch.cuda.synchronize(dev)
        if world > 1 and gather:
            dist.barrier()
        t0 = time.perf_counter()
        out = None
        for _ in range(reps):
            frame.render(stream)
            out = frame.gather() if gather else frame.shard[: frame.rows]
        torch.cuda.synchronize(dev)
        if world > 1 and gather:
            dist.barrier()
        return (time.perf_counter() - t0) / reps, out

    # T_N: the split, exactly as the line's frames are split
    frame = ShardedFrame(rk, 0, 1, device=dev) if single_process_multi else ShardedFrame(rk, rank, world, device=dev)
    tn, full_n = timed(frame, gather=True)
    if world > 1:
        t = torch.tensor([tn], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        tn = float(t.item())
    del frame
    rk.width, rk.height, rk.render_samples, rk.max_bounces = saved
    # T_1: the whole frame on GPU 0 alone (a single-device context; the other ranks wait)
    t1, bitwise = None, None
    if rank == 0:
        k1 = rt_amd.RenderKernel(W4, H4, spp4, nb4, rt_amd.Image(1, 1), P.triangles, P.materials,
                                 P.emissive_triangle_indices, P.material_indices, None, rt_amd.BVH(P.triangles),
                                 rt_amd.Image.from_rgb(sky), None, device=dev.index)
        k1.set_camera(rt_amd.Camera(cam17[:16], cam17[16]))
        t1, full_1 = timed(ShardedFrame(k1, 0, 1, device=dev), gather=False)
        # the gathered N-GPU frame against the 1-GPU frame, every pixel, bit for bit
        bitwise = frame_compare(full_n, full_1, torch)
        bitwise["against"] = "the same cfg4 frame rendered by GPU 0 alone (T_1's frame), every pixel"
        del k1, full_1
    del full_n
    if world > 1:
        dist.barrier()
    if rank != 0:
        return None
    return {"workload": f"cfg4: {desc4}", "W": W4, "H": H4, "spp": spp4, "bounces": nb4,
            "ms_1gpu": round(t1 * 1e3, 2), "ms_n_gpus": round(tn * 1e3, 2), "n_gpus": n,
            "msamples_per_s_n_gpus": round(W4 * H4 * spp4 / tn / 1e6, 1),
            "efficiency": round(t1 / (n * tn), 4),
            "bitwise": bitwise,
            "measured": "one render each after a warm-up; T_N = max over ranks incl. the RCCL exchange; "
                        "T_1 = the same frame on GPU 0 alone"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--scaling", default="weak", choices=("weak", "strong"),
                    help="N > 1: weak = N x the config's pixels (per-GPU work fixed), strong = the config's frame")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-strong-cfg4", action="store_true", help="N > 1: skip the strong_cfg4 object")
    ap.add_argument("--no-stats", action="store_true", help="skip the counter pass (roofline.achieved = null)")
    ap.add_argument("--no-roofline-pass", action="store_true", help="skip the 1-lane per-launch timing render")
    ap.add_argument("--roofline-only", action="store_true",
                    help="counter pass + the 1-lane timing renders only (the command profiled under profiles/)")
    ap.add_argument("--cpu-row-step", type=int, default=10)
    ap.add_argument("--sim-world", type=int, default=0,
                    help="diagnostic: render only one rank's rows (cfg5sweep: variants) of an N-GPU strong-scaling "
                         "split of the config's frame, on this one GPU (not a bench line)")
    ap.add_argument("--sim-rank", type=int, default=0, help="--sim-world: which rank's share")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world > 1 and world != args.gpus:
        fail(f"WORLD_SIZE={world} but --gpus={args.gpus}: launch with --nproc-per-node {args.gpus}")
    if args.sim_world and (world > 1 or args.gpus > 1):
        fail("--sim-world is a one-GPU diagnostic")

    import torch
    import torch.distributed as dist

    n_gpus = args.gpus
    single_process_multi = world == 1 and n_gpus > 1
    # (RT_BENCH_LOOPBACK=1: rehearse the one-process multi-device driver on one GPU — the
    # device list repeats GPU 0 and the shards move by device copies, rt_create_multi_loopback;
    # never set for a measurement)
    loopback = single_process_multi and os.environ.get("RT_BENCH_LOOPBACK") == "1"
    if single_process_multi and not loopback:
        have = torch.cuda.device_count()
        if have < n_gpus:
            fail(f"--gpus {n_gpus} but only {have} HIP device(s) visible")
    # (RT_BENCH_DEVICE_MOD / RT_BENCH_BACKEND: rehearse the multi-process path with several ranks on one
    # GPU and gloo; never set for a measurement)
    if os.environ.get("RT_BENCH_DEVICE_MOD"):
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("RT_BENCH_BACKEND", "nccl")
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)

    if args.config == "cfg5sweep":
        return run_sweep(args, rank, world, dev, single_process_multi, torch, dist)

    import rt_amd
    from rt_amd.dist import ShardedFrame
    scene, sky_kind, cam, _, _, spp, nb, desc = CONFIGS[args.config]
    W, H = frame_dims(args.config, n_gpus, args.scaling)

    t0 = time.time()
    if rank == 0:
        build_inputs(args.config)  # materialise the scene file once
    if world > 1:
        dist.barrier()
    P, sky, cam17 = build_inputs(args.config)
    devices = ([0] * n_gpus if loopback else list(range(n_gpus))) if single_process_multi else local
    rk = rt_amd.RenderKernel(W, H, spp, nb, rt_amd.Image(1, 1), P.triangles, P.materials,
                             P.emissive_triangle_indices, P.material_indices, None, rt_amd.BVH(P.triangles),
                             rt_amd.Image.from_rgb(sky), None, device=devices, loopback=loopback)
    rk.set_camera(rt_amd.Camera(cam17[:16], cam17[16]))
    if single_process_multi:
        frame = ShardedFrame(rk, 0, 1, device=dev)  # the root's full frame; the context shards it
    else:
        frame = ShardedFrame(rk, args.sim_rank if args.sim_world else rank, args.sim_world or world, device=dev)
    setup_s = time.time() - t0
    info = rk.bvh_info()
    log(f"[rank {rank}] setup {setup_s:.1f}s  devices {rk.n_devices}  frame {W}x{H}  bvh {info}")

    stream = torch.cuda.current_stream(dev).cuda_stream

    # counter pass (same workload, stats kernel variant) -> algorithmic bytes
    stats, stats_seq = None, None
    if not args.no_stats:
        rk.set_stats(True)
        frame.render(stream)
        torch.cuda.synchronize(dev)
        stats = rk.stats()
        log(f"[rank {rank}] counters {stats}  iterations {rk.last_iterations()}")
        if n_gpus == 1:
            # the same frame with unpaired occlusion walks: the box tests a walk must make
            # (the product pairs the stack top's node into a trip; same answers)
            rk.set_stats(2)
            frame.render(stream)
            torch.cuda.synchronize(dev)
            stats_seq = rk.stats()
        rk.set_stats(False)

    elapsed, full, kernel_ms, handovers = None, None, None, None
    if not args.roofline_only:
        for _ in range(args.warmup):
            frame.render(stream)
            if not args.sim_world:
                frame.gather()
        torch.cuda.synchronize(dev)

        rk.exact_handovers(reset=True)  # (waits for the device: before the timed region)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
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
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if world == 1 or dist.get_backend() == "nccl" else "cpu")
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        kernel_ms = float(np.mean(kms))
        handovers = rk.exact_handovers()  # (this rank's devices, the timed renders)

    # roofline pass: one lane (one stream), HIP events around every launch
    ktime, lane1_ms = None, None
    if not args.no_roofline_pass or args.roofline_only:
        rk.set_lanes(1)
        # (no fast lane either: its tail kernel would run on a second stream beside the
        # k_trace launches being timed; the pass is one stream, launches never overlap)
        rk.test_schedule(fast_k=0)
        frame.render(stream)  # (warm: the 1-lane wave buffers)
        torch.cuda.synchronize(dev)
        rk.kernel_timing(1)
        t1 = time.perf_counter()
        frame.render(stream)
        torch.cuda.synchronize(dev)
        lane1_ms = (time.perf_counter() - t1) * 1e3
        ktime = rk.kernel_timing(0)
        rk.set_lanes(0)  # (auto)
        rk.test_schedule(reset=1)  # (the product's schedule again)
        log(f"[rank {rank}] 1-lane render {lane1_ms:.1f} ms, kernel time per class {ktime}")

    samples_rank = frame.rows * W * spp if not single_process_multi else W * H * spp
    roofline = None
    if stats is not None and ktime is not None:
        tot_ms, launches = ktime["trace"]
        algo = algo_bytes(stats, "trace") / max(launches, 1)  # per launch (the stats pass rendered the same frame)
        avg_ms = tot_ms / max(launches, 1)
        achieved = algo / (avg_ms * 1e-3) / 1e9
        necessary = None
        if stats_seq is not None:
            necessary = algo_bytes(stats_seq, "trace") / max(launches, 1) / (avg_ms * 1e-3) / 1e9
        tkey = f"{args.config}_1lane"
        tsrc = traffic_source(tkey) if (n_gpus == 1 and not args.sim_world) else None
        # (the committed PMC bytes count only if they were taken on the running build)
        traffic = load_traffic(tkey) if (tsrc and tsrc["same_build"]) else None
        roofline = {"bound": "hbm", "kernel": "k_trace", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "achieved_necessary": None if necessary is None else round(necessary, 1),
                    "frac_necessary": None if necessary is None else round(necessary / HBM_PEAK_GBS, 4),
                    "necessary_model": "as byte_model, but the box tests of a counter render whose occlusion walks "
                                       "take one node per trip (rt_set_stats 2: the tests a walk must make; the "
                                       "product's paired trips also test the stack top's node, counted in frac)",
                    "occlusion_box_tests": None if stats_seq is None else
                    {"executed": stats["any_vol"] - stats.get("tail_any_vol", 0),
                     "necessary": stats_seq["any_vol"] - stats_seq.get("tail_any_vol", 0)},
                    "byte_model": "records a query must read (bench.py BYTES): 48 B per search-BVH box test (one "
                                  "child record + its 16-B oriented slab), 48 B per triangle test, 64 B per octree verification slab test, "
                                  "40 B per query (queue ray + result); box tests counted as executed, incl. the "
                                  "paired occlusion trips' stack-top node",
                    "traffic": traffic,
                    "traffic_source": tsrc,
                    # (the measured fabric bytes per launch / the launch's time / peak: what HBM actually
                    # moved, vs frac's algorithmic bytes; most records are served by L2 and the MALL;
                    # null when the committed profile is of another build)
                    "traffic_frac": (round(traffic / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                                     if (traffic and avg_ms > 0) else None),
                    "measured": "1-lane render after the timed steps, fast lane off (one stream: launches do "
                                "not overlap); HIP events around each launch",
                    "algo_bytes_per_launch": round(algo), "avg_launch_ms": round(avg_ms, 4),
                    "launches_per_render": launches,
                    "kernel_ms_per_render_1lane": {k: round(v[0], 2) for k, v in ktime.items()},
                    "render_ms_1lane": round(lane1_ms, 2),
                    "bytes_per_sample_all_kernels": round(sum(algo_bytes(stats, k) for k in ktime) / samples_rank, 1),
                    "closest_rays_per_sample": round(stats["rays"] / samples_rank, 3),
                    "any_rays_per_sample": round(stats["any_rays"] / samples_rank, 3)}
        # k_step against its byte models: the scene records alone (material, env texel, CDF
        # fences) and with the wavefront's slot records; traffic = committed FETCH_SIZE pass
        sm = step_model_bytes(stats, samples_rank)
        s_launches = ktime["step"][1]
        tr = load_traffic_class(f"{args.config}_1lane", "k_step") if (tsrc and tsrc["same_build"]) else None
        roofline["k_step"] = {
            "model_scene_bytes_per_launch": round(sm["scene"] / max(s_launches, 1)),
            "model_with_slots_bytes_per_launch": round((sm["scene"] + sm["slot"]) / max(s_launches, 1)),
            "avg_launch_ms": round(ktime["step"][0] / max(s_launches, 1), 4),
            "traffic": tr,
            "traffic_over_model_with_slots": round(tr / ((sm["scene"] + sm["slot"]) / max(s_launches, 1)), 3) if tr else None,
        }
        if kernel_ms:
            # all kernels' algorithmic bytes over the timed (3-lane, overlapped) render
            roofline["render_ms"] = round(kernel_ms, 3)
            roofline["frame_achieved_GBps"] = round(sum(algo_bytes(stats, k) for k in ktime) / (kernel_ms * 1e-3) / 1e9, 1)

    samples_per_step = W * H * spp if not args.sim_world else frame.rows * W * spp
    value = samples_per_step * args.steps / elapsed / 1e6 if elapsed else None

    cpu, parity = None, None
    if rank == 0 and world == 1 and n_gpus == 1 and not args.sim_world and not args.no_cpu_baseline and full is not None:
        omp = os.environ.get("OMP_NUM_THREADS")
        aff = len(os.sched_getaffinity(0))
        threads = min(int(omp or 0) or aff, aff)
        gpu_frame = full.cpu().numpy()
        cpu, parity, ref = cpu_baseline(P, sky, cam17, W, H, spp, nb, gpu_frame, threads, args.cpu_row_step)
        # where the core count comes from: the box sets OMP_NUM_THREADS (its CPU share), capped
        # by this process's affinity mask; the model string names the whole socket
        cpu["cores_source"] = (f"OMP_NUM_THREADS={omp} (the host's CPU share for this job) capped by the process's "
                               f"CPU affinity ({aff} CPUs, os.sched_getaffinity); os.cpu_count() = {os.cpu_count()}"
                               if omp else f"the process's CPU affinity ({aff} CPUs, os.sched_getaffinity); "
                                           f"os.cpu_count() = {os.cpu_count()}")
        if roofline is not None:
            roofline.update(ref)
            # the reference walk's bytes at this throughput: above 8 TB/s, because the search BVH + octree
            # verification does ~5x fewer node tests than the reference's octree walk
            roofline["ref_model_rate_GBps"] = round(ref["ref_model_bytes_per_sample"] * value * 1e6 / 1e9, 1)

    # N > 1: the gathered frame's rows against one device's render of the same rows (rank 0)
    if n_gpus > 1 and not args.sim_world and full is not None and rank == 0:
        solo = solo_kernel(rk, P, sky, cam17, dev, single_process_multi)
        parity = multi_parity(full, solo, dev, torch)
        if solo is not rk:
            del solo
    if world > 1:
        dist.barrier()

    strong = None
    if n_gpus > 1 and not args.sim_world and not args.no_strong_cfg4:
        strong = strong_cfg4(args, rk, P, sky, cam17, rank, world, dev, single_process_multi, torch, dist)
    if world > 1:
        dist.barrier()
    if rank == 0:
        if loopback:
            par = (f"REHEARSAL, not a measurement: one process, rt_create_multi_loopback over GPU 0 x {n_gpus}: "
                   f"rows y%{n_gpus}, device-copy exchange")
        elif single_process_multi:
            par = f"one process, rt_create_multi over {n_gpus} GPUs: rows y%{n_gpus} + RCCL scatter/gather"
        elif world > 1:
            par = f"{world} processes (torchrun): rows y%{world} per GPU + {dist.get_backend()} gather"
        else:
            par = "1 GPU"
        out = {
            "metric": "Msamples/sec (W×H×spp/s) at 1080p; per-channel L∞ vs CPU ref",
            "value": None if value is None else round(value, 3), "unit": "Msamples/s", "n_gpus": n_gpus,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": None if elapsed is None else round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": args.scaling,
            "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: procedural 1,000,002-triangle stand-in for the absent pbrt_dragon.obj and a "
                    "synthetic 2048x1024 env map (SURVEY.md §8d)",
            "config": {"workload": f"{args.config}: {desc}" + (f"; frame {W}x{H} = {n_gpus}x the config's pixels "
                                                                 f"(weak scaling)" if (W, H) != CONFIGS[args.config][3:5]
                                                                 else ""),
                       "W": W, "H": H, "spp": spp, "bounces": nb, "parallelism": par},
            "setup_s": round(setup_s, 2),
            "build": build_commit(),
            "roofline": roofline,
            "cpu_baseline": cpu,
            "parity": parity,
        }
        if handovers is not None:
            # the search-BVH walks' health: queries the timed renders handed to the exact octree
            # walk (ties, failed verifications, overflows), rank 0's devices; ~2e-6 per sample
            ms = samples_rank * args.steps / 1e6
            out["exact_handovers"] = {"per_frame": round(handovers / args.steps, 1),
                                      "per_msample": round(handovers / ms, 3) if ms > 0 else None}
        if strong is not None:
            out["strong_cfg4"] = strong
            # the north star's fixed-size figure beside the weak-scaling value: cfg4 (its 8-GPU
            # config) split over these N GPUs against the same frame on one, T_1 / (N T_N)
            out["scaling_fixed_size"] = {"config": "cfg4", "kind": "strong", "n_gpus": n_gpus,
                                         "efficiency": strong["efficiency"], "ms_1gpu": strong["ms_1gpu"],
                                         "ms_n_gpus": strong["ms_n_gpus"],
                                         "note": f"`value` is {args.scaling} scaling ({args.config}); this is "
                                                 f"cfg4's fixed-size split over the same {n_gpus} GPUs"}
        print(json.dumps(out), flush=True)
    # a frame that differs from the reference's (N = 1: the CPU port's rows, 1e-4 per channel
    # after tone-map; N > 1: the gathered frame against one device's, bitwise) fails the run
    bad = []
    if rank == 0 and parity is not None:
        if n_gpus > 1 and not parity.get("ok", False):
            bad.append(f"gathered frame rows differ from one device's ({parity})")
        if n_gpus == 1 and (parity["nan_mismatch"] or parity["linf"] > 1e-4):
            bad.append(f"frame rows differ from the CPU port's ({parity})")
    if rank == 0 and strong is not None and not strong["bitwise"]["ok"]:
        bad.append(f"strong_cfg4: the {n_gpus}-GPU frame differs from the 1-GPU frame ({strong['bitwise']})")
    if world > 1:
        dist.destroy_process_group()
    if bad:
        fail("PARITY FAILURE: " + "; ".join(bad), code=3)


if __name__ == "__main__":
    main()
