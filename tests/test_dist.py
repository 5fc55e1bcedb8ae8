"""Multi-process framebuffer sharding + gather (rt_amd.dist) with the gloo
backend on CPU, world_size 2 and 3, using the hostsim build of the kernel:
the gathered frame must equal the reference's golden single-process render
bit for bit."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    import conftest  # noqa: F401  (paths)
    import json
    import torch.distributed as dist
    import rt_cases
    from rt_amd.dist import ShardedFrame
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import numpy as np_
        manifest = json.load(open(os.path.join(here, "golden", "manifest.json")))
        cams = dict(np_.load(os.path.join(here, "golden", "cameras.npz")))
        e = rt_cases.golden_case("cornell32_128", manifest)
        rk, _ = rt_cases.make_kernel(e, cams, hostsim=True)
        f = ShardedFrame(rk, rank, world, device="cpu")
        f.render()
        full = f.gather(dst=0)
        if rank == 0:
            # bench.py's N > 1 self-check: the gathered frame's rows against one device's
            # render of the same rows (bitwise), and the same check on a frame whose rows
            # were permuted (as a broken gather would leave them) must fail
            import torch
            sys.path.insert(0, os.path.dirname(here))
            import bench
            good = bench.multi_parity(full, rk, "cpu", torch, rows_every=5, first=2)
            bad_frame = full.clone()
            bad_frame[[2, 7]] = full[[7, 2]]
            bad = bench.multi_parity(bad_frame, rk, "cpu", torch, rows_every=5, first=2)
            q.put((full.numpy().copy(), good["ok"], good["bitwise_fraction"], bad["ok"], bad["bitwise_fraction"]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_render_matches_golden(world):
    import conftest
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, good_ok, good_frac, bad_ok, bad_frac = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want = conftest.load_golden("render_cornell32_128.npz")["rgba"]
    np.testing.assert_array_equal(full.view(np.uint32), want.view(np.uint32))
    assert good_ok and good_frac == 1.0
    assert not bad_ok and bad_frac < 1.0
