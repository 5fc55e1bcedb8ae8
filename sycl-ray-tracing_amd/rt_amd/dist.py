"""Multi-GPU render driver: framebuffer rows shard across ranks, one process
per GPU, and the tone-mapped HDR shards are gathered to one rank over RCCL
(torch.distributed backend "nccl" on ROCm) — SURVEY.md §8(e).

Partition: image row y belongs to rank y mod world (row-interleaved, so the
sky rows and the object rows spread evenly over the GPUs). Pixels are
independent (the RNG seed is 31 + x*y*spp, render_kernel.cpp:77), so the
gathered frame is bit-identical to a single-GPU render at any world size.

Exchange: one gather of each rank's [rows_local, W, 4] f32 shard to the
destination rank, then an un-permute of the interleaved rows. At 4K that is
16.6 MB per rank over xGMI; the render itself is the cost.

The same code runs on CPU tensors with the gloo backend and the hostsim
build of the kernel (tests/test_dist.py), because rt_render_device only needs
a pointer in the memory space of the library that renders.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def rows_of(height: int, rank: int, world: int) -> int:
    return len(range(rank, height, world))


class ShardedFrame:
    """This rank's share of a RenderKernel frame.

    kernel: rt_amd.RenderKernel bound to this rank's device (or hostsim).
    device: torch device of the shard ("cuda:k" for the product, "cpu" for hostsim).
    """

    def __init__(self, kernel, rank: int = 0, world: int = 1, device: str | torch.device = "cuda"):
        self.k = kernel
        self.rank, self.world = rank, world
        self.W, self.H = kernel.width, kernel.height
        self.rows_max = rows_of(self.H, 0, world)
        self.rows = rows_of(self.H, rank, world)
        self.device = torch.device(device)
        # the reference's fresh Image: black, alpha 1 (image.h:27-33)
        self.init = torch.zeros((self.rows_max, self.W, 4), dtype=torch.float32, device=self.device)
        self.init[..., 3] = 1.0
        self.shard = self.init.clone()

    def render(self, stream: int | None = None, reset: bool = True) -> torch.Tensor:
        """Renders this rank's rows into self.shard (accumulating into its
        contents like RenderKernel::render mutates its Image, unless reset)."""
        if reset:
            self.shard.copy_(self.init)
        if self.device.type == "cuda" and stream is None:
            stream = torch.cuda.current_stream(self.device).cuda_stream
        if self.rows:
            self.k.render_device(self.shard.data_ptr(), self.rank, self.world, stream)
        return self.shard

    def gather(self, dst: int = 0, group=None) -> torch.Tensor | None:
        """Gathers every rank's shard to `dst` and returns the [H, W, 4] frame
        there (None elsewhere)."""
        if self.world == 1:
            return self.shard[: self.rows]
        src = self.shard
        if src.is_cuda and dist.get_backend(group) == "gloo":  # (gloo gathers host tensors: rehearsals)
            src = src.cpu()
        parts = [torch.empty_like(src) for _ in range(self.world)] if self.rank == dst else None
        dist.gather(src, parts, dst=dst, group=group)
        if parts is not None and parts[0].device != self.device:
            parts = [x.to(self.device) for x in parts]
        if self.rank != dst:
            return None
        full = torch.empty((self.H, self.W, 4), dtype=torch.float32, device=self.device)
        for r, p in enumerate(parts):
            full[r:: self.world] = p[: rows_of(self.H, r, self.world)]
        return full
