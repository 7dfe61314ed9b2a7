"""One-process-per-GPU helpers for the benchmark (torchrun env contract).

The exporter itself never uses a collective library; RCCL
(torch.distributed backend ``nccl`` on ROCm) appears only here, to line the
benchmark ranks up (barriers) and reduce their timings (MAX over ranks) — and
as an optional xGMI load.  CPU runs (mock provider, tests) use ``gloo``.
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass
class Ctx:
    rank: int = 0
    local_rank: int = 0
    world: int = 1
    local_world: int = 1
    backend: str = ""
    cuda: bool = False
    cpu_group: object = None  # gloo group: waits that must not put a kernel on the GPU

    @property
    def is_dist(self) -> bool:
        return self.world > 1


def init_from_env(use_cuda: bool) -> Ctx:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    ctx = Ctx(rank, local_rank, world, local_world, "", use_cuda)
    if world > 1:
        import torch
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if use_cuda:
            torch.cuda.set_device(local_rank)
            ctx.backend = "nccl"  # RCCL over xGMI on ROCm
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
            # An RCCL barrier is a kernel that spins on every GPU until the last rank
            # arrives: a rank waiting on it is not idle.  Waits that must leave the
            # GPUs idle (bench phase Q) go through a CPU-only gloo group.
            ctx.cpu_group = dist.new_group(backend="gloo")
        else:
            ctx.backend = "gloo"
            dist.init_process_group("gloo")
    elif use_cuda:
        import torch

        torch.cuda.set_device(local_rank)
    return ctx


def barrier(ctx: Ctx) -> None:
    if ctx.is_dist:
        import torch.distributed as dist

        if ctx.cuda:
            import torch

            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def cpu_barrier(ctx: Ctx) -> None:
    """Barrier that launches nothing on the GPU (gloo over TCP)."""
    if ctx.is_dist:
        import torch.distributed as dist

        dist.barrier(group=ctx.cpu_group) if ctx.cpu_group is not None else dist.barrier()


def all_reduce(ctx: Ctx, values: list[float], op: str = "max") -> list[float]:
    if not ctx.is_dist:
        return list(values)
    import torch
    import torch.distributed as dist

    dev = torch.device("cuda", torch.cuda.current_device()) if ctx.cuda else torch.device("cpu")
    t = torch.tensor(values, dtype=torch.float64, device=dev)
    dist.all_reduce(t, op={"max": dist.ReduceOp.MAX, "sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN}[op])
    return [float(x) for x in t.cpu().tolist()]


def all_gather_object(ctx: Ctx, obj):
    if not ctx.is_dist:
        return [obj]
    import torch.distributed as dist

    out = [None] * ctx.world
    dist.all_gather_object(out, obj)
    return out


def broadcast_object(ctx: Ctx, obj, src: int = 0):
    if not ctx.is_dist:
        return obj
    import torch.distributed as dist

    box = [obj]
    dist.broadcast_object_list(box, src=src)
    return box[0]


def destroy(ctx: Ctx) -> None:
    if ctx.is_dist:
        import torch.distributed as dist

        dist.destroy_process_group()
