"""Data-parallel training support for the Generator (BASELINE config 4).

One process per GPU.  Each rank runs the reference training step on its own shard of utterance
minibatches; the only exchange is ONE all-reduce (sum, then /world) of the flat 113.7 MB
gradient per step, after which every rank applies the same fused clip/Adam/EMA update, so the
parameters stay bit-identical across ranks.  BatchNorm batch statistics stay per rank (no
SyncBN); the running buffers are broadcast from rank 0 before a checkpoint is written.
With the nccl backend torch.distributed is RCCL over xGMI on MI355X.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def average_gradients(flat_grad: torch.Tensor) -> torch.Tensor:
    """In-place mean of the flat gradient over all ranks (one collective)."""
    ws = world()
    if ws > 1:
        dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM)
        flat_grad.div_(ws)
    return flat_grad


def broadcast_buffers(module: torch.nn.Module, src: int = 0) -> None:
    """Make every rank's BN running statistics equal to rank `src`'s (before saving)."""
    if world() > 1:
        for b in module.buffers():
            dist.broadcast(b, src)


def params_in_sync(flat_param: torch.Tensor) -> bool:
    """True when every rank holds bitwise the same parameters (max/min all-reduce of a checksum)."""
    if world() == 1:
        return True
    v = flat_param.detach().double()
    ck = torch.stack([v.sum(), (v * v).sum(), v.abs().max()])
    lo, hi = ck.clone(), ck.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    return bool(torch.equal(lo, hi))


def shard_indices(n: int, r: int | None = None, ws: int | None = None) -> range:
    """Contiguous, equal-size shard of n utterance minibatches for rank r (drops the remainder
    so every rank runs the same number of steps, as the collective requires)."""
    r = rank() if r is None else r
    ws = world() if ws is None else ws
    per = n // ws
    return range(r * per, (r + 1) * per)
