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


def broadcast_seed(src: int = 0) -> int:
    """A 63-bit seed drawn from rank `src`'s torch RNG, the same on every rank."""
    seed = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64)
    if world() > 1:
        dist.broadcast(seed, src)
    return int(seed.item())


def shard_loader(loader, seed: int | None = None):
    """The caller's DataLoader (voice_converter.py:282-285 builds it: dataloader.py:123-144,
    batch_size utterances per batch, shuffle=True, zero-padding collate_fn) re-built over a
    DistributedSampler: rank r loads only its own 1/world of the utterances, in batches of the
    same batch_size (the per-GPU batch of BASELINE config 4), every rank runs the same number of
    steps (drop_last on the shard), and all ranks draw their shuffles from one seed broadcast from
    rank 0 (call set_epoch(epoch) on the returned loader's sampler each epoch, as learn() does).
    World 1: the loader itself."""
    from torch.utils.data import DataLoader, DistributedSampler, RandomSampler
    if world() == 1:
        return loader
    if not isinstance(loader, DataLoader) or loader.batch_size is None:
        raise TypeError("data-parallel learn() needs a torch DataLoader with a batch_size (dataloader.py:137)")
    seed = broadcast_seed() if seed is None else seed
    sampler = DistributedSampler(loader.dataset, num_replicas=world(), rank=rank(),
                                 shuffle=isinstance(loader.sampler, RandomSampler), seed=seed, drop_last=True)
    return DataLoader(loader.dataset, batch_size=loader.batch_size, sampler=sampler,
                      collate_fn=loader.collate_fn, num_workers=loader.num_workers,
                      pin_memory=loader.pin_memory, drop_last=loader.drop_last)


def set_epoch(loader, epoch: int) -> None:
    from torch.utils.data import DistributedSampler
    if isinstance(getattr(loader, "sampler", None), DistributedSampler):
        loader.sampler.set_epoch(epoch)


def shard_indices(n: int, r: int | None = None, ws: int | None = None) -> range:
    """Contiguous, equal-size shard of n utterance minibatches for rank r (drops the remainder
    so every rank runs the same number of steps, as the collective requires)."""
    r = rank() if r is None else r
    ws = world() if ws is None else ws
    per = n // ws
    return range(r * per, (r + 1) * per)
