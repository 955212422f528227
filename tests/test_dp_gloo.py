"""Data-parallel orchestration on CPU with the gloo backend, world_size 2 (the GPU path uses the
same code over RCCL).  Checks: gradient averaging is one exact mean; ranks that apply the same
averaged gradient with the oracle's Adam stay bit-identical; BN buffers are broadcast from rank 0;
shards are equal-sized and disjoint."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from autovc_amd import dp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        torch.manual_seed(100 + rank)
        g = torch.randn(1000, dtype=torch.float32)
        allg = [torch.zeros_like(g) for _ in range(ws)]
        dist.all_gather(allg, g)
        expect = torch.stack(allg).sum(0) / ws
        dp.average_gradients(g)
        ok_mean = torch.allclose(g, expect, rtol=0, atol=1e-6)
        # identical updates keep ranks in sync; a per-rank perturbation is detected
        torch.manual_seed(0)
        p = torch.randn(1000)
        for step in range(3):
            torch.manual_seed(1000 * step + rank)
            gr = torch.randn(1000)
            dp.average_gradients(gr)
            p -= 1e-3 * gr / (gr.abs() + 1e-8)
        in_sync = dp.params_in_sync(p)
        p2 = p.clone()
        if rank == 1:
            p2[0] += 1e-3
        detects = not dp.params_in_sync(p2)
        bn = torch.nn.BatchNorm1d(4)
        bn.running_mean.fill_(float(rank))
        dp.broadcast_buffers(bn)
        bcast = float(bn.running_mean[0]) == 0.0
        sh = list(dp.shard_indices(11))
        q.put((rank, ok_mean, in_sync, detects, bcast, sh))
    finally:
        dist.destroy_process_group()


def test_dp_gloo_world2():
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(ws)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    for rank, ok_mean, in_sync, detects, bcast, sh in res:
        assert ok_mean and in_sync and detects and bcast, (rank, ok_mean, in_sync, detects, bcast)
    assert res[0][5] == list(range(0, 5)) and res[1][5] == list(range(5, 10))


def test_shard_single_process():
    assert list(dp.shard_indices(7, 0, 1)) == list(range(7))
    assert dp.world() == 1 and dp.rank() == 0
