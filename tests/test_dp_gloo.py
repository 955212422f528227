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


class _Toy(torch.utils.data.Dataset):
    def __len__(self):
        return 23

    def __getitem__(self, i):
        return torch.full((80, 4), float(i)), torch.zeros(256)


def _loader_worker(rank, ws, port, q, tmp):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        torch.manual_seed(7 + rank)  # ranks' own RNGs differ; the shuffle seed comes from rank 0
        loader = torch.utils.data.DataLoader(_Toy(), batch_size=3, shuffle=True)
        sh = dp.shard_loader(loader)
        epochs = []
        for e in range(2):
            dp.set_epoch(sh, e)
            epochs.append([[int(v) for v in X[:, 0, 0]] for X, _ in sh])
        # save(): the BN buffers come from rank 0 and only rank 0 writes
        from autovc_amd.auto_encoder import AutoEncoder
        ae = AutoEncoder(device="cpu", verbose=False)
        for m in ae.modules():
            if isinstance(m, torch.nn.BatchNorm1d):
                m.running_mean.fill_(float(rank + 1))
        ae.configure_optimizer()
        calls = []
        real = torch.save
        torch.save = lambda obj, path: (calls.append(path), real(obj, path))
        os.chdir(tmp)  # save() paths are relative like the reference's (save_dir.strip("/"))
        try:
            ae.save("ae.pt", save_dir="ckpt")
        finally:
            torch.save = real
        bn = float(ae.encoder.convolutions[0][1].running_mean[0])
        q.put((rank, epochs, len(calls), bn))
    except Exception as e:  # report instead of leaving the parent waiting
        q.put((rank, repr(e), -1, -1.0))
        raise
    finally:
        dist.destroy_process_group()


def test_learn_sharding_and_save_world2(tmp_path):
    """learn()'s data-parallel pieces: dp.shard_loader gives every rank a disjoint, equal-size
    share of the caller's loader with the same batch size, reshuffled per epoch from one seed
    broadcast by rank 0; AutoEncoder.save broadcasts rank 0's BN buffers and writes on rank 0 only."""
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    (tmp_path / "ckpt").mkdir()
    procs = [ctx.Process(target=_loader_worker, args=(r, ws, port, q, str(tmp_path))) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in range(ws)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    assert all(r[2] >= 0 for r in res), res
    assert all(p.exitcode == 0 for p in procs)
    (_, e0, calls0, bn0), (_, e1, calls1, bn1) = res
    for e in range(2):
        a = [i for b in e0[e] for i in b]
        b = [i for b in e1[e] for i in b]
        assert len(a) == len(b) == 11 and not set(a) & set(b)
        assert [len(x) for x in e0[e]] == [len(x) for x in e1[e]] == [3, 3, 3, 2]
    assert e0[0] != e0[1]  # reshuffled per epoch
    assert (calls0, calls1) == (1, 0) and bn0 == bn1 == 1.0
    assert (tmp_path / "ckpt" / "ae.pt").exists()


def _flat_model(seed):
    """A small stack whose first block is used twice per loss (like the encoder, which the
    reference loss runs again on the postnet output), with flat parameter/gradient storage."""
    torch.manual_seed(seed)
    net = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 32),
                              torch.nn.Tanh(), torch.nn.Linear(32, 16))
    params = list(net.parameters())
    total = sum(p.numel() for p in params)
    flat, grad, off = torch.empty(total), torch.zeros(total), 0
    with torch.no_grad():
        for p in params:
            n = p.numel()
            flat[off:off + n].copy_(p.reshape(-1))
            p.data = flat[off:off + n].view_as(p)
            p.grad = grad[off:off + n].view_as(p)
            off += n
    return net, params, grad


def _loss(net, x):
    y = net(x)
    return (y ** 2).mean() + net[0](y).abs().mean()  # block 0 used a second time


def _bucket_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        net, params, grad = _flat_model(0)
        torch.manual_seed(50 + rank)
        x = torch.randn(8, 16)
        # reference: plain backward, then one all-reduce of the whole flat gradient
        _loss(net, x).backward()
        expect = dp.average_gradients(grad.clone())
        grad.zero_()
        # the product path: buckets issued from the post-accumulate hooks during backward
        red = dp.GradBuckets(params, grad, bucket_bytes=4 * 300)
        with red.armed():
            _loss(net, x).backward()
        log = list(red.launch_log)
        red.finish()
        same = torch.equal(grad, expect)
        # disarmed: a backward outside train_step issues no collective
        grad.zero_()
        _loss(net, x).backward()
        quiet = len(red.handles) == 0 and red.launch_log == log
        q.put((rank, same, red.buckets, log, quiet, grad.numel()))
    finally:
        dist.destroy_process_group()


def test_grad_buckets_overlap_world2():
    """dp.GradBuckets gives exactly the single flat all-reduce's mean, its buckets cover the flat
    gradient back to front, and buckets are issued while backward still has gradients pending."""
    ws = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(ws))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, same, buckets, log, quiet, total in res:
        assert same, rank
        assert quiet, rank
        assert len(buckets) >= 3
        assert buckets[0][1] == total and buckets[-1][0] == 0
        assert all(buckets[i][0] == buckets[i + 1][1] for i in range(len(buckets) - 1))
        assert [b for b, _ in log] == list(range(len(log)))   # strictly in bucket order
        assert log[0][1] > 0, "first bucket was only issued after backward finished"
    assert res[0][3] == res[1][3]  # same issue order on both ranks


def test_nccl_branch_places_collective_tensors_on_the_gpu(monkeypatch):
    """The nccl (RCCL) branch, forced on CPU: RCCL has no CPU backend, so collective_device() must
    name the current GPU, and broadcast_seed / params_in_sync must hand the collectives tensors on
    that device (the round-2 fix of the seed broadcast).  The GPU itself is stood in for
    by a recorder: the collectives record the device of what they are given."""
    monkeypatch.setattr(dp, "world", lambda: 2)
    monkeypatch.setattr(dist, "get_backend", lambda *a, **k: "nccl")
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 5)
    assert dp.collective_device() == torch.device("cuda", 5)

    # the helpers must route through collective_device(); a CPU-only box cannot hold a CUDA
    # tensor, so the recorder hands out a stand-in device and checks every collective sees it
    stand_in = torch.device("cpu")
    asked, seen = [], []
    monkeypatch.setattr(dp, "collective_device", lambda: asked.append(1) or stand_in)
    monkeypatch.setattr(dist, "broadcast", lambda t, src, *a, **k: seen.append(("broadcast", t.device)))
    monkeypatch.setattr(dist, "all_reduce", lambda t, *a, **k: seen.append(("all_reduce", t.device)))
    seed = dp.broadcast_seed()
    assert isinstance(seed, int) and 0 <= seed < 2 ** 62
    assert dp.params_in_sync(torch.randn(64))
    assert len(asked) == 2
    assert [s[0] for s in seen] == ["broadcast", "all_reduce", "all_reduce"]
    assert all(d == stand_in for _, d in seen)
