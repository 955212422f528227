"""The bucketed gradient exchange over RCCL itself (dp.GradBuckets with the nccl backend).

The driver's multi-GPU run is the only place two RCCL ranks meet; the test box has one MI355X and
RCCL refuses two ranks on one device.  What does run here is a world-1 nccl process group: every
bucket's `dist.all_reduce(async_op=True)` then launches a real RCCL kernel on the GPU, with the
same stream semantics as at N ranks -- issued from the post-accumulate / param_ready hooks while
backward runs, held back while a persistent BPTT is still to come, issued on the side stream behind
the library's after-launch event (avc_persist_notify), and waited for by a stream wait in finish().
A sum over one rank is the identity and /1 is exact, so two C4-plan training steps (B = 256,
T = 128: lstm1 forward + three persistent BPTTs) through that exchange must leave every parameter,
the EMA copy and the BN buffers bit-identical to the same steps without any exchange.  Reference training
loop: autovc/auto_encoder/model.py:303-321."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

B, T = 256, 128


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, q, out_dir, comm):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        if comm:
            dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        from autovc_amd import _lib, dp
        from autovc_amd.auto_encoder import AutoEncoder
        from autovc_amd.weights import onehot_embedding, synthetic_mel, torch_state_dict
        ae = AutoEncoder(device=dev, verbose=False)
        ae.load_state_dict(torch_state_dict(0))
        ae.to(dev).train()
        ae.configure_optimizer()
        if comm:  # the real bucketed exchange (dist.all_reduce on the nccl group), world 1
            ae.grad_comm = dict(world_size=1)
        launches = _lib.persist_launches(dev)
        rec = {"losses": [], "issued": 0}
        for s in range(2):
            X = torch.from_numpy(synthetic_mel(90 + s, B, T)).to(dev)
            c = torch.from_numpy(onehot_embedding(B, offset=5 * s)).to(dev)
            loss, _ = ae.train_step(X, c)
            rec["losses"].append(float(loss))
            if comm:
                rec["issued"] += len(ae._reducer.launch_log)
        ae.check_health()
        rec["persist"] = _lib.persist_launches(dev) - launches
        if comm:
            rec["backend"] = dist.get_backend()
            rec["buckets"] = len(ae._reducer.buckets)
            rec["in_sync"] = dp.params_in_sync(ae._flat_param)
        torch.save({"flat": ae._flat_param.cpu(), "ema": ae.avg_params.cpu(),
                    "state": {k: v.cpu() for k, v in ae.state_dict().items()}},
                   os.path.join(out_dir, f"comm{int(comm)}.pt"))
        q.put(rec)
        if comm:
            dist.destroy_process_group()
    except Exception as e:
        q.put({"error": repr(e)})
        raise


def _run(tmp_path, comm):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q, str(tmp_path), comm))
    p.start()
    rec = q.get(timeout=300)
    p.join(timeout=60)
    assert "error" not in rec, rec
    assert p.exitcode == 0
    return rec


@pytest.mark.timeout(600)
def test_rccl_bucketed_exchange_world1_is_exact(tmp_path):
    plain = _run(tmp_path, False)
    rccl = _run(tmp_path, True)
    print(f"RCCL world 1: backend {rccl['backend']}, {rccl['buckets']} buckets, {rccl['issued']} all-reduces "
          f"issued over 2 steps, persistent launches {rccl['persist']}; losses {rccl['losses']} vs {plain['losses']}")
    assert rccl["backend"] == "nccl"
    assert rccl["issued"] == 2 * rccl["buckets"]  # every bucket went through RCCL on every step
    assert rccl["persist"] >= 8 and rccl["persist"] == plain["persist"]  # the co-residency path ran
    assert rccl["in_sync"]
    assert rccl["losses"] == plain["losses"]
    a = torch.load(tmp_path / "comm0.pt", weights_only=True)
    b = torch.load(tmp_path / "comm1.pt", weights_only=True)
    assert torch.equal(a["flat"], b["flat"])
    assert torch.equal(a["ema"], b["ema"])
    for k in a["state"]:
        assert torch.equal(a["state"][k], b["state"][k]), k
