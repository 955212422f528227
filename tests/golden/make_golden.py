"""Generate the golden fixtures from the REFERENCE AutoEncoder (run in the build container only).

The reference has no tests and no golden vectors of its own, so parity is pinned
here: the reference class autovc/auto_encoder/model.py:27 is imported straight from
/root/reference with `wandb` and the package __init__ stubbed (SURVEY §8c loader recipe), loaded
with seeded synthetic weights (autovc_amd.weights, seed 0), and run on seeded inputs.  Only
small inputs/outputs are written (tests/golden/*.npz); the weights are re-generated from the
seed and checked against a stored checksum.

    python tests/golden/make_golden.py          # rewrites tests/golden/*.npz

Nothing on the GPU box runs this file (it needs /root/reference).
"""
from __future__ import annotations

import importlib
import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from autovc_amd.weights import (onehot_embedding, state_checksum, synthetic_embedding,  # noqa: E402
                                synthetic_mel, torch_state_dict)

REF = "/root/reference"


def load_reference():
    sys.modules.setdefault("wandb", types.ModuleType("wandb"))
    for name, path in [("autovc", REF + "/autovc"), ("autovc.auto_encoder", REF + "/autovc/auto_encoder")]:
        m = types.ModuleType(name)
        m.__path__ = [path]
        sys.modules[name] = m
    model = importlib.import_module("autovc.auto_encoder.model")
    hp = importlib.import_module("autovc.utils.hparams")
    return model.AutoEncoder, hp.AutoEncoderParams


def make_ae(AE, seed=0):
    torch.manual_seed(1234)
    ae = AE(device="cpu", verbose=False)
    sd = torch_state_dict(seed)
    ae.load_state_dict(sd)
    return ae, state_checksum(sd)


def bn_buffers(ae):
    out = {}
    for k, v in ae.state_dict().items():
        if k.endswith("running_mean") or k.endswith("running_var") or k.endswith("num_batches_tracked"):
            out["bn/" + k] = v.detach().numpy().copy()
    return out


def fwd_case(AE, B, T, train, x_seed, lengths=None):
    ae, ck = make_ae(AE)
    ae.train(train)
    x = synthetic_mel(x_seed, B, T)
    if lengths is not None:  # collate_fn zero-pad semantics (dataloader.py:112-121)
        for i, L in enumerate(lengths):
            x[i, :, L:] = 0.0
    c_org = synthetic_embedding(x_seed + 100, B)
    c_trg = synthetic_embedding(x_seed + 200, B)
    with torch.no_grad():
        mel, mel_post, codes = ae(torch.from_numpy(x), torch.from_numpy(c_org), torch.from_numpy(c_trg))
    d = dict(x=x, c_org=c_org, c_trg=c_trg, mel=mel.numpy(), mel_post=mel_post.numpy(),
             codes=codes.numpy(), train=np.array(train), weights_checksum=np.array(ck), seed=np.array(0))
    if lengths is not None:
        d["lengths"] = np.array(lengths)
    d.update(bn_buffers(ae))
    return d


def batch_forward_case(AE):
    ae, ck = make_ae(AE)
    ae.train(True)
    M, N = 5, 128
    batch = synthetic_mel(7, M, N)
    c_org = synthetic_embedding(107, 1)
    c_trg = synthetic_embedding(207, 1)
    with torch.no_grad():
        out = ae.batch_forward(torch.from_numpy(batch), torch.from_numpy(c_org), torch.from_numpy(c_trg), overlap=0.5)
    return dict(batch=batch, c_org=c_org, c_trg=c_trg, out=out.numpy(), overlap=np.array(0.5),
                weights_checksum=np.array(ck))


def c1_case(AE):
    """BASELINE config 1 / SURVEY §8c: a (1, 80, 128) mel of data/samples/mette_183.wav through the
    reference Generator on the CPU.  The mel comes from the float64 restatement of the reference's
    librosa frontend (oracle/audio_oracle.py; librosa is absent, so that step is unpinned) applied
    to the committed waveform head (tests/golden/mette_183_head.npz), first 128 frames; the
    Generator outputs are the reference class's own.  Both BN modes."""
    from oracle import audio_oracle as ao
    head = np.load(os.path.join(HERE, "mette_183_head.npz"))
    mel = ao.mel_spec_auto_encoder(head["wav"].astype(np.float64), sr=int(head["sr"]))[:, :128]
    x = np.asarray(mel, dtype=np.float32)[None]
    c_org = synthetic_embedding(301, 1)
    c_trg = synthetic_embedding(302, 1)
    d = dict(x=x, c_org=c_org, c_trg=c_trg, weights_checksum=np.array(0), seed=np.array(0))
    for train in (True, False):
        ae, ck = make_ae(AE)
        ae.train(train)
        with torch.no_grad():
            mel_o, post, codes = ae(torch.from_numpy(x), torch.from_numpy(c_org), torch.from_numpy(c_trg))
        tag = "train" if train else "eval"
        d[f"mel_{tag}"], d[f"mel_post_{tag}"], d[f"codes_{tag}"] = mel_o.numpy(), post.numpy(), codes.numpy()
        d["weights_checksum"] = np.array(ck)
    return d


TRACE_TENSORS = ["encoder.convolutions.0.0.conv.weight", "encoder.lstm.weight_hh_l0_reverse",
                 "decoder.lstm2.weight_hh_l1", "decoder.linear_projection.linear_layer.bias",
                 "postnet.convolutions.4.1.weight"]


def train_case(AE, hparams, steps=3, B=4, T=128):
    """Replays model.py:303-321 with the reference's own forward/_loss/Adam/clip/EMA, then checks
    the same batches through the reference `learn()` give the same parameters."""
    ae, ck = make_ae(AE)
    xs = [synthetic_mel(30 + s, B, T) for s in range(steps)]
    cs = [onehot_embedding(B, offset=4 * s) for s in range(steps)]
    opt_params = {k: v for k, v in hparams["optimizer"].items() if k not in ("lr_scheduler", "n_warmup_steps")}

    ae.train()
    ae.criterion1 = torch.nn.MSELoss()
    ae.criterion2 = torch.nn.L1Loss()
    ae.optimiser = torch.optim.Adam(ae.parameters(), **opt_params)
    avg = ae.flatten_params()
    losses, norms = [], []
    for s in range(steps):
        X, c = torch.from_numpy(xs[s]), torch.from_numpy(cs[s])
        out_dec, out_post, codes = ae(X, c, c)
        loss = ae._loss(X=X, c_org=c, out_decoder=out_dec, out_postnet=out_post, content_codes=codes)
        ae.optimiser.zero_grad()
        loss.backward()
        norms.append(float(torch.nn.utils.clip_grad_norm_(ae.parameters(), max_norm=1)))
        ae.optimiser.step()
        avg = 0.9999 * avg + (1 - 0.9999) * ae.flatten_params()
        losses.append(float(loss.detach()))
    sd = ae.state_dict()
    d = dict(losses=np.array(losses), grad_norms=np.array(norms), weights_checksum=np.array(ck),
             ema_sum=np.array(float(avg.double().sum())), ema_abs=np.array(float(avg.double().abs().sum())),
             B=np.array(B), T=np.array(T), steps=np.array(steps))
    for s in range(steps):
        d[f"x{s}"] = xs[s]
        d[f"c{s}"] = cs[s]
    for k, v in sd.items():
        a = v.detach().double().numpy()
        d["sum/" + k] = np.array(a.sum())
        d["abs/" + k] = np.array(np.abs(a).sum())
    for k in TRACE_TENSORS:
        d["val/" + k] = sd[k].detach().numpy().ravel()[:256].copy()

    # Cross-check against the reference training loop itself (model.py:218-361).
    ae2, _ = make_ae(AE)
    hp_opt = hparams["optimizer"]
    saved = dict(hp_opt)
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        os.makedirs("ckpt")
        try:
            ae2.learn([(torch.from_numpy(xs[s]), torch.from_numpy(cs[s])) for s in range(steps)],
                      n_epochs=1, save_dir="ckpt", model_name="m.pt")
        finally:
            os.chdir(cwd)
            hp_opt.clear()
            hp_opt.update(saved)
    for k, v in ae2.state_dict().items():
        assert torch.equal(v, sd[k]), f"learn() diverged from the replayed loop at {k}"
    return d


def curve_case(AE, hparams, steps=12, B=256, T=128):
    """The training-loss curve of BASELINE config 3 (B = 256, T = 128) from the reference's own
    learn() (model.py:218-361), one epoch over `steps` seeded batches: per-step loss and pre-clip
    gradient norm, recorded by wrapping the instance's _loss and torch.nn.utils.clip_grad_norm_
    (the values the loop computes; nothing else changes).  Only the batch seeds and the two curves
    are stored.  The same steps are also run through the oracle's Trainer in float64 (exact
    arithmetic up to 1e-16): its distance from the fp32 reference is the run-to-run spread any
    correct fp32 implementation has, which the GPU test's tolerance is built from."""
    seeds = [500 + s for s in range(steps)]

    def batch(s):
        return (torch.from_numpy(synthetic_mel(seeds[s], B, T)), torch.from_numpy(onehot_embedding(B, offset=s)))

    ae, ck = make_ae(AE)
    losses, norms = [], []
    inner_loss = ae._loss

    def loss_rec(*a, **k):
        out = inner_loss(*a, **k)
        losses.append(float(out.detach()))
        return out
    ae._loss = loss_rec
    clip = torch.nn.utils.clip_grad_norm_

    def clip_rec(*a, **k):
        n = clip(*a, **k)
        norms.append(float(n))
        return n
    hp_opt = hparams["optimizer"]
    saved = dict(hp_opt)
    torch.nn.utils.clip_grad_norm_ = clip_rec
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        os.makedirs("ckpt")
        try:
            ae.learn([batch(s) for s in range(steps)], n_epochs=1, save_dir="ckpt", model_name="m.pt")
        finally:
            torch.nn.utils.clip_grad_norm_ = clip
            os.chdir(cwd)
            hp_opt.clear()
            hp_opt.update(saved)
    assert len(losses) == steps and len(norms) == steps

    from oracle import autovc_oracle as orc
    sd64 = {k: v.double() if v.is_floating_point() else v for k, v in torch_state_dict(0).items()}
    tr = orc.Trainer(sd64)
    l64, n64 = [], []
    for s in range(steps):
        X, c = batch(s)
        l, g = tr.grads(X.double(), c.double(), tr.bufs)
        l64.append(l)
        n64.append(tr._apply(list(g)))
    return dict(seeds=np.array(seeds), onehot_offsets=np.arange(steps), B=np.array(B), T=np.array(T),
                losses=np.array(losses), grad_norms=np.array(norms), losses_f64=np.array(l64),
                grad_norms_f64=np.array(n64), weights_checksum=np.array(ck), lr=np.array(saved.get("lr", 1e-3)))


def checkpoint_layout_case(AE, hparams, B=2, T=64):
    """The checkpoint dict the reference's learn() writes through save() (model.py:158-176): one
    training step, then the file's structure (model_state keys/shapes/dtypes, optimizer_state's
    torch.optim.Adam layout and param_groups, step) and a few value sums.  Written as JSON."""
    ae, ck = make_ae(AE)
    hp_opt = hparams["optimizer"]
    saved = dict(hp_opt)
    X, c = torch.from_numpy(synthetic_mel(91, B, T)), torch.from_numpy(onehot_embedding(B))
    with tempfile.TemporaryDirectory() as tmp:
        cwd = os.getcwd()
        os.chdir(tmp)
        os.makedirs("ckpt")
        try:
            ae.learn([(X, c)], n_epochs=1, save_dir="ckpt", model_name="m.pt")
            ckpt = torch.load("ckpt/m.pt", weights_only=True)
        finally:
            os.chdir(cwd)
            hp_opt.clear()
            hp_opt.update(saved)
    ms = ckpt["model_state"]
    opt = ckpt["optimizer_state"]
    st0 = opt["state"][0]
    return {
        "top_keys": sorted(ckpt.keys()),
        "step": ckpt["step"],
        "model_state": [[k, list(v.shape), str(v.dtype)] for k, v in ms.items()],
        "optimizer_state_keys": sorted(opt.keys()),
        "n_state": len(opt["state"]),
        "state_entry_keys": sorted(st0.keys()),
        "state_step_dtype": str(st0["step"].dtype), "state_step_shape": list(st0["step"].shape),
        "param_groups": [{k: (len(v) if k == "params" else v) for k, v in g.items()} for g in opt["param_groups"]],
        "exp_avg_abs_sum": float(sum(float(s["exp_avg"].double().abs().sum()) for s in opt["state"].values())),
        "weights_checksum": ck,
    }


def main():
    AE, hparams = load_reference()
    if sys.argv[1:] == ["reference_checkpoint_layout"]:
        import json
        d = checkpoint_layout_case(AE, hparams)
        path = os.path.join(HERE, "reference_checkpoint_layout.json")
        with open(path, "w") as fh:
            json.dump(d, fh, indent=1, default=str)
        print(f"wrote {path}")
        return
    torch.set_num_threads(8)
    cases = {
        "fwd_b2_t128_train": lambda: fwd_case(AE, 2, 128, True, 1),
        "fwd_b2_t128_eval": lambda: fwd_case(AE, 2, 128, False, 1),
        "fwd_b2_t100_train": lambda: fwd_case(AE, 2, 100, True, 2),
        "fwd_b1_t128_train": lambda: fwd_case(AE, 1, 128, True, 3),
        "fwd_b3_t33_train": lambda: fwd_case(AE, 3, 33, True, 4),
        "fwd_b2_t1024_ragged": lambda: fwd_case(AE, 2, 1024, True, 5, lengths=[1024, 700]),
        "batch_forward_m5_n128": lambda: batch_forward_case(AE),
        "c1_mette_183_b1_t128": lambda: c1_case(AE),
        "train_b4_t128_3steps": lambda: train_case(AE, hparams),
        "train_b256_t128_curve": lambda: curve_case(AE, hparams),
    }
    only = sys.argv[1:]
    for name, fn in cases.items():
        if only and name not in only:
            continue
        d = fn()
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **d)
        print(f"wrote {path} ({os.path.getsize(path) / 1024:.0f} KiB)")


if __name__ == "__main__":
    main()
