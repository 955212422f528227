"""ORACLE — test infrastructure only (never imported by the product path).

CPU restatement of the AutoVC Generator hot path in stock torch-CPU functional ops
(F.conv1d / torch.lstm / F.batch_norm / F.linear) composed in the reference's order.
It is pinned against tests/golden/*.npz, which were produced by the reference class itself
(tests/golden/make_golden.py).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module.

Every function cites the reference lines it restates (paths relative to /root/reference).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor
FREQ = 32
DIM_NECK = 32


def conv_bn(x: Tensor, sd: Dict[str, Tensor], prefix: str, training: bool,
            bufs: Optional[Dict[str, Tensor]] = None) -> Tensor:
    """ConvNorm (net_layers.py:39-49, k=5 p=2) followed by nn.BatchNorm1d (encoder.py:40-46).

    Train mode normalises with the biased batch variance over (B,T) and updates the running
    stats with momentum 0.1 and the unbiased variance, exactly as nn.BatchNorm1d.
    """
    y = F.conv1d(x, sd[prefix + ".0.conv.weight"], sd[prefix + ".0.conv.bias"], padding=2)
    rm = (bufs or sd)[prefix + ".1.running_mean"]
    rv = (bufs or sd)[prefix + ".1.running_var"]
    y = F.batch_norm(y, rm, rv, sd[prefix + ".1.weight"], sd[prefix + ".1.bias"],
                     training=training, momentum=0.1, eps=1e-5)
    if training and bufs is not None and prefix + ".1.num_batches_tracked" in bufs:
        bufs[prefix + ".1.num_batches_tracked"] += 1
    return y


def lstm(x: Tensor, sd: Dict[str, Tensor], prefix: str, num_layers: int, bidirectional: bool) -> Tensor:
    """nn.LSTM(batch_first=True) with zero initial state (encoder.py:51,75; decoder.py:37,53)."""
    params: List[Tensor] = []
    for l in range(num_layers):
        for sfx in ([""] + (["_reverse"] if bidirectional else [])):
            params += [sd[f"{prefix}.weight_ih_l{l}{sfx}"], sd[f"{prefix}.weight_hh_l{l}{sfx}"],
                       sd[f"{prefix}.bias_ih_l{l}{sfx}"], sd[f"{prefix}.bias_hh_l{l}{sfx}"]]
    H = sd[f"{prefix}.weight_hh_l0"].shape[1]
    D = 2 if bidirectional else 1
    h0 = x.new_zeros(num_layers * D, x.shape[0], H)
    out, _, _ = torch.lstm(x, (h0, h0.clone()), params, True, num_layers, 0.0, False, bidirectional, True)
    return out


def encoder(sd, x: Tensor, c_org: Tensor, training: bool, bufs=None) -> Tuple[List[Tensor], List[Tensor]]:
    """Encoder.forward (encoder.py:53-97): concat speaker embedding, 3x relu(BN(conv)), BiLSTM,
    downsample forward outputs at 31,63,.. and backward outputs at 0,32,.."""
    c = c_org.unsqueeze(-1).expand(-1, -1, x.size(-1))
    h = torch.cat((x, c), dim=1)
    for i in range(3):
        h = F.relu(conv_bn(h, sd, f"encoder.convolutions.{i}", training, bufs))
    out = lstm(h.transpose(1, 2), sd, "encoder.lstm", 2, True)
    fwd, bwd = out[:, :, :DIM_NECK], out[:, :, DIM_NECK:]
    codes_a = [fwd[:, i, :] for i in range(FREQ - 1, out.size(1), FREQ)]
    codes_b = [bwd[:, i, :] for i in range(0, out.size(1), FREQ)]
    return codes_a, codes_b


def content_codes(codes_a, codes_b) -> Tensor:
    """model.py:99 / :143."""
    return torch.cat([torch.cat(codes_a, dim=-1), torch.cat(codes_b, dim=-1)], dim=-1)


def upsample(codes_a, codes_b, T: int) -> Tensor:
    """model.py:115-123: repeat each code over its 32-frame block; forward tail repeats the last
    code, backward stream truncated to T."""
    up_a = torch.cat([c.unsqueeze(-1).expand(-1, -1, FREQ) for c in codes_a], dim=-1)
    tail = codes_a[-1].unsqueeze(-1).expand(-1, -1, T - up_a.size(-1))
    up_a = torch.cat([up_a, tail], dim=-1)
    up_b = torch.cat([c.unsqueeze(-1).expand(-1, -1, FREQ) for c in codes_b], dim=-1)[:, :, :T]
    return torch.cat([up_a, up_b], dim=1)


def decoder(sd, x: Tensor, training: bool, bufs=None) -> Tensor:
    """Decoder.forward (decoder.py:58-79). x: (B,T,320) -> (B,T,80)."""
    h = lstm(x, sd, "decoder.lstm1", 1, False).transpose(1, 2)
    for i in range(3):
        h = F.relu(conv_bn(h, sd, f"decoder.convolutions.{i}", training, bufs))
    out = lstm(h.transpose(1, 2), sd, "decoder.lstm2", 2, False)
    return F.linear(out, sd["decoder.linear_projection.linear_layer.weight"],
                    sd["decoder.linear_projection.linear_layer.bias"])


def postnet(sd, x: Tensor, training: bool, bufs=None) -> Tensor:
    """Postnet.forward (postnet.py:50-63): 4x tanh(BN(conv)), then BN(conv)."""
    for i in range(4):
        x = torch.tanh(conv_bn(x, sd, f"postnet.convolutions.{i}", training, bufs))
    return conv_bn(x, sd, "postnet.convolutions.4", training, bufs)


def forward(sd, x: Tensor, c_org: Tensor, c_trg: Optional[Tensor], training: bool = True, bufs=None):
    """AutoEncoder.forward (model.py:68-146).  x is channel-first (B,80,T)."""
    codes_a, codes_b = encoder(sd, x, c_org, training, bufs)
    if c_trg is None:
        return content_codes(codes_a, codes_b)
    T = x.size(-1)
    code_exp = upsample(codes_a, codes_b, T)
    enc_out = torch.cat((code_exp, c_trg.unsqueeze(-1).expand(-1, -1, T)), dim=1)
    mel = decoder(sd, enc_out.transpose(1, 2), training, bufs).transpose(2, 1)
    mel_post = mel + postnet(sd, mel, training, bufs)
    return mel, mel_post, content_codes(codes_a, codes_b)


def batch_forward(sd, batch: Tensor, c_org: Tensor, c_trg: Tensor, overlap: float = 0.5,
                  training: bool = True, bufs=None) -> Tensor:
    """AutoEncoder.batch_forward (model.py:395-437): NaN-pad each slice by its offset and nanmean."""
    c_org = c_org.expand(batch.size(0), -1)
    c_trg = c_trg.expand(batch.size(0), -1)
    _, out, _ = forward(sd, batch, c_org, c_trg, training, bufs)
    N = batch.size(-1)
    M = out.size(0)
    step = int(N * (1 - overlap))
    frames = [F.pad(out[i], (i * step, (M - i - 1) * step), mode="constant", value=math.nan) for i in range(M)]
    return torch.stack(frames).nanmean(dim=0)


# ---- training (model.py:184-215, 286-321) -----------------------------------------------

def loss_fn(sd, X, c_org, out_dec, out_post, codes, bufs=None):
    """_loss: MSE(post,X) + MSE(dec,X) + L1(Enc(post,c_org), codes), nothing detached."""
    rec_codes = forward(sd, out_post, c_org, None, True, bufs)
    return F.mse_loss(out_post, X) + F.mse_loss(out_dec, X) + F.l1_loss(rec_codes, codes)


def param_names(sd) -> List[str]:
    return [k for k in sd.keys() if not (k.endswith("running_mean") or k.endswith("running_var")
                                         or k.endswith("num_batches_tracked"))]


class Trainer:
    """One reference training step (model.py:303-321) on CPU: fwd, _loss, backward,
    clip_grad_norm_(1), Adam(lr 1e-3, betas (.9,.999), eps 1e-8) and the EMA of flatten_params."""

    def __init__(self, sd, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, ema_decay=0.9999):
        self.names = param_names(sd)
        self.p = {k: sd[k].detach().clone().requires_grad_(True) for k in self.names}
        self.bufs = {k: v.detach().clone() for k, v in sd.items() if k not in self.p}
        self.m = {k: torch.zeros_like(v) for k, v in self.p.items()}
        self.v = {k: torch.zeros_like(v) for k, v in self.p.items()}
        self.lr, self.betas, self.eps, self.ema_decay = lr, betas, eps, ema_decay
        self.t = 0
        self.avg = self.flatten()

    def sd(self):
        d = dict(self.p)
        d.update(self.bufs)
        return d

    def flatten(self):
        return torch.cat([self.p[k].detach().reshape(-1) for k in self.names])

    def grads(self, X, c, bufs):
        """Loss and parameter gradients of one batch; `bufs` takes the BN running-stat updates."""
        sd = dict(self.p)
        sd.update(bufs)
        out_dec, out_post, codes = forward(sd, X, c, c, True, bufs)
        loss = loss_fn(sd, X, c, out_dec, out_post, codes, bufs)
        return float(loss.detach()), torch.autograd.grad(loss, [self.p[k] for k in self.names])

    def step_dp(self, shards, bufs_per_rank):
        """Data-parallel form of step() (BASELINE config 4): every rank r computes
        the gradient of its own shard (its own BN batch statistics and running buffers), the
        gradients are averaged (the all-reduce), then clip_grad_norm_(1) + Adam + EMA exactly as
        the single-process step (model.py:313-321).  Returns (per-rank losses, pre-clip norm)."""
        losses, acc = [], None
        for (X, c), bufs in zip(shards, bufs_per_rank):
            l, g = self.grads(X, c, bufs)
            losses.append(l)
            acc = list(g) if acc is None else [a + b for a, b in zip(acc, g)]
        grads = [a / len(shards) for a in acc]
        return losses, self._apply(grads)

    def _apply(self, grads):
        norm = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g) for g in grads]))
        coef = torch.clamp(1.0 / (norm + 1e-6), max=1.0)
        self.t += 1
        b1, b2 = self.betas
        with torch.no_grad():
            for k, g in zip(self.names, grads):
                g = g * coef
                self.m[k].mul_(b1).add_(g, alpha=1 - b1)
                self.v[k].mul_(b2).addcmul_(g, g, value=1 - b2)
                bc1 = 1 - b1 ** self.t
                bc2 = 1 - b2 ** self.t
                denom = (self.v[k].sqrt() / math.sqrt(bc2)).add_(self.eps)
                self.p[k].addcdiv_(self.m[k], denom, value=-self.lr / bc1)
            self.avg = self.ema_decay * self.avg + (1 - self.ema_decay) * self.flatten()
        return float(norm)

    def step(self, X, c):
        sd = self.sd()
        out_dec, out_post, codes = forward(sd, X, c, c, True, self.bufs)
        loss = loss_fn(sd, X, c, out_dec, out_post, codes, self.bufs)
        grads = torch.autograd.grad(loss, [self.p[k] for k in self.names])
        norm = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g) for g in grads]))
        coef = torch.clamp(1.0 / (norm + 1e-6), max=1.0)
        self.t += 1
        b1, b2 = self.betas
        with torch.no_grad():
            for k, g in zip(self.names, grads):
                g = g * coef
                self.m[k].mul_(b1).add_(g, alpha=1 - b1)
                self.v[k].mul_(b2).addcmul_(g, g, value=1 - b2)
                bc1 = 1 - b1 ** self.t
                bc2 = 1 - b2 ** self.t
                denom = (self.v[k].sqrt() / math.sqrt(bc2)).add_(self.eps)
                self.p[k].addcdiv_(self.m[k], denom, value=-self.lr / bc1)
            self.avg = self.ema_decay * self.avg + (1 - self.ema_decay) * self.flatten()
        return float(loss.detach()), float(norm)
