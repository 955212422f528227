"""Drop-in WaveRNN vocoder (inference) — `autovc/wavernn/model.py:16-496`.

Same constructor, submodule names, state_dict keys and checkpoint format as the reference
(`upsample.resnet.*`, `upsample.up_layers.{1,3,5}`, `I`, `rnn1`, `rnn2`, `fc1..3`, `step`), so a
reference checkpoint loads unchanged.  `generate` runs entirely in the HIP library
(`avc_wavernn_generate`, csrc/wavernn.hip): up-sampling, the per-sample GRU loop over every fold
row at once with MOL / RAW sampling, and the cross-fade; `forward(x, mels)` runs the same
per-step kernels teacher-forced and returns the logits.

Differences a caller can observe:
* sampling draws from a counter-based stream seeded from torch's default generator (one draw per
  call), not from torch's per-op RNG; `torch.manual_seed` therefore still makes `generate`
  reproducible, and the samples follow the same distributions (tests/test_gpu_wavernn.py);
* `forward` does not build an autograd graph (vocoder training is out of scope, SURVEY §8f row 4
  names `generate`), and the progress display of `gen_display` is not printed.
"""
from __future__ import annotations

import ctypes
import math
from pathlib import Path
from typing import Union

import numpy as np
import torch
import torch.nn as nn

from .. import _lib
from ..hparams import WaveRNNParams

_M = WaveRNNParams["model"]
_G = WaveRNNParams["generate"]


class ResBlock(nn.Module):
    """model.py:16-31 (parameter holder; computed by wr_frame_layer_kernel)."""

    def __init__(self, dims):
        super().__init__()
        self.conv1 = nn.Conv1d(dims, dims, kernel_size=1, bias=False)
        self.conv2 = nn.Conv1d(dims, dims, kernel_size=1, bias=False)
        self.batch_norm1 = nn.BatchNorm1d(dims)
        self.batch_norm2 = nn.BatchNorm1d(dims)


class MelResNet(nn.Module):
    """model.py:34-49."""

    def __init__(self, res_blocks, in_dims, compute_dims, res_out_dims, pad):
        super().__init__()
        self.conv_in = nn.Conv1d(in_dims, compute_dims, kernel_size=pad * 2 + 1, bias=False)
        self.batch_norm = nn.BatchNorm1d(compute_dims)
        self.layers = nn.ModuleList([ResBlock(compute_dims) for _ in range(res_blocks)])
        self.conv_out = nn.Conv1d(compute_dims, res_out_dims, kernel_size=1)


class Stretch2d(nn.Module):
    """model.py:52-63 (no parameters; the stretch is index arithmetic in the kernels)."""

    def __init__(self, x_scale, y_scale):
        super().__init__()
        self.x_scale = x_scale
        self.y_scale = y_scale


class UpsampleNetwork(nn.Module):
    """model.py:66-93: up_layers alternate Stretch2d / Conv2d(1, 1, (1, 2s+1)) initialised to 1/k."""

    def __init__(self, feat_dims, upsample_factors, compute_dims, res_blocks, res_out_dims, pad):
        super().__init__()
        total_scale = int(np.prod(upsample_factors))
        self.indent = pad * total_scale
        self.resnet = MelResNet(res_blocks, feat_dims, compute_dims, res_out_dims, pad)
        self.resnet_stretch = Stretch2d(total_scale, 1)
        self.up_layers = nn.ModuleList()
        for scale in upsample_factors:
            k_size = (1, scale * 2 + 1)
            conv = nn.Conv2d(1, 1, kernel_size=k_size, padding=(0, scale), bias=False)
            conv.weight.data.fill_(1.0 / k_size[1])
            self.up_layers.append(Stretch2d(scale, 1))
            self.up_layers.append(conv)


class WaveRNN(nn.Module):
    """Class for the WaveRNN vocoder (model.py:95-496)."""

    def __init__(self, hop_length=_M["hop_length"], rnn_dims=_M["rnn_dims"], res_out_dims=_M["res_out_dims"],
                 feat_dims=_M["feat_dims"], fc_dims=_M["fc_dims"], bits=_M["bits"],
                 upsample_factors=_M["upsample_factors"], compute_dims=_M["compute_dims"], pad=_M["pad"],
                 res_blocks=_M["res_blocks"], mode=_M["mode"], device=None):
        super().__init__()
        assert mode in ["RAW", "MOL"]
        if device is None:
            device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.hop_length = hop_length
        self.rnn_dims = rnn_dims
        self.res_out_dims = res_out_dims
        self.feat_dims = feat_dims
        self.fc_dims = fc_dims
        self.bits = bits
        self.upsample_factors = upsample_factors
        self.compute_dims = compute_dims
        self.pad = pad
        self.res_blocks = res_blocks
        self.mode = mode
        self.aux_dims = res_out_dims // 4
        self.n_classes = 2 * bits if mode == "RAW" else 30
        self.device = device if not isinstance(device, str) else torch.device(device)
        self.upsample = UpsampleNetwork(feat_dims, upsample_factors, compute_dims, res_blocks, res_out_dims, pad)
        self.I = nn.Linear(feat_dims + self.aux_dims + 1, rnn_dims)
        self.rnn1 = nn.GRU(rnn_dims, rnn_dims, batch_first=True)
        self.rnn2 = nn.GRU(rnn_dims + self.aux_dims, rnn_dims, batch_first=True)
        self.fc1 = nn.Linear(rnn_dims + self.aux_dims, fc_dims)
        self.fc2 = nn.Linear(fc_dims + self.aux_dims, fc_dims)
        self.fc3 = nn.Linear(fc_dims, self.n_classes)
        self.register_buffer("step", torch.zeros(1, dtype=torch.long))
        self.to(self.device)
        self.num_params()

    # ---- library plumbing ------------------------------------------------------------------
    def _dims(self):
        if len(self.upsample_factors) != 3:
            raise NotImplementedError("the HIP up-sampling runs exactly three stretch stages (the reference's "
                                      "(5, 5, 11) layout)")
        if int(np.prod(self.upsample_factors)) != self.hop_length:
            raise ValueError("upsample_factors must factorise hop_length (hparams.py:102)")
        d = [self.feat_dims, self.compute_dims, self.res_out_dims, self.res_blocks, self.rnn_dims, self.fc_dims,
             self.n_classes, self.pad] + [int(f) for f in self.upsample_factors]
        return (ctypes.c_int * 11)(*d)

    def _param_ptrs(self):
        ts = [v for k, v in self.state_dict().items() if k != "step" and not k.endswith("num_batches_tracked")]
        n = _lib.load().avc_wavernn_param_count(self.res_blocks)
        if len(ts) != n:
            raise RuntimeError(f"WaveRNN parameter layout: {len(ts)} tensors, library expects {n}")
        ts = [t if t.is_contiguous() else t.contiguous() for t in ts]
        self._keep = ts
        return (ctypes.c_void_p * n)(*[_lib.ptr(t) for t in ts])

    def _run(self, mel, batched, target, overlap, seed, x_teacher=None, want_samples=False):
        dev = next(self.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("autovc_amd's WaveRNN runs on the GPU only (HIP kernels); move it with .to('cuda')")
        mel = torch.as_tensor(mel, device=dev, dtype=torch.float32).contiguous()
        if mel.dim() != 3 or mel.size(1) != self.feat_dims:
            raise ValueError(f"expected a mel of shape (1, {self.feat_dims}, T), got {tuple(mel.shape)}")
        T = mel.size(-1)
        n_pos = (T if x_teacher is None else T - 2 * self.pad) * self.hop_length
        rows, steps = ctypes.c_long(), ctypes.c_long()
        _lib.call("avc_wavernn_fold_shape", n_pos, int(batched), int(target), int(overlap), ctypes.byref(rows),
                  ctypes.byref(steps))
        samples = torch.empty(rows.value, steps.value, device=dev, dtype=torch.float32)
        logits = wave = xt = None
        if x_teacher is not None:
            xt = x_teacher.to(dev, torch.float32).contiguous()
            logits = torch.empty(rows.value, steps.value, self.n_classes, device=dev, dtype=torch.float32)
        else:
            wave = torch.empty(max(0, (T - 1) * self.hop_length), device=dev, dtype=torch.float32)
        with torch.cuda.device(dev):
            _lib.call("avc_wavernn_generate", _lib.context(dev), self._dims(), T, self._param_ptrs(),
                      _lib.ptr(mel[:1].contiguous()), int(batched), int(target), int(overlap),
                      int(self.mode == "MOL"), ctypes.c_ulonglong(seed), _lib.ptr(xt), _lib.ptr(logits),
                      _lib.ptr(samples), _lib.ptr(wave), _lib.stream(dev))
        return samples, logits, wave

    def upsample_features(self, mel):
        """generate()'s up-sampling (model.py:249-252: `pad` zero frames each side, then
        UpsampleNetwork in eval mode): mel (1, F, T) -> (m (L, F), aux (T, res_out_dims)) with
        L = T * hop; aux stays at frame rate (the x hop stretch is an index in the kernels)."""
        dev = next(self.parameters()).device
        mel = torch.as_tensor(mel, device=dev, dtype=torch.float32).contiguous()
        T = mel.size(-1)
        m = torch.empty(T * self.hop_length, self.feat_dims, device=dev)
        aux = torch.empty(T, self.res_out_dims, device=dev)
        with torch.cuda.device(dev):
            _lib.call("avc_wavernn_upsample", _lib.context(dev), self._dims(), T, self._param_ptrs(),
                      _lib.ptr(mel), _lib.ptr(m), _lib.ptr(aux), _lib.stream(dev))
        return m, aux

    # ---- reference API -----------------------------------------------------------------------
    def forward(self, x, mels):
        """model.py:180-211, teacher-forced (the same per-step kernels as generate): x (1, L)
        previous samples, mels (1, F, T) with L = (T - 2 pad) * hop -> logits (1, L, n_classes).
        No autograd graph is built (training the vocoder is out of scope)."""
        self.step += 1
        mels = torch.as_tensor(mels, dtype=torch.float32)
        L = (mels.size(-1) - 2 * self.pad) * self.hop_length
        x = torch.as_tensor(x, dtype=torch.float32)
        if mels.dim() != 3 or mels.size(0) != 1 or x.dim() != 2 or x.size(0) != 1 or x.size(1) != L:
            raise ValueError(f"forward expects x (1, {L}) and mels (1, F, T); got {tuple(x.shape)}, {tuple(mels.shape)}")
        with torch.no_grad():
            _, logits, _ = self._run(mels, False, 0, 0, 0, x_teacher=x)
        return logits

    def generate(self, melspectrogram, batched=_G["batched"], target=_G["target"], overlap=_G["overlap"],
                 mu_law=_G["mu_law"]):
        """model.py:214-329: waveform (np.float32) from a (1, F, T) mel spectrogram."""
        self.eval()
        mu_law = mu_law if self.mode == "RAW" else False
        if mu_law:
            raise NotImplementedError  # as the reference (model.py:318-320)
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        with torch.no_grad():
            mel = torch.as_tensor(melspectrogram, dtype=torch.float32)
            if mel.dim() == 2:
                mel = mel[None]
            if mel.size(-1) < 21:
                raise ValueError("generate() fades out the last 20 hops (model.py:326-328): need >= 21 frames")
            _, _, wave = self._run(mel, batched, target, overlap, seed)
        torch.cuda.synchronize(wave.device)
        return wave.cpu().numpy().astype(np.float32)

    def get_gru_cell(self, gru):
        """model.py:273-280."""
        cell = nn.GRUCell(gru.input_size, gru.hidden_size).to(gru.weight_hh_l0.device)
        cell.weight_hh.data = gru.weight_hh_l0.data
        cell.weight_ih.data = gru.weight_ih_l0.data
        cell.bias_hh.data = gru.bias_hh_l0.data
        cell.bias_ih.data = gru.bias_ih_l0.data
        return cell

    def pad_tensor(self, x, pad, side="both"):
        """model.py:282-294."""
        b, t, c = x.size()
        total = t + 2 * pad if side == "both" else t + pad
        padded = torch.zeros(b, total, c, device=x.device, dtype=x.dtype)
        if side in ("before", "both"):
            padded[:, pad:pad + t, :] = x
        elif side == "after":
            padded[:, :t, :] = x
        return padded

    def fold_with_overlap(self, x, target, overlap):
        """model.py:296-339 (the generate path folds by index arithmetic in the kernels)."""
        _, total_len, features = x.size()
        num_folds = (total_len - overlap) // (target + overlap)
        extended_len = num_folds * (overlap + target) + overlap
        remaining = total_len - extended_len
        if remaining != 0:
            num_folds += 1
            x = self.pad_tensor(x, target + 2 * overlap - remaining, side="after")
        starts = torch.arange(num_folds, device=x.device) * (target + overlap)
        idx = starts[:, None] + torch.arange(target + 2 * overlap, device=x.device)[None, :]
        return x[0][idx]

    def xfade_and_unfold(self, y, target, overlap):
        """model.py:341-399 (host numpy float64, as the reference; generate() cross-fades on the GPU)."""
        num_folds, length = y.shape
        target = length - 2 * overlap
        total_len = num_folds * (target + overlap) + overlap
        silence_len = overlap // 2
        fade_len = overlap - silence_len
        t = np.linspace(-1, 1, fade_len, dtype=np.float64)
        fade_in = np.concatenate([np.zeros(silence_len, dtype=np.float64), np.sqrt(0.5 * (1 + t))])
        fade_out = np.concatenate([np.ones(silence_len, dtype=np.float64), np.sqrt(0.5 * (1 - t))])
        y[:, :overlap] *= fade_in
        y[:, -overlap:] *= fade_out
        unfolded = np.zeros(total_len, dtype=np.float64)
        for i in range(num_folds):
            start = i * (target + overlap)
            unfolded[start:start + target + 2 * overlap] += y[i]
        return unfolded

    def get_step(self):
        return self.step.data.item()

    def log(self, path, msg):
        with open(path, "a") as f:
            print(msg, file=f)

    def load(self, model_name, model_dir=WaveRNNParams["model_dir"], device=None):
        """model.py:436-447 (a state_dict checkpoint; loaded with weights_only=True)."""
        device = next(self.parameters()).device if device is None else device
        model_path = model_dir.strip("/") + "/" + model_name
        self.load_state_dict(torch.load(model_path, map_location=device, weights_only=True))
        print('Loaded vocoder "%s"' % model_path)

    def save(self, path: Union[str, Path]):
        torch.save(self.state_dict(), path)

    def num_params(self, print_out=False):
        n = sum(int(np.prod(p.size())) for p in self.parameters() if p.requires_grad) / 1_000_000
        if print_out:
            print("Trainable Parameters: %.3fM" % n)
        return n

    def _flatten_parameters(self):
        for m in (self.rnn1, self.rnn2):
            m.flatten_parameters()
