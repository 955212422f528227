"""Drop-in speaker encoder (inference) — `autovc/speaker_encoder/model.py:21-194,437-456`.

Same constructor, attribute names (`lstm`, `linear`, `relu`, `speakers`), state_dict keys and
checkpoint dict as the reference; `forward` runs the whole network in ONE library call
(`avc_speaker_encoder_forward`: the 3-layer LSTM on the split-f16 step kernels — layers 0/1 as
one two-layer wavefront — then Linear + ReLU and the row L2 normalisation), and
`embed_utterance` chains the GPU mel frontend, the batched partial forward and the
mean + normalise reduction without leaving the device.

Out of scope (SURVEY §8f row 3 covers `embed_utterance`): GE2E training (`learn`, `_loss`,
`batch_forward`, `do_gradient_ops`) and its TSNE/wandb logging; those raise
NotImplementedError.  `hidden_init` must be None (zero initial state, the only value the
reference passes).
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.nn as nn

from .. import _lib
from ..audio import load_wav
from ..audio.spectrogram import mel_spec_speaker_encoder
from ..hparams import SpeakerEncoderParams

_P = SpeakerEncoderParams["model"]


def retrieve_file_paths(paths, excluded=()):
    """autovc/utils/__init__.py:4-38: files under `paths` (a file, a directory or a list of
    them), minus those under `excluded`."""
    ex = set(retrieve_file_paths(list(excluded))) if excluded else set()
    if isinstance(paths, (list, tuple)):
        out = []
        for p in paths:
            out.extend(retrieve_file_paths(p, excluded))
        return out
    if os.path.isfile(paths):
        return [paths] if paths not in ex else []
    if os.path.isdir(paths):
        out = []
        for root, _, files in os.walk(paths):
            out.extend(os.path.join(root, f) for f in sorted(files) if os.path.join(root, f) not in ex)
        return out
    return []


class SpeakerEncoder(nn.Module):
    def __init__(self, input_size=_P["input_size"], hidden_size=_P["hidden_size"],
                 embedding_size=_P["embedding_size"], num_layers=_P["num_layers"], batch_first=_P["batch_first"],
                 device=None, verbose=True):
        super().__init__()
        if device is None:
            device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.verbose = verbose
        self.device = device if not isinstance(device, str) else torch.device(device)
        self.speakers = {}
        self.logging = {}
        self.lstm = nn.LSTM(input_size=input_size, hidden_size=hidden_size, num_layers=num_layers,
                            batch_first=batch_first).to(self.device)
        self.linear = nn.Linear(in_features=hidden_size, out_features=embedding_size).to(self.device)
        self.relu = nn.ReLU().to(self.device)

    # ---- network ----------------------------------------------------------------------------
    def _params(self):
        names = [f"{n}_l{l}" for l in range(self.lstm.num_layers)
                 for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
        ps = [getattr(self.lstm, n) for n in names] + [self.linear.weight, self.linear.bias]
        return [p.detach().float().contiguous() for p in ps]

    def forward(self, utterances, hidden_init=None):
        """model.py:71-91: (B, n_frames, n_mels) -> L2-normalised (B, embedding_size).
        Inference only (no autograd graph is recorded)."""
        if hidden_init is not None:
            raise NotImplementedError("autovc_amd SpeakerEncoder: hidden_init must be None (zero initial state)")
        if self.lstm.num_layers != 3 or not self.lstm.batch_first or self.lstm.bidirectional:
            raise NotImplementedError("autovc_amd SpeakerEncoder: 3-layer unidirectional batch_first LSTM only")
        x = utterances
        if x.dim() != 3:
            raise ValueError(f"expected (batch, frames, channels), got {tuple(x.shape)}")
        dev = self.linear.weight.device
        x = x.to(device=dev, dtype=torch.float32).contiguous()
        B, T, C = x.shape
        if C != self.lstm.input_size:
            raise ValueError(f"expected {self.lstm.input_size} input channels, got {C}")
        params = self._params()
        arr = (_lib._P * len(params))(*[_lib.ptr(p) for p in params])
        out = torch.empty(B, self.linear.out_features, device=dev, dtype=torch.float32)
        _lib.call("avc_speaker_encoder_forward", _lib.context(dev), T, B, C, self.lstm.hidden_size,
                  self.linear.out_features, arr, _lib.ptr(x), _lib.ptr(out), _lib.stream(dev))
        return out

    def embed_frames_batch(self, frames_batch):
        """model.py:126-139: numpy/tensor (B, n_frames, n_mels) -> CPU embeddings (B, E)."""
        frames = torch.as_tensor(np.asarray(frames_batch) if not torch.is_tensor(frames_batch) else frames_batch)
        return self.forward(frames).detach().cpu()

    def embed_utterance(self, wav, using_partials=True, return_partials=False, **kwargs):
        """model.py:142-194: the utterance embedding (CPU tensor (E,), as the reference) from the
        normalised mean of the embeddings of its 160-frame partials (or of the whole utterance
        with using_partials=False)."""
        if isinstance(wav, str):
            wav, _ = load_wav(wav)
        dev = self.linear.weight.device
        if not using_partials:
            frames = mel_spec_speaker_encoder(wav, cut=False, device=dev, **kwargs)
            embed = self.forward(frames[None])[0].cpu()
            return (embed, None, None) if return_partials else embed
        frames_batch, wave_slices, _ = mel_spec_speaker_encoder(wav, cut=True, return_slices=True, device=dev,
                                                                **kwargs)
        partial = self.forward(torch.stack(frames_batch))
        embed = torch.empty(partial.shape[1], device=dev, dtype=torch.float32)
        _lib.call("avc_embedding_mean_normalize", partial.shape[0], partial.shape[1], _lib.ptr(partial),
                  _lib.ptr(embed), _lib.stream(dev))
        if return_partials:
            return embed.cpu(), partial.cpu(), wave_slices
        return embed.cpu()

    def learn_speaker(self, speaker, speaker_path, speaker_path_excluded=()):
        """model.py:437-453: mean embedding of a speaker's wav files, stored in self.speakers."""
        files = retrieve_file_paths(speaker_path, speaker_path_excluded)
        if not files:
            raise ValueError(f"no files under {speaker_path!r}")
        emb = torch.stack([self.embed_utterance(f) for f in files])
        self.speakers[speaker] = emb.mean(axis=0, keepdim=True).squeeze()

    # ---- checkpoints ------------------------------------------------------------------------
    def load(self, model_name, model_dir=SpeakerEncoderParams["model_dir"], device=None):
        """model.py:93-105 (state dict loaded with weights_only=True)."""
        self.device = device if device is not None else self.device
        path = model_dir.strip("/") + "/" + model_name
        ckpt = torch.load(path, map_location=self.device, weights_only=True)
        self.load_state_dict(ckpt["model_state"], strict=False)
        self.speakers.update(ckpt.get("speakers", {}))
        if self.verbose:
            print('Loaded speaker encoder "%s" trained to step %s' % (path, ckpt.get("step")))

    def save(self, model_name, save_dir=SpeakerEncoderParams["learn"]["save_dir"], wandb_run=None, step=None):
        """model.py:107-120 (wandb artifact logging not included)."""
        path = save_dir.strip("/") + "/" + model_name
        torch.save({"step": self.logging.get("step") if step is None else step,
                    "model_state": self.state_dict(), "speakers": self.speakers}, path)

    # ---- GE2E training: out of scope --------------------------------------------------------
    def learn(self, *args, **kwargs):
        raise NotImplementedError("SpeakerEncoder training (GE2E) is outside this package's scope (SURVEY §8f)")

    _loss = batch_forward = do_gradient_ops = learn
