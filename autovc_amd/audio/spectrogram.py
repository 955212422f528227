"""Mel frontends on the HIP path — drop-in for `autovc/audio/spectrogram.py`.

The arithmetic (framing, DFT, magnitude/power, mel projection, dB + normalisation) runs in
`avc_mel_spectrogram` (autovc_amd/csrc/audio.hip): two fp32 MFMA products and three small
kernels per call, the dB/normalise step fused into the mel product's epilogue.  librosa is not
used (and not importable here): its stft / filters.mel algorithms are restated in the kernels.

Differences from the reference, all deliberate:
* results stay on the GPU: `mel_spec_auto_encoder` returns a CUDA tensor (the reference returns
  a CPU tensor that convert() moves to the GPU anyway), `mel_spec_speaker_encoder` returns CUDA
  tensors instead of numpy arrays (its only caller, `SpeakerEncoder.embed_utterance`, feeds them
  straight to the GPU);
* the STFT edge padding is `pad_mode="reflect"`: the reference's positional
  `librosa.feature.melspectrogram(wav, sr, ...)` call (spectrogram.py:200-205) only runs on
  librosa < 0.10, whose stft pads with "reflect" (0.10 switched to "constant").  Pass
  `pad_mode="constant"` for the newer behaviour.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .. import _lib
from ..hparams import AutoEncoderParams, SpeakerEncoderParams

_AE = AutoEncoderParams["spectrogram"]
_SE = SpeakerEncoderParams["spectrogram"]
_PAD = {"constant": 0, "reflect": 1}
_basis_cache: dict = {}


def normalize_spec(spectrogram, min_level_db=-100):
    """spectrogram.py:14-31 (host helper on numpy arrays, as in the reference)."""
    return np.clip((spectrogram - min_level_db) / -min_level_db, 0, 1)


def denormalize_spec(spectrogram, min_level_db=-100):
    """spectrogram.py:33-51"""
    return (np.clip(spectrogram, 0, 1) * -min_level_db) + min_level_db


def amp_to_db(amplitude):
    """spectrogram.py:53-55"""
    return 20 * np.log10(np.maximum(1e-5, amplitude))


def db_to_amp(power):
    """spectrogram.py:57-59"""
    return np.power(10.0, power * 0.05)


def _device(device):
    if device is None:
        if not torch.cuda.is_available():
            raise RuntimeError("autovc_amd mel frontends run on the GPU only (HIP kernels)")
        return torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    if device.type != "cuda":
        raise RuntimeError("autovc_amd mel frontends run on the GPU only (HIP kernels)")
    return device


def mel_basis(sr, n_fft, n_mels, fmin=0.0, fmax=None, device=None) -> torch.Tensor:
    """librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax) built on the device (avc_mel_basis),
    cached per configuration; rows padded to ld = (n_fft//2 + 1) rounded up to 4."""
    device = _device(device)
    fmax = sr / 2.0 if fmax is None else float(fmax)
    key = (device.index, float(sr), int(n_fft), int(n_mels), float(fmin), fmax)
    b = _basis_cache.get(key)
    if b is None:
        ld = (n_fft // 2 + 1 + 3) & ~3
        b = torch.empty(n_mels, ld, device=device, dtype=torch.float32)
        _lib.call("avc_mel_basis", float(sr), int(n_fft), int(n_mels), float(fmin), fmax, ld, _lib.ptr(b),
                  _lib.stream(device))
        _basis_cache[key] = b
    return b


def _wav_tensor(wav, device, pad_to=None):
    y = torch.as_tensor(wav).to(device=device, dtype=torch.float32).reshape(-1)
    if pad_to is not None and pad_to > y.numel():
        yp = torch.zeros(pad_to, device=device, dtype=torch.float32)
        yp[: y.numel()] = y
        y = yp
    if y.numel() == 0:
        raise ValueError("empty waveform")
    return y.contiguous()


def _mel(y, sr, n_fft, hop, win, n_mels, fmin, power, db, channels_first, pad_mode):
    if pad_mode not in _PAD:
        raise ValueError(f"pad_mode must be one of {sorted(_PAD)}")
    dev = y.device
    basis = mel_basis(sr, n_fft, n_mels, fmin, device=dev)
    F = 1 + y.numel() // hop
    out = torch.empty((n_mels, F) if channels_first else (F, n_mels), device=dev, dtype=torch.float32)
    _lib.call("avc_mel_spectrogram", _lib.context(dev), _lib.ptr(y), y.numel(), n_fft, hop, win, _PAD[pad_mode],
              power, _lib.ptr(basis), n_mels, basis.shape[1], int(db), int(channels_first), _lib.ptr(out),
              _lib.stream(dev))
    return out


def mel_spec_auto_encoder(wav, sr=_AE["sr"], cut=False, n_mels=_AE["n_mels"], n_fft=_AE["n_fft"],
                          hop_length=_AE["hop_length"], window_length=_AE["window_length"], fmin=_AE["fmin"],
                          device=None, pad_mode="reflect", **kwargs):
    """spectrogram.py:62-142: normalised dB mel of |STFT| -> (n_mels, frames) float32 on the
    GPU, or a list of (n_mels, partial_utterance_n_frames) slices when `cut`."""
    device = _device(device)
    pad_to = None
    if cut:
        wave_slices, mel_slices = compute_partial_slices(
            len(wav), sr=sr, mel_window_step=kwargs.pop("mel_window_step", _AE["mel_window_step"]),
            partial_utterance_n_frames=kwargs.pop("partial_utterance_n_frames", _AE["partial_utterance_n_frames"]),
            **kwargs)
        pad_to = wave_slices[-1].stop
    y = _wav_tensor(wav, device, pad_to)
    mel = _mel(y, sr, n_fft, hop_length, window_length, n_mels, fmin, 1, True, True, pad_mode)
    if cut:
        return [mel[:, s] for s in mel_slices]
    return mel


def mel_spec_speaker_encoder(wav, sr=_SE["sr"], n_mels=_SE["n_mels"], mel_window_length=_SE["mel_window_length"],
                             mel_window_step=_SE["mel_window_step"], cut=False, return_slices=False,
                             device=None, pad_mode="reflect", **kwargs):
    """spectrogram.py:144-218: mel of the POWER spectrogram (n_fft = sr·25 ms, hop = sr·10 ms,
    full-length Hann, fmin 0), frame-major (frames, n_mels) on the GPU; with `cut` a list of
    (partial_utterance_n_frames, n_mels) slices."""
    device = _device(device)
    wave_slices = mel_slices = None
    pad_to = None
    if cut:
        wave_slices, mel_slices = compute_partial_slices(len(wav), sr=sr, **kwargs)
        pad_to = wave_slices[-1].stop
    y = _wav_tensor(wav, device, pad_to)
    n_fft = int(sr * mel_window_length / 1000)
    hop = int(sr * mel_window_step / 1000)
    mel = _mel(y, sr, n_fft, hop, n_fft, n_mels, 0.0, 2, False, False, pad_mode)
    if cut:
        mel = [mel[s] for s in mel_slices]
    if return_slices:
        return mel, wave_slices, mel_slices
    return mel


def mel_spectrogram(wav, model, **kwargs):
    """spectrogram.py:220-246"""
    if model == "auto_encoder":
        return mel_spec_auto_encoder(wav, **kwargs)
    if model == "speaker_encoder":
        return mel_spec_speaker_encoder(wav, **kwargs)
    raise ValueError(f"'{model}' is not a valid model type. Must be either 'auto_encoder' or 'speaker_encoder'")


def compute_partial_slices(n_samples, sr, partial_utterance_n_frames=160, min_pad_coverage=0.75, overlap=0.5,
                           mel_window_step=10):
    """spectrogram.py:248-311 (host-side index arithmetic): windows of
    `partial_utterance_n_frames` mel frames every round(n·(1 - overlap)) frames; the last window
    is kept only if the audio covers at least `min_pad_coverage` of it (always >= 1 window)."""
    assert 0 <= overlap < 1
    assert 0 < min_pad_coverage <= 1
    spf = int(sr * mel_window_step / 1000)
    n_frames = int(math.ceil((n_samples + 1) / spf))
    frame_step = max(int(np.round(partial_utterance_n_frames * (1 - overlap))), 1)
    last = max(1, n_frames - partial_utterance_n_frames + frame_step + 1)
    mel_slices = [slice(int(i), int(i) + partial_utterance_n_frames) for i in range(0, last, frame_step)]
    wav_slices = [slice(s.start * spf, s.stop * spf) for s in mel_slices]
    tail = wav_slices[-1]
    if (n_samples - tail.start) / (tail.stop - tail.start) < min_pad_coverage and len(mel_slices) > 1:
        mel_slices, wav_slices = mel_slices[:-1], wav_slices[:-1]
    return wav_slices, mel_slices
