"""ORACLE — test infrastructure only (never imported by the product path).

CPU restatement of the rows either side of the Generator: the mel frontends
(`autovc/audio/spectrogram.py`), the partial-slice arithmetic and the speaker encoder's
`forward` / `embed_utterance` (`autovc/speaker_encoder/model.py`).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.

Pinning:
* `compute_partial_slices` and the speaker-encoder forward are pinned against fixtures made by
  importing the reference itself (tests/golden/make_golden_audio.py).
* The spectrogram math lives in librosa, which is absent here and unpinned by the reference
  (`requirements.txt:7`).  The functions below restate librosa's published algorithm (stft with
  `center=True`, periodic Hann window zero-padded to n_fft, `filters.mel` with the Slaney mel
  scale and Slaney area normalisation) in float64.  **Parity unpinned** for those: no librosa
  output exists to check them against.  pad_mode defaults to "reflect": the reference calls
  `librosa.feature.melspectrogram(wav, sr, ...)` positionally (spectrogram.py:200-205), which
  only librosa < 0.10 accepts, and < 0.10 pads with "reflect".

Every function cites the reference lines it restates (paths relative to /root/reference).
"""
from __future__ import annotations

import math
from typing import Dict, List, Tuple

import numpy as np
import torch

# hparams.py:5-14 (AutoEncoderParams["spectrogram"]) and hparams.py:52-58 (SpeakerEncoderParams)
AE_SPEC = dict(sr=22050, n_mels=80, n_fft=2048, hop_length=275, window_length=1100, fmin=40,
               mel_window_step=12.5, partial_utterance_n_frames=400)
SE_SPEC = dict(sr=16000, n_mels=40, mel_window_step=10, mel_window_length=25,
               partial_utterance_n_frames=160)


# ---- librosa restatements (parity unpinned) ------------------------------------------------

def hz_to_mel(f):
    """Slaney mel scale (librosa.core.convert.hz_to_mel, htk=False): linear below 1 kHz
    (200/3 Hz per mel), logarithmic above (27 mels per factor 6.4)."""
    f = np.asarray(f, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, math.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-300) / min_log_hz) / logstep,
                    f / f_sp)


def mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, math.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


def mel_filterbank(sr: float, n_fft: int, n_mels: int, fmin: float = 0.0, fmax: float | None = None) -> np.ndarray:
    """librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax, htk=False, norm='slaney') -> float32
    [n_mels][1 + n_fft//2]: triangles between consecutive points of n_mels+2 mel-spaced
    frequencies, each scaled by 2 / (its upper - lower edge in Hz)."""
    fmax = sr / 2.0 if fmax is None else fmax
    fft_f = np.linspace(0.0, sr / 2.0, 1 + n_fft // 2)
    mel_f = mel_to_hz(np.linspace(hz_to_mel(fmin), hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fft_f[None, :]
    lower = -ramps[:-2] / fdiff[:-1, None]
    upper = ramps[2:] / fdiff[1:, None]
    w = np.maximum(0.0, np.minimum(lower, upper))
    w *= (2.0 / (mel_f[2:] - mel_f[:-2]))[:, None]
    return w.astype(np.float32)


def stft(y: np.ndarray, n_fft: int, hop: int, win_length: int | None = None,
         pad_mode: str = "reflect") -> np.ndarray:
    """librosa.stft(y, n_fft, hop_length, win_length, window='hann', center=True) in float64:
    periodic Hann of win_length centred in n_fft, signal padded by n_fft//2 both sides,
    1 + len(y)//hop frames.  Returns complex128 [1 + n_fft//2][frames]."""
    win_length = n_fft if win_length is None else win_length
    n = np.arange(win_length)
    w = 0.5 - 0.5 * np.cos(2.0 * np.pi * n / win_length)
    off = (n_fft - win_length) // 2
    window = np.zeros(n_fft)
    window[off:off + win_length] = w
    y = np.asarray(y, dtype=np.float64)
    yp = np.pad(y, n_fft // 2, mode=pad_mode)
    n_frames = 1 + (len(yp) - n_fft) // hop
    idx = np.arange(n_fft)[None, :] + hop * np.arange(n_frames)[:, None]
    frames = yp[idx] * window[None, :]
    return np.fft.rfft(frames, axis=1).T


def amp_to_db(a):
    """spectrogram.py:53-55"""
    return 20 * np.log10(np.maximum(1e-5, a))


def normalize_spec(s, min_level_db=-100):
    """spectrogram.py:14-31"""
    return np.clip((s - min_level_db) / -min_level_db, 0, 1)


def compute_partial_slices(n_samples: int, sr: int, partial_utterance_n_frames: int = 160,
                           min_pad_coverage: float = 0.75, overlap: float = 0.5,
                           mel_window_step: float = 10) -> Tuple[List[slice], List[slice]]:
    """spectrogram.py:248-311: windows of partial_utterance_n_frames mel frames every
    round(n·(1-overlap)) frames; the last one is dropped when its audio coverage is below
    min_pad_coverage (unless it is the only one)."""
    assert 0 <= overlap < 1 and 0 < min_pad_coverage <= 1
    spf = int(sr * mel_window_step / 1000)
    n_frames = int(math.ceil((n_samples + 1) / spf))
    step = max(int(round(partial_utterance_n_frames * (1 - overlap))), 1)
    starts = range(0, max(1, n_frames - partial_utterance_n_frames + step + 1), step)
    mel = [slice(i, i + partial_utterance_n_frames) for i in starts]
    wav = [slice(s.start * spf, s.stop * spf) for s in mel]
    cov = (n_samples - wav[-1].start) / (wav[-1].stop - wav[-1].start)
    if cov < min_pad_coverage and len(mel) > 1:
        mel, wav = mel[:-1], wav[:-1]
    return wav, mel


def mel_spec_auto_encoder(wav: np.ndarray, sr=AE_SPEC["sr"], cut=False, pad_mode="reflect", **kw):
    """spectrogram.py:62-142: |stft| (n_fft 2048, hop 275, win 1100) -> mel (80, fmin 40, Slaney)
    of the MAGNITUDE -> 20·log10(max(1e-5, ·)) -> clip((·+100)/100, 0, 1); float32 (80, frames),
    or a list of (80, 400) slices when cut."""
    p = AE_SPEC
    wav = np.asarray(wav, dtype=np.float32)
    if cut:
        ws, ms = compute_partial_slices(len(wav), sr=sr,
                                        mel_window_step=kw.pop("mel_window_step", p["mel_window_step"]),
                                        partial_utterance_n_frames=kw.pop("partial_utterance_n_frames",
                                                                          p["partial_utterance_n_frames"]), **kw)
        if ws[-1].stop >= len(wav):
            wav = np.pad(wav, (0, ws[-1].stop - len(wav)))
    S = np.abs(stft(wav, p["n_fft"], p["hop_length"], p["window_length"], pad_mode))
    mel = mel_filterbank(sr, p["n_fft"], p["n_mels"], p["fmin"]).astype(np.float64) @ S
    out = torch.from_numpy(normalize_spec(amp_to_db(mel)).astype(np.float32))
    return [out[:, s] for s in ms] if cut else out


def mel_spec_speaker_encoder(wav: np.ndarray, sr=SE_SPEC["sr"], cut=False, return_slices=False,
                             pad_mode="reflect", **kw):
    """spectrogram.py:144-218: melspectrogram(y, sr, n_fft=sr·25ms, hop=sr·10ms, n_mels=40) —
    POWER spectrogram (|stft|^2), full-length Hann, fmin 0 — as float32 (frames, 40)."""
    p = SE_SPEC
    wav = np.asarray(wav, dtype=np.float32)
    ws = ms = None
    if cut:
        ws, ms = compute_partial_slices(len(wav), sr=sr, **kw)
        if ws[-1].stop >= len(wav):
            wav = np.pad(wav, (0, ws[-1].stop - len(wav)))
    n_fft = int(sr * p["mel_window_length"] / 1000)
    hop = int(sr * p["mel_window_step"] / 1000)
    S = np.abs(stft(wav, n_fft, hop, n_fft, pad_mode)) ** 2
    mel = (mel_filterbank(sr, n_fft, p["n_mels"]).astype(np.float64) @ S).astype(np.float32).T
    if cut:
        mel = [mel[s] for s in ms]
    return (mel, ws, ms) if return_slices else mel


# ---- speaker encoder (pinned by the reference import) --------------------------------------

def se_forward(sd: Dict[str, torch.Tensor], utterances: torch.Tensor) -> torch.Tensor:
    """speaker_encoder/model.py:71-91: 3-layer nn.LSTM(40->256, batch_first, zero state) ->
    Linear(256->256) on the last layer's final hidden state -> ReLU -> L2 normalise per row."""
    flat = [sd[f"lstm.{n}_l{l}"] for l in range(3) for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
    B = utterances.shape[0]
    H = sd["lstm.weight_hh_l0"].shape[1]
    h0 = torch.zeros(3, B, H, dtype=utterances.dtype)
    _, h, _ = torch.lstm(utterances, (h0, h0.clone()), flat, True, 3, 0.0, False, False, True)
    raw = torch.relu(torch.nn.functional.linear(h[-1], sd["linear.weight"], sd["linear.bias"]))
    return raw / torch.norm(raw, dim=1, keepdim=True)


def embed_utterance(sd: Dict[str, torch.Tensor], wav: np.ndarray, pad_mode="reflect") -> np.ndarray:
    """speaker_encoder/model.py:142-194 (using_partials=True): partial 160-frame mels ->
    per-partial embeddings -> mean -> L2 normalise."""
    frames, _, _ = mel_spec_speaker_encoder(wav, cut=True, return_slices=True, pad_mode=pad_mode)
    with torch.no_grad():
        pe = se_forward(sd, torch.from_numpy(np.array(frames))).numpy()
    raw = pe.mean(axis=0)
    return raw / np.linalg.norm(raw, 2)
