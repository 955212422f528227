"""CPU tests of the rows either side of the Generator: the oracle against the
reference's own outputs (partial slices, speaker-encoder forward), known answers for the
librosa restatements (whose parity is otherwise unpinned), and the host-side logic and
drop-in surface of autovc_amd.audio / autovc_amd.speaker_encoder."""
import json
import math
import os

import numpy as np
import pytest
import torch

from autovc_amd import _lib
from autovc_amd.audio import spectrogram as sp
from autovc_amd.speaker_encoder import SpeakerEncoder
from autovc_amd.weights import speaker_encoder_state_dict, state_checksum
from oracle import audio_oracle as ao

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _slices_cases():
    with open(os.path.join(GOLD, "partial_slices.json")) as fh:
        return json.load(fh)


@pytest.mark.parametrize("impl", ["oracle", "package"])
def test_partial_slices_match_reference(impl):
    fn = ao.compute_partial_slices if impl == "oracle" else sp.compute_partial_slices
    for case in _slices_cases():
        kw = dict(case["args"])
        n = kw.pop("n_samples")
        ws, ms = fn(n, **kw)
        assert [[s.start, s.stop] for s in ws] == case["wav"], case["args"]
        assert [[s.start, s.stop] for s in ms] == case["mel"], case["args"]


def test_partial_slices_argument_checks():
    with pytest.raises(AssertionError):
        sp.compute_partial_slices(1000, 16000, overlap=1.0)
    with pytest.raises(AssertionError):
        sp.compute_partial_slices(1000, 16000, min_pad_coverage=0.0)


def test_speaker_encoder_oracle_matches_reference():
    d = np.load(os.path.join(GOLD, "speaker_encoder_fwd.npz"))
    sd = speaker_encoder_state_dict(0)
    assert abs(state_checksum(sd) - float(d["checksum"])) < 1e-6
    for name in ("b3_t160", "b1_t37", "b8_t160"):
        with torch.no_grad():
            e = ao.se_forward(sd, torch.from_numpy(d[f"{name}_x"]))
        np.testing.assert_allclose(e.numpy(), d[f"{name}_embeds"], atol=1e-6, rtol=0)


def test_speaker_encoder_dropin_surface():
    d = np.load(os.path.join(GOLD, "speaker_encoder_fwd.npz"))
    se = SpeakerEncoder(device="cpu", verbose=False)
    sdict = se.state_dict()
    assert list(sdict.keys()) == [str(k) for k in d["keys"]]
    for v, s in zip(sdict.values(), d["shapes"].tolist()):
        assert list(v.shape) == [x for x in s if x]
    se.load_state_dict(speaker_encoder_state_dict(0))
    assert se.linear.out_features == 256 and se.lstm.num_layers == 3 and se.speakers == {}
    with pytest.raises(NotImplementedError):
        se.learn(None)
    with pytest.raises(NotImplementedError):
        se(torch.zeros(1, 10, 40), hidden_init=torch.zeros(3, 1, 256))


def test_mel_scale_known_answers():
    # Slaney: linear (200/3 Hz per mel) below 1 kHz, 27 mels per factor 6.4 above
    assert ao.hz_to_mel(1000.0) == pytest.approx(15.0)
    assert ao.hz_to_mel(200.0 / 3) == pytest.approx(1.0)
    assert ao.hz_to_mel(6400.0) == pytest.approx(15.0 + 27.0)
    f = np.array([0.0, 40.0, 999.0, 1000.0, 5000.0, 11025.0])
    np.testing.assert_allclose(ao.mel_to_hz(ao.hz_to_mel(f)), f, rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("sr,n_fft,n_mels,fmin", [(22050, 2048, 80, 40), (16000, 400, 40, 0)])
def test_mel_filterbank_properties(sr, n_fft, n_mels, fmin):
    w = ao.mel_filterbank(sr, n_fft, n_mels, fmin).astype(np.float64)
    assert w.shape == (n_mels, n_fft // 2 + 1) and (w >= 0).all()
    freqs = np.linspace(0, sr / 2, n_fft // 2 + 1)
    pts = ao.mel_to_hz(np.linspace(ao.hz_to_mel(fmin), ao.hz_to_mel(sr / 2), n_mels + 2))
    for m in range(n_mels):
        nz = np.nonzero(w[m])[0]
        if len(nz):  # support strictly inside (f_m, f_m+2), slaney height 2/(f_m+2 - f_m)
            assert freqs[nz[0]] > pts[m] - 1e-9 and freqs[nz[-1]] < pts[m + 2] + 1e-9
            assert w[m].max() <= 2.0 / (pts[m + 2] - pts[m]) + 1e-9
    # a triangle of area 1 (Hz·weight) once it spans many bins
    df = freqs[1] - freqs[0]
    wide = [m for m in range(n_mels) if (pts[m + 2] - pts[m]) > 20 * df]
    for m in wide:
        assert w[m].sum() * df == pytest.approx(1.0, rel=0.02)


def test_stft_known_answers():
    # a cosine exactly on bin 5 of n_fft 64 (full Hann): |X[5]| = sum(w)/2 in every interior frame
    n_fft, hop = 64, 16
    t = np.arange(2048)
    y = np.cos(2 * np.pi * 5 * t / n_fft)
    S = ao.stft(y, n_fft, hop, n_fft, pad_mode="reflect")
    assert S.shape == (n_fft // 2 + 1, 1 + len(y) // hop)
    w = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(n_fft) / n_fft)
    np.testing.assert_allclose(np.abs(S[5, 4:-4]), w.sum() / 2, rtol=1e-9)
    assert np.abs(S[8, 4:-4]).max() < 1e-9
    # window shorter than n_fft is centred: equals the direct DFT of the zero-padded frame
    win = 40
    S2 = ao.stft(y[:256], n_fft, hop, win, pad_mode="constant")
    yp = np.pad(y[:256], n_fft // 2)
    wc = np.zeros(n_fft)
    wc[(n_fft - win) // 2:(n_fft - win) // 2 + win] = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(win) / win)
    f = 3
    frame = yp[f * hop:f * hop + n_fft] * wc
    k = np.arange(n_fft)
    X = np.array([(frame * np.exp(-2j * np.pi * b * k / n_fft)).sum() for b in range(n_fft // 2 + 1)])
    np.testing.assert_allclose(S2[:, f], X, atol=1e-10)


def test_ae_frontend_oracle_shapes_and_range():
    d = np.load(os.path.join(GOLD, "mette_183_head.npz"))
    mel = ao.mel_spec_auto_encoder(d["wav"])
    assert mel.shape == (80, 1 + len(d["wav"]) // 275) == (80, 128)
    assert mel.dtype == torch.float32 and float(mel.min()) >= 0.0 and float(mel.max()) <= 1.0
    parts = ao.mel_spec_auto_encoder(d["wav"], cut=True, partial_utterance_n_frames=64)
    assert all(p.shape == (80, 64) for p in parts)
    se = ao.mel_spec_speaker_encoder(np.zeros(16000, np.float32) + 0.1, cut=True)
    assert all(p.shape == (160, 40) for p in se)


def test_frontend_abi_exports():
    lib = _lib.load()
    for name in ("avc_stft_frames", "avc_mel_basis", "avc_mel_spectrogram", "avc_speaker_encoder_forward",
                 "avc_speaker_encoder_param_count", "avc_embedding_mean_normalize"):
        assert hasattr(lib, name)
    assert lib.avc_speaker_encoder_param_count() == 14
    assert lib.avc_stft_frames(34926, 275) == 128 and lib.avc_stft_frames(0, 160) == 1
    assert lib.avc_stft_frames(10, 0) == -1


def test_frontend_refuses_cpu():
    with pytest.raises(RuntimeError):
        sp.mel_spec_auto_encoder(np.zeros(1000, np.float32), device="cpu")
