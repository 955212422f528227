"""GPU parity of the rows either side of the Generator through the C ABI:
mel filterbank, the two mel frontends and the speaker encoder.

Pins: the speaker-encoder forward against the reference's own outputs (golden fixture); the
frontends against the float64 oracle restatement of librosa (parity unpinned: librosa is
absent).  Tolerances (written per test):
* normalised AE mel (values in [0, 1]): max |Δ| <= 1e-4, the Generator's own bar;
* SE power mel: relative to each frame's largest band, |Δ| <= 2e-5 (fp32 DFT accumulation);
* embeddings (unit vectors): max |Δ| <= 2e-5 against the reference outputs."""
import os

import numpy as np
import pytest
import torch

from autovc_amd.audio import spectrogram as sp
from autovc_amd.speaker_encoder import SpeakerEncoder
from autovc_amd.weights import speaker_encoder_state_dict, synthetic_speech
from oracle import audio_oracle as ao

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("sr,n_fft,n_mels,fmin", [(22050, 2048, 80, 40), (16000, 400, 40, 0)])
def test_mel_basis(cuda_device, sr, n_fft, n_mels, fmin):
    b = sp.mel_basis(sr, n_fft, n_mels, fmin, device=cuda_device).cpu().numpy()
    ref = ao.mel_filterbank(sr, n_fft, n_mels, fmin)
    nb = n_fft // 2 + 1
    assert b.shape == (n_mels, (nb + 3) & ~3) and (b[:, nb:] == 0).all()
    np.testing.assert_allclose(b[:, :nb], ref, rtol=2e-6, atol=1e-9)


def _ae_err(wav, dev, pad_mode="reflect"):
    got = sp.mel_spec_auto_encoder(wav, device=dev, pad_mode=pad_mode).cpu()
    ref = ao.mel_spec_auto_encoder(wav, pad_mode=pad_mode)
    assert got.shape == ref.shape
    return (got - ref).abs().max().item()


def test_ae_frontend_c1_excerpt(cuda_device):
    """C1: the head of data/samples/mette_183.wav (128 frames)."""
    d = np.load(os.path.join(GOLD, "mette_183_head.npz"))
    err = _ae_err(d["wav"], cuda_device)
    print(f"AE mel (mette_183 head) max |d| = {err:.2e}")
    assert err <= 1e-4


@pytest.mark.parametrize("n,pad_mode", [(22050 * 3, "reflect"), (22050 * 3 + 17, "constant"), (700, "reflect"),
                                        (1, "reflect"), (5000, "constant")])
def test_ae_frontend_synthetic(cuda_device, n, pad_mode):
    """Synthetic speech (spectra spanning > 80 dB), ragged lengths, signals shorter than the
    n_fft/2 edge padding (repeated reflection) and a single sample."""
    wav = synthetic_speech(3, n, 22050)
    err = _ae_err(wav, cuda_device, pad_mode)
    assert err <= 1e-4, err


def test_ae_frontend_cut_matches_slices(cuda_device):
    wav = synthetic_speech(4, 22050 * 7, 22050)
    parts = sp.mel_spec_auto_encoder(wav, cut=True, device=cuda_device)
    ref = ao.mel_spec_auto_encoder(wav, cut=True)
    assert len(parts) == len(ref) >= 2
    for a, b in zip(parts, ref):
        assert a.shape == b.shape == (80, 400)
        assert (a.cpu() - b).abs().max().item() <= 1e-4


@pytest.mark.parametrize("n", [16000 * 2 + 123, 300])
def test_se_frontend(cuda_device, n):
    wav = synthetic_speech(5, n, 16000)
    got = sp.mel_spec_speaker_encoder(wav, device=cuda_device).cpu().numpy()
    ref = ao.mel_spec_speaker_encoder(wav)
    assert got.shape == ref.shape == (1 + n // 160, 40)
    scale = ref.max(axis=1, keepdims=True) + 1e-30
    err = np.abs(got - ref) / scale
    print(f"SE power mel max rel-to-frame-peak |d| = {err.max():.2e}")
    assert err.max() <= 2e-5


def test_speaker_encoder_forward_matches_reference(cuda_device):
    d = np.load(os.path.join(GOLD, "speaker_encoder_fwd.npz"))
    se = SpeakerEncoder(device=cuda_device, verbose=False)
    se.load_state_dict(speaker_encoder_state_dict(0))
    for name in ("b3_t160", "b1_t37", "b8_t160"):
        e = se(torch.from_numpy(d[f"{name}_x"]).to(cuda_device)).cpu().numpy()
        err = np.abs(e - d[f"{name}_embeds"]).max()
        print(f"speaker encoder {name}: max |d| vs reference = {err:.2e}")
        assert err <= 2e-5
        np.testing.assert_allclose(np.linalg.norm(e, axis=1), 1.0, atol=1e-6)


@pytest.mark.parametrize("n,partials", [(16000 * 3 + 500, True), (16000 * 2, False), (1000, True)])
def test_embed_utterance(cuda_device, n, partials):
    sd = speaker_encoder_state_dict(0)
    se = SpeakerEncoder(device=cuda_device, verbose=False)
    se.load_state_dict(sd)
    wav = synthetic_speech(6, n, 16000)
    if partials:
        e, pe, ws = se.embed_utterance(wav, return_partials=True)
        ref = ao.embed_utterance(sd, wav)
        frames, ws_ref, _ = ao.mel_spec_speaker_encoder(wav, cut=True, return_slices=True)
        assert ws == ws_ref and pe.shape == (len(frames), 256)
    else:
        e = se.embed_utterance(wav, using_partials=False)
        with torch.no_grad():
            r = ao.se_forward(sd, torch.from_numpy(ao.mel_spec_speaker_encoder(wav))[None])[0]
        ref = r.numpy()
    assert e.device.type == "cpu" and e.shape == (256,)
    err = np.abs(e.numpy() - ref).max()
    print(f"embed_utterance n={n}: max |d| = {err:.2e}")
    assert err <= 2e-5
