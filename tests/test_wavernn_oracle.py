"""The WaveRNN oracle (oracle/wavernn_oracle.py) pinned against the reference class's own outputs
(tests/golden/make_golden_wavernn.py), plus known answers for the sampler and the counter-based
uniform stream the GPU path shares with it."""
import json
import os

import numpy as np
import pytest
import torch

from autovc_amd.weights import wavernn_state_dict
from oracle import wavernn_oracle as wo
from tests.conftest import load_golden

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def sd():
    return wavernn_state_dict(0)


@pytest.fixture(scope="module")
def g():
    return load_golden("wavernn_ref")


def test_state_dict_layout_matches_reference(sd):
    with open(os.path.join(GOLD, "wavernn_state_layout.json")) as fh:
        ref = json.load(fh)
    assert [[k, list(v.shape), str(v.dtype)] for k, v in sd.items()] == ref


def test_upsample_matches_reference(sd, g):
    mel = torch.from_numpy(g["up_mel_in"])
    padded = wo.pad_tensor(mel.transpose(1, 2), wo.PAD).transpose(1, 2)
    with torch.no_grad():
        m, aux = wo.upsample(sd, padded)
    np.testing.assert_allclose(m.numpy(), g["up_m"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(aux.numpy(), g["up_aux"], rtol=0, atol=2e-6)


def test_teacher_forced_network_matches_reference(sd, g):
    with torch.no_grad():
        logits = wo.forward(sd, torch.from_numpy(g["fwd_x"]), torch.from_numpy(g["fwd_mels"]))
    np.testing.assert_allclose(logits.numpy(), g["fwd_logits"], rtol=0, atol=2e-5)


def test_fold_and_xfade_match_reference(g):
    f = wo.fold_with_overlap(torch.from_numpy(g["fold_in"]), 400, 50)
    np.testing.assert_array_equal(f.numpy(), g["fold_out"])
    np.testing.assert_array_equal(wo.xfade_and_unfold(g["xfade_in"], 400, 50), g["xfade_out"])


def test_mol_sampler_matches_reference_given_its_uniforms(g):
    s = wo.sample_mol(torch.from_numpy(g["mol_logits"]), torch.from_numpy(g["mol_u_mix"]),
                      torch.from_numpy(g["mol_u_log"]))
    np.testing.assert_allclose(s.numpy(), g["mol_sample"], rtol=0, atol=1e-6)


def test_uniform_stream_known_answers():
    u = wo.uniforms(0, np.arange(4), 0, 11)
    assert u.dtype == np.float32 and u.shape == (4, 11)
    assert (u >= np.float32(1e-5)).all() and (u <= np.float32(1 - 1e-5)).all()
    # distinct per (row, step, draw) and per seed; reproducible
    v = wo.uniforms(0, np.arange(4), 1, 11)
    w = wo.uniforms(1, np.arange(4), 0, 11)
    assert not np.array_equal(u, v) and not np.array_equal(u, w)
    np.testing.assert_array_equal(u, wo.uniforms(0, np.arange(4), 0, 11))
    big = wo.uniforms(3, np.arange(20000), 5, 1)[:, 0].astype(np.float64)
    assert abs(big.mean() - 0.5) < 0.01 and abs(big.var() - 1 / 12) < 0.003


def test_generate_short_run_is_finite_and_bounded(sd):
    mel = torch.rand(1, 80, 6)
    y = wo.generate(sd, mel, batched=True, target=400, overlap=50, steps=64)
    assert y.shape[1] == 64 and np.isfinite(y).all() and np.abs(y).max() <= 1.0
