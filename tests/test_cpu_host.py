"""CPU-side checks: the C-ABI library loads and exports every symbol include/autovc_hip.h
declares; the drop-in module mirrors the reference's state_dict and call surface."""
import ctypes
import inspect
import os
import re

import pytest
import torch

from autovc_amd import _lib
from autovc_amd.auto_encoder import AutoEncoder
from autovc_amd.weights import param_specs, torch_state_dict
from tests.conftest import REPO, load_golden


def header_symbols(name="autovc_hip.h"):
    h = open(os.path.join(REPO, "include", name)).read()
    h = re.sub(r"/\*.*?\*/", "", h, flags=re.S)
    return sorted(set(re.findall(r"\b(avc_\w+)\s*\(", h)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    product, debug = header_symbols(), header_symbols("autovc_hip_debug.h")
    assert len(product) >= 25
    assert not set(product) & set(debug), "a symbol is declared as product and as debug"
    syms = sorted(product + debug)
    for s in syms:
        assert hasattr(lib, s), s
    # and the ctypes table binds exactly the two headers' functions
    assert sorted(_lib.exported_symbols()) == syms
    assert lib.avc_abi_version() == 1
    assert lib.avc_generator_param_count() == 96


def test_no_cpu_fallback():
    ae = AutoEncoder(device="cpu", verbose=False)
    with pytest.raises(RuntimeError):
        ae(torch.rand(1, 80, 64), torch.rand(1, 256), torch.rand(1, 256))


def test_state_dict_matches_reference_layout():
    ae = AutoEncoder(device="cpu", verbose=False)
    sd = ae.state_dict()
    specs = param_specs()
    assert [s[0] for s in specs] == list(sd.keys())
    for name, shape, _, _ in specs:
        assert tuple(sd[name].shape) == tuple(shape), name
    ae.load_state_dict(torch_state_dict(0))
    assert sum(p.numel() for p in ae.parameters()) == 28_422_464
    # reference init distributions (net_layers.py:15-17,44-45; nn.LSTM default)
    torch.manual_seed(0)
    fresh = AutoEncoder(device="cpu", verbose=False)
    w = fresh.encoder.convolutions[0][0].conv.weight
    bound = (2 ** 0.5) * (6 / (336 * 5 + 512 * 5)) ** 0.5
    assert w.abs().max().item() <= bound and w.abs().max().item() > 0.9 * bound
    h = fresh.decoder.lstm2.weight_hh_l1
    assert h.abs().max().item() <= 1 / 32 + 1e-7


def test_call_surface_matches_reference():
    assert AutoEncoder.learn.__allowed_args__ == [
        "self", "trainloader", "n_epochs", "log_freq", "save_freq", "save_dir", "model_name", "ema_decay",
        "wandb_run", "voice_converter", "source_examples", "target_examples"]
    assert "lr" in AutoEncoder.learn.__allowed_kw__
    sig = inspect.signature(AutoEncoder.__init__)
    assert list(sig.parameters)[1:] == ["dim_neck", "dim_emb", "dim_pre", "freq", "verbose", "device"]
    ae = AutoEncoder(device="cpu", verbose=False)
    assert ae.encoder.freq == 32
    assert ae.decoder.linear_projection.linear_layer.out_features == 80
    for m in ("forward", "load", "save", "_loss", "learn", "flatten_params", "load_flattened_params",
              "batch_forward"):
        assert callable(getattr(ae, m))


def test_flatten_roundtrip_cpu():
    ae = AutoEncoder(device="cpu", verbose=False)
    ae.load_state_dict(torch_state_dict(0))
    flat = ae.flatten_params()
    assert flat.numel() == 28_422_464
    ae2 = AutoEncoder(device="cpu", verbose=False)
    ae2.load_flattened_params(flat)
    for (k, a), (_, b) in zip(ae.named_parameters(), ae2.named_parameters()):
        assert torch.equal(a, b), k


def test_golden_fixture_shapes():
    g = load_golden("fwd_b3_t33_train")
    assert g["codes"].shape == (3, 96)
    g = load_golden("fwd_b2_t100_train")
    assert g["codes"].shape == (2, 224)
    g = load_golden("batch_forward_m5_n128")
    assert g["out"].shape == (80, 4 * 64 + 128)


def test_bench_refuses_fewer_gpus_than_requested():
    """bench.py --gpus N without torchrun spawns N ranks itself, and never measures a multi-GPU
    request on fewer GPUs (here: none visible) -> non-zero exit, no JSON line."""
    import subprocess
    import sys
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0 and "GPU(s) are visible" in (r.stdout + r.stderr)
    assert '"metric"' not in r.stdout


def test_grad_sink_counts_uses():
    """ops.GradSink (in-place parameter gradients): a parameter is reported complete only after the
    backward of its last forward use (the encoder's parameters are used twice per loss)."""
    import torch
    from autovc_amd import ops
    done = []
    sink = ops.GradSink(notify=done.append)
    a = torch.nn.Parameter(torch.zeros(3))
    b = torch.nn.Parameter(torch.zeros(2))
    sink.use(a, b, None)
    sink.use(a)
    sink.done(a)
    assert done == []
    sink.done(b)
    assert done == [b]
    sink.done(a)
    assert done == [b, a]


def test_unit_bound_mark_follows_the_tensor_version():
    """ops._unit_bounded: an LSTMLayer output carries the |h| <= 1 mark until it is modified."""
    from autovc_amd import ops
    t = torch.zeros(4)
    assert not ops._unit_bounded(t)
    t._avc_unit = t._version
    assert ops._unit_bounded(t)
    t.add_(1.0)  # an in-place change voids the bound
    assert not ops._unit_bounded(t)


def test_wgrad_image_shape_rule():
    """avc_conv_wgrad_image_bytes (host logic, no device call): the conv forward can hand its weight
    gradient x's split image when B % 16 == 0, T*B % 32 == 0 and cin % 64 == 0, sized rows = cin by
    K = T*B in 2 KiB fragment blocks; 0 otherwise (ops.wgrad_image_bytes then takes the _frag path)."""
    lib = _lib.load()
    f = lib.avc_conv_wgrad_image_bytes
    f.restype = ctypes.c_size_t
    assert f(128, 64, 512, 512) == 512 * 128 * 64 * 4
    assert f(128, 256, 512, 512) == 512 * 128 * 256 * 4
    assert f(64, 32, 256, 128) == 256 * 64 * 32 * 4
    assert f(20, 8, 512, 512) == 0       # B % 16 != 0
    assert f(128, 64, 336, 512) == 0     # the first encoder conv (80 + 256 channels)
    assert f(128, 64, 80, 512) == 0      # postnet's first conv
    assert f(0, 64, 512, 512) == 0 and f(128, 64, 512, 0) == 0
