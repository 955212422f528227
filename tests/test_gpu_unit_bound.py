"""The stacked LSTM backward's W_ih gradient of layer 1 splits its input x = layer 0's h with the
bound |h| <= 1 instead of a max scan of x (avc_lstm_backward_ex x_unit, round 5; ops._unit_bounded).

A bound above max |x| by 2^k moves every element k binades down inside f16's range: the product
keeps the 3xf16 accuracy unless elements sit ~2^-28 below the bound.  Checked against an fp64
evaluation of the same two-layer recurrence, beside the scanned form.  Reference:
autovc/auto_encoder/decoder.py:53,74 (lstm2 = nn.LSTM(512, 1024, 2))."""
import pytest
import torch

from autovc_amd import ops

pytestmark = pytest.mark.gpu


def _stack(dev, B, T, din, H, seed):
    g = torch.Generator().manual_seed(seed)
    k = 1.0 / H ** 0.5
    layers = []
    for d in (din, H):
        layers.append([((torch.rand(*s, generator=g) * 2 - 1) * k) for s in [(4 * H, d), (4 * H, H), (4 * H,), (4 * H,)]])
    x = torch.randn(T * B, din, generator=g) * 0.5
    dy = torch.randn(T * B, H, generator=g)
    return layers, x, dy


def _ours(dev, layers, x, dy, T, B, check=True):
    ws = [[w.to(dev).requires_grad_(True) for w in lw] for lw in layers]
    h = ops.LSTMLayer.apply(x.to(dev), *ws[0], T, B, True)
    assert ops._unit_bounded(h) or not check
    y = ops.LSTMLayer.apply(h, *ws[1], T, B, True)
    y.backward(dy.to(dev))
    torch.cuda.synchronize()
    return ws[1][0].grad.double().cpu()


def _fp64(layers, x, dy, T, B, H):
    lstm = torch.nn.LSTM(x.shape[1], H, 2).double()
    with torch.no_grad():
        for l, (wi, wh, bi, bh) in enumerate(layers):
            getattr(lstm, f"weight_ih_l{l}").copy_(wi.double())
            getattr(lstm, f"weight_hh_l{l}").copy_(wh.double())
            getattr(lstm, f"bias_ih_l{l}").copy_(bi.double())
            getattr(lstm, f"bias_hh_l{l}").copy_(bh.double())
    y, _ = lstm(x.double().view(T, B, -1))
    y.backward(dy.double().view(T, B, H))
    return lstm.weight_ih_l1.grad


@pytest.mark.parametrize("B,T,din,H", [(64, 16, 512, 1024), (256, 12, 512, 1024), (32, 20, 512, 512)])
def test_layer1_input_weight_gradient_with_unit_bound(cuda_device, monkeypatch, B, T, din, H):
    layers, x, dy = _stack(cuda_device, B, T, din, H, B + T)
    ref = _fp64(layers, x, dy, T, B, H)
    bound = _ours(cuda_device, layers, x, dy, T, B)
    monkeypatch.setattr(ops, "_unit_bounded", lambda t: False)  # the scanned form
    scanned = _ours(cuda_device, layers, x, dy, T, B, check=False)
    scale = float(ref.abs().max())
    e_bound = float((bound - ref).abs().max()) / scale
    e_scan = float((scanned - ref).abs().max()) / scale
    print(f"B={B} T={T} H={H}: dW_ih(l1) rel err bound {e_bound:.2e}, scanned {e_scan:.2e}")
    assert e_bound < 2e-6, e_bound
    assert e_bound <= 2 * e_scan + 1e-7
