"""Split-image hand-over between consecutive convs of the per-layer (training) path
(ops.ConvBNAct emit_frag / avc_conv_bn_act_forward_frag): the producing conv's BN apply also
writes its output as the split-f16 fragment image the next conv's product streams, so the
consumer skips its range scan and its own split of x.  Outputs, loss and every parameter gradient
must be bit-identical to the fp32-only hand-over (the default; AUTOVC_FRAG_CHAIN=1 turns the chain
on)."""
import pytest
import torch

from autovc_amd import _lib, ops
from autovc_amd.auto_encoder import AutoEncoder
from autovc_amd.weights import onehot_embedding, synthetic_mel, torch_state_dict

pytestmark = pytest.mark.gpu


def _step(dev, chain, B, T):
    ops._FRAG_CHAIN = chain
    try:
        ae = AutoEncoder(device=dev, verbose=False)
        ae.load_state_dict(torch_state_dict(0))
        ae.to(dev).train()
        X = torch.from_numpy(synthetic_mel(81, B, T)).to(dev)
        c = torch.from_numpy(onehot_embedding(B)).to(dev)
        md, mp, mc = ae._forward_layers(X, c, c)
        loss = ae._loss(X, c, md, mp, mc)
        loss.backward()
        torch.cuda.synchronize()
        return [loss.detach(), md.detach(), mp.detach()] + [p.grad.detach().clone() for p in ae.parameters()]
    finally:
        ops._FRAG_CHAIN = False  # the default


@pytest.mark.parametrize("B,T", [(32, 64), (64, 96)])
def test_frag_chain_is_bit_identical(cuda_device, B, T):
    assert _lib.load().avc_conv_frag_chain_ok(T, B, 512, 512) == 1
    ref = _step(cuda_device, False, B, T)
    got = _step(cuda_device, True, B, T)
    for i, (a, b) in enumerate(zip(got, ref)):
        assert torch.equal(a, b), (i, float((a.double() - b.double()).abs().max()))


def test_frag_is_taken_once_and_dropped_on_modification(cuda_device):
    """The record travels with the very tensor: an in-place change (version bump) voids it, and a
    consumer takes it (the image is freed with the record)."""
    T, B = 64, 32
    g = torch.Generator().manual_seed(3)
    dev = cuda_device
    ops._FRAG_CHAIN = True
    try:
        _taken_once(dev, g, T, B)
    finally:
        ops._FRAG_CHAIN = False


def _taken_once(dev, g, T, B):
    W = ((torch.rand(512, 512, 5, generator=g) - 0.5) * 0.1).to(dev)
    z, o = torch.zeros(512, device=dev), torch.ones(512, device=dev)
    x = torch.rand(T * B, 512, generator=g).to(dev)
    y = ops.ConvBNAct.apply(x, W, z, o, z, None, None, True, 0.1, 1e-5, ops.ACT_RELU, None, T, B, True)
    assert hasattr(y, "_avc_frag")
    y2 = y.clone()
    y.mul_(1.0)  # version bump: the image no longer describes y
    a = ops.ConvBNAct.apply(y, W, z, o, z, None, None, True, 0.1, 1e-5, ops.ACT_NONE, None, T, B)
    assert not hasattr(y, "_avc_frag")
    b = ops.ConvBNAct.apply(y2, W, z, o, z, None, None, True, 0.1, 1e-5, ops.ACT_NONE, None, T, B)
    assert torch.equal(a, b)
