"""Content encoder (reference: autovc/auto_encoder/encoder.py:7-97) on HIP kernels."""
import torch.nn as nn

from .. import ops
from .net_layers import ConvNorm, LSTMParams


def conv_bn(seq, x, T, B, act, residual=None, emit_frag=False):
    """Sequential(ConvNorm, BatchNorm1d) + act on time-major frames, honouring bn.training.
    emit_frag: the next op is another conv (its input also handed over as a split image)."""
    conv, bn = seq[0].conv, seq[1]
    training = bn.training or bn.running_mean is None
    if bn.training and bn.track_running_stats and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
    momentum = 0.1 if bn.momentum is None else bn.momentum
    return ops.ConvBNAct.apply(x, conv.weight, conv.bias, bn.weight, bn.bias, bn.running_mean,
                               bn.running_var, training, momentum, bn.eps, act, residual, T, B, emit_frag)


class Encoder(nn.Module):
    """3 x relu(BN(Conv1d k5)) over [mel ++ c_org], 2-layer BiLSTM(H=dim_neck), codes every `freq`."""

    def __init__(self, dim_neck, dim_emb, freq):
        super().__init__()
        self.dim_neck = dim_neck
        self.freq = freq
        if dim_neck != 32 or freq != 32:
            raise NotImplementedError("HIP encoder kernels are built for dim_neck = freq = 32 (hparams.py:17-20)")
        convolutions = []
        for i in range(3):
            convolutions.append(nn.Sequential(
                ConvNorm(80 + dim_emb if i == 0 else 512, 512, kernel_size=5, stride=1, padding=2,
                         dilation=1, w_init_gain="relu"),
                nn.BatchNorm1d(512)))
        self.convolutions = nn.ModuleList(convolutions)
        self.lstm = LSTMParams(512, dim_neck, 2, batch_first=True, bidirectional=True)

    def frames(self, x, c_org, save):
        """x (B,80,T), c_org (B,256) -> BiLSTM outputs [T*B][64] (fwd || bwd)."""
        B, _, T = x.shape
        h = ops.FramesFromMel.apply(x, c_org)
        for i, conv in enumerate(self.convolutions):
            h = conv_bn(conv, h, T, B, ops.ACT_RELU, emit_frag=i + 1 < len(self.convolutions))
        for l in range(2):
            h = ops.BiLSTMLayer.apply(h, *self.lstm.layer(l), *self.lstm.layer(l, True), T, B, save)
        return h

    def forward(self, x, c_org):
        """Same return as the reference: (codesA list of (B,32) at t=31,63,..; codesB at t=0,32,..)."""
        B, _, T = x.shape
        if T < self.freq:
            raise ValueError("torch.cat(): expected a non-empty list of Tensors")
        codes = ops.Codes.apply(self.frames(x, c_org, True), T, B)
        nA = T // self.freq
        chunks = codes.split(self.dim_neck, dim=-1)
        return list(chunks[:nA]), list(chunks[nA:])
