"""Decoder (reference: autovc/auto_encoder/decoder.py:5-79) on HIP kernels."""
import torch.nn as nn

from .. import ops
from .encoder import conv_bn
from .net_layers import ConvNorm, LinearNorm, LSTMParams


class Decoder(nn.Module):
    """LSTM(320->512), 3 x relu(BN(Conv1d)), 2-layer LSTM(512->1024), Linear(1024->80)."""

    def __init__(self, dim_neck, dim_emb, dim_pre):
        super().__init__()
        self.lstm1 = LSTMParams(dim_neck * 2 + dim_emb, dim_pre, 1, batch_first=True)
        convolutions = []
        for i in range(3):
            convolutions.append(nn.Sequential(
                ConvNorm(dim_pre, dim_pre, kernel_size=5, stride=1, padding=2, dilation=1,
                         w_init_gain="relu"),
                nn.BatchNorm1d(dim_pre)))
        self.convolutions = nn.ModuleList(convolutions)
        self.lstm2 = LSTMParams(dim_pre, 1024, 2, batch_first=True)
        self.linear_projection = LinearNorm(1024, 80)

    def frames(self, x, T, B, save):
        """x [T*B][320] time-major frames -> decoder output frames [T*B][80]."""
        h = ops.LSTMLayer.apply(x, *self.lstm1.layer(0), T, B, save)
        for i, conv in enumerate(self.convolutions):
            h = conv_bn(conv, h, T, B, ops.ACT_RELU, emit_frag=i + 1 < len(self.convolutions))
        for l in range(2):
            h = ops.LSTMLayer.apply(h, *self.lstm2.layer(l), T, B, save)
        lin = self.linear_projection.linear_layer
        return ops.Linear.apply(h, lin.weight, lin.bias)

    def forward(self, x):
        """Reference signature: x (B, T, 320) batch-first -> (B, T, 80)."""
        B, T, C = x.shape
        fr = x.transpose(0, 1).reshape(T * B, C)
        out = self.frames(fr, T, B, True)
        return out.reshape(T, B, -1).transpose(0, 1)
