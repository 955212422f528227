"""Postnet (reference: autovc/auto_encoder/postnet.py:6-63) on HIP kernels."""
import torch.nn as nn

from .. import ops
from .encoder import conv_bn
from .net_layers import ConvNorm


class Postnet(nn.Module):
    """4 x tanh(BN(Conv1d k5)) 80->512->..->512, then BN(Conv1d 512->80)."""

    def __init__(self):
        super().__init__()
        self.convolutions = nn.ModuleList()
        self.convolutions.append(nn.Sequential(
            ConvNorm(80, 512, kernel_size=5, stride=1, padding=2, dilation=1, w_init_gain="tanh"),
            nn.BatchNorm1d(512)))
        for _ in range(1, 5 - 1):
            self.convolutions.append(nn.Sequential(
                ConvNorm(512, 512, kernel_size=5, stride=1, padding=2, dilation=1, w_init_gain="tanh"),
                nn.BatchNorm1d(512)))
        self.convolutions.append(nn.Sequential(
            ConvNorm(512, 80, kernel_size=5, stride=1, padding=2, dilation=1, w_init_gain="linear"),
            nn.BatchNorm1d(80)))

    def frames(self, x, T, B, residual=None):
        """x [T*B][80] -> postnet(x) (+ residual) frames [T*B][80]."""
        for i in range(len(self.convolutions) - 1):
            x = conv_bn(self.convolutions[i], x, T, B, ops.ACT_TANH, emit_frag=True)
        return conv_bn(self.convolutions[-1], x, T, B, ops.ACT_NONE, residual)

    def forward(self, x):
        """Reference signature: x (B, 80, T) -> (B, 80, T)."""
        B, _, T = x.shape
        fr = ops.FramesFromMel.apply(x, None)
        return ops.MelFromFrames.apply(self.frames(fr, T, B), T, B)
