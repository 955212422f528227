"""Parameter-holding layers with the reference's names and init (net_layers.py:3-49).

ConvNorm / LinearNorm keep `.conv` / `.linear_layer` (torch Conv1d / Linear) so state_dict keys,
shapes and Xavier-uniform init match the reference exactly; their arithmetic never runs through
torch: the Generator calls the HIP kernels in autovc_amd.ops on these parameters.
"""
import math

import torch
import torch.nn as nn


class LinearNorm(nn.Module):
    """Linear layer holder, xavier_uniform init with `w_init_gain` (net_layers.py:3-20)."""

    def __init__(self, in_dim, out_dim, bias=True, w_init_gain="linear"):
        super().__init__()
        self.linear_layer = nn.Linear(in_dim, out_dim, bias=bias)
        nn.init.xavier_uniform_(self.linear_layer.weight, gain=nn.init.calculate_gain(w_init_gain))


class ConvNorm(nn.Module):
    """Conv1d holder, xavier_uniform init with `w_init_gain` (net_layers.py:23-49)."""

    def __init__(self, in_channels, out_channels, kernel_size=1, stride=1, padding=None, dilation=1,
                 bias=True, w_init_gain="linear"):
        super().__init__()
        if padding is None:
            assert kernel_size % 2 == 1
            padding = int(dilation * (kernel_size - 1) / 2)
        if (kernel_size, stride, padding, dilation) != (5, 1, 2, 1):
            raise NotImplementedError("the HIP Conv1d implements the Generator's k=5, stride 1, pad 2")
        self.conv = nn.Conv1d(in_channels, out_channels, kernel_size=kernel_size, stride=stride,
                              padding=padding, dilation=dilation, bias=bias)
        nn.init.xavier_uniform_(self.conv.weight, gain=nn.init.calculate_gain(w_init_gain))


class LSTMParams(nn.Module):
    """Holds nn.LSTM's parameters under nn.LSTM's names (weight_ih_l{k}[_reverse], ...) and its
    default U(+-1/sqrt(H)) init, without nn.LSTM's cuDNN/MIOpen weight flattening."""

    def __init__(self, input_size, hidden_size, num_layers=1, batch_first=True, bidirectional=False):
        super().__init__()
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.batch_first, self.bidirectional = batch_first, bidirectional
        D = 2 if bidirectional else 1
        for l in range(num_layers):
            for sfx in ([""] + (["_reverse"] if bidirectional else [])):
                din = input_size if l == 0 else hidden_size * D
                self.register_parameter(f"weight_ih_l{l}{sfx}", nn.Parameter(torch.empty(4 * hidden_size, din)))
                self.register_parameter(f"weight_hh_l{l}{sfx}", nn.Parameter(torch.empty(4 * hidden_size, hidden_size)))
                self.register_parameter(f"bias_ih_l{l}{sfx}", nn.Parameter(torch.empty(4 * hidden_size)))
                self.register_parameter(f"bias_hh_l{l}{sfx}", nn.Parameter(torch.empty(4 * hidden_size)))
        self.reset_parameters()

    def reset_parameters(self):
        stdv = 1.0 / math.sqrt(self.hidden_size)
        for p in self.parameters():
            nn.init.uniform_(p, -stdv, stdv)

    def layer(self, l, reverse=False):
        sfx = "_reverse" if reverse else ""
        return (getattr(self, f"weight_ih_l{l}{sfx}"), getattr(self, f"weight_hh_l{l}{sfx}"),
                getattr(self, f"bias_ih_l{l}{sfx}"), getattr(self, f"bias_hh_l{l}{sfx}"))

    def flatten_parameters(self):  # encoder.py:74 calls this on nn.LSTM; nothing to do here
        return None
