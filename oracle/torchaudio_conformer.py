"""nn.Module shell with torchaudio.models.Conformer's parameter names whose
forward is oracle.tsvad_ref.conformer — TEST INFRASTRUCTURE ONLY.

torchaudio (2.5.1 pinned by the reference requirements) is not installed, so
the golden script installs this class as `torchaudio.models.Conformer` to run
the reference's own forward_common_ots_vad (model.py:669-756) end to end.  That
pins everything around the conformer; the conformer arithmetic itself is
"parity unpinned" (restated from the published torchaudio algorithm).
"""
import torch
from torch import nn

from .tsvad_ref import conformer as _conformer


class _FFN(nn.Module):
    def __init__(self, d, h):
        super().__init__()
        self.sequential = nn.Sequential(nn.LayerNorm(d), nn.Linear(d, h), nn.SiLU(), nn.Dropout(0.0),
                                        nn.Linear(h, d), nn.Dropout(0.0))


class _Conv(nn.Module):
    def __init__(self, d, k, group_norm):
        super().__init__()
        self.layer_norm = nn.LayerNorm(d)
        self.sequential = nn.Sequential(
            nn.Conv1d(d, 2 * d, 1), nn.GLU(dim=1), nn.Conv1d(d, d, k, padding=(k - 1) // 2, groups=d),
            nn.GroupNorm(1, d) if group_norm else nn.BatchNorm1d(d), nn.SiLU(), nn.Conv1d(d, d, 1), nn.Dropout(0.0))


class _Layer(nn.Module):
    def __init__(self, d, ffn, nh, k, group_norm):
        super().__init__()
        self.ffn1 = _FFN(d, ffn)
        self.self_attn_layer_norm = nn.LayerNorm(d)
        self.self_attn = nn.MultiheadAttention(d, nh)
        self.self_attn_dropout = nn.Dropout(0.0)
        self.conv_module = _Conv(d, k, group_norm)
        self.ffn2 = _FFN(d, ffn)
        self.final_layer_norm = nn.LayerNorm(d)


class Conformer(nn.Module):
    def __init__(self, input_dim, num_heads, ffn_dim, num_layers, depthwise_conv_kernel_size,
                 dropout=0.0, use_group_norm=False, convolution_first=False):
        super().__init__()
        assert not convolution_first
        self.num_heads = num_heads
        self.use_group_norm = use_group_norm
        self.num_layers = num_layers
        self.conformer_layers = nn.ModuleList(
            [_Layer(input_dim, ffn_dim, num_heads, depthwise_conv_kernel_size, use_group_norm)
             for _ in range(num_layers)])

    def forward(self, x, lengths):
        sd = {k: v.detach() for k, v in self.state_dict().items()}
        return _conformer(x, lengths.cpu(), sd, "", num_layers=self.num_layers, nh=self.num_heads,
                           group_norm=self.use_group_norm), lengths
