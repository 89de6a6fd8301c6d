"""FS-EEND / plain-EEND inference restated on CPU — TEST INFRASTRUCTURE ONLY.

FS-EEND (speaker_diarization/fs_eend/fs_eend.py):
  OnlineTransformerDADiarization.test          :79-96
  MaskedTransformerEncoderModel.forward        :178-204 (BatchNorm1d, Linear, LN, causal encoder)
  _generate_square_subsequent_mask             :168-171 / 120-123 (mask_delay)
  MaskedTransformerDecoderModel.forward        :125-134 (convert(cat(emb, slot PE)))
  PositionalEncoding.forward                   :234-240 (returns only the slot PE)
  TransformerEncoderFusionLayer.forward        :343-478 (slow path: src is 4-D)
Plain EEND (speaker_diarization/eend/models.py):
  TransformerModel.forward                     :69-101 (activation=sigmoid from eend_infer.py:69)
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .tsvad_ref import mha, transformer_layer


def causal_mask(T, mask_delay=0):
    m = (torch.triu(torch.ones(T, T), diagonal=-mask_delay) == 1).transpose(0, 1)
    return m.float().masked_fill(m == 0, float("-inf")).masked_fill(m == 1, 0.0)


@torch.no_grad()
def encoder(sd, cfg, src):
    """MaskedTransformerEncoderModel.forward: list of (T_i, in) -> (B, T, E)."""
    x = torch.nn.utils.rnn.pad_sequence(list(src), padding_value=-1, batch_first=True).float()
    x = F.batch_norm(x.transpose(1, 2), sd["enc.bn.running_mean"], sd["enc.bn.running_var"],
                     sd["enc.bn.weight"], sd["enc.bn.bias"], False, 0.0, 1e-5).transpose(1, 2)
    mask = causal_mask(x.shape[1], cfg.mask_delay) if cfg.has_mask else None
    x = F.linear(x, sd["enc.encoder.weight"], sd["enc.encoder.bias"])
    x = F.layer_norm(x, (cfg.n_units,), sd["enc.encoder_norm.weight"], sd["enc.encoder_norm.bias"], 1e-5)
    x = x.transpose(0, 1)
    for i in range(cfg.enc_n_layers):
        x = transformer_layer(x, sd, f"enc.transformer_encoder.layers.{i}.", cfg.n_heads, causal_mask=mask)
    return x.transpose(0, 1)


def _mha_bf(x, sd, p, nh, mask=None):
    """batch_first MultiheadAttention on (N, L, E)."""
    return mha(x.transpose(0, 1), sd, p, nh, causal_mask=mask).transpose(0, 1)


@torch.no_grad()
def fusion_layer(src, sd, p, nh, t_mask):
    """TransformerEncoderFusionLayer.forward, norm_first=False (fs_eend.py:456-478)."""
    B, T, C, D = src.shape
    ln = lambda x, n: F.layer_norm(x, (D,), sd[p + n + ".weight"], sd[p + n + ".bias"], 1e-5)
    x = src.transpose(1, 2).reshape(B * C, T, D)
    x = ln(x + _mha_bf(x, sd, p + "self_attn1.", nh, t_mask), "norm11")
    x = x.reshape(B, C, T, D).transpose(1, 2).reshape(B * T, C, D)
    x = ln(x + _mha_bf(x, sd, p + "self_attn2.", nh), "norm21")
    h = F.linear(F.relu(F.linear(x, sd[p + "linear1.weight"], sd[p + "linear1.bias"])),
                 sd[p + "linear2.weight"], sd[p + "linear2.bias"])
    x = ln(x + h, "norm22")
    return x.reshape(B, T, C, D)


@torch.no_grad()
def decoder(sd, cfg, emb, max_nspks):
    """MaskedTransformerDecoderModel.forward (the same layer object dec_n_layers times;
    torch's load_state_dict leaves the LAST index's tensors in it)."""
    B, T, D = emb.shape
    pe = sd["dec.pos_enc.pe"][:, :max_nspks, :]
    pe = pe.unsqueeze(0).repeat(B, T, 1, 1)
    x = torch.cat([emb.unsqueeze(2).repeat(1, 1, max_nspks, 1), pe], dim=-1)
    x = F.linear(x, sd["dec.convert.weight"], sd["dec.convert.bias"])
    t_mask = causal_mask(T, cfg.mask_delay)
    p = f"dec.attractor_decoder.{cfg.dec_n_layers - 1}."
    for _ in range(cfg.dec_n_layers):
        x = fusion_layer(x, sd, p, cfg.n_heads, t_mask)
    return x


@torch.no_grad()
def fseend_test(sd, cfg, src, ilens, max_nspks=6):
    """OnlineTransformerDADiarization.test -> (output list (T_i, C), emb list, attractors list)."""
    emb = encoder(sd, cfg, src)
    emb = torch.nn.utils.rnn.pad_sequence([e[:n] for e, n in zip(emb, ilens)], padding_value=0, batch_first=True)
    k = sd["cnn.weight"].shape[-1]
    emb = F.conv1d(emb.transpose(1, 2), sd["cnn.weight"], sd["cnn.bias"], padding=9).transpose(1, 2)
    emb = emb / torch.norm(emb, dim=-1, keepdim=True)
    att = decoder(sd, cfg, emb, max_nspks)
    att = att / torch.norm(att, dim=-1, keepdim=True)
    out = torch.matmul(emb.unsqueeze(-2), att.transpose(-1, -2)).squeeze(-2)
    return ([o[:n] for o, n in zip(out, ilens)], [e[:n] for e, n in zip(emb, ilens)],
            [a[:n] for a, n in zip(att, ilens)])


@torch.no_grad()
def eend_forward(sd, n_layers, n_heads, src, activation=torch.sigmoid):
    """eend/models.py TransformerModel.forward(src, has_mask=False, activation)."""
    ilens = [x.shape[0] for x in src]
    x = torch.nn.utils.rnn.pad_sequence(list(src), padding_value=-1, batch_first=True).float()
    x = F.linear(x, sd["encoder.weight"], sd["encoder.bias"])
    x = F.layer_norm(x, (x.shape[-1],), sd["encoder_norm.weight"], sd["encoder_norm.bias"], 1e-5)
    x = x.transpose(0, 1)
    for i in range(n_layers):
        x = transformer_layer(x, sd, f"transformer_encoder.layers.{i}.", n_heads)
    x = F.linear(x.transpose(0, 1), sd["decoder.weight"], sd["decoder.bias"])
    if activation:
        x = activation(x)
    return [o[:n] for o, n in zip(x, ilens)]
