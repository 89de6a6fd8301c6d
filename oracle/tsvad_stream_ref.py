"""Chunk-streaming TS-VAD restated with torch.nn.functional on CPU (fp32) — oracle.

Follows egs/alimeeting/ts_vad2_streaming/model.py (TSVADModel.forward_chunk_by_chunk_temp1
:594-655, forward_chunk :657-744, forward_chunk_layer :746-882, Subsampling4 :1274-1366,
PositionalEncoding :1182-1266) and transformer_chunk_streaming.py (TransformerEncoderLayer
:435-514, MultiHeadedAttention :154-432, PositionwiseFeedForward :112-150).  `sd` is a flat
state_dict of torch tensors under the reference key names.  Pinned against
tests/golden/tsvad_stream_*.npz (the reference run here).  Test infrastructure only.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from oracle.tsvad_ref import _bn, campplus_time_out


def embed(sd, chunk_xs, n_lab):
    """Subsampling4.forward (:1321-1366): CAM++ (get_time_out) -> Conv1d k5 s2 + BN + ReLU,
    trimmed to the chunk's label count.  chunk_xs (1, T, 80) -> (1, T', 192)."""
    x = campplus_time_out(sd, chunk_xs, pre="embed.speech_encoder.")
    x = F.conv1d(x, sd["embed.speech_down_or_up.0.weight"], sd["embed.speech_down_or_up.0.bias"], stride=2, padding=2)
    x = F.relu(_bn(x, sd, "embed.speech_down_or_up.1.bn"))
    diff = x.size(-1) - n_lab
    assert -1 <= diff <= 2, f"label and ref_speech(mix speech) diff: {diff}"
    if diff == -1:
        # the reference calls nn.functinal.pad here (model.py:1358, typo): AttributeError
        raise AttributeError("module 'torch.nn' has no attribute 'functinal'")
    return x[:, :, :n_lab].transpose(1, 2)


def mha(x, sd, p, nh, cache):
    """MultiHeadedAttention.forward (:375-432) with the KV cache concatenated in front
    (_update_kv_and_cache :305-373), no mask.  x (1, T, D); cache (k, v) (1, h, t, dk) or None."""
    B, T, D = x.shape
    dk = D // nh
    q = F.linear(x, sd[p + "linear_q.weight"], sd[p + "linear_q.bias"]).view(B, T, nh, dk).transpose(1, 2)
    k = F.linear(x, sd[p + "linear_k.weight"], sd[p + "linear_k.bias"]).view(B, T, nh, dk).transpose(1, 2)
    v = F.linear(x, sd[p + "linear_v.weight"], sd[p + "linear_v.bias"]).view(B, T, nh, dk).transpose(1, 2)
    if cache is not None:
        k = torch.cat([cache[0], k], dim=2)
        v = torch.cat([cache[1], v], dim=2)
    scores = torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(dk)
    o = torch.matmul(torch.softmax(scores, dim=-1), v).transpose(1, 2).reshape(B, T, D)
    return F.linear(o, sd[p + "linear_out.weight"], sd[p + "linear_out.bias"]), (k, v)


def layer(x, sd, p, nh, cache, eps=1e-5):
    """TransformerEncoderLayer.forward, normalize_before=True (:473-514)."""
    D = x.shape[-1]
    h = F.layer_norm(x, (D,), sd[p + "norm1.weight"], sd[p + "norm1.bias"], eps)
    a, new_cache = mha(h, sd, p + "self_attn.", nh, cache)
    x = x + a
    h = F.layer_norm(x, (D,), sd[p + "norm2.weight"], sd[p + "norm2.bias"], eps)
    f = F.linear(F.relu(F.linear(h, sd[p + "feed_forward.w_1.weight"], sd[p + "feed_forward.w_1.bias"])),
                 sd[p + "feed_forward.w_2.weight"], sd[p + "feed_forward.w_2.bias"])
    return x + f, new_cache


def forward_chunk_by_chunk(sd, xs, target_speech, n_labels, decoding_chunk_size, num_decoding_left_chunks=-1,
                           nh=4, n_layers=2, ns=4):
    """forward_chunk_by_chunk_temp1: xs (1, T_fb, 80), target_speech (1, ns, 192) -> logits (1, ns, T')."""
    sub = 4
    if xs.size(1) != sub * n_labels:     # pad (or trim, when the gap is negative) to 4 * labels
        xs = F.pad(xs.permute(0, 2, 1), (0, sub * n_labels - xs.size(1))).permute(0, 2, 1)
    num_frames = xs.size(1)
    stride = sub * decoding_chunk_size
    required = decoding_chunk_size * num_decoding_left_chunks
    pe = sd["pos_encoder.pe"][0]
    E = pe.shape[-1]
    s_cache = [[None] * n_layers for _ in range(ns)]
    m_cache = [None] * n_layers
    offset, outs = 0, []
    for cur in range(0, num_frames, stride):
        end = min(cur + stride, num_frames)
        lab = math.ceil(end / 4) - math.ceil(cur / 4)
        x = embed(sd, xs[:, cur:end, :], lab)                       # (1, T, 192)
        T = x.shape[1]
        cache_t1 = 0 if s_cache[0][0] is None else s_cache[0][0][0].shape[2]
        key_size = cache_t1 + T
        nxt = 0 if required < 0 else (key_size if required == 0 else max(key_size - required, 0))
        pos = offset - cache_t1                                      # PositionalEncoding offset (:774-776)
        per_spk = []
        for j in range(ns):
            c = torch.cat([target_speech[:, j:j + 1, :].expand(1, T, -1), x], dim=2)   # (1, T, 384)
            c = c * math.sqrt(E) + pe[pos:pos + T]
            for i in range(n_layers):
                c, kv = layer(c, sd, f"single_backend.{i}.", nh, s_cache[j][i])
                s_cache[j][i] = (kv[0][:, :, nxt:], kv[1][:, :, nxt:])
            per_spk.append(c)
        cat = torch.stack(per_spk).permute(1, 0, 3, 2).reshape(1, ns * E, T)   # channel j*E + f
        y = F.conv1d(cat, sd["backend_down.0.weight"], sd["backend_down.0.bias"], padding=2)
        y = F.relu(_bn(y, sd, "backend_down.1.bn")).permute(0, 2, 1)
        for i in range(n_layers):
            y, kv = layer(y, sd, f"multi_backend.{i}.", nh, m_cache[i])
            m_cache[i] = (kv[0][:, :, nxt:], kv[1][:, :, nxt:])
        outs.append(F.linear(y, sd["fc.weight"], sd["fc.bias"]).transpose(1, 2))
        offset += T
    return torch.cat(outs, dim=2)
