"""TS-VAD forward restated with torch.nn.functional on CPU (fp32) — oracle.

Follows egs/alimeeting/ts_vad2/model.py and cam_pplus_wespeaker.py of the
reference.  `sd` is a flat state_dict of torch tensors under the reference key
names.  Pinned against tests/golden/tsvad_*.npz (reference outputs), except the
torchaudio Conformer block (parity unpinned: torchaudio 2.5.1 is absent; see
conformer() below).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F


def _bn(x, sd, p, eps=1e-5):
    """Eval BatchNorm over dim 1 (nn.BatchNorm1d/2d in eval())."""
    w = sd.get(p + ".weight")
    b = sd.get(p + ".bias")
    return F.batch_norm(x, sd[p + ".running_mean"], sd[p + ".running_var"], w, b, False, 0.0, eps)


def _bn1d_nan_bypass(x, sd, p):
    """BatchNorm1D (model.py:161-171): the wrapped eval BatchNorm1d runs only when the WHOLE input tensor
    (the forward's batch) holds no NaN; otherwise the input passes through unchanged for every window."""
    return _bn(x, sd, p) if int(torch.isnan(x).sum()) == 0 else x


# ----------------------------------------------------------------------------- CAM++
def fcm(sd, x, pre="speech_encoder.head."):
    """FCM.forward (cam_pplus_wespeaker.py:299-308). x: (B, F, T) -> (B, 320, T)."""
    x = x.unsqueeze(1)
    out = F.relu(_bn(F.conv2d(x, sd[pre + "conv1.weight"], padding=1), sd, pre + "bn1"))
    for layer in (1, 2):
        for blk in (0, 1):
            q = f"{pre}layer{layer}.{blk}."
            stride = 2 if blk == 0 else 1
            # BasicResBlock.forward (236-268)
            y = F.relu(_bn(F.conv2d(out, sd[q + "conv1.weight"], stride=(stride, 1), padding=1), sd, q + "bn1"))
            y = _bn(F.conv2d(y, sd[q + "conv2.weight"], padding=1), sd, q + "bn2")
            if q + "shortcut.0.weight" in sd:
                sc = _bn(F.conv2d(out, sd[q + "shortcut.0.weight"], stride=(stride, 1)), sd, q + "shortcut.1")
            else:
                sc = out
            out = F.relu(y + sc)
    out = F.relu(_bn(F.conv2d(out, sd[pre + "conv2.weight"], stride=(2, 1), padding=1), sd, pre + "bn2"))
    b, c, f, t = out.shape
    return out.reshape(b, c * f, t)


def cam_layer(sd, q, x, dilation):
    """CAMLayer.forward (cam_pplus_wespeaker.py:106-123)."""
    y = F.conv1d(x, sd[q + "linear_local.weight"], sd.get(q + "linear_local.bias"),
                 padding=dilation, dilation=dilation)
    seg = F.avg_pool1d(x, kernel_size=100, stride=100, ceil_mode=True)
    seg = seg.unsqueeze(-1).expand(*seg.shape, 100).reshape(*seg.shape[:-1], -1)[..., : x.shape[-1]]
    context = x.mean(-1, keepdim=True) + seg
    context = F.relu(F.conv1d(context, sd[q + "linear1.weight"], sd[q + "linear1.bias"]))
    m = torch.sigmoid(F.conv1d(context, sd[q + "linear2.weight"], sd[q + "linear2.bias"]))
    return y * m


def campplus_time_out(sd, fbank, pre="speech_encoder."):
    """CAMPPlus.forward(x, get_time_out=True) (cam_pplus_wespeaker.py:388-399):
    (B, T, 80) -> (B, 512, T')  = xvector[:-2] (no stats / dense)."""
    x = fcm(sd, fbank.permute(0, 2, 1), pre + "head.")
    xv = pre + "xvector."
    x = F.relu(_bn(F.conv1d(x, sd[xv + "tdnn.linear.weight"], stride=2, padding=2), sd, xv + "tdnn.nonlinear.batchnorm"))
    for b, (n, dil) in enumerate(zip((12, 24, 16), (1, 2, 2))):
        for i in range(n):
            q = f"{xv}block{b + 1}.tdnnd{i + 1}."
            # CAMDenseTDNNLayer.forward (158-167), CAMDenseTDNNBlock.forward (199-202)
            h = F.conv1d(F.relu(_bn(x, sd, q + "nonlinear1.batchnorm")), sd[q + "linear1.weight"])
            h = cam_layer(sd, q + "cam_layer.", F.relu(_bn(h, sd, q + "nonlinear2.batchnorm")), dil)
            x = torch.cat([x, h], dim=1)
        q = f"{xv}transit{b + 1}."
        # TransitLayer.forward (213-216)
        x = F.conv1d(F.relu(_bn(x, sd, q + "nonlinear.batchnorm")), sd[q + "linear.weight"], sd.get(q + "linear.bias"))
    return F.relu(_bn(x, sd, xv + "out_nonlinear.batchnorm"))


def campplus_embedding(sd, fbank, pre=""):
    """CAMPPlus.forward(x) (get_time_out=False, cam_pplus_wespeaker.py:388-399): xvector[:-2]
    -> StatsPool (mean, unbiased std over time, :28-39) -> DenseLayer(1024 -> E, batchnorm_)
    (:219-233).  (B, T, 80) -> (B, E)."""
    x = campplus_time_out(sd, fbank, pre)
    stats = torch.cat([x.mean(dim=-1), x.std(dim=-1, unbiased=True)], dim=-1)
    y = F.conv1d(stats.unsqueeze(-1), sd[pre + "xvector.dense.linear.weight"]).squeeze(-1)
    return _bn(y, sd, pre + "xvector.dense.nonlinear.batchnorm")


def embedding_chunks(n_samples, length_embedding=6.0, step_embedding=1.0, sr=16000):
    """Chunk plan of extract_embed (generate_chunk_..._for_diarization.py:271-299): starts
    range(0, N - L, step) when N > L (so a chunk ending exactly at N is never taken), else the
    whole file as one chunk.  Returns [(start, stop)]."""
    L, S = int(length_embedding * sr), int(step_embedding * sr)
    if n_samples > L:
        return [(s, s + L) for s in range(0, n_samples - L, S)]
    return [(0, n_samples)]


def extract_embed(sd, wav, length_embedding=6.0, step_embedding=1.0, batch_size=96):
    """extract_embed (:271-304) with FBank(80, mean_nor=True) (:307-331, :336): wav float64
    in [-1, 1) -> (n_chunks, E) float32 (the tensor torch.save writes, :351)."""
    from oracle.fbank_ref import embed_fbank
    feats = [embed_fbank(wav[a:b]) for a, b in embedding_chunks(len(wav), length_embedding, step_embedding)]
    out = []
    for i in range(0, len(feats), batch_size):
        out.append(campplus_embedding(sd, torch.from_numpy(np.stack(feats[i:i + batch_size]))))
    return torch.cat(out)


# ----------------------------------------------------------------------------- encoders
def mha(x, sd, p, nh, key_padding_mask=None, causal_mask=None):
    """nn.MultiheadAttention (batch_first=False, need_weights=False) on (T, B, E)."""
    T, B, E = x.shape
    hd = E // nh
    qkv = F.linear(x, sd[p + "in_proj_weight"], sd[p + "in_proj_bias"])
    q, k, v = qkv.split(E, dim=-1)

    def heads(t):
        return t.reshape(T, B * nh, hd).transpose(0, 1)  # (B*nh, T, hd)

    q, k, v = heads(q), heads(k), heads(v)
    s = torch.bmm(q, k.transpose(1, 2)) / math.sqrt(hd)
    if causal_mask is not None:
        s = s + causal_mask
    if key_padding_mask is not None:
        s = s.view(B, nh, T, T).masked_fill(key_padding_mask[:, None, None, :], float("-inf")).view(B * nh, T, T)
    a = torch.softmax(s, dim=-1)
    o = torch.bmm(a, v).transpose(0, 1).reshape(T, B, E)
    return F.linear(o, sd[p + "out_proj.weight"], sd[p + "out_proj.bias"])


def transformer_layer(x, sd, p, nh, eps=1e-5, causal_mask=None):
    """nn.TransformerEncoderLayer (post-LN, ReLU, eval) on (T, B, E)."""
    e = x.shape[-1]
    x = F.layer_norm(x + mha(x, sd, p + "self_attn.", nh, causal_mask=causal_mask), (e,),
                     sd[p + "norm1.weight"], sd[p + "norm1.bias"], eps)
    h = F.linear(F.relu(F.linear(x, sd[p + "linear1.weight"], sd[p + "linear1.bias"])),
                 sd[p + "linear2.weight"], sd[p + "linear2.bias"])
    return F.layer_norm(x + h, (e,), sd[p + "norm2.weight"], sd[p + "norm2.bias"], eps)


def conformer(x, lengths, sd, p, num_layers=6, nh=8, eps=1e-5, group_norm=True):
    """torchaudio.models.Conformer(input_dim, num_heads, ffn_dim, num_layers,
    depthwise_conv_kernel_size=31, use_group_norm).forward in eval (GroupNorm(1, D)
    for TS-VAD ots_vad, model.py:259-267; BatchNorm1d for EendEdaModel, models.py:502) —
    restated from the published torchaudio 2.5.1 algorithm (parity unpinned:
    torchaudio is not installed here).  x: (B, T, D) -> (B, T, D)."""
    B, T, E = x.shape
    kpm = torch.arange(T)[None, :] >= lengths[:, None]
    x = x.transpose(0, 1)  # (T, B, E)

    def ffn(y, q):
        h = F.layer_norm(y, (E,), sd[q + "sequential.0.weight"], sd[q + "sequential.0.bias"], eps)
        h = F.silu(F.linear(h, sd[q + "sequential.1.weight"], sd[q + "sequential.1.bias"]))
        return F.linear(h, sd[q + "sequential.4.weight"], sd[q + "sequential.4.bias"])

    for i in range(num_layers):
        q = f"{p}conformer_layers.{i}."
        x = ffn(x, q + "ffn1.") * 0.5 + x
        r = x
        h = F.layer_norm(x, (E,), sd[q + "self_attn_layer_norm.weight"], sd[q + "self_attn_layer_norm.bias"], eps)
        x = mha(h, sd, q + "self_attn.", nh, key_padding_mask=kpm) + r
        # _ConvolutionModule (input (B, T, D))
        r = x
        c = F.layer_norm(x.transpose(0, 1), (E,), sd[q + "conv_module.layer_norm.weight"],
                         sd[q + "conv_module.layer_norm.bias"], eps).transpose(1, 2)  # (B, E, T)
        c = F.conv1d(c, sd[q + "conv_module.sequential.0.weight"], sd[q + "conv_module.sequential.0.bias"])
        c = F.glu(c, dim=1)
        k = sd[q + "conv_module.sequential.2.weight"].shape[-1]
        c = F.conv1d(c, sd[q + "conv_module.sequential.2.weight"], sd[q + "conv_module.sequential.2.bias"],
                     padding=(k - 1) // 2, groups=E)
        n = q + "conv_module.sequential.3."
        if group_norm:
            c = F.group_norm(c, 1, sd[n + "weight"], sd[n + "bias"], eps)
        else:
            c = F.batch_norm(c, sd[n + "running_mean"], sd[n + "running_var"], sd[n + "weight"], sd[n + "bias"],
                             False, 0.0, eps)
        c = F.silu(c)
        c = F.conv1d(c, sd[q + "conv_module.sequential.5.weight"], sd[q + "conv_module.sequential.5.bias"])
        x = c.permute(2, 0, 1) + r
        x = ffn(x, q + "ffn2.") * 0.5 + x
        x = F.layer_norm(x, (E,), sd[q + "final_layer_norm.weight"], sd[q + "final_layer_norm.bias"], eps)
    return x.transpose(0, 1)


def lstm(x, sd, p, bidirectional=True, h0=None, c0=None, lengths=None):
    """torch.nn.LSTM(batch_first=True) single layer, gate order i,f,g,o.
    x: (B, T, I) -> out (B, T, ndir*H), (h_n, c_n) each (ndir, B, H).
    With `lengths`, follows pack_padded_sequence semantics."""
    B, T, _ = x.shape
    outs, hs, cs = [], [], []
    for d, sfx in enumerate(("", "_reverse") if bidirectional else ("",)):
        wih, whh = sd[f"{p}weight_ih_l0{sfx}"], sd[f"{p}weight_hh_l0{sfx}"]
        b = sd[f"{p}bias_ih_l0{sfx}"] + sd[f"{p}bias_hh_l0{sfx}"]
        H = whh.shape[1]
        gx = F.linear(x, wih, b)
        h = torch.zeros(B, H) if h0 is None else h0[d].clone()
        c = torch.zeros(B, H) if c0 is None else c0[d].clone()
        out = torch.zeros(B, T, H)
        L = torch.full((B,), T) if lengths is None else torch.as_tensor(lengths)
        for s in range(T):
            active = s < L
            t = torch.where(torch.tensor(d == 0), torch.full((B,), s), L - 1 - s).clamp(min=0)
            z = gx[torch.arange(B), t] + h @ whh.t()
            i, f, g, o = z.chunk(4, dim=-1)
            cn = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
            hn = torch.sigmoid(o) * torch.tanh(cn)
            m = active[:, None]
            c = torch.where(m, cn, c)
            h = torch.where(m, hn, h)
            out[torch.arange(B)[active], t[active]] = hn[active]
        outs.append(out)
        hs.append(h)
        cs.append(c)
    return torch.cat(outs, dim=-1), (torch.stack(hs), torch.stack(cs))


def positional_encoding(x, sd):
    """PositionalEncoding.forward (model.py:152-158), dropout off: x (T, B, E)."""
    return x + sd["pos_encoder.pe"][: x.size(0)]


# ----------------------------------------------------------------------------- TS-VAD
def speech_encoder_out(sd, ref_speech):
    """CAM++ time output + speech_down_or_up (model.py:844-848 / 683-687) -> (B, 192, T')."""
    x = campplus_time_out(sd, ref_speech)
    x = F.conv1d(x, sd["speech_down_or_up.0.weight"], sd["speech_down_or_up.0.bias"], stride=2, padding=2)
    return F.relu(_bn1d_nan_bypass(x, sd, "speech_down_or_up.1.bn"))


@torch.no_grad()
def tsvad_forward(sd, cfg, ref_speech, target_speech, max_len):
    """TSVADModel.forward in eval (model.py:899-921): ref_speech (B, T_fb, 80),
    target_speech (B, NS, 192) -> logits (B, NS, max_len)."""
    ns = cfg.max_num_speaker
    x = speech_encoder_out(sd, ref_speech)
    if cfg.variant == 1:
        # forward_common_ots_vad (model.py:669-756)
        mean = x.mean(dim=1, keepdim=True)
        std = x.std(dim=1, keepdim=True)
        stats = torch.cat([mean, std], dim=1).permute(0, 2, 1)
        x = F.linear(stats, sd["gsp_fc.weight"], sd["gsp_fc.bias"]).permute(0, 2, 1)
        gap = x.size(-1) - max_len
        assert abs(gap) <= 3, f"label and ref_speech(mix speech) diff: {gap}"
        if gap < 0:
            x = F.pad(x, (0, -gap))
        x = x[:, :, :max_len]
        mix = x.transpose(1, 2)
        B, T, _ = mix.shape
        outs = []
        for i in range(ns):
            cat = torch.cat((target_speech[:, i, None, :].expand(B, T, -1), mix), 2)
            outs.append(conformer(cat, torch.full((B,), T), sd, "single_backend."))
        cat = torch.cat(outs, dim=-1)
        h, _ = lstm(cat, sd, "multi_backend.", bidirectional=True)
        return F.linear(h, sd["fc.weight"], sd["fc.bias"]).transpose(1, 2)
    # forward_common (model.py:758-897)
    gap = x.size(-1) - max_len
    assert -1 <= gap <= 2, f"label and ref_speech(mix speech) diff: {gap}"
    if gap == -1:
        x = F.pad(x, (0, 1))   # intended behaviour of model.py:853 (`nn.functinal` typo there)
    x = x[:, :, :max_len]
    mix = x.transpose(1, 2)
    B, T, _ = mix.shape
    nh = cfg.num_attention_head
    outs = []
    for i in range(ns):
        cat = torch.cat((target_speech[:, i, None, :].expand(B, T, -1), mix), 2).transpose(0, 1)
        cat = positional_encoding(cat, sd)
        for l in range(cfg.num_transformer_layer):
            cat = transformer_layer(cat, sd, f"single_backend.layers.{l}.", nh)
        outs.append(cat.transpose(0, 1))
    cat = torch.stack(outs).permute(1, 0, 3, 2).reshape(B, -1, T)
    cat = F.relu(_bn1d_nan_bypass(F.conv1d(cat, sd["backend_down.0.weight"], sd["backend_down.0.bias"], padding=2),
                                  sd, "backend_down.1.bn"))
    cat = positional_encoding(cat.permute(2, 0, 1), sd)
    for l in range(cfg.num_transformer_layer):
        cat = transformer_layer(cat, sd, f"multi_backend.layers.{l}.", nh)
    return F.linear(cat.transpose(0, 1), sd["fc.weight"], sd["fc.bias"]).transpose(1, 2)
