"""SSND inference restated with torch.nn.functional on CPU (fp32) — TEST INFRASTRUCTURE ONLY.

Follows egs/alimeeting/ssnd/ssnd_model.py of the reference:
  ResNetExtractor 'CAM++_wo_gsp'      :107-124, :164-170  (CAMPPlusWithGSP.forward,
                                                            cam_pplus_wespeaker.py:513-525)
  SSNDConformerEncoder                :172-195             (torchaudio Conformer, unpinned)
  FqFusion / FkFusion                 :198-222
  SWDecoderBlockV2                    :224-272
  DetectionDecoder                    :274-296
  RepresentationDecoder               :343-370
  SSNDModel.infer                     :752-776
  SSNDModel.offline_diarization       :778-800
Pinned by tests/golden/ssnd_*.npz (tests/golden/make_ssnd_golden.py imports the reference
module here): the decoders bit-for-bit in fp32 arithmetic, the whole infer with the restated
torchaudio Conformer injected (as for C2, parity of that block is unpinned).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .tsvad_ref import _bn, campplus_time_out, conformer


def mha_bf(q_in, k_in, v_in, sd, p, nh):
    """nn.MultiheadAttention(batch_first=True, need_weights unused) on (B, Nq, D) x (B, Tk, D)."""
    B, Nq, D = q_in.shape
    Tk = k_in.shape[1]
    hd = D // nh
    W, b = sd[p + "in_proj_weight"], sd[p + "in_proj_bias"]
    q = F.linear(q_in, W[:D], b[:D]).view(B, Nq, nh, hd).transpose(1, 2)
    k = F.linear(k_in, W[D:2 * D], b[D:2 * D]).view(B, Tk, nh, hd).transpose(1, 2)
    v = F.linear(v_in, W[2 * D:], b[2 * D:]).view(B, Tk, nh, hd).transpose(1, 2)
    a = torch.softmax(q @ k.transpose(-2, -1) / math.sqrt(hd), dim=-1)
    o = (a @ v).transpose(1, 2).reshape(B, Nq, D)
    return F.linear(o, sd[p + "out_proj.weight"], sd[p + "out_proj.bias"])


def decoder_block(sd, p, x_dec, x_fea, q_aux, k_pos, nh):
    """SWDecoderBlockV2.forward (ssnd_model.py:246-272), eval (dropout off)."""
    D = x_dec.shape[-1]
    s = D ** 0.5
    Q = x_dec + F.linear(q_aux, sd[p + "fq.linear.weight"], sd[p + "fq.linear.bias"]) / s
    K = x_fea + F.linear(k_pos, sd[p + "fk.linear.weight"], sd[p + "fk.linear.bias"]) / s
    x = F.layer_norm(x_dec + mha_bf(Q, K, x_fea, sd, p + "cross_attn.", nh), (D,), sd[p + "norm1.weight"],
                     sd[p + "norm1.bias"], 1e-5)
    x = F.layer_norm(x + mha_bf(x, x, x, sd, p + "self_attn.", nh), (D,), sd[p + "norm2.weight"],
                     sd[p + "norm2.bias"], 1e-5)
    h = F.linear(F.relu(F.linear(x, sd[p + "ffn.0.weight"], sd[p + "ffn.0.bias"])), sd[p + "ffn.3.weight"],
                 sd[p + "ffn.3.bias"])
    return F.layer_norm(x + h, (D,), sd[p + "norm3.weight"], sd[p + "norm3.bias"], 1e-5)


def detection_decoder(sd, cfg, x_dec, x_fea, q_aux, k_pos, pre="det_decoder."):
    """DetectionDecoder.forward (:286-296): L2-normalised auxiliary queries -> layers -> out_proj."""
    q_aux = F.normalize(q_aux, p=2, dim=-1)
    for i in range(cfg.num_layers):
        x_dec = decoder_block(sd, f"{pre}layers.{i}.", x_dec, x_fea, q_aux, k_pos, cfg.nhead)
    return F.linear(x_dec, sd[pre + "out_proj.weight"], sd[pre + "out_proj.bias"])


def representation_decoder(sd, cfg, x_dec, x_fea, q_aux, k_pos, pre="rep_decoder."):
    """RepresentationDecoder.forward (:356-370)."""
    x_fea = F.linear(x_fea, sd[pre + "input_proj.weight"], sd[pre + "input_proj.bias"])
    x = F.linear(x_dec.mean(-1, keepdim=True), sd[pre + "xdec_proj.weight"], sd[pre + "xdec_proj.bias"])
    qa = F.linear(q_aux.mean(-1, keepdim=True), sd[pre + "qaux_proj.weight"], sd[pre + "qaux_proj.bias"])
    for i in range(cfg.num_layers):
        x = decoder_block(sd, f"{pre}layers.{i}.", x, x_fea, qa, k_pos, cfg.nhead)
    return F.linear(x, sd[pre + "out_proj.weight"], sd[pre + "out_proj.bias"])


def extractor(sd, feats, pre="extractor."):
    """ResNetExtractor('CAM++_wo_gsp').forward (:164-170): CAMPPlusWithGSP (xvector[:-2] incl.
    out_nonlinear, then output_proj; cam_pplus_wespeaker.py:513-525) -> Conv1d k5 s2 + BN + ReLU."""
    x = campplus_time_out(sd, feats, pre + "speech_encoder.")            # (B, 512, T')
    x = F.linear(x.permute(0, 2, 1), sd[pre + "speech_encoder.output_proj.weight"],
                 sd[pre + "speech_encoder.output_proj.bias"])              # (B, T', 256)
    x = F.conv1d(x.permute(0, 2, 1), sd[pre + "speech_down_or_up.0.weight"], sd[pre + "speech_down_or_up.0.bias"],
                 stride=2, padding=2)
    return F.relu(_bn(x, sd, pre + "speech_down_or_up.1.bn")).permute(0, 2, 1)


def encoder(sd, cfg, x, pre="encoder."):
    """SSNDConformerEncoder.forward (:186-195): input_proj -> Conformer(lengths = T)."""
    x = F.linear(x, sd[pre + "input_proj.weight"], sd[pre + "input_proj.bias"])
    lengths = torch.full((x.shape[0],), x.shape[1], dtype=torch.long)
    return conformer(x, lengths, sd, pre + "encoder.", num_layers=cfg.num_layers, nh=cfg.nhead,
                     group_norm=False)


def decode(sd, cfg, enc_out, x, speaker_embs):
    """infer (:762-776) after the encoder: (vad_pred (B, N, T), emb_pred (B, N, S))."""
    B, T, _ = enc_out.shape
    N = speaker_embs.shape[1]
    pos = sd["pos_emb"][:, :T, :].expand(B, T, cfg.pos_emb_dim)
    x_det = sd["det_query_emb"].unsqueeze(0).expand(B, N, cfg.d_model)
    x_rep = sd["rep_query_emb"].unsqueeze(0).expand(B, N, T)
    vad = detection_decoder(sd, cfg, x_det, enc_out, speaker_embs, pos)
    emb = representation_decoder(sd, cfg, x_rep, x, torch.sigmoid(vad), pos)
    return vad, emb


@torch.no_grad()
def infer(sd, cfg, feats, speaker_embs):
    """SSNDModel.infer (:752-776): feats (B, T_fb, 80) -> (vad_pred, emb_pred)."""
    x = extractor(sd, feats)
    enc = encoder(sd, cfg, x)
    return decode(sd, cfg, enc, x, speaker_embs)
