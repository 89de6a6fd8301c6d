"""Chunk-streaming TS-VAD oracle pinned to the reference (tests/golden/tsvad_stream_*.npz, made by
tests/golden/make_golden.py from ts_vad2_streaming/model.py forward_chunk_by_chunk_temp1), plus
the identity the GPU path relies on: the per-chunk KV-cache loop equals one forward with
block-causal attention masks."""
import math
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from make_golden import TSVAD_STREAM_CASES, tsvad_stream_inputs
from oracle import tsvad_stream_ref as R
from oracle.tsvad_ref import _bn
from speaker_diarization_amd.weights import TSVADStreamingConfig, to_torch, tsvad_streaming_state_dict

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("name", list(TSVAD_STREAM_CASES))
def test_stream_oracle_matches_reference(name):
    T_lab, dcs, left, T_fb, iseed, wseed = TSVAD_STREAM_CASES[name]
    sd = to_torch(tsvad_streaming_state_dict(TSVADStreamingConfig(), seed=wseed))
    xs, ts = tsvad_stream_inputs(T_fb, iseed)
    with torch.no_grad():
        y = R.forward_chunk_by_chunk(sd, torch.from_numpy(xs), torch.from_numpy(ts), T_lab, dcs, left).numpy()
    g = np.load(os.path.join(GOLD, name + ".npz"))["logits"]
    assert y.shape == g.shape == (1, 4, T_lab)
    np.testing.assert_allclose(y, g, atol=2e-5, rtol=1e-5)


def _block_mha(x, sd, p, nh, C, left):
    B, T, D = x.shape
    dk = D // nh
    q, k, v = (F.linear(x, sd[p + f"linear_{n}.weight"], sd[p + f"linear_{n}.bias"]).view(B, T, nh, dk).transpose(1, 2)
               for n in ("q", "k", "v"))
    s = q @ k.transpose(-2, -1) / math.sqrt(dk)
    qc = torch.arange(T)[:, None] // C
    kc = torch.arange(T)[None, :] // C
    vis = (kc <= qc) & ((kc >= qc - left) if left >= 0 else torch.ones_like(kc, dtype=torch.bool))
    s = s.masked_fill(~vis, float("-inf"))
    o = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B, T, D)
    return F.linear(o, sd[p + "linear_out.weight"], sd[p + "linear_out.bias"])


def _block_layer(x, sd, p, C, left):
    D = x.shape[-1]
    x = x + _block_mha(F.layer_norm(x, (D,), sd[p + "norm1.weight"], sd[p + "norm1.bias"]), sd, p + "self_attn.", 4,
                       C, left)
    h = F.layer_norm(x, (D,), sd[p + "norm2.weight"], sd[p + "norm2.bias"])
    return x + F.linear(F.relu(F.linear(h, sd[p + "feed_forward.w_1.weight"], sd[p + "feed_forward.w_1.bias"])),
                        sd[p + "feed_forward.w_2.weight"], sd[p + "feed_forward.w_2.bias"])


@pytest.mark.parametrize("name", list(TSVAD_STREAM_CASES))
def test_cache_loop_equals_block_causal_forward(name):
    """What libsdiar computes: chunk-batched embed, block-causal attention, PE offsets
    max(0, c - left) * C (0 with the whole history cached), chunk-local backend_down."""
    T_lab, C, left, T_fb, iseed, wseed = TSVAD_STREAM_CASES[name]
    sd = to_torch(tsvad_streaming_state_dict(TSVADStreamingConfig(), seed=wseed))
    xs, ts = tsvad_stream_inputs(T_fb, iseed)
    xs = torch.from_numpy(xs)
    xs = F.pad(xs.permute(0, 2, 1), (0, 4 * T_lab - xs.size(1))).permute(0, 2, 1)
    ts = torch.from_numpy(ts)
    bounds = [(c0, min(c0 + C, T_lab)) for c0 in range(0, T_lab, C)]
    with torch.no_grad():
        mix = torch.cat([R.embed(sd, xs[:, 4 * a:4 * b], b - a) for a, b in bounds], 1)      # (1, T, 192)
        pe = sd["pos_encoder.pe"][0]
        pos = torch.tensor([(0 if left < 0 else max(0, t // C - left) * C) + t % C for t in range(T_lab)])
        spk = []
        for j in range(4):
            x = torch.cat([ts[:, j:j + 1].expand(1, T_lab, -1), mix], 2) * math.sqrt(384) + pe[pos]
            for i in range(2):
                x = _block_layer(x, sd, f"single_backend.{i}.", C, left)
            spk.append(x)
        cat = torch.stack(spk).permute(1, 0, 3, 2).reshape(1, 4 * 384, T_lab)
        y = torch.cat([F.relu(_bn(F.conv1d(cat[:, :, a:b], sd["backend_down.0.weight"], sd["backend_down.0.bias"],
                                           padding=2), sd, "backend_down.1.bn")) for a, b in bounds], 2).permute(0, 2, 1)
        for i in range(2):
            y = _block_layer(y, sd, f"multi_backend.{i}.", C, left)
        out = F.linear(y, sd["fc.weight"], sd["fc.bias"]).transpose(1, 2).numpy()
    g = np.load(os.path.join(GOLD, name + ".npz"))["logits"]
    np.testing.assert_allclose(out, g, atol=5e-5, rtol=1e-4)
