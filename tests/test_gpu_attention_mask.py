"""In-kernel attention masks, dumped pair by pair (sd_probe_attention_mask).

Round-1's verdict asked for the chunk-mask failure to be root-caused: a per-key division form of
the chunk-visibility term (chunk(key) <= chunk(query), chunk(x) = x / chunk) was replaced by the
per-query key window without a reproducer, while the same unrolled predicate also carries the
causal and key_len terms.  These tests record every (query, key) decision the kernels make for
sequence 0 / head 0 and compare it with the host mask of

  ts_vad2_streaming/model.py:594-655 (forward_chunk_by_chunk's KV caches = block-causal mask),
  fs_eend/fs_eend.py:163-171 (causal with delay), nn.MultiheadAttention key_padding_mask,

for the product's key-window form in all three kernel instantiations the product uses (fp32 long,
bf16 long with fp32 io, bf16 short with bf16 io).  (Round 2 also ran the per-key division form and
that form over the unclipped key range through this probe: both agreed with the host mask, so the
round-1 "miscompile" diagnosis was wrong — DESIGN.md §5; round 3 removed those diagnostic forms from
the shipping kernels.)
"""
import math

import numpy as np
import pytest
import torch

from speaker_diarization_amd import _lib

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _host_visible(T, klen, causal, delay, chunk, left):
    q = np.arange(T)[:, None]
    k = np.arange(T)[None, :]
    vis = k < klen
    if causal:
        vis = vis & (k <= q + delay)
    if chunk:
        vis = vis & (k // chunk <= q // chunk)
        if left >= 0:
            vis = vis & (k // chunk >= q // chunk - left)
    return np.broadcast_to(vis, (T, T))


def _torch_ref(qkv, S, T, D, nh, vis):
    hd = D // nh
    q, k, v = qkv.view(S, T, 3, nh, hd).permute(2, 0, 3, 1, 4)
    sc = (q @ k.transpose(-1, -2) / math.sqrt(hd)).masked_fill(~torch.from_numpy(vis.copy()), float("-inf"))
    p = torch.softmax(sc, -1).nan_to_num(0.0)
    return (p @ v).permute(0, 2, 1, 3).reshape(S * T, D)


CASES = [
    # S, T, D, nh, causal, delay, klen, chunk, left
    (4, 100, 384, 4, 0, 0, None, 25, -1),      # tsvad_stream_c25 shape (the round-1 failure)
    (4, 100, 384, 4, 0, 0, None, 25, 1),
    (2, 300, 384, 4, 0, 0, None, 16, 0),
    (3, 250, 384, 4, 0, 0, None, 50, 2),
    (1, 77, 256, 4, 0, 0, None, 10, 3),
    (2, 60, 384, 4, 0, 0, None, 10, 2),        # tsvad_stream_c10_l2 shape
    (2, 70, 384, 4, 0, 0, None, 25, -1),       # ragged last chunk
    (2, 200, 256, 4, 1, 0, None, 0, -1),       # FS-EEND causal
    (2, 200, 256, 4, 1, 5, None, 0, -1),       # causal with look-ahead
    (3, 150, 384, 8, 0, 0, 97, 0, -1),         # key padding
    (2, 130, 384, 8, 0, 0, 61, 20, 1),         # key padding + chunk window
]


@pytest.mark.parametrize("precision", [0, 1, 2])
@pytest.mark.parametrize("S,T,D,nh,causal,delay,klen,chunk,left", CASES)
def test_kernel_mask_matches_host(gpu, precision, S, T, D, nh, causal, delay, klen, chunk, left):
    g = torch.Generator().manual_seed(T * 7 + chunk + 3 * causal + delay)
    qkv = torch.randn(S * T, 3 * D, generator=g)
    key_len = None
    kl_host = T
    if klen is not None:
        key_len = torch.full((S,), T, dtype=torch.int32)
        key_len[0] = klen
        kl_host = klen
    dump = torch.zeros(T * T, dtype=torch.int32, device=gpu)
    out = torch.empty(S * T, D, device=gpu)
    kld = key_len.to(gpu) if key_len is not None else None
    _lib.call("sd_probe_attention_mask", qkv.to(gpu).data_ptr(), S, T, D, nh, causal, delay,
              kld.data_ptr() if kld is not None else None, chunk, left, dump.data_ptr(), out.data_ptr(),
              precision, _lib.stream_ptr(gpu))
    torch.cuda.synchronize()
    d = dump.cpu().numpy().reshape(T, T)
    vis = _host_visible(T, kl_host, causal, delay, chunk, left)
    visited = d != 0
    # every visible pair was visited and judged visible; every visited pair agrees with the host
    bad_missed = np.argwhere(vis & ~visited)
    assert bad_missed.size == 0, f"visible pairs never visited (query, key): {bad_missed[:8].tolist()}"
    got = d == 1
    wrong = np.argwhere(visited & (got != vis))
    assert wrong.size == 0, f"mask decisions differ from the host at (query, key): {wrong[:8].tolist()}"
    # and the output of sequence 0 follows from that mask
    vis_all = np.broadcast_to(vis, (T, T))
    ref = _torch_ref(qkv[:T], 1, T, D, nh, vis_all)
    o = out.cpu()[:T]
    if precision == 0:
        torch.testing.assert_close(o, ref, rtol=1e-3, atol=1e-3)
    else:
        assert (o - ref).norm() / ref.norm().clamp_min(1e-12) < 2e-2
