"""Kernel-level parity through the C ABI vs torch-CPU fp32 references."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from speaker_diarization_amd import _lib, frontend

pytestmark = pytest.mark.gpu

FP32_TOL = dict(atol=1e-4, rtol=1e-4)
BF16_TOL = dict(atol=3e-2, rtol=3e-2)


def _tol(precision):
    return FP32_TOL if precision == 0 else BF16_TOL


_ALIVE = []


def _d(t, gpu):
    """Device copy kept alive until the test ends (a temporary's block could be
    reused by the caching allocator before the kernel reads it)."""
    x = t.to(gpu).contiguous()
    _ALIVE.append(x)
    return x.data_ptr()


@pytest.fixture(autouse=True)
def _release():
    yield
    torch.cuda.synchronize()
    _ALIVE.clear()


def _rel_err(a, b):
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


@pytest.mark.parametrize("precision", [0, 1, 2])
@pytest.mark.parametrize("M,K,N,act", [(1, 32, 4, 0), (257, 384, 1152, 0), (1000, 1536, 384, 1),
                                       (64, 512, 4, 0), (333, 96, 130, 3), (4096, 256, 2048, 2),
                                       # weight-resident streaming path (bf16 A, K % 64 == 0, M >= 2048):
                                       (20000, 384, 512, 3), (9001, 384, 1152, 0), (7777, 512, 384, 0),
                                       (5003, 448, 200, 1), (3000, 768, 96, 0), (2048, 64, 130, 2),
                                       # skinny weight-streaming path (M <= 16, streaming FS-EEND chunks):
                                       (1, 2048, 256, 0), (6, 256, 2048, 1), (16, 768, 256, 3),
                                       (12, 352, 256, 0), (3, 4864, 256, 0), (9, 256, 768, 2)])
def test_linear(gpu, precision, M, K, N, act):
    g = torch.Generator().manual_seed(M * 7 + N)
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) / math.sqrt(K)
    b = torch.randn(N, generator=g) * 0.1
    ref = F.linear(x, w, b)
    ref = [ref, F.relu(ref), torch.sigmoid(ref), F.silu(ref)][act]
    out = torch.empty(M, N, device=gpu)
    xd, wd, bd = x.to(gpu), w.to(gpu), b.to(gpu)
    _lib.call("sd_op_linear", xd.data_ptr(), M, K, wd.data_ptr(), bd.data_ptr(), N, act, out.data_ptr(),
              precision, _lib.stream_ptr(gpu))
    torch.cuda.synchronize()
    if precision == 0:
        torch.testing.assert_close(out.cpu(), ref, **FP32_TOL)
    else:
        assert _rel_err(out.cpu(), ref) < 1e-2


@pytest.mark.parametrize("precision", [0, 1, 2])
@pytest.mark.parametrize("B,T,Cin,Cout,k,stride,pad,dil", [
    (2, 299, 128, 32, 3, 1, 2, 2),     # CAM dense k3 dilation 2
    (3, 598, 320, 128, 5, 2, 2, 1),    # TDNN
    (2, 299, 512, 192, 5, 2, 2, 1),    # speech_down_or_up
    (2, 100, 1536, 384, 5, 1, 2, 1),   # backend_down
    (1, 7, 64, 40, 1, 1, 0, 1),
    (3, 150, 384, 768, 1, 1, 0, 1),    # conformer pointwise
    (2, 50, 64, 130, 3, 1, 1, 1),      # Cin % 64 == 0 multi-tap, N tail
    (2, 299, 136, 32, 1, 1, 0, 1),     # K tail (136 = 2*64 + 8)
    (1, 19, 256, 256, 19, 1, 0, 1),    # FS-EEND look-ahead conv, streaming window of 1 frame (skinny)
    (1, 26, 256, 256, 19, 1, 0, 1),    # ... 8 frames
])
def test_conv1d(gpu, precision, B, T, Cin, Cout, k, stride, pad, dil):
    g = torch.Generator().manual_seed(B * T + Cout)
    x = torch.randn(B, Cin, T, generator=g)
    w = torch.randn(Cout, Cin, k, generator=g) / math.sqrt(Cin * k)
    b = torch.randn(Cout, generator=g)
    ref = F.conv1d(x, w, b, stride=stride, padding=pad, dilation=dil).permute(0, 2, 1)
    xd = x.permute(0, 2, 1).contiguous().to(gpu)
    out = torch.empty(ref.shape, device=gpu)
    _lib.call("sd_op_conv1d", xd.data_ptr(), B, T, Cin, _d(w, gpu), _d(b, gpu), Cout, k,
              stride, pad, dil, 0, out.data_ptr(), precision, _lib.stream_ptr(gpu))
    torch.cuda.synchronize()
    if precision == 0:
        torch.testing.assert_close(out.cpu(), ref, **FP32_TOL)
    else:
        assert _rel_err(out.cpu(), ref) < 1e-2


@pytest.mark.parametrize("precision", [0, 1, 2])
@pytest.mark.parametrize("B,H,W,sh,kh,pad", [(2, 80, 50, 2, 3, 1), (1, 40, 37, 1, 3, 1), (2, 40, 21, 2, 1, 0),
                                             (2, 20, 33, 2, 3, 1), (1, 40, 300, 1, 3, 1), (3, 9, 257, 2, 3, 1),
                                             (2, 10, 598, 1, 3, 1), (2, 11, 600, 2, 3, 1)])
def test_conv2d(gpu, precision, B, H, W, sh, kh, pad):
    g = torch.Generator().manual_seed(H * W)
    x = torch.randn(B, 32, H, W, generator=g)
    w = torch.randn(32, 32, kh, kh, generator=g) / math.sqrt(32 * kh * kh)
    ref = F.conv2d(x, w, stride=(sh, 1), padding=pad).permute(0, 2, 3, 1)
    out = torch.empty(ref.shape, device=gpu)
    xd = x.permute(0, 2, 3, 1).contiguous().to(gpu)
    _lib.call("sd_op_conv2d", xd.data_ptr(), B, H, W, 32, _d(w, gpu), 32, kh, kh, sh, 1, pad, pad,
              out.data_ptr(), precision, _lib.stream_ptr(gpu))
    torch.cuda.synchronize()
    if precision == 0:
        torch.testing.assert_close(out.cpu(), ref, **FP32_TOL)
    else:
        assert _rel_err(out.cpu(), ref) < 1e-2


def _attn_ref(qkv, S, T, D, nh, causal=0, delay=0, key_len=None):
    hd = D // nh
    q, k, v = qkv.view(S, T, 3, nh, hd).permute(2, 0, 3, 1, 4)
    s = q @ k.transpose(-1, -2) / math.sqrt(hd)
    if causal:
        m = torch.ones(T, T).triu(1 + delay).bool()
        s = s.masked_fill(m, float("-inf"))
    if key_len is not None:
        km = torch.arange(T)[None, :] >= key_len[:, None]
        s = s.masked_fill(km[:, None, None, :], float("-inf"))
    return (torch.softmax(s, -1) @ v).permute(0, 2, 1, 3).reshape(S * T, D)


@pytest.mark.parametrize("precision", [0, 1, 2])
@pytest.mark.parametrize("S,T,D,nh,causal", [(8, 100, 384, 4, 0), (6, 150, 384, 8, 0), (1, 777, 256, 4, 0),
                                             (2, 300, 256, 4, 1), (3, 33, 512, 4, 0), (5, 256, 256, 4, 1),
                                             (40, 6, 256, 4, 0), (2, 129, 1024, 8, 0), (7, 3, 128, 2, 1),
                                             (33, 16, 256, 4, 1), (9, 11, 512, 4, 0)])
def test_attention(gpu, precision, S, T, D, nh, causal):
    g = torch.Generator().manual_seed(S * T)
    qkv = torch.randn(S * T, 3 * D, generator=g)
    ref = _attn_ref(qkv, S, T, D, nh, causal)
    out = torch.empty(S * T, D, device=gpu)
    _lib.call("sd_op_attention", _d(qkv, gpu), S, T, D, nh, causal, 0, None, out.data_ptr(), precision,
              _lib.stream_ptr(gpu))
    torch.cuda.synchronize()
    if precision == 0:
        torch.testing.assert_close(out.cpu(), ref, **FP32_TOL)
    else:
        assert _rel_err(out.cpu(), ref) < 2e-2


@pytest.mark.parametrize("precision", [0, 2])
@pytest.mark.parametrize("T,kls", [(70, (70, 41, 1)), (9, (9, 4, 1))])   # T <= 16: the tiny-sequence kernel
def test_attention_key_len(gpu, precision, T, kls):
    S, D, nh = 3, 384, 8
    g = torch.Generator().manual_seed(5)
    qkv = torch.randn(S * T, 3 * D, generator=g)
    kl = torch.tensor(kls, dtype=torch.int32)
    ref = _attn_ref(qkv, S, T, D, nh, key_len=kl)
    out = torch.empty(S * T, D, device=gpu)
    kld = kl.to(gpu)
    _lib.call("sd_op_attention", _d(qkv, gpu), S, T, D, nh, 0, 0, kld.data_ptr(), out.data_ptr(), precision,
              _lib.stream_ptr(gpu))
    torch.cuda.synchronize()
    if precision == 0:
        torch.testing.assert_close(out.cpu(), ref, **FP32_TOL)
    else:
        assert _rel_err(out.cpu(), ref) < 2e-2


@pytest.mark.parametrize("S,T,D,nh,causal,delay,kl", [(1, 6000, 256, 4, 1, 0, None), (2, 1000, 256, 4, 1, 3, None),
                                                       (3, 513, 128, 4, 0, 0, (513, 300, 257)),
                                                       (2, 700, 512, 4, 1, 0, (650, 700)), (1, 2000, 256, 4, 0, 0, None)])
def test_attention_long_bf16(gpu, S, T, D, nh, causal, delay, kl):
    """attn_long_kernel (T > 256, bf16 in/out: FS-EEND's causal T = 6000 encoder, the EDA T = 2000 chunks),
    incl. causal look-ahead, key lengths and head dims 32 / 64 / 128, vs the fp32 torch reference."""
    g = torch.Generator().manual_seed(T + S)
    qkv = torch.randn(S * T, 3 * D, generator=g)
    klt = None if kl is None else torch.tensor(kl, dtype=torch.int32)
    ref = _attn_ref(qkv, S, T, D, nh, causal, delay, key_len=klt)
    out = torch.empty(S * T, D, device=gpu)
    kld = None if klt is None else klt.to(gpu)
    _lib.call("sd_op_attention", _d(qkv, gpu), S, T, D, nh, causal, delay, None if kld is None else kld.data_ptr(),
              out.data_ptr(), 2, _lib.stream_ptr(gpu))
    torch.cuda.synchronize()
    assert _rel_err(out.cpu(), ref) < 2e-2


@pytest.mark.parametrize("S,T,C,D,nh,delay", [(1, 3000, 6, 256, 4, 0), (1, 2200, 4, 256, 4, 2), (2, 1100, 6, 256, 4, 0)])
def test_attention_grid_large_bf16(gpu, S, T, C, D, nh, delay):
    """The FS-EEND decoder's time attention (fs_eend.py:459-478): causal MHA per speaker slot over a
    (T, C) token grid, tokens C rows apart, bf16 io — at >= 512 workgroups (ceil(T / 64) x S*C*nh:
    1128 / 560 / 816), i.e. the large-grid attn_long_kernel variant (K / V hoisted, XCD-aware block
    order) the C5 decoder launches run, vs the fp32 torch reference of each slot's sequence."""
    g = torch.Generator().manual_seed(T + C)
    qkv = torch.randn(S, T, C, 3 * D, generator=g)
    out = torch.empty(S * T * C, D, device=gpu)
    _lib.call("sd_op_attention_grid", _d(qkv.reshape(-1, 3 * D), gpu), S, T, C, D, nh, 1, delay, out.data_ptr(), 2,
              _lib.stream_ptr(gpu))
    torch.cuda.synchronize()
    assert ((T + 63) // 64) * S * C * nh >= 512
    got = out.cpu().view(S, T, C, D)
    for c in range(C):
        seq = qkv[:, :, c].reshape(S * T, 3 * D)
        ref = _attn_ref(seq, S, T, D, nh, 1, delay).view(S, T, D)
        assert _rel_err(got[:, :, c], ref) < 2e-2, c


def _chunk_mask(T, chunk, left):
    """Key visibility of forward_chunk_by_chunk's KV caches (ts_vad2_streaming/model.py:594-655,
    transformer_chunk_streaming.py:305-373): chunks max(0, c - left) .. c."""
    c = torch.arange(T) // chunk
    vis = c[None, :] <= c[:, None]
    if left >= 0:
        vis &= c[None, :] >= c[:, None] - left
    return ~vis


@pytest.mark.parametrize("precision", [0, 1, 2])
@pytest.mark.parametrize("S,T,D,nh,chunk,left", [(4, 100, 384, 4, 25, -1), (4, 100, 384, 4, 25, 1),
                                                  (1, 64, 96, 1, 1000, -1), (2, 300, 384, 4, 16, 0),
                                                  (3, 250, 384, 4, 50, 2), (1, 77, 256, 4, 10, 3)])
def test_attention_chunk(gpu, precision, S, T, D, nh, chunk, left):
    g = torch.Generator().manual_seed(T + chunk)
    qkv = torch.randn(S * T, 3 * D, generator=g)
    hd = D // nh
    q, k, v = qkv.view(S, T, 3, nh, hd).permute(2, 0, 3, 1, 4)
    sc = (q @ k.transpose(-1, -2) / math.sqrt(hd)).masked_fill(_chunk_mask(T, chunk, left), float("-inf"))
    ref = (torch.softmax(sc, -1) @ v).permute(0, 2, 1, 3).reshape(S * T, D)
    out = torch.empty(S * T, D, device=gpu)
    _lib.call("sd_op_attention_chunk", _d(qkv, gpu), S, T, D, nh, chunk, left, out.data_ptr(), precision,
              _lib.stream_ptr(gpu))
    torch.cuda.synchronize()
    if precision == 0:
        torch.testing.assert_close(out.cpu(), ref, **FP32_TOL)
    else:
        assert _rel_err(out.cpu(), ref) < 2e-2


def test_attention_large_logits(gpu):
    """Online-softmax rescale path: a key tile far later in the sequence dominates."""
    S, T, D, nh = 1, 200, 256, 4
    g = torch.Generator().manual_seed(9)
    qkv = torch.randn(S * T, 3 * D, generator=g)
    qkv[150, D:2 * D] *= 30.0     # spike one key
    ref = _attn_ref(qkv, S, T, D, nh)
    out = torch.empty(S * T, D, device=gpu)
    _lib.call("sd_op_attention", _d(qkv, gpu), S, T, D, nh, 0, 0, None, out.data_ptr(), 0,
              _lib.stream_ptr(gpu))
    torch.cuda.synchronize()
    torch.testing.assert_close(out.cpu(), ref, atol=2e-4, rtol=2e-4)


@pytest.mark.parametrize("rows,D", [(1000, 384), (7, 256), (65, 1000)])
def test_layernorm(gpu, rows, D):
    g = torch.Generator().manual_seed(rows)
    x = torch.randn(rows, D, generator=g) * 3 + 1
    w = torch.randn(D, generator=g)
    b = torch.randn(D, generator=g)
    ref = F.layer_norm(x, (D,), w, b, 1e-5)
    out = torch.empty(rows, D, device=gpu)
    _lib.call("sd_op_layernorm", _d(x, gpu), rows, D, _d(w, gpu), _d(b, gpu), 1e-5,
              out.data_ptr(), _lib.stream_ptr(gpu))
    torch.cuda.synchronize()
    torch.testing.assert_close(out.cpu(), ref, **FP32_TOL)


def _bf16_round(x):
    return x.to(torch.bfloat16).to(torch.float32)


# (M, N, K, lda, a_coff, pre, act): ring path (tall, K <= 1024, N >= 96, bf16 out), its K
# tail / partial-N / multi-n-tile cases, the stream path (no prologue), the DMA path
# (K > 1024 or short M).  act 1 = relu (CAM++ nonlinear2).
GEMM_BF16_CASES = [(5000, 128, 640, 1024, 32, True, 1), (4096, 128, 256, 256, 0, True, 1),
                   (3000, 512, 1024, 1024, 0, True, 0), (2100, 132, 360, 400, 8, True, 1),
                   (5000, 384, 512, 512, 0, False, 0), (3000, 128, 1536, 1536, 0, True, 1),
                   (700, 128, 256, 512, 64, True, 1)]


@pytest.mark.parametrize("M,N,K,lda,a_coff,pre,act", GEMM_BF16_CASES)
def test_gemm_bf16(gpu, M, N, K, lda, a_coff, pre, act):
    g = torch.Generator().manual_seed(M + N + K)
    x = _bf16_round(torch.randn(M, lda, generator=g))
    w = torch.randn(N, K, generator=g) / K ** 0.5
    s = torch.rand(K, generator=g) + 0.5
    h = torch.randn(K, generator=g) * 0.3
    al = torch.rand(N, generator=g) + 0.5
    be = torch.randn(N, generator=g) * 0.1
    a = x[:, a_coff:a_coff + K]
    if pre:
        a = _bf16_round(torch.relu(a * s + h))
    ref = (a @ _bf16_round(w).t()) * al + be
    if act == 1:
        ref = torch.relu(ref)
    xd = x.to(torch.bfloat16).view(torch.int16).to(gpu)
    out = torch.zeros(M, N, dtype=torch.int16, device=gpu)
    _lib.call("sd_op_gemm_bf16", xd.data_ptr(), M, K, lda, a_coff, _d(w, gpu), N,
              _d(s, gpu) if pre else None, _d(h, gpu) if pre else None, _d(al, gpu), _d(be, gpu), act,
              out.data_ptr(), N, _lib.stream_ptr(gpu))
    torch.cuda.synchronize()
    got = out.cpu().view(torch.bfloat16).float()
    torch.testing.assert_close(got, _bf16_round(ref), atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("rows,D", [(1000, 384), (9, 256), (65, 1000), (333, 512)])
@pytest.mark.parametrize("t_bf16,y_bf16", [(False, False), (True, True), (True, False)])
def test_add_layernorm(gpu, rows, D, t_bf16, y_bf16):
    g = torch.Generator().manual_seed(rows + D)
    x = torch.randn(rows, D, generator=g) * 3 + 1
    t = torch.randn(rows, D, generator=g)
    w = torch.randn(D, generator=g)
    b = torch.randn(D, generator=g)
    t_in = _bf16_round(t) if t_bf16 else t
    s = x + t_in
    ref = F.layer_norm(s, (D,), w, b, 1e-5)
    xd = x.to(gpu)
    td = (t.to(torch.bfloat16).view(torch.int16) if t_bf16 else t).to(gpu)
    y = torch.empty(rows, D, device=gpu, dtype=torch.int16 if y_bf16 else torch.float32)
    _lib.call("sd_op_add_layernorm", xd.data_ptr(), td.data_ptr(), int(t_bf16), rows, D, _d(w, gpu), _d(b, gpu),
              1e-5, 1, y.data_ptr(), int(y_bf16), _lib.stream_ptr(gpu))
    torch.cuda.synchronize()
    torch.testing.assert_close(xd.cpu(), s, atol=1e-6, rtol=1e-6)
    got = y.cpu().view(torch.bfloat16).float() if y_bf16 else y.cpu()
    torch.testing.assert_close(got, _bf16_round(ref) if y_bf16 else ref, **(dict(atol=2e-2, rtol=1e-2) if y_bf16
                                                                           else FP32_TOL))


@pytest.mark.parametrize("B,T,H,ndir,lengths", [(64, 150, 256, 2, None), (1, 300, 256, 1, None),
                                                (5, 40, 256, 2, [40, 17, 1, 33, 40])])
def test_lstm(gpu, B, T, H, ndir, lengths):
    from oracle.tsvad_ref import lstm
    g = torch.Generator().manual_seed(B + T)
    I = 64
    x = torch.randn(B, T, I, generator=g)
    sd = {}
    for d, sfx in enumerate(("", "_reverse")[:ndir]):
        sd[f"l.weight_ih_l0{sfx}"] = torch.randn(4 * H, I, generator=g) / 16
        sd[f"l.weight_hh_l0{sfx}"] = torch.randn(4 * H, H, generator=g) / 16
        sd[f"l.bias_ih_l0{sfx}"] = torch.randn(4 * H, generator=g) * 0.1
        sd[f"l.bias_hh_l0{sfx}"] = torch.randn(4 * H, generator=g) * 0.1
    ref, (hn, cn) = lstm(x, sd, "l.", bidirectional=ndir == 2, lengths=lengths)
    sfxs = ("", "_reverse")[:ndir]
    gx = torch.cat([F.linear(x, sd[f"l.weight_ih_l0{s}"], sd[f"l.bias_ih_l0{s}"] + sd[f"l.bias_hh_l0{s}"])
                    for s in sfxs], -1).contiguous()
    whh = torch.stack([sd[f"l.weight_hh_l0{s}"] for s in sfxs]).contiguous()
    out = torch.zeros(B, T, ndir * H, device=gpu)
    hT = torch.empty(ndir, B, H, device=gpu)
    cT = torch.empty(ndir, B, H, device=gpu)
    work = torch.empty(3 * ndir * B * H, device=gpu)
    ld = torch.tensor(lengths, dtype=torch.int32, device=gpu) if lengths else None
    _lib.call("sd_op_lstm", _d(gx, gpu), B, T, H, ndir, _d(whh, gpu),
              ld.data_ptr() if ld is not None else None, out.data_ptr(), hT.data_ptr(), cT.data_ptr(),
              work.data_ptr(), _lib.stream_ptr(gpu))
    torch.cuda.synchronize()
    torch.testing.assert_close(out.cpu(), ref, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(hT.cpu(), hn, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(cT.cpu(), cn, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("n", [400, 16000 * 3 + 123, 16000 * 60])
def test_fbank(gpu, n):
    from oracle import fbank_ref
    rng = np.random.default_rng(n)
    wav = (rng.standard_normal(n) * 0.1).astype(np.float32)
    ref = fbank_ref.fbank(wav)
    out = frontend.kaldi_fbank(torch.from_numpy(wav).to(gpu)).cpu().numpy()
    assert out.shape == ref.shape
    np.testing.assert_allclose(out, ref, atol=2e-3, rtol=1e-4)


def test_window_cmn(gpu):
    g = torch.Generator().manual_seed(3)
    feats = torch.randn(1000, 80, generator=g) * 4 + 2
    starts = torch.tensor([0, 100, 400, 900], dtype=torch.int32)
    ns = torch.tensor([398, 398, 198, 100], dtype=torch.int32)
    out = frontend.window_cmn(feats.to(gpu), starts.to(gpu), ns.to(gpu), 398).cpu()
    for i in range(4):
        s, n = int(starts[i]), int(ns[i])
        w = feats[s:s + n]
        torch.testing.assert_close(out[i, :n], w - w.mean(0, keepdim=True), atol=1e-5, rtol=1e-5)
        assert (out[i, n:] == 0).all()


def _np_mean_lists(prob, plan):
    """infer.py:90-94 literally: per frame, np.mean of the float32 list of window values in
    window order (what res_dict[name-spk][start+t].append(p) builds, model.py:960-966)."""
    from collections import defaultdict
    ns = prob.shape[1]
    res = [defaultdict(list) for _ in range(ns)]
    for w in range(plan.n_win):
        for t in range(int(plan.lens[w])):
            for i in range(ns):
                res[i][int(plan.starts[w]) + t].append(prob[w, i, t])
    ref = np.full((ns, plan.n_labels), np.nan, np.float32)
    for i in range(ns):
        for t, v in res[i].items():
            ref[i, t] = np.mean(v)
    return ref


@pytest.mark.parametrize("n_lab,rs,shift", [(1000, 6, 1), (777, 4, 1), (613, 6, 2), (3, 4, 1), (1500, 10, 1),
                                            (901, 16, 1), (4000, 140, 1)])
def test_overlap_mean_bit_exact(gpu, n_lab, rs, shift):
    """sd_overlap_mean == np.mean over the res_dict lists, bit for bit (values chosen to make
    float32 rounding order matter).  Up to 6 windows per frame numpy sums in order; the
    streaming recipe's rs_len 10 (10 per frame), 16 and 140 (numpy's > 128 split) exercise its
    pairwise summation."""
    from speaker_diarization_amd.ts_vad.pipeline import TSVADPipeline
    from speaker_diarization_amd.ts_vad.windows import plan_windows
    plan = plan_windows(n_lab, rs, shift)
    rng = np.random.default_rng(n_lab)
    prob = rng.random((plan.n_win, 4, plan.chunk)).astype(np.float32)
    prob[:, 1] = (prob[:, 1] * 1e-4 + np.float32(0.5)).astype(np.float32)    # many ulp-level carries
    prob[:, 2] = np.float32(0.1)                                              # 0.1 is inexact in binary
    out = TSVADPipeline.mean_probs(torch.from_numpy(prob).to(gpu), plan).cpu().numpy()
    ref = _np_mean_lists(prob, plan)
    np.testing.assert_array_equal(out, ref)


def test_overlap_average(gpu):
    """sigmoid on the GPU + the same bit-exact mean: equals np.mean over torch-CPU sigmoid
    probabilities up to the sigmoid's own last-ulp differences (expf implementations differ)."""
    from speaker_diarization_amd.ts_vad.windows import plan_windows
    from speaker_diarization_amd.ts_vad.pipeline import TSVADPipeline
    plan = plan_windows(1000, 6, 1)
    g = torch.Generator().manual_seed(4)
    logits = torch.randn(plan.n_win, 4, plan.chunk, generator=g)
    out = TSVADPipeline.average(logits.to(gpu), plan).cpu().numpy()
    ref = _np_mean_lists(torch.sigmoid(logits).numpy(), plan)
    np.testing.assert_array_max_ulp(out, ref, maxulp=4)
