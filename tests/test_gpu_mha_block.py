"""mha_block (the C2 conformer's in-projection + multi-head attention in one launch, mha_block.hip) through
sd_op_mha_block against a plain torch fp32 restatement of torchaudio's MHA core (ts_vad2/model.py:259-267 ->
torch.nn.MultiheadAttention: q/k/v = y W^T + b, softmax(q k^T / sqrt(48)) v per head, key_padding_mask from
the lengths), on bf16 inputs.  Every kernel layout sd_op_mha_block can launch (0: the shipped <SEQ 2, 8 waves,
3-slot ring, 48-wide Q / K rows>; 1-7: the round-5 sweep's other layouts, mha_block.hip) must agree with the
reference within bf16 rounding and with each other bit for bit."""
import numpy as np
import pytest
import torch

from speaker_diarization_amd import _lib

pytestmark = pytest.mark.gpu


def _ref(y, w, b, key_len):
    S, T, D = y.shape
    qkv = y.float() @ w.t() + b
    q, k, v = qkv.split(D, -1)
    q = q.view(S, T, 8, 48).transpose(1, 2) / np.sqrt(48.0)
    k = k.view(S, T, 8, 48).transpose(1, 2)
    v = v.view(S, T, 8, 48).transpose(1, 2)
    sc = q @ k.transpose(-1, -2)
    if key_len is not None:
        mask = torch.arange(T, device=y.device)[None, :] >= key_len[:, None]
        sc = sc.masked_fill(mask[:, None, None, :], float("-inf"))
    return (sc.softmax(-1) @ v).transpose(1, 2).reshape(S, T, D)


def _run(y, w, b, key_len, variant, flags=0):
    S, T, D = y.shape
    out = torch.zeros(S, T, D, device=y.device, dtype=torch.bfloat16)
    _lib.call("sd_op_mha_block", _lib.ptr(y), _lib.ptr(w), _lib.ptr(b), S, T,
              _lib.ptr(key_len) if key_len is not None else None, _lib.ptr(out), variant, flags,
              _lib.stream_ptr(y.device))
    torch.cuda.synchronize()
    return out


def _tile(x):
    """(S, T, 384) rows -> the row programs' MFMA-fragment layout (kernels.h RowProgArgs::a_tiled): 16-row group g,
    fragment kk (features 32 kk ..), lane l = row % 16 + 16 q holds features 32 kk + 8 q .. + 7 of row 16 g + l % 16."""
    S, T, D = x.shape
    r = x.reshape(S * T // 16, 16, D // 32, 4, 8)          # (group, row, kk, q, 8)
    return r.permute(0, 2, 3, 1, 4).contiguous().reshape(S, T, D)


def _untile(x):
    S, T, D = x.shape
    r = x.reshape(S * T // 16, D // 32, 4, 16, 8)           # (group, kk, q, row, 8)
    return r.permute(0, 3, 1, 2, 4).contiguous().reshape(S, T, D)


@pytest.mark.parametrize("S,T,lens", [(4, 150, False), (7, 150, True), (3, 100, False), (5, 37, True), (1, 160, False)])
def test_mha_block_layouts(gpu, S, T, lens):
    g = torch.Generator().manual_seed(S * 1000 + T)
    y = torch.randn(S, T, 384, generator=g).to(torch.bfloat16).to(gpu)
    w = (torch.randn(1152, 384, generator=g) * 384 ** -0.5).to(gpu)
    b = (torch.randn(1152, generator=g) * 0.1).to(gpu)
    key_len = torch.randint(1, T + 1, (S,), generator=g, dtype=torch.int32).to(gpu) if lens else None
    ref = _ref(y, w.to(torch.bfloat16).float(), b, key_len)
    outs = [_run(y, w, b, key_len, v) for v in range(8)]   # every layout mha_block() can launch
    for v, o in enumerate(outs):
        err = (o.float() - ref).abs()
        print(f"layout {v}: max err {err.max().item():.3e}; worst (seq, token, feature) {np.unravel_index(int(err.argmax()), err.shape)}")
        assert err.max().item() < 3e-2, v
    for v in range(1, 8):
        assert torch.equal(outs[0], outs[v]), v



@pytest.mark.parametrize("S,T", [(8, 150), (3, 160), (2, 96)])
def test_mha_block_tiled_layouts_bit_identical(gpu, S, T):
    """The production hand-offs: y read in the row programs' fragment layout and the output written in
    it (encoder.cpp's tiled_y / tiled_a) give the row-major call's bits once de-tiled on the host."""
    g = torch.Generator().manual_seed(S * 7 + T)
    y = torch.randn(S, T, 384, generator=g).to(torch.bfloat16).to(gpu)
    w = (torch.randn(1152, 384, generator=g) * 384 ** -0.5).to(gpu)
    b = (torch.randn(1152, generator=g) * 0.1).to(gpu)
    key_len = torch.randint(1, T + 1, (S,), generator=g, dtype=torch.int32).to(gpu)
    base = _run(y, w, b, key_len, -1)
    assert torch.equal(_untile(_tile(y)), y)
    for flags in (1, 2, 3):
        yin = _tile(y) if flags & 1 else y
        out = _run(yin, w, b, key_len, -1, flags)
        out = _untile(out) if flags & 2 else out
        assert torch.equal(out, base), flags


def test_mha_block_nonfinite_masked_rows(gpu):
    """Rows past key_len holding Inf / NaN (with 48-wide Q / K rows a key row's features 0..15 meet the
    zeroed Q lanes of the key before it, and 0 * Inf = NaN).  The kernel never reads a 32-key tile that starts at or
    past key_len, so non-finite rows there leave every visible query finite and equal to the reference computed with
    those rows replaced by finite values -- where torch's MHA returns NaN for the whole sequence (the masked key's
    weight 0 times its non-finite value row).  A non-finite row inside the last visited tile (past key_len) turns the
    sequence NaN, as it does in torch.  The product never sees either case: a TS-VAD window with a non-finite input
    is poisoned to NaN upstream (tsvad.cpp nonfinite_windows / poison_windows) and its sequences are whole (no
    key_len).  (Zeroing the masked K / V rows in the projection epilogue was measured: +9 % mha_block time on C2.)"""
    S, T = 5, 150
    g = torch.Generator().manual_seed(99)
    y = torch.randn(S, T, 384, generator=g)
    key_len = torch.tensor([150, 120, 90, 150, 90], dtype=torch.int32)
    clean = y.clone()
    y[1, 130:] = float("inf")         # past the last visited tile (keys 96..127)
    y[2, 100, 5] = float("nan")       # past the last visited tile (keys 64..95)
    y[4, 91, 0] = float("-inf")       # inside the last visited tile, past key_len
    w = (torch.randn(1152, 384, generator=g) * 384 ** -0.5).to(gpu)
    b = (torch.randn(1152, generator=g) * 0.1).to(gpu)
    kl = key_len.to(gpu)
    ref = _ref(clean.to(torch.bfloat16).to(gpu), w.to(torch.bfloat16).float(), b, kl)
    ref_raw = _ref(y.to(torch.bfloat16).to(gpu), w.to(torch.bfloat16).float(), b, kl)
    out = _run(y.to(torch.bfloat16).to(gpu), w, b, kl, -1).float()
    for s_ in range(4):
        n = int(key_len[s_])                       # the visible queries (every row past key_len is padding)
        o, r = out[s_, :n], ref[s_, :n]
        assert torch.isfinite(o).all(), s_
        assert (o - r).abs().max().item() < 3e-2, s_
    assert torch.isnan(ref_raw[1:3]).all()         # torch: NaN for those sequences
    n = int(key_len[4])
    assert torch.isnan(out[4, :n]).all() and torch.isnan(ref_raw[4, :n]).all()
