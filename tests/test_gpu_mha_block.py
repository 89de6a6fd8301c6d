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


def _run(y, w, b, key_len, variant):
    S, T, D = y.shape
    out = torch.zeros(S, T, D, device=y.device, dtype=torch.bfloat16)
    _lib.call("sd_op_mha_block", _lib.ptr(y), _lib.ptr(w), _lib.ptr(b), S, T,
              _lib.ptr(key_len) if key_len is not None else None, _lib.ptr(out), variant, _lib.stream_ptr(y.device))
    torch.cuda.synchronize()
    return out


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
