"""Debug helper: long-sequence attention (sd_op_attention, bf16 io) vs a torch fp32 reference on the GPU,
reporting which query rows / head dims are off.  python tools/attn_dbg.py"""
import math, sys, torch
sys.path.insert(0, '.')
from speaker_diarization_amd import _lib
dev = torch.device('cuda', 0)
def ref(qkv, S, T, D, nh, causal=0):
    hd = D // nh
    q, k, v = qkv.view(S, T, 3, nh, hd).permute(2, 0, 3, 1, 4)
    s = q @ k.transpose(-1, -2) / math.sqrt(hd)
    if causal:
        m = torch.ones(T, T, device=qkv.device).triu(1).bool()
        s = s.masked_fill(m, float('-inf'))
    return (torch.softmax(s, -1) @ v).permute(0, 2, 1, 3).reshape(S * T, D)
for (S, T, D, nh, c) in [(1, 300, 256, 4, 0), (1, 320, 256, 4, 1), (1, 384, 256, 4, 0), (1, 300, 64, 1, 0)]:
    g = torch.Generator().manual_seed(T)
    qkv = torch.randn(S * T, 3 * D, generator=g).to(dev)
    r = ref(qkv, S, T, D, nh, c)
    out = torch.empty(S * T, D, device=dev)
    _lib.call("sd_op_attention", qkv.data_ptr(), S, T, D, nh, c, 0, None, out.data_ptr(), 2, _lib.stream_ptr(dev))
    torch.cuda.synchronize()
    e = (out - r).abs()
    print(S, T, D, nh, c, 'max err', round(e.max().item(), 4), 'ref max', round(r.abs().max().item(), 4))
    rows = e.max(1).values
    bad = (rows > 0.05).nonzero().flatten().cpu()
    if bad.numel():
        print('  bad rows', bad.numel(), 'wave hist', torch.bincount((bad % 64) // 16, minlength=4).tolist(),
              'l15 hist', torch.bincount(bad % 16, minlength=16).tolist(), 'qblock hist',
              torch.bincount(bad // 64, minlength=(T + 63) // 64).tolist())
        cols = e[bad].max(0).values
        print('  bad cols per head-dim group', [(int(x), round(float(cols[x]), 3)) for x in (cols > 0.05).nonzero().flatten()[:12]])
