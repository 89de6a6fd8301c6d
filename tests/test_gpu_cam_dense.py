"""The fused CAM++ dense layer (cam_dense.hip, sd_op_cam_dense) against a torch-CPU restatement of
CAMDenseTDNNLayer + CAMLayer (egs/alimeeting/ts_vad2/cam_pplus_wespeaker.py:79-168) that rounds to bf16
where the kernel does (the BN-ReLU'd input and the bottleneck output h, both MFMA operands; the weights),
so the comparison isolates the kernel's arithmetic from bf16 storage.  Shapes cover the one-workgroup
items (T <= 160) and the two-part items (T > 160: the parts meet through a per-item record), dilation 1
and 2, the cut next to a ragged last tile, batches that leave a partial group of 8 items, and repeated
launches on the same monotonic counters (bit-identical each time)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from speaker_diarization_amd import _lib

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16).to(torch.float32)


def _params(cin, seed):
    g = torch.Generator().manual_seed(seed)
    r = lambda *s: torch.randn(*s, generator=g)
    return dict(s1=1 + 0.2 * r(cin), h1=0.1 * r(cin), wb=r(128, cin) / math.sqrt(cin), a2=1 + 0.2 * r(128),
                b2=0.1 * r(128), wl=r(32, 128, 3) / math.sqrt(384), bl=0.1 * r(32), w1=r(64, 128) / math.sqrt(128),
                c1=0.1 * r(64), w2=r(32, 64) / 8.0, c2=0.1 * r(32))


def _reference(x, cin, dil, p):
    """x: (B, T, ld) float (bf16 values) -> (B, T, 32) fp32 layer output (before the bf16 store)."""
    B, T, _ = x.shape
    xa = _bf(F.relu(x[:, :, :cin].double() * p["s1"].double() + p["h1"].double()).float())
    h = xa.double() @ _bf(p["wb"]).double().T
    h = _bf(F.relu(h * p["a2"].double() + p["b2"].double()).float()).double()          # (B, T, 128)
    nseg = (T + 99) // 100
    seg = torch.stack([h[:, 100 * s:min(T, 100 * (s + 1))].mean(1) for s in range(nseg)], 1)
    ctx = h.mean(1, keepdim=True) + seg                                              # (B, nseg, 128)
    hid = F.relu(ctx @ p["w1"].double().T + p["c1"].double())
    gate = torch.sigmoid(hid @ p["w2"].double().T + p["c2"].double())                 # (B, nseg, 32)
    conv = F.conv1d(h.transpose(1, 2), _bf(p["wl"]).double(), p["bl"].double(), padding=dil, dilation=dil)
    conv = conv.transpose(1, 2)                                                       # (B, T, 32)
    idx = torch.arange(T) // 100
    return (conv * gate[:, idx]).float()


def _run(gpu, x, cin, dil, p, repeats=1):
    B, T, ld = x.shape
    xd = x.to(torch.bfloat16).to(gpu).contiguous()
    dp = {k: v.float().to(gpu).contiguous() for k, v in p.items()}
    out = xd.data_ptr() + 2 * cin                       # the new channels' slice of the same map
    _lib.call("sd_op_cam_dense", _lib.ptr(xd), B, T, ld, cin, dil, *(_lib.ptr(dp[k]) for k in ("s1", "h1", "wb", "a2", "b2", "wl")),
              _lib.ptr(dp["bl"]), *(_lib.ptr(dp[k]) for k in ("w1", "c1", "w2", "c2")), out, repeats,
              _lib.stream_ptr(gpu))
    torch.cuda.synchronize()
    return xd.cpu().float()


CASES = [  # B, T, cin, dil
    (3, 299, 128, 1), (3, 299, 992, 2), (5, 160, 256, 2), (4, 161, 512, 1), (4, 162, 512, 2),
    (2, 175, 96, 2), (9, 320, 320, 2), (1, 40, 64, 1), (17, 299, 128, 2), (2, 7, 32, 1), (6, 250, 448, 1),
]


@pytest.mark.parametrize("B,T,cin,dil", CASES)
def test_cam_dense_matches_reference(gpu, B, T, cin, dil):
    ld = cin + 32 + 64                                   # channels beyond the new slice must stay untouched
    g = torch.Generator().manual_seed(B * 1000 + T + cin)
    x = _bf(torch.randn(B, T, ld, generator=g))
    p = _params(cin, T + cin)
    got = _run(gpu, x, cin, dil, p)
    ref = _reference(x, cin, dil, p)
    assert torch.equal(got[:, :, :cin], x[:, :, :cin]) and torch.equal(got[:, :, cin + 32:], x[:, :, cin + 32:])
    new = got[:, :, cin:cin + 32]
    scale = float(ref.abs().max())
    err = float((new - ref).abs().max())
    # bf16 output rounding (2^-9 relative) plus the odd 1-ulp flip of a bf16 h value between fp32 orders
    assert err <= 1.2e-2 * scale, (err, scale)
    assert float((new - ref).abs().mean()) <= 2e-3 * scale


@pytest.mark.parametrize("B,T,cin,dil", [(3, 299, 256, 2), (9, 161, 128, 1), (2, 100, 64, 2)])
def test_cam_dense_repeats_and_batch_invariance(gpu, B, T, cin, dil):
    ld = cin + 32
    g = torch.Generator().manual_seed(7 + T)
    x = _bf(torch.randn(B, T, ld, generator=g))
    p = _params(cin, 3)
    once = _run(gpu, x, cin, dil, p, repeats=1)
    again = _run(gpu, x, cin, dil, p, repeats=4)          # four launches on one set of counters / records
    assert torch.equal(once, again)
    for i in (0, B - 1):                                  # an item alone == the same item in the batch
        alone = _run(gpu, x[i:i + 1], cin, dil, p)
        assert torch.equal(alone[0], once[i])


def test_cam_dense_rejects_unsupported(gpu):
    x = torch.zeros(1, 330, 160, dtype=torch.bfloat16, device=gpu)
    p = {k: v.float().to(gpu) for k, v in _params(128, 1).items()}
    with pytest.raises(ValueError):                       # T > 320
        _lib.call("sd_op_cam_dense", _lib.ptr(x), 1, 330, 160, 128, 1, *(_lib.ptr(p[k]) for k in ("s1", "h1", "wb", "a2", "b2", "wl")),
                  _lib.ptr(p["bl"]), *(_lib.ptr(p[k]) for k in ("w1", "c1", "w2", "c2")), _lib.ptr(x), 1, _lib.stream_ptr(gpu))


HANDOVER = r"""
import sys, torch
sys.path.insert(0, {repo!r}); sys.path.insert(0, {repo!r} + "/tests")
import test_gpu_cam_dense as t
g = torch.Generator().manual_seed(5)
x = t._bf(torch.randn(5, 299, 352, generator=g))
out = t._run(torch.device("cuda", 0), x, 320, 2, t._params(320, 9), repeats=2)
torch.save(out, {path!r})
"""


def test_cam_dense_handover_matches_meet(gpu, tmp_path):
    """The first part's two ways of finishing (meet: each part its own frames; hand-over past its deadline:
    the last part finishes both from the published pre-gate conv) give the same bits.
    SDIAR_CAM_DENSE_MEET_TICKS=0 forces every hand-over (child process: the setting is read once)."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = []
    for ticks in (None, "0"):
        env = dict(os.environ)
        env.pop("SDIAR_CAM_DENSE_MEET_TICKS", None)
        if ticks is not None:
            env["SDIAR_CAM_DENSE_MEET_TICKS"] = ticks
        path = str(tmp_path / f"out_{ticks}.pt")
        r = subprocess.run([sys.executable, "-c", HANDOVER.format(repo=repo, path=path)], env=env,
                           capture_output=True, text=True, timeout=110)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(torch.load(path, weights_only=True))
    assert torch.equal(outs[0], outs[1])
    ref = _reference(_bf(torch.randn(5, 299, 352, generator=torch.Generator().manual_seed(5))), 320, 2, _params(320, 9))
    assert float((outs[1][:, :, 320:352] - ref).abs().max()) <= 1.2e-2 * float(ref.abs().max())
