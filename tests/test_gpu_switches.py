"""Every kernel A/B switch the shipping library reads from the environment (SDIAR_NO_* and friends)
selects another implementation of the same op; each is exercised here against the reference goldens,
so no environment-reachable path goes untested.  Round 6 deleted every switch whose variant DESIGN.md records
as measured and dropped (and, where nothing else reached it, the variant's code): 17 remain -- the 8 kernel
fallbacks below (SDIAR_NO_ROWPROG, _CAM_DENSE, _ATTN_LONG, _MHA_BLOCK, _AREG_GEMM, _RING_GEMM, _STREAM_GEMM,
_LSTM_SEQ), SDIAR_LSTM_FP32 (the exact recurrence in bf16 mode, a precision diagnostic), SDIAR_CAM_ONE_STREAM (one
launch sequence, bit-identical: test below), SDIAR_CAM_DENSE_MEET_TICKS (test_gpu_cam_dense.py), the LSTM spin
limits (test_gpu_lstm_status.py), SDIAR_PROF_DETAIL (profiler key names), and the build / A-B plumbing
SDIAR_LIB, SDIAR_ARCH, SDIAR_TSS_WINDOWS (bench.py).  A switch is read once per process, so each group
runs in ONE child process (sequentially, one at a time) over the bf16 model goldens it affects:
TS-VAD ots_vad v1 (C2: CAM++ trunk, conformer, BiLSTM) and CAM++/transformer v0, FS-EEND (causal
encoder, fusion decoder, T = 700 long-attention case vs the oracle) and EEND-EDA.  Tolerances are the
bf16 bounds of test_gpu_tsvad.py / test_gpu_fseend.py / test_gpu_eda.py.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

GROUPS = {
    "rowprog_off+camdense_off+long_off": {"SDIAR_NO_ROWPROG": "1", "SDIAR_NO_CAM_DENSE": "1", "SDIAR_NO_ATTN_LONG": "1"},
    "mha_off+areg_off+lstm_fp32": {"SDIAR_NO_MHA_BLOCK": "1", "SDIAR_NO_AREG_GEMM": "1", "SDIAR_LSTM_FP32": "1"},
    "ring_off+stream_off+lstmseq_off": {"SDIAR_NO_RING_GEMM": "1", "SDIAR_NO_STREAM_GEMM": "1", "SDIAR_NO_LSTM_SEQ": "1"},
}

CHILD = r"""
import json, os, sys
import numpy as np, torch
sys.path.insert(0, {repo!r}); sys.path.insert(0, os.path.join({repo!r}, "tests", "golden"))
from make_golden import TSVAD_CASES, FSEEND_CASES, EDA_CASES, tsvad_inputs, eda_inputs
from oracle import fseend_ref
from speaker_diarization_amd.ts_vad.model import TSVADModel
from speaker_diarization_amd.fs_eend.model import OnlineTransformerDADiarization
from speaker_diarization_amd.eend_eda.models import EendEdaModel, TransformerEdaModel
from speaker_diarization_amd.weights import (TSVADConfig, tsvad_state_dict, FSEENDConfig, fseend_state_dict,
                                             EDAConfig, eda_state_dict, to_torch)
G = os.path.join({repo!r}, "tests", "golden")
dev = torch.device("cuda", 0)
res = {{}}
for name, (v, rs, B, T, nl, iseed, wseed) in TSVAD_CASES.items():
    cfg = TSVADConfig(rs_len=rs) if v == 0 else TSVADConfig.ots_vad_v1(rs_len=rs)
    m = TSVADModel(cfg, device=dev, precision="bf16", max_batch=8)
    m.load_state_dict(to_torch(tsvad_state_dict(cfg, seed=wseed)))
    x, ts = tsvad_inputs(B, T, nl, seed=iseed)
    for rep in range(2):      # a repeated call reuses the handle's workspaces
        out = m.forward(torch.from_numpy(x).to(dev), torch.from_numpy(ts).to(dev), nl).cpu().numpy()
    # the main test's bf16 bound (test_gpu_tsvad.py BF16_ATOL): every switch setting is held to it
    res["tsvad/" + name] = (float(np.abs(out - np.load(os.path.join(G, name + ".npz"))["logits"]).max()), 1.5e-2)
def fse(delay, wseed, T=512):
    m = OnlineTransformerDADiarization(None, 345, 256, 4, 4, 2, 0.1, True, 10000, 2048, conv_delay=9,
                                       mask_delay=delay, precision="bf16", max_seqs=2, max_frames=T, max_nspks=6)
    m.load_state_dict(to_torch(fseend_state_dict(FSEENDConfig(mask_delay=delay), seed=wseed)))
    return m
for name, (lens, C, delay, iseed, wseed) in FSEEND_CASES.items():
    g = np.load(os.path.join(G, name + ".npz"))
    out, emb, att = fse(delay, wseed).test([torch.from_numpy(x) for x in eda_inputs(lens, seed=iseed)], lens, max_nspks=C)
    res["fseend/" + name] = (float(np.abs(torch.cat(out).cpu().numpy() - g["out"]).max()), 3e-2)
T = 700
x = eda_inputs([T], seed=77)
out, _, _ = fse(0, 797, T).test([torch.from_numpy(x[0])], [T], max_nspks=6)
ro, _, _ = fseend_ref.fseend_test(to_torch(fseend_state_dict(FSEENDConfig(), seed=797)), FSEENDConfig(),
                                  [torch.from_numpy(x[0])], [T], 6)
res["fseend/T700_vs_oracle"] = (float(np.abs(out[0].cpu().numpy() - ro[0].numpy()).max()), 3e-2)
for name, (mtype, L, lens, nspk, iseed, wseed) in EDA_CASES.items():
    torch.manual_seed(777)
    if mtype == "TransformerEda":
        m = TransformerEdaModel(n_speakers=2, in_size=345, n_heads=4, n_units=256, n_layers=L, has_pos=False,
                                precision="bf16")
    else:
        m = EendEdaModel(n_speakers=2, in_size=345, n_heads=4, n_units=256, n_layers=L,
                         encoder_type="conformer" if mtype == "ConformerEda" else "transformer", precision="bf16")
    m.load_state_dict(to_torch(eda_state_dict(EDAConfig(model_type=mtype, n_layers=L), seed=wseed)))
    g = np.load(os.path.join(G, name + ".npz"))
    offs = np.cumsum([0] + lens)
    err = 0.0
    for i, xi in enumerate(eda_inputs(lens, seed=iseed)):
        feats, ilens = m._pad_src([torch.from_numpy(xi)])
        act, probs = m.forward_infer(feats, ilens, [torch.from_numpy(g["perms"][offs[i]:offs[i + 1]])], 15,
                                     key_len=ilens if mtype == "ConformerEda" else None)
        err = max(err, float(np.abs(act[0].cpu().numpy() - g["act"][i, : lens[i]]).max()),
                  float(np.abs(probs[0].cpu().numpy() - g["probs"][i]).max()))
    res["eda/" + name] = (err, 3e-2)
print("RESULT " + json.dumps(res))
"""


@pytest.mark.parametrize("group", list(GROUPS))
def test_switch_group_matches_goldens(gpu, group):
    env = dict(os.environ)
    env.update(GROUPS[group])
    r = subprocess.run([sys.executable, "-c", CHILD.format(repo=REPO)], capture_output=True, text=True,
                       timeout=110, env=env)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert r.returncode == 0 and line, (r.stdout[-2000:], r.stderr[-3000:])
    res = json.loads(line[0][len("RESULT "):])
    bad = {k: v for k, v in res.items() if not v[0] < v[1]}
    print(group, {k: round(v[0], 5) for k, v in res.items()})
    assert not bad, bad


TSVAD_BITS_CHILD = r"""
import hashlib, os, sys
import numpy as np, torch
sys.path.insert(0, {repo!r}); sys.path.insert(0, os.path.join({repo!r}, "tests", "golden"))
from make_golden import tsvad_inputs
from speaker_diarization_amd.ts_vad.model import TSVADModel
from speaker_diarization_amd.weights import TSVADConfig, tsvad_state_dict, to_torch
dev = torch.device("cuda", 0)
h = hashlib.sha256()
for v in (1, 0):
    cfg = TSVADConfig(rs_len=4) if v == 0 else TSVADConfig.ots_vad_v1(rs_len=4)
    B = 400
    m = TSVADModel(cfg, device=dev, precision="bf16", max_batch=B)
    m.load_state_dict(to_torch(tsvad_state_dict(cfg, seed=11)))
    x, ts = tsvad_inputs(B, 398, 100, seed=5)
    out = m.forward(torch.from_numpy(x).to(dev), torch.from_numpy(ts).to(dev), 100)
    h.update(out.float().cpu().numpy().tobytes())
print("HASH " + h.hexdigest())
"""


def test_cam_two_stream_slices_bit_identical(gpu):
    """TS-VAD batches of >= 384 windows run the CAM++ trunk as two window slices on two streams
    (tsvad.cpp); the logits must be bit-identical to one launch sequence over the whole batch."""
    hashes = []
    for one in (False, True):
        env = dict(os.environ)
        env.pop("SDIAR_CAM_ONE_STREAM", None)
        if one:
            env["SDIAR_CAM_ONE_STREAM"] = "1"
        r = subprocess.run([sys.executable, "-c", TSVAD_BITS_CHILD.format(repo=REPO)], capture_output=True,
                           text=True, timeout=110, env=env)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("HASH ")]
        assert r.returncode == 0 and line, (r.stdout[-2000:], r.stderr[-3000:])
        hashes.append(line[0])
    assert hashes[0] == hashes[1], hashes
