"""Where the bf16 TS-VAD (C2: ots_vad v1) error comes from: the same windows through an fp32 and a bf16
handle, stage buffers compared (sd_tsvad_debug_buffer: 0 mix = speech_down_or_up conv + bias, 1 mixg =
gsp_fc, 2 X2 = conformer stack output (bf16 in bf16 mode), 3 H = BiLSTM input projection (gates), 4 Y =
BiLSTM output) plus logits and posteriors (GPU box).  With a weight variant ('plain', 'dynamic', 'spread') the
inputs are the bench meeting's first B windows (product fbank + window CMN) and every stage's error is also quoted
against that stage's variation across frames (the signal a DER decision rides on).
    python3 tools/parity_stages.py [B] [variant]"""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from speaker_diarization_amd import _lib
from speaker_diarization_amd.ts_vad.model import TSVADModel
from speaker_diarization_amd.weights import TSVADConfig, to_torch, tsvad_state_dict

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
VAR = sys.argv[2] if len(sys.argv) > 2 else None
dev = torch.device("cuda", 0)
cfg = TSVADConfig.ots_vad_v1(rs_len=6)
T = 150
if VAR is None:
    sd = to_torch(tsvad_state_dict(cfg, seed=779))
    g = torch.Generator().manual_seed(11)
    x = (torch.randn(B, 598, 80, generator=g) * 3 + 1).to(dev)
    ts = torch.randn(B, 4, 192, generator=g).to(dev)
else:
    from speaker_diarization_amd.frontend import kaldi_fbank, window_cmn
    from speaker_diarization_amd.synth import make_meeting, speaker_embeddings
    from speaker_diarization_amd.ts_vad.windows import plan_windows
    sd = to_torch(tsvad_state_dict(cfg, seed=777, spread=VAR == "spread", dynamic=VAR == "dynamic"))
    m = make_meeting(600.0, n_spk=4, seed=777)
    plan = plan_windows(m.labels.shape[1], 6, 1, 25, 16000)
    wav = torch.from_numpy(m.wav.astype(np.float32)).to(dev)
    feats = kaldi_fbank(wav[: (B + 6) * 16000])
    fs = torch.from_numpy(plan.fbank_start[:B].astype(np.int32)).to(dev)
    fn = torch.from_numpy(plan.fbank_n[:B].astype(np.int32)).to(dev)
    x = window_cmn(feats, fs, fn, 598).contiguous()
    ts = torch.from_numpy(speaker_embeddings(4, seed=777)).to(dev)[None].expand(B, -1, -1).contiguous()
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]


def run(prec):
    m = TSVADModel(cfg, device=dev, precision=prec, max_batch=B)
    m.load_state_dict(sd)
    out = m.forward(x, ts, T).cpu().numpy()
    st = []
    for i in range(5):
        p, n = ctypes.c_void_p(), ctypes.c_int64()
        _lib.call("sd_tsvad_debug_buffer", m._h, i, ctypes.byref(p), ctypes.byref(n))
        h = np.empty(n.value // 4, np.float32)
        assert hip.hipMemcpy(h.ctypes.data, p.value, n.value, 2) == 0
        st.append(h)
    return out, st


f_out, f_st = run("fp32")
b_out, b_st = run("bf16")
E, NS = 384, 4
T3 = 150
# valid extents: mix/mixg (B, T3, 192) fp32; X2 (B, T, NS*E) bf16 in bf16 mode (fp32 in fp32 mode); H (B*T, 2048) fp32
# gates; Y (B, T, 512) fp32
def bf16_to_f32(a):
    u = a.view(np.uint32)
    lo = (u & 0xffff).astype(np.uint32) << 16
    hi = (u & 0xffff0000).astype(np.uint32)
    return np.stack([lo.view(np.float32), hi.view(np.float32)], -1).reshape(-1)


n_mix = B * T3 * 192
rows = [("mix (conv+bias)", f_st[0][:n_mix], b_st[0][:n_mix]),
        ("mixg (gsp_fc)", f_st[1][:n_mix], b_st[1][:n_mix]),
        ("X2 (conformer out)", f_st[2][:B * T * NS * E], bf16_to_f32(b_st[2])[:B * T * NS * E]),
        ("H (LSTM gates)", f_st[3][:B * T * 2048], b_st[3][:B * T * 2048]),
        ("Y (BiLSTM out)", f_st[4][:B * T * 512], b_st[4][:B * T * 512]),
        ("logits", f_out.ravel(), b_out.ravel())]
frames = {"mix (conv+bias)": (B, T3, 192), "mixg (gsp_fc)": (B, T3, 192), "X2 (conformer out)": (B, T, NS * E),
          "H (LSTM gates)": (B, T, 2048), "Y (BiLSTM out)": (B, T, 512), "logits": (B, NS, T)}
for name, a, b in rows:
    d = np.abs(a.astype(np.float64) - b)
    sh = frames[name]
    ax = 2 if name == "logits" else 1
    if a.size != np.prod(sh):      # the gate buffer is not (B, T, 2048) row-major in every build
        print(f"{name:22s} max|d| {d.max():.3e}  mean|d| {d.mean():.3e}", flush=True)
        continue
    var = a.reshape(sh).astype(np.float64).std(axis=ax).mean()     # mean over features of the std across frames
    rms = np.sqrt((d ** 2).mean())
    print(f"{name:22s} max|d| {d.max():.3e}  mean|d| {d.mean():.3e}  max|ref| {np.abs(a).max():.3e}  "
          f"rel {d.max() / max(np.abs(a).max(), 1e-12):.2e}  rms|d| / frame-std {rms / max(var, 1e-12):.2e}", flush=True)
sig = lambda v: 1 / (1 + np.exp(-v.astype(np.float64)))
dp = np.abs(sig(f_out) - sig(b_out))
print(f"posteriors max|d| {dp.max():.3e} mean {dp.mean():.3e}  flips@0.5 {int(((sig(f_out) > .5) != (sig(b_out) > .5)).sum())}")
