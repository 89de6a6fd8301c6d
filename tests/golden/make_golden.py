"""Generate golden vectors by running the REFERENCE modules (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Imports shanguanma/speaker_diarization from /root/reference with stub modules
for packages absent here (torchaudio, soundfile, librosa, whisper,
sherpa_onnx), loads seeded synthetic weights (speaker_diarization_amd.weights,
strict=True so the key layout is pinned), runs the reference forward in eval on
seeded inputs and writes inputs' seeds + outputs to tests/golden/*.npz.
Nothing from the reference is copied; only its outputs are stored.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

REF = os.environ.get("SDIAR_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)


def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def install_stubs(conformer_cls=None):
    ta = _stub("torchaudio")
    ta.models = _stub("torchaudio.models", Conformer=conformer_cls)
    ta.compliance = _stub("torchaudio.compliance")
    ta.compliance.kaldi = _stub("torchaudio.compliance.kaldi")
    for n in ("whisper", "soundfile", "librosa", "sherpa_onnx"):
        _stub(n)


def tsvad_inputs(B, T_fb, n_lab, ns=4, seed=1234):
    """Deterministic (PCG64) inputs shared by the golden script and the tests."""
    rng = np.random.default_rng(seed)
    ref_speech = rng.standard_normal((B, T_fb, 80)).astype(np.float32)
    ts = rng.standard_normal((B, ns, 192)).astype(np.float32)
    return ref_speech, ts


TSVAD_CASES = {
    # name: (variant, rs_len, B, T_fb, n_label, input seed, weight seed)
    "tsvad_v0_rs4": (0, 4, 2, 398, 100, 1234, 777),
    "tsvad_v0_rs4_short": (0, 4, 3, 198, 50, 4321, 778),
    "tsvad_v1_rs6": (1, 6, 2, 598, 150, 99, 779),
}

# BatchNorm1D's NaN bypass (model.py:161-171): one window of the batch carries a NaN fbank value, so the
# reference skips speech_down_or_up's (and variant 0's backend_down's) BatchNorm for EVERY window of the
# batch.  name: (base TSVAD_CASES entry, window, fbank frame, mel bin of the NaN)
TSVAD_NAN_CASES = {
    "tsvad_v1_rs6_nan": ("tsvad_v1_rs6", 1, 300, 17),
    "tsvad_v0_rs4_nan": ("tsvad_v0_rs4_short", 2, 5, 0),
    # round 5: an infinite fbank value instead (the reference tests isnan on the BatchNorm INPUT, the conv
    # output, model.py:166-170; these pin what the CAM++ trunk's arithmetic turns the Inf into)
    "tsvad_v1_rs6_inf": ("tsvad_v1_rs6", 1, 300, 17, np.inf),
    "tsvad_v0_rs4_inf": ("tsvad_v0_rs4_short", 2, 5, 0, np.inf),
    "tsvad_v0_rs4_ninf": ("tsvad_v0_rs4_short", 0, 100, 40, -np.inf),
}


# round 6: the 'dynamic' weight variant (weights.py dynamic_weights, tests/golden/calibrate_dynamic.py) on real windows
# of the bench meeting (synth.make_meeting(600, seed 777), the restated kaldi fbank + per-window CMN of
# oracle/pipeline_ref.py), so the reference run pins the variant's arithmetic in the regime it was calibrated
# for.  The window fbanks are stored in the fixture (data).  name: (variant, rs_len, first window, n windows)
TSVAD_DYN_CASES = {
    "tsvad_v1_rs6_dyn": (1, 6, 20, 3),
    "tsvad_v0_rs4_dyn": (0, 4, 30, 3),
}


def tsvad_dyn_inputs(name):
    """(ref_speech (B, T_fb, 80), ts (B, 4, 192), n_label) of a TSVAD_DYN_CASES entry, built from the meeting."""
    from oracle.pipeline_ref import plan, window_batches
    from speaker_diarization_amd.synth import make_meeting, speaker_embeddings
    v, rs, w0, n = TSVAD_DYN_CASES[name]
    m = make_meeting(600.0, n_spk=4, seed=777)
    ws = plan(m.labels.shape[1], rs, 1)[w0:w0 + n]
    (_, _, ref, tsb, L), = list(window_batches(m.wav, speaker_embeddings(4, seed=777), ws, n))
    return ref.numpy(), tsb.numpy(), int(L)


def make_tsvad_dyn(name):
    import torch
    from speaker_diarization_amd.weights import TSVADConfig, tsvad_state_dict, to_torch
    from oracle.torchaudio_conformer import Conformer

    variant, rs_len = TSVAD_DYN_CASES[name][:2]
    ref_speech, ts, n_lab = tsvad_dyn_inputs(name)
    install_stubs(Conformer)
    sys.path.insert(0, os.path.join(REF, "egs/alimeeting/ts_vad2"))
    import model as ref_model  # reference TSVADModel
    ref_model.TSVADModel.load_speaker_encoder = lambda self, *a, **k: None
    mcfg = ref_model.TSVADConfig()
    dcfg = ref_model.TSVADDataConfig()
    dcfg.rs_len = rs_len
    cfg = TSVADConfig(rs_len=rs_len)
    if variant == 1:
        mcfg.speech_encoder_type = "CAM++_ots_vad"
        mcfg.single_backend_type = "conformer_ots_vad"
        mcfg.multi_backend_type = "lstm_ots_vad"
        mcfg.ots_vad_style = "v1"
        cfg = TSVADConfig.ots_vad_v1(rs_len=rs_len)
    torch.manual_seed(0)
    m = ref_model.TSVADModel(cfg=mcfg, task_cfg=dcfg)
    m.eval()
    m.load_state_dict(to_torch(tsvad_state_dict(cfg, seed=777, dynamic=True)), strict=True)
    B = ref_speech.shape[0]
    with torch.no_grad():
        logits = m(torch.from_numpy(ref_speech), torch.from_numpy(ts), torch.zeros(B, 4, n_lab), num_updates=0)
    out = dict(logits=logits.numpy().astype(np.float32), ref_speech=ref_speech.astype(np.float32),
               ts=ts.astype(np.float32), variant=np.int64(variant), rs_len=np.int64(rs_len), n_label=np.int64(n_lab))
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(name, {k: v.shape for k, v in out.items() if hasattr(v, "shape")},
          "logit std over frames", logits.std(-1).mean().item())
    sys.path.remove(os.path.join(REF, "egs/alimeeting/ts_vad2"))
    for mod in ("model", "cam_pplus_wespeaker", "build_datasets", "ts_vad_dataset"):
        sys.modules.pop(mod, None)


def tsvad_case_inputs(name):
    """(case tuple, ref_speech, ts) of a TSVAD_CASES or TSVAD_NAN_CASES name."""
    base, nan_at = (TSVAD_NAN_CASES[name][0], TSVAD_NAN_CASES[name][1:4]) if name in TSVAD_NAN_CASES else (name, None)
    case = TSVAD_CASES[base]
    _, _, B, T_fb, n_lab, iseed, _ = case
    ref_speech, ts = tsvad_inputs(B, T_fb, n_lab, seed=iseed)
    if nan_at is not None:
        ref_speech[nan_at] = TSVAD_NAN_CASES[name][4] if len(TSVAD_NAN_CASES[name]) > 4 else np.nan
    return case, ref_speech, ts


def make_tsvad(name):
    import torch
    from speaker_diarization_amd.weights import TSVADConfig, tsvad_state_dict, to_torch
    from oracle.torchaudio_conformer import Conformer

    (variant, rs_len, B, T_fb, n_lab, iseed, wseed), ref_speech, ts = tsvad_case_inputs(name)
    install_stubs(Conformer)
    sys.path.insert(0, os.path.join(REF, "egs/alimeeting/ts_vad2"))
    import model as ref_model  # reference TSVADModel
    ref_model.TSVADModel.load_speaker_encoder = lambda self, *a, **k: None

    mcfg = ref_model.TSVADConfig()
    dcfg = ref_model.TSVADDataConfig()
    dcfg.rs_len = rs_len
    cfg = TSVADConfig(rs_len=rs_len)
    if variant == 1:
        for k in ("speech_encoder_type", "single_backend_type", "multi_backend_type", "ots_vad_style"):
            pass
        mcfg.speech_encoder_type = "CAM++_ots_vad"
        mcfg.single_backend_type = "conformer_ots_vad"
        mcfg.multi_backend_type = "lstm_ots_vad"
        mcfg.ots_vad_style = "v1"
        cfg = TSVADConfig.ots_vad_v1(rs_len=rs_len)
    torch.manual_seed(0)
    m = ref_model.TSVADModel(cfg=mcfg, task_cfg=dcfg)
    m.eval()
    sd = to_torch(tsvad_state_dict(cfg, seed=wseed))
    m.load_state_dict(sd, strict=True)
    labels = torch.zeros(B, 4, n_lab)
    with torch.no_grad():
        logits = m(torch.from_numpy(ref_speech), torch.from_numpy(ts), labels, num_updates=0)
        enc = m.speech_down_or_up(m.speech_encoder(torch.from_numpy(ref_speech), get_time_out=True))
    out = dict(logits=logits.numpy().astype(np.float32), speech_enc=enc.numpy().astype(np.float32),
               variant=np.int64(variant), rs_len=np.int64(rs_len), B=np.int64(B), T_fb=np.int64(T_fb),
               n_label=np.int64(n_lab), input_seed=np.int64(iseed), weight_seed=np.int64(wseed))
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(name, {k: v.shape for k, v in out.items() if hasattr(v, "shape")})
    sys.path.remove(os.path.join(REF, "egs/alimeeting/ts_vad2"))
    for mod in ("model", "cam_pplus_wespeaker", "build_datasets", "ts_vad_dataset"):
        sys.modules.pop(mod, None)


# ----------------------------------------------------------------------------- CAM++ embeddings
CAMPP_CASES = {
    # name: (B, T_fbank, embedding_size, input seed, weight seed)
    "campp_emb": (3, 598, 192, 51, 801),
    "campp_emb_vox": (2, 200, 512, 52, 802),
}
# extract_embed over whole wav files: (seconds per file, batch_size, wav seed, weight seed)
CAMPP_EXTRACT = {"campp_extract": ([9.5, 4.0], 3, 53, 803)}


def campp_inputs(B, T, seed):
    return np.random.default_rng(seed).standard_normal((B, T, 80)).astype(np.float32)


def _import_campp():
    install_stubs()
    d = os.path.join(REF, "egs/alimeeting/ts_vad2")
    if d not in sys.path:
        sys.path.insert(0, d)
    import cam_pplus_wespeaker as C  # reference CAMPPlus
    return C


def make_campp(name):
    import torch
    from speaker_diarization_amd.weights import campplus_state_dict, to_torch
    B, T, E, iseed, wseed = CAMPP_CASES[name]
    C = _import_campp()
    torch.manual_seed(0)
    m = C.CAMPPlus(feat_dim=80, embedding_size=E)
    m.eval()
    m.load_state_dict(to_torch(campplus_state_dict(wseed, E)), strict=True)
    x = torch.from_numpy(campp_inputs(B, T, iseed))
    with torch.no_grad():
        emb = m(x)
        tout = m(x, get_time_out=True)
    # time_out (B, 512, T'): the first 64 frames keep the fixture small
    out = dict(emb=emb.numpy().astype(np.float32), time_out=tout[:, :, :64].numpy().astype(np.float32))
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(name, {k: v.shape for k, v in out.items()})


def embed_wav(seconds, seed, sr=16000):
    """int16-valued speech-like noise (what soundfile returns for a 16-bit wav)."""
    rng = np.random.default_rng(seed)
    n = int(seconds * sr)
    env = 0.3 + 0.7 * np.abs(np.sin(np.arange(n) / sr * 2.1))
    return (np.round(rng.standard_normal(n) * 2500 * env).clip(-32768, 32767) / 32768.0).astype(np.float64)


def make_campp_extract(name):
    """Runs the reference extract_embed (generate_chunk_..._for_diarization.py:271-304) on
    wav files written to a temp dir, with the downloaded model replaced by the seeded
    CAMPPlus and kaldi.fbank by the restated oracle (torchaudio is absent: unpinned)."""
    import tempfile
    import wave as wave_mod
    import torch
    from oracle import fbank_ref
    from speaker_diarization_amd.weights import campplus_state_dict, to_torch
    secs, bs, wseed_wav, wseed = CAMPP_EXTRACT[name]
    C = _import_campp()

    def kaldi_fbank(waveform, num_mel_bins=23, sample_frequency=16000.0, dither=0.0, window_type="povey", **kw):
        assert dither == 0.0 and not kw, kw
        x = waveform[0].numpy().astype(np.float64)
        return torch.from_numpy(fbank_ref.fbank(x, num_mel_bins, int(sample_frequency), scale=1.0,
                                                window=window_type))

    sys.modules["torchaudio.compliance.kaldi"].fbank = kaldi_fbank

    def sf_read(path, start=0, stop=None):
        with wave_mod.open(path, "rb") as w:
            a = np.frombuffer(w.readframes(w.getnframes()), np.int16).astype(np.float64) / 32768.0
        return a[start:stop], 16000

    sys.modules["soundfile"].read = sf_read
    for n in ("modelscope", "modelscope.hub", "modelscope.hub.snapshot_download"):
        _stub(n, snapshot_download=None)
    import generate_chunk_speaker_embedding_from_modelscope_for_diarization as G
    torch.manual_seed(0)
    m = C.CAMPPlus(feat_dim=80, embedding_size=192)
    m.eval()
    m.load_state_dict(to_torch(campplus_state_dict(wseed, 192)), strict=True)
    batches = []

    def extract_embeddings(args, batch):     # :215-268 minus the download
        batches.append(len(batch))
        with torch.no_grad():
            return m(torch.stack(batch)).detach()

    G.extract_embeddings = extract_embeddings
    args = types.SimpleNamespace(length_embedding=6, step_embedding=1, batch_size=bs)
    fe = G.FBank(80, sample_rate=16000, mean_nor=True)
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for i, s in enumerate(secs):
            wav = embed_wav(s, wseed_wav + i)
            path = os.path.join(td, f"spk{i}.wav")
            with wave_mod.open(path, "wb") as w:
                w.setnchannels(1)
                w.setsampwidth(2)
                w.setframerate(16000)
                w.writeframes(np.round(wav * 32768).astype(np.int16).tobytes())
            out[f"emb{i}"] = G.extract_embed(args, path, fe).numpy().astype(np.float32)
    out["batches"] = np.array(batches, np.int64)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(name, {k: v.shape for k, v in out.items()}, batches)


# ----------------------------------------------------------------------------- streaming TS-VAD
TSVAD_STREAM_CASES = {
    # name: (T_label, decoding_chunk_size, num_decoding_left_chunks, T_fbank, input seed, weight seed)
    "tsvad_stream_c25": (100, 25, -1, 400, 61, 811),
    "tsvad_stream_c10_l2": (60, 10, 2, 240, 62, 812),
    "tsvad_stream_tail": (70, 25, -1, 277, 63, 813),     # short last chunk; xs padded to 4 * T_label
    "tsvad_stream_tail1": (76, 25, -1, 304, 64, 814),    # 1-label last chunk: 4 fbank frames -> CAM++ 2 -> 1
}


def tsvad_stream_inputs(T_fb, seed):
    rng = np.random.default_rng(seed)
    return (rng.standard_normal((1, T_fb, 80)).astype(np.float32),
            rng.standard_normal((1, 4, 192)).astype(np.float32))


def make_tsvad_stream(name):
    """ts_vad2_streaming/model.py TSVADModel.forward_chunk_by_chunk_temp1 (the path infer_debug
    takes with simulate_streaming, model.py:951-975), B = 1."""
    import torch
    from speaker_diarization_amd.weights import TSVADStreamingConfig, to_torch, tsvad_streaming_state_dict
    T_lab, dcs, left, T_fb, iseed, wseed = TSVAD_STREAM_CASES[name]
    install_stubs()
    d = os.path.join(REF, "egs/alimeeting/ts_vad2_streaming")
    sys.path.insert(0, d)
    for mod in ("model", "cam_pplus_wespeaker", "datasets", "ts_vad_dataset", "mask", "transformer_chunk_streaming"):
        sys.modules.pop(mod, None)
    import model as M
    M.Subsampling4.load_speaker_encoder = lambda self, *a, **k: None
    torch.manual_seed(0)
    m = M.TSVADModel()
    m.eval()
    cfg = TSVADStreamingConfig()
    m.load_state_dict(to_torch(tsvad_streaming_state_dict(cfg, seed=wseed)), strict=True)
    xs, ts = tsvad_stream_inputs(T_fb, iseed)
    labels = torch.zeros(1, 4, T_lab)
    import contextlib, io
    with torch.no_grad(), contextlib.redirect_stdout(io.StringIO()):
        ys = m.forward_chunk_by_chunk_temp1(torch.from_numpy(xs), torch.from_numpy(ts), labels,
                                            decoding_chunk_size=dcs, num_decoding_left_chunks=left)
    out = dict(logits=ys.numpy().astype(np.float32))
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(name, out["logits"].shape)
    sys.path.remove(d)
    for mod in ("model", "cam_pplus_wespeaker", "datasets", "ts_vad_dataset", "mask", "transformer_chunk_streaming"):
        sys.modules.pop(mod, None)


# ----------------------------------------------------------------------------- EEND-EDA
EDA_CASES = {
    # name: (model_type, n_layers, chunk lengths, infer_num_speakers, input seed, weight seed)
    "eda_tfm_l2": ("TransformerEda", 2, [300, 300, 157], 2, 11, 781),
    "eda_tfm_l2_thr": ("TransformerEda", 2, [256, 99], None, 14, 784),
    "eda_eend_l4": ("EendEda", 4, [240, 240, 99], 3, 12, 782),
    "eda_conformer_l2": ("ConformerEda", 2, [200, 77], None, 13, 783),
}


def eda_inputs(lens, in_size=345, seed=11):
    rng = np.random.default_rng(seed)
    return [rng.standard_normal((n, in_size)).astype(np.float32) for n in lens]


def _import_eda():
    from oracle.torchaudio_conformer import Conformer
    install_stubs(Conformer)
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from speaker_diarization.eend_eda import models as eda_models
    return eda_models


def make_eda(name):
    import torch
    from speaker_diarization_amd.weights import EDAConfig, eda_state_dict, to_torch

    mtype, L, lens, nspk, iseed, wseed = EDA_CASES[name]
    M = _import_eda()
    cfg = EDAConfig(model_type=mtype, n_layers=L)
    torch.manual_seed(777)     # infer_eda.py:39-43, before construction
    if mtype == "TransformerEda":
        m = M.TransformerEdaModel(n_speakers=2, in_size=345, n_units=256, n_heads=4, n_layers=L, has_pos=False)
    else:
        m = M.EendEdaModel(n_speakers=2, in_size=345, n_units=256, n_heads=4, n_layers=L,
                           encoder_type="conformer" if mtype == "ConformerEda" else "transformer", eda_type="lstm")
    m.eval()
    m.load_state_dict(to_torch(eda_state_dict(cfg, seed=wseed)), strict=True)
    xs = eda_inputs(lens, seed=iseed)
    perms, cap = [], {}
    orig_randperm = torch.randperm

    def rec_randperm(n, *a, **k):
        p = orig_randperm(n, *a, **k)
        perms.append(p.clone())
        return p

    orig_emb = m.forward_embedding

    def emb_hook(src):
        r = orig_emb(src)
        cap["emb"] = r[1]
        return r

    m.forward_embedding = emb_hook
    m.eda.register_forward_hook(lambda mod, inp, out: cap.__setitem__("eda", out))
    T = max(lens)
    act = np.zeros((len(lens), T, 14), np.float32)
    probs = np.zeros((len(lens), 15), np.float32)
    ys, index_error = [], np.zeros(len(lens), np.int64)
    torch.randperm = rec_randperm
    try:
        with torch.no_grad():
            for i, x in enumerate(xs):     # one chunk per infer() call, infer_eda.py:99-112
                try:
                    y = m.infer([torch.from_numpy(x)], infer_num_speakers=nspk, max_n_speakers=15,
                                attractor_threshold=0.5)
                    ys.append(y[0].numpy())
                except IndexError:           # models.py:338-339
                    index_error[i] = 1
                    ys.append(np.zeros((lens[i], 0), np.float32))
                att, pr = cap["eda"]
                act[i, : lens[i]] = torch.sigmoid(torch.bmm(cap["emb"], att[:, :-1, :].permute(0, 2, 1)))[0].numpy()
                probs[i] = pr[0].numpy()
    finally:
        torch.randperm = orig_randperm
    nsel = np.array([y.shape[1] for y in ys], np.int64)
    out = dict(lens=np.array(lens, np.int64), perms=np.concatenate([p.numpy() for p in perms]).astype(np.int64),
               act=act, probs=probs, nsel=nsel, index_error=index_error,
               ys=np.concatenate([y.reshape(-1) for y in ys]).astype(np.float32),
               n_layers=np.int64(L), input_seed=np.int64(iseed), weight_seed=np.int64(wseed),
               infer_num_speakers=np.int64(-1 if nspk is None else nspk))
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(name, "perm0", perms[0][:8].tolist(), "nsel", nsel.tolist(), "index_error", index_error.tolist())


def make_eda_batch(name="eda_tfm_batch"):
    """One infer() call on a 2-element list of different lengths: pad_sequence(-1)
    and no key mask (models.py:216-225) — the reference's B>1 semantics."""
    import torch
    from speaker_diarization_amd.weights import EDAConfig, eda_state_dict, to_torch
    M = _import_eda()
    cfg = EDAConfig(model_type="TransformerEda", n_layers=2)
    torch.manual_seed(777)
    m = M.TransformerEdaModel(n_speakers=2, in_size=345, n_units=256, n_heads=4, n_layers=2, has_pos=False)
    m.eval()
    m.load_state_dict(to_torch(eda_state_dict(cfg, seed=785)), strict=True)
    lens = [180, 131]
    xs = eda_inputs(lens, seed=15)
    cap = {}
    m.eda.register_forward_hook(lambda mod, inp, out: cap.__setitem__("eda", out))
    with torch.no_grad():
        ys = m.infer([torch.from_numpy(x) for x in xs], infer_num_speakers=None, max_n_speakers=15,
                     attractor_threshold=0.5)
    out = dict(lens=np.array(lens, np.int64), probs=torch.stack(cap["eda"][1]).numpy(),
               nsel=np.array([y.shape[1] for y in ys], np.int64),
               ys=np.concatenate([y.numpy().reshape(-1) for y in ys]).astype(np.float32))
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(name, out["nsel"])


# ----------------------------------------------------------------------------- feature.py glue
FEATURE_CASES = {
    # name: (n_samples, sample_rate, transform, frame_size, frame_shift, context, subsampling, seed)
    "feat_logmel23_mn_16k": (48123, 16000, "logmel23_mn", 400, 160, 7, 10, 21),
    "feat_logmel23_mn_16k_div": (48000, 16000, "logmel23_mn", 400, 160, 7, 10, 22),
}


def feature_wav(n, seed):
    rng = np.random.default_rng(seed)
    # int16-valued samples / 32768 like soundfile's float64 read (kaldi_data.py:82)
    return (np.round(rng.standard_normal(n) * 3000).clip(-32768, 32767) / 32768.0).astype(np.float64)


def make_feature(name):
    from oracle import eend_ref
    install_stubs()
    lib = sys.modules["librosa"]
    lib.stft = lambda y, n_fft, win_length, hop_length: eend_ref.librosa_stft(y, n_fft, hop_length, win_length)
    lib.filters = types.SimpleNamespace(mel=lambda sr, n_fft, n_mels: eend_ref.slaney_mel(sr, n_fft, n_mels))
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from speaker_diarization import feature
    n, sr, tr, fs, fsh, ctx, sub, seed = FEATURE_CASES[name]
    wav = feature_wav(n, seed)
    Y = feature.stft(wav, fs, fsh)
    Y = feature.transform(Y, transform_type=tr, sample_rate=sr)
    Y = feature.splice(Y, context_size=ctx)
    Y = np.ascontiguousarray(Y[::sub])
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), feats=Y.astype(np.float32), seed=np.int64(seed),
                        n_samples=np.int64(n))
    print(name, Y.shape)


# ----------------------------------------------------------------------------- FS-EEND / EEND
FSEEND_CASES = {
    # name: (lengths of the src list, max_nspks, mask_delay, input seed, weight seed)
    "fseend_T240": ([240], 6, 0, 31, 791),
    "fseend_batch": ([150, 97], 6, 0, 32, 792),
    "fseend_delay2": ([130], 5, 2, 33, 793),
}
EEND_CASES = {
    # name: (n_speakers, n_layers, lengths, input seed, weight seed)
    "eend_tfm_l2": (2, 2, [200], 41, 795),
    "eend_tfm_batch": (3, 2, [120, 77], 42, 796),
}


def make_fseend(name):
    import torch
    from speaker_diarization_amd.weights import FSEENDConfig, fseend_state_dict, to_torch
    lens, C, delay, iseed, wseed = FSEEND_CASES[name]
    d = os.path.join(REF, "speaker_diarization/fs_eend")
    sys.path.insert(0, d)
    import fs_eend as F  # reference module (plain torch)
    cfg = FSEENDConfig(mask_delay=delay)
    torch.manual_seed(0)
    m = F.OnlineTransformerDADiarization(n_speakers=None, in_size=345, n_units=256, n_heads=4, enc_n_layers=4,
                                         dec_n_layers=2, dropout=0.1, has_mask=True, max_seqlen=10000,
                                         dec_dim_feedforward=2048, conv_delay=9, mask_delay=delay)
    m.eval()
    m.load_state_dict(to_torch(fseend_state_dict(cfg, seed=wseed)), strict=True)
    xs = [torch.from_numpy(x) for x in eda_inputs(lens, seed=iseed)]
    with torch.no_grad():
        out, emb, att = m.test(xs, lens, max_nspks=C)
    res = dict(lens=np.array(lens, np.int64), max_nspks=np.int64(C), mask_delay=np.int64(delay),
               out=np.concatenate([o.numpy() for o in out]).astype(np.float32),
               emb=np.concatenate([e.numpy() for e in emb]).astype(np.float32),
               att_head=np.concatenate([a.numpy()[:24] for a in att]).astype(np.float32))   # first 24 frames
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **res)
    print(name, res["out"].shape, res["att_head"].shape)
    sys.path.remove(d)
    sys.modules.pop("fs_eend", None)


def make_eend(name):
    import torch
    from speaker_diarization_amd.weights import EDAConfig, eend_layout, synthetic_state_dict, to_torch
    nspk, L, lens, iseed, wseed = EEND_CASES[name]
    install_stubs()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from speaker_diarization.eend import models as M
    cfg = EDAConfig(n_speakers=nspk, n_layers=L)
    torch.manual_seed(0)
    m = M.TransformerModel(n_speakers=nspk, in_size=345, n_heads=4, n_units=256, n_layers=L)
    m.eval()
    m.load_state_dict(to_torch(synthetic_state_dict(eend_layout(cfg), wseed)), strict=True)
    xs = [torch.from_numpy(x) for x in eda_inputs(lens, seed=iseed)]
    with torch.no_grad():
        ys = m(xs, activation=torch.sigmoid)     # eend_infer.py:69
    res = dict(lens=np.array(lens, np.int64), ys=np.concatenate([y.numpy() for y in ys]).astype(np.float32))
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **res)
    print(name, res["ys"].shape)


if __name__ == "__main__":
    import torch
    torch.set_num_threads(8)
    names = sys.argv[1:] or (list(TSVAD_CASES) + list(EDA_CASES) + ["eda_tfm_batch"] + list(FEATURE_CASES)
                             + list(FSEEND_CASES) + list(EEND_CASES) + list(CAMPP_CASES) + list(CAMPP_EXTRACT) + list(TSVAD_STREAM_CASES))
    for n in names:
        if n in TSVAD_CASES or n in TSVAD_NAN_CASES:
            make_tsvad(n)
        elif n in TSVAD_DYN_CASES:
            make_tsvad_dyn(n)
        elif n in CAMPP_CASES:
            make_campp(n)
        elif n in TSVAD_STREAM_CASES:
            make_tsvad_stream(n)
        elif n in CAMPP_EXTRACT:
            make_campp_extract(n)
        elif n in EDA_CASES:
            make_eda(n)
        elif n == "eda_tfm_batch":
            make_eda_batch(n)
        elif n in FSEEND_CASES:
            make_fseend(n)
        elif n in EEND_CASES:
            make_eend(n)
        else:
            make_feature(n)
