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


def make_tsvad(name):
    import torch
    from speaker_diarization_amd.weights import TSVADConfig, tsvad_state_dict, to_torch
    from oracle.torchaudio_conformer import Conformer

    variant, rs_len, B, T_fb, n_lab, iseed, wseed = TSVAD_CASES[name]
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
    ref_speech, ts = tsvad_inputs(B, T_fb, n_lab, seed=iseed)
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


if __name__ == "__main__":
    import torch
    torch.set_num_threads(8)
    names = sys.argv[1:] or list(TSVAD_CASES)
    for n in names:
        make_tsvad(n)
