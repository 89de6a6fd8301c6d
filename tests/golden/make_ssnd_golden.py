"""SSND goldens from the reference module (egs/alimeeting/ssnd/ssnd_model.py), imported and run
here only (stubs: torchaudio with the restated Conformer injected, soundfile/librosa/whisper;
the CAM++ speaker-encoder checkpoint loader is a no-op because the pretrained file is a cluster
path).  Seeded weights come from speaker_diarization_amd.weights.ssnd_state_dict, loaded with
strict=True into the reference model (pins every key name).

  ssnd_decode_*: DetectionDecoder + sigmoid + RepresentationDecoder exactly as SSNDModel.infer
                 calls them (:762-776), on seeded encoder outputs / extractor features / speaker
                 embeddings — pure torch, fully pinned.
  ssnd_infer_*:  the whole SSNDModel.infer (:752-776) on seeded fbank blocks (the Conformer is
                 the restated torchaudio algorithm: that block is parity-unpinned, as for C2).

    python tests/golden/make_ssnd_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import REF, REPO, install_stubs  # noqa: E402

SSND_DIR = os.path.join(REF, "egs/alimeeting/ssnd")

# name: (kind, B, T (label frames) or T_fb (fbank frames), max_speakers, input seed, weight seed)
SSND_CASES = {
    "ssnd_decode_n4": ("decode", 3, 200, 4, 31, 901),
    "ssnd_decode_n6": ("decode", 2, 200, 6, 32, 902),
    "ssnd_infer_n4": ("infer", 2, 800, 4, 33, 903),
}


def ssnd_cfg(n_spk):
    from speaker_diarization_amd.weights import SSNDConfig
    return SSNDConfig(max_speakers=n_spk, vad_out_len=200)


def ssnd_inputs(kind, B, T, N, seed, cfg):
    rng = np.random.default_rng(seed)
    if kind == "decode":
        enc = rng.standard_normal((B, T, cfg.d_model)).astype(np.float32)
        x = rng.standard_normal((B, T, cfg.emb_dim)).astype(np.float32)
        spk = rng.standard_normal((B, N, cfg.emb_dim)).astype(np.float32)
        return enc, x, spk
    feats = rng.standard_normal((B, T, 80)).astype(np.float32)
    spk = rng.standard_normal((B, N, cfg.emb_dim)).astype(np.float32)
    return feats, spk


def _import():
    from oracle.torchaudio_conformer import Conformer
    install_stubs(Conformer)
    sys.path.insert(0, SSND_DIR)
    for mod in ("ssnd_model", "cam_pplus_wespeaker", "resnet_wespeaker", "pooling_layers_wespeaker"):
        sys.modules.pop(mod, None)
    import ssnd_model as M
    M.ResNetExtractor.load_speaker_encoder = lambda self, *a, **k: None
    return M


def make(name, M):
    import torch
    from speaker_diarization_amd.weights import ssnd_state_dict, to_torch
    kind, B, T, N, iseed, wseed = SSND_CASES[name]
    cfg = ssnd_cfg(N)
    torch.manual_seed(0)
    m = M.SSNDModel(None, max_speakers=N, vad_out_len=cfg.vad_out_len, training=False)
    m.eval()
    m.load_state_dict(to_torch(ssnd_state_dict(cfg, seed=wseed)), strict=True)
    with torch.no_grad():
        if kind == "decode":
            enc, x, spk = (torch.from_numpy(a) for a in ssnd_inputs(kind, B, T, N, iseed, cfg))
            pos = m.pos_emb[:, :T, :].expand(B, T, m.pos_emb_dim)
            x_det = m.det_query_emb.unsqueeze(0).expand(B, N, m.d_model)
            x_rep = m.rep_query_emb.unsqueeze(0).expand(B, N, T)
            vad = m.det_decoder(x_det, enc, spk, pos)
            emb = m.rep_decoder(x_rep, x, torch.sigmoid(vad), pos)
        else:
            feats, spk = (torch.from_numpy(a) for a in ssnd_inputs(kind, B, T, N, iseed, cfg))
            vad, emb = m.infer(feats, spk)
            enc = None
    out = dict(vad_pred=vad.numpy().astype(np.float32), emb_pred=emb.numpy().astype(np.float32))
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(name, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    import torch
    torch.set_num_threads(8)
    M = _import()
    for n in sys.argv[1:] or list(SSND_CASES):
        make(n, M)
