"""Target-speaker embedding extraction on the MI355X path.

Drop-in for the step before TS-VAD inference:
  * `CAMPPlus` — egs/alimeeting/ts_vad2/cam_pplus_wespeaker.py:311-399 (same constructor
    arguments, same standalone state_dict keys, forward(x) -> (B, E) and
    forward(x, get_time_out=True) -> (B, 512, T')), run by libsdiar (`sd_campp_*`).
  * `FBank` — the extractor's FBank (generate_chunk_speaker_embedding_from_modelscope_for_
    diarization.py:307-331): kaldi fbank with the povey window, dither 0, no 2^15 scale,
    mean_nor over the chunk.
  * `extract_embed` — :271-304: 6 s chunks every 1 s (starts range(0, N - L, step)), or the
    whole file when it is not longer than one chunk; returns the (n_chunks, E) tensor the
    script `torch.save`s (:351).  The fbank is computed once per file and each chunk is a
    slice of it (chunk starts are whole frames: 16000 samples = 100 frames), then the
    per-chunk mean is subtracted on the device (`sd_window_cmn`).
  * `load_ts_embed` — TSVADDataset.load_alimeeting_ts_embed at inference
    (ts_vad_dataset.py:494-537): mean over chunks, zeros for speaker ids -1 / -2.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .. import _lib
from ..frontend import FRAME_LEN, FRAME_SHIFT, _mel_device, num_frames
from ..weights import unwrap_checkpoint

POVEY = 1


class CAMPPlus:
    def __init__(self, feat_dim: int = 80, embedding_size: int = 192, growth_rate: int = 32, bn_size: int = 4,
                 init_channels: int = 128, config_str: str = "batchnorm-relu", memory_efficient: bool = True,
                 *, device=None, precision: str = "bf16", max_batch: int = 96, max_frames: int = 598):
        import torch
        if (growth_rate, bn_size, init_channels, config_str) != (32, 4, 128, "batchnorm-relu"):
            raise ValueError("the MI355X CAM++ supports the shipped CAMPPlus topology only")
        if precision not in ("bf16", "fp32"):
            raise ValueError(f"precision must be bf16 or fp32, got {precision}")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise ValueError("CAMPPlus (MI355X backend) runs on a HIP device only")
        self.feat_dim, self.embedding_size = feat_dim, embedding_size
        self.precision, self.max_batch, self.max_frames = precision, max_batch, max_frames
        conf = _lib.CamppConfig(feat_dim=feat_dim, embedding_size=embedding_size, max_batch=max_batch,
                                max_frames=max_frames, precision=1 if precision == "bf16" else 0)
        h = ctypes.c_void_p()
        _lib.call("sd_campp_create", ctypes.byref(conf), ctypes.byref(h))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib._lib is not None:
            _lib.load().sd_campp_destroy(h)
            self._h = None

    def load_state_dict(self, state_dict, strict: bool = True):
        import torch
        if not strict:
            raise ValueError("the MI355X backend only supports strict=True loading")
        state_dict = unwrap_checkpoint(state_dict, kind="campp")
        with torch.device("cpu"):
            for k, v in state_dict.items():
                t = torch.as_tensor(np.asarray(v.cpu() if hasattr(v, "cpu") else v)).to(torch.float32).contiguous()
                shape = (ctypes.c_int64 * max(t.dim(), 1))(*t.shape)
                _lib.call("sd_campp_set_param", self._h, k.encode(), ctypes.c_void_p(t.data_ptr()), shape, t.dim())
        _lib.call("sd_campp_finalize", self._h)
        return self

    def eval(self):
        return self

    def to(self, device):
        import torch
        if torch.device(device) != self.device:
            raise ValueError("re-create the model on the target device")
        return self

    @property
    def device_bytes(self) -> int:
        return int(_lib.load().sd_campp_device_bytes(self._h))

    def forward(self, x, get_time_out: bool = False, out=None):
        """x (B, T, 80) -> (B, E), or (B, 512, (T-1)//2+1) with get_time_out (cam_pplus_wespeaker.py:388-399)."""
        import torch
        B, T, F = x.shape
        if F != self.feat_dim:
            raise ValueError(f"expected {self.feat_dim}-dim fbank, got {F}")
        x = x.to(self.device, torch.float32).contiguous()
        if B > self.max_batch:
            return torch.cat([self.forward(x[s:s + self.max_batch], get_time_out)
                              for s in range(0, B, self.max_batch)])
        st = _lib.stream_ptr(self.device)
        if get_time_out:
            t2 = (T - 1) // 2 + 1
            tout = torch.empty(B, t2, 512, device=self.device, dtype=torch.float32)
            _lib.call("sd_campp_forward", self._h, _lib.ptr(x), B, T, None, _lib.ptr(tout), st)
            return tout.permute(0, 2, 1)
        if out is None:
            out = torch.empty(B, self.embedding_size, device=self.device, dtype=torch.float32)
        _lib.call("sd_campp_forward", self._h, _lib.ptr(x), B, T, _lib.ptr(out), None, st)
        return out

    __call__ = forward


def kaldi_fbank_povey(wav, n_mels: int = 80, out=None):
    """Kaldi.fbank(wav, num_mel_bins, sample_frequency=16000, dither=0) (povey window,
    samples as read, no 2^15 scale): 1-D float32 CUDA tensor -> (n_frames, n_mels)."""
    import torch
    assert wav.is_cuda and wav.dtype == torch.float32 and wav.dim() == 1
    n = num_frames(wav.numel())
    if out is None:
        out = torch.empty(n, n_mels, device=wav.device, dtype=torch.float32)
    fb = _mel_device(n_mels, wav.device)
    _lib.call("sd_fbank_kaldi_ex", _lib.ptr(wav.contiguous()), wav.numel(), 1.0, n, _lib.ptr(fb), n_mels, POVEY,
              _lib.ptr(out), _lib.stream_ptr(wav.device))
    return out


class FBank:
    """generate_chunk_..._for_diarization.py:307-331 (16 kHz only, as the reference asserts)."""

    def __init__(self, n_mels: int, sample_rate: int, mean_nor: bool = False):
        self.n_mels, self.sample_rate, self.mean_nor = n_mels, sample_rate, mean_nor

    def __call__(self, wav, dither=0):
        import torch
        assert self.sample_rate == 16000
        if dither != 0:
            raise ValueError("the MI355X fbank is deterministic (dither 0, the extractor's default)")
        if wav.dim() == 2:
            wav = wav[0]
        feat = kaldi_fbank_povey(wav.to(torch.float32).contiguous(), self.n_mels)
        if self.mean_nor:
            feat = feat - feat.mean(0, keepdim=True)
        return feat


def embedding_chunks(n_samples: int, length_embedding: float = 6.0, step_embedding: float = 1.0,
                     sample_rate: int = 16000):
    """[(start, stop)] of extract_embed (:274-299)."""
    L, S = int(length_embedding * sample_rate), int(step_embedding * sample_rate)
    if n_samples > L:
        return [(s, s + L) for s in range(0, n_samples - L, S)]
    return [(0, n_samples)]


def extract_embed(wav, model: CAMPPlus, length_embedding: float = 6.0, step_embedding: float = 1.0,
                  batch_size: int = 96, n_mels: int = 80):
    """wav: 1-D float samples in [-1, 1) (numpy or tensor; soundfile values cast to float32
    like torch.FloatTensor at :283) -> (n_chunks, E) float32 embeddings on the model device."""
    import torch
    dev = model.device
    w = torch.as_tensor(np.asarray(wav) if not isinstance(wav, torch.Tensor) else wav)
    w = w.to(dev, torch.float32).contiguous()
    chunks = embedding_chunks(w.numel(), length_embedding, step_embedding)
    if any(a % FRAME_SHIFT for a, _ in chunks):
        raise ValueError("chunk starts must be whole fbank frames (step_embedding * 16000 % 160 == 0)")
    if num_frames(chunks[0][1] - chunks[0][0]) < 8:
        raise ValueError("audio shorter than CAM++'s minimum of 8 fbank frames")
    feats = kaldi_fbank_povey(w, n_mels)
    nf = num_frames(chunks[0][1] - chunks[0][0])           # every chunk has the same length
    starts = torch.tensor([a // FRAME_SHIFT for a, _ in chunks], dtype=torch.int32, device=dev)
    lens = torch.full((len(chunks),), nf, dtype=torch.int32, device=dev)
    win = torch.empty(len(chunks), nf, n_mels, device=dev, dtype=torch.float32)
    _lib.call("sd_window_cmn", _lib.ptr(feats), n_mels, _lib.ptr(starts), _lib.ptr(lens), len(chunks), nf,
              _lib.ptr(win), _lib.stream_ptr(dev))
    out = torch.empty(len(chunks), model.embedding_size, device=dev, dtype=torch.float32)
    step = min(batch_size, model.max_batch)
    for s in range(0, len(chunks), step):
        model.forward(win[s:s + step], out=out[s:s + step])
    return out


def load_ts_embed(spk_path: str, file: str, speaker_ids, speaker_embed_dim: int = 192):
    """TSVADDataset.load_alimeeting_ts_embed at inference (ts_vad_dataset.py:494-537, is_train
    False): <spk_path>/<file>/<id>.pt, (n_chunks, E) averaged over chunks; -1 / -2 -> zeros.
    Loads with weights_only=True (the files hold one tensor)."""
    import torch
    feats = []
    for sid in speaker_ids:
        if sid in (-1, -2):
            feats.append(torch.zeros(speaker_embed_dim))
            continue
        f = torch.load(os.path.join(spk_path, file, f"{sid}.pt"), map_location="cpu", weights_only=True)
        feats.append(f.mean(dim=0) if f.dim() == 2 else f)
    return torch.stack(feats)
