"""TransformerModel — drop-in for speaker_diarization/eend/models.py:17-101 (plain EEND,
self-attention encoder + per-frame Linear decoder), inference surface only.

eend/eend_infer.py:66-70 calls model([chunk], activation=torch.sigmoid) per
chunk; the forward (Linear, LayerNorm, TransformerEncoder, decoder Linear,
sigmoid) runs in libsdiar as variant 3 of the EDA runner.
"""
from __future__ import annotations

import ctypes

import torch

from .. import _lib
from ..weights import EDAConfig


class TransformerModel:
    def __init__(self, n_speakers, in_size, n_heads, n_units, n_layers, dim_feedforward=2048, dropout=0.5,
                 has_pos=False, *, device=None, precision: str = "fp32", max_seqs: int = 8,
                 max_frames: int = 2000):
        if has_pos:
            raise NotImplementedError("has_pos=True is not on the inference path")
        if precision not in ("bf16", "fp32", "bf16x3"):
            raise ValueError(f"precision must be bf16, fp32 or bf16x3, got {precision}")
        self.cfg = EDAConfig(n_speakers=n_speakers, in_size=in_size, n_heads=n_heads, n_units=n_units,
                             n_layers=n_layers, dim_feedforward=dim_feedforward)
        self.n_speakers = n_speakers
        self.precision = precision
        self.max_seqs, self.max_frames = max_seqs, max_frames
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise ValueError("EEND (MI355X backend) runs on a HIP device only")
        self._h = None

    def load_state_dict(self, state_dict, strict: bool = True):
        if not strict:
            raise ValueError("strict=False is not supported by the MI355X backend")
        c = self.cfg
        conf = _lib.EdaConfig(variant=3, in_size=c.in_size, n_units=c.n_units, n_heads=c.n_heads,
                              n_layers=c.n_layers, dim_feedforward=c.dim_feedforward, max_seqs=self.max_seqs,
                              max_frames=self.max_frames, max_n_speakers=2,
                              precision={"fp32": 0, "bf16": 1, "bf16x3": 2}[self.precision], n_speakers=c.n_speakers)
        h = _lib.create_handle("eda", conf, _lib.host_state(state_dict))
        self._release()
        self._h = h
        self.in_ld = _lib.load().sd_eda_input_stride(h)
        return self

    def _release(self):
        if self._h is not None:
            _lib.load().sd_eda_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass

    def eval(self):
        return self

    def to(self, device):
        if torch.device(device).type != "cuda":
            raise ValueError("EEND (MI355X backend) runs on a HIP device only")
        return self

    def __call__(self, src, has_mask=False, activation=None):
        return self.forward(src, has_mask, activation)

    def forward(self, src, has_mask=False, activation=None):
        """models.py:69-101.  src: list of (T_i, in_size) -> list of (T_i, n_speakers)."""
        if has_mask:
            # models.py:70-73 reads src.device / src.size(1) on the list argument
            raise AttributeError("'list' object has no attribute 'device'")
        if activation is not torch.sigmoid:
            raise NotImplementedError("the MI355X EEND forward fuses activation=torch.sigmoid (eend_infer.py:69)")
        if self._h is None:
            raise RuntimeError("load_state_dict() must be called before forward()")
        ilens = [int(x.shape[0]) for x in src]
        S, T = len(src), max(ilens)
        if S > self.max_seqs or T > self.max_frames:
            raise ValueError(f"batch ({S}, {T}) exceeds the handle workspace ({self.max_seqs}, {self.max_frames})")
        buf = torch.full((S, T, self.in_ld), -1.0, device=self.device, dtype=torch.float32)   # pad_sequence(-1)
        for i, x in enumerate(src):
            buf[i, : ilens[i], : self.cfg.in_size] = x.to(self.device, torch.float32)
        buf[:, :, self.cfg.in_size:] = 0.0
        out = torch.empty(S, T, self.n_speakers, device=self.device, dtype=torch.float32)
        _lib.call("sd_eda_forward", self._h, _lib.ptr(buf), self.in_ld, S, T, None, None, None, None,
                  _lib.ptr(out), _lib.stream_ptr(self.device))
        return [out[i, : ilens[i]] for i in range(S)]
