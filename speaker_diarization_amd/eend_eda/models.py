"""TransformerEdaModel / EendEdaModel — drop-ins for speaker_diarization/eend_eda/models.py
(inference surface: constructor, load_state_dict, eval/to, infer).

The forward (Linear+LN -> transformer/conformer encoder -> frame shuffle -> EDA
LSTM encoder/decoder -> attractor probabilities and sigmoid activities) runs in
libsdiar (HIP, gfx950); this module only moves state_dict tensors across the C
ABI, draws the frame permutations and does the speaker selection on the 15
attractor probabilities, exactly where the reference does them.

Random-number parity: the reference shuffles frames with torch.randperm on the
CPU default generator (models.py:229-233 / 532-536), and its constructor's
parameter inits advance that generator after infer_eda.py seeds it
(infer_eda.py:39-43 -> :51-71).  The constructor here therefore replays the
reference's module construction on the CPU (the parameters are discarded) so a
seeded script draws the same permutations.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import numpy as np

from .. import _lib
from ..weights import EDAConfig


def _replay_construction_rng(cfg: EDAConfig, dropout: float):
    """Run the reference constructor's RNG-consuming inits in its order."""
    import torch
    from torch import nn
    e = cfg.n_units
    with torch.no_grad():
        nn.Linear(cfg.in_size, e)                                   # encoder / linear
        nn.LayerNorm(e)
        if cfg.variant in (0, 1):
            layer = nn.TransformerEncoderLayer(e, cfg.n_heads, cfg.dim_feedforward, dropout, batch_first=True)
            nn.TransformerEncoder(layer, cfg.n_layers)
        else:
            _replay_torchaudio_conformer(e, cfg.n_heads, cfg.dim_feedforward, cfg.n_layers, 31)
        nn.LSTM(e, e, 1, batch_first=True)                         # eda.encoder
        nn.LSTM(e, e, 1, batch_first=True)                         # eda.decoder
        nn.Linear(e, 1)                                             # eda.linear
        if cfg.variant == 0:                                        # init_weights (models.py:207-210)
            torch.empty(e, cfg.in_size).uniform_(-0.1, 0.1)


def _replay_torchaudio_conformer(d, nh, ffn, layers, k):
    """torchaudio.models.Conformer construction order (2.5.1, use_group_norm=False)."""
    from torch import nn
    for _ in range(layers):
        nn.LayerNorm(d); nn.Linear(d, ffn); nn.Linear(ffn, d)      # ffn1
        nn.LayerNorm(d); nn.MultiheadAttention(d, nh)              # self_attn
        nn.LayerNorm(d); nn.Conv1d(d, 2 * d, 1); nn.Conv1d(d, d, k, padding=(k - 1) // 2, groups=d)
        nn.BatchNorm1d(d); nn.Conv1d(d, d, 1)                      # conv_module
        nn.LayerNorm(d); nn.Linear(d, ffn); nn.Linear(ffn, d)      # ffn2
        nn.LayerNorm(d)                                             # final_layer_norm


class _EdaBase:
    """Shared handle management for the two reference classes."""

    def __init__(self, cfg: EDAConfig, dropout: float, device=None, precision: str = "fp32",
                 max_seqs: int = 8, max_frames: int = 2000):
        import torch
        cfg.variant  # validates model/encoder type like the reference constructor
        if precision not in ("bf16", "fp32", "bf16x3"):
            raise ValueError(f"precision must be bf16, fp32 or bf16x3, got {precision}")
        self.cfg = cfg
        self.precision = precision
        self.max_seqs = max_seqs
        self.max_frames = max_frames
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise ValueError("EEND-EDA (MI355X backend) runs on a HIP device only")
        _replay_construction_rng(cfg, dropout)
        self._state = None
        self._h = None
        self._n_att = None

    # ------------------------------------------------------------------ handle
    def _build(self, max_n_speakers: int):
        c = self.cfg
        conf = _lib.EdaConfig(variant=c.variant, in_size=c.in_size, n_units=c.n_units, n_heads=c.n_heads,
                              n_layers=c.n_layers, dim_feedforward=c.dim_feedforward, max_seqs=self.max_seqs,
                              max_frames=self.max_frames, max_n_speakers=max_n_speakers,
                              precision={"fp32": 0, "bf16": 1, "bf16x3": 2}[self.precision])
        h = ctypes.c_void_p()
        _lib.call("sd_eda_create", ctypes.byref(conf), ctypes.byref(h))
        try:
            for k, v in self._state.items():
                a = np.ascontiguousarray(np.asarray(v, dtype=np.float32))
                shape = (ctypes.c_int64 * max(a.ndim, 1))(*a.shape)
                _lib.call("sd_eda_set_param", h, k.encode(), a.ctypes.data_as(ctypes.c_void_p), shape, a.ndim)
            _lib.call("sd_eda_finalize", h)
        except Exception:
            _lib.load().sd_eda_destroy(h)
            raise
        self._release()
        self._h, self._n_att = h, max_n_speakers
        self.in_ld = _lib.load().sd_eda_input_stride(h)

    def _release(self):
        if self._h is not None:
            _lib.load().sd_eda_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self._release()
        except Exception:
            pass

    def load_state_dict(self, state_dict, strict: bool = True):
        """Same keys as the reference module (torch.load of the model file,
        infer_eda.py:88).  Missing/unexpected keys raise RuntimeError."""
        if not strict:
            raise ValueError("strict=False is not supported by the MI355X backend")
        self._state = {k: (v.detach().cpu().float().numpy() if hasattr(v, "detach") else np.asarray(v))
                       for k, v in state_dict.items()}
        self._build(15)
        return self

    def eval(self):
        return self

    def to(self, device):
        import torch
        if torch.device(device).type != "cuda":
            raise ValueError("EEND-EDA (MI355X backend) runs on a HIP device only")
        return self

    def device_bytes(self) -> int:
        return int(_lib.load().sd_eda_device_bytes(self._h)) if self._h is not None else 0

    # ------------------------------------------------------------------ forward
    def forward_infer(self, feats, lengths: List[int], perms, max_n_speakers: int = 15,
                      key_len: Optional[List[int]] = None, act=None, probs=None, check: bool = True):
        """Device-level forward of S equal-stride sequences.
        feats: CUDA (S, T, ld>=in_ld) f32; perms: list of S int tensors (randperm(lengths[s])).
        Returns (act (S, T, max_n-1), probs (S, max_n)) CUDA f32.  check: wait for the stream and
        raise RuntimeError here if an EDA LSTM recurrence lost co-residency (its outputs are NaN);
        check=False leaves that to a later status() (batched callers check once)."""
        import torch
        if self._h is None:
            raise RuntimeError("load_state_dict() must be called before infer()")
        if max_n_speakers != self._n_att:
            self._build(max_n_speakers)
        S, T, ld = feats.shape
        if S > self.max_seqs or T > self.max_frames:
            # split into workspace-sized pieces
            raise ValueError(f"batch ({S}, {T}) exceeds the handle workspace ({self.max_seqs}, {self.max_frames})")
        dev = self.device
        perm = np.tile(np.arange(T, dtype=np.int32), (S, 1))
        for s, p in enumerate(perms):
            perm[s, : lengths[s]] = np.asarray(p, dtype=np.int32)
        perm_d = torch.from_numpy(perm).to(dev)
        len_d = torch.tensor(lengths, dtype=torch.int32, device=dev)
        kl_d = torch.tensor(key_len, dtype=torch.int32, device=dev) if key_len is not None else None
        if act is None:
            act = torch.empty(S, T, max_n_speakers - 1, device=dev, dtype=torch.float32)
        if probs is None:
            probs = torch.empty(S, max_n_speakers, device=dev, dtype=torch.float32)
        feats = feats.contiguous()
        _lib.call("sd_eda_forward", self._h, _lib.ptr(feats), ld, S, T, _lib.ptr(len_d),
                  _lib.ptr(kl_d) if kl_d is not None else None, _lib.ptr(perm_d), _lib.ptr(probs), _lib.ptr(act),
                  _lib.stream_ptr(dev))
        if check:
            self.status()
        return act, probs

    def status(self):
        """sd_eda_status: wait for the device stream, raise RuntimeError if a persistent LSTM
        recurrence of the forwards enqueued so far timed out."""
        _lib.call("sd_eda_status", self._h, _lib.stream_ptr(self.device))

    def _pad_src(self, src):
        """pad_sequence(src, padding_value=-1, batch_first=True) into in_ld-wide rows."""
        import torch
        ilens = [int(x.shape[0]) for x in src]
        T = max(ilens)
        buf = torch.full((len(src), T, self.in_ld), -1.0, device=self.device, dtype=torch.float32)
        for i, x in enumerate(src):
            if x.shape[-1] != self.cfg.in_size:
                raise RuntimeError(f"mat1 and mat2 shapes cannot be multiplied (feature dim {x.shape[-1]} "
                                   f"!= in_size {self.cfg.in_size})")
            buf[i, : ilens[i], : self.cfg.in_size] = x.to(self.device, torch.float32)
        buf[:, :, self.cfg.in_size:] = 0.0
        return buf, ilens

    def infer(self, src: List, infer_num_speakers=None, max_n_speakers=15, attractor_threshold=0.5):
        """models.py:297-347 (TransformerEda) / 601-652 (EendEda): list of (T_i, in_size)
        -> list of (T_i, n_spk) sigmoid activities (CUDA)."""
        import torch
        feats, ilens = self._pad_src(src)
        perms = [torch.randperm(n) for n in ilens]      # CPU generator, batch order (models.py:231)
        key_len = ilens if self.cfg.variant == 2 else None
        act, probs = self.forward_infer(feats, ilens, perms, max_n_speakers, key_len=key_len)
        return self.select(act, probs.cpu(), ilens, infer_num_speakers, attractor_threshold)

    def select(self, act, probs_cpu, ilens, infer_num_speakers, attractor_threshold):
        """Speaker selection on the attractor probabilities (host)."""
        import torch
        out = []
        n_cols = act.shape[-1]
        for b in range(act.shape[0]):
            p, y = probs_cpu[b], act[b, : ilens[b]]
            if infer_num_speakers is not None:
                if self.cfg.variant == 0:
                    # models.py:337-339: the order of 15 probs indexes 14 columns
                    order = torch.sort(p, descending=True)[1][:infer_num_speakers]
                    bad = order[order >= n_cols]
                    if bad.numel():
                        raise IndexError(f"index {int(bad[0])} is out of bounds for dimension 1 with size {n_cols}")
                    out.append(y[:, order.to(y.device)])
                else:
                    out.append(y[:, :infer_num_speakers])    # models.py:644
            elif attractor_threshold is not None:
                silence = np.where(p.numpy() < attractor_threshold)[0]
                n_spk = silence[0] if silence.size else None
                out.append(y[:, :n_spk])
            else:
                NotImplementedError("infer_num_speakers or attractor_threshold has to be given.")
        return out


class TransformerEdaModel(_EdaBase):
    """eend_eda/models.py:160-347."""

    def __init__(self, n_speakers, in_size, n_heads, n_units, n_layers, dim_feedforward=2048, dropout=0.5,
                 has_pos=False, diar_weight: float = 1.0, attractor_weight: float = 1.0, *, device=None,
                 precision: str = "fp32", max_seqs: int = 8, max_frames: int = 2000):
        if has_pos:
            raise NotImplementedError("has_pos=True is not on the inference path (infer_eda.py:56)")
        self.n_speakers = n_speakers
        cfg = EDAConfig(model_type="TransformerEda", n_speakers=n_speakers, in_size=in_size, n_heads=n_heads,
                        n_units=n_units, n_layers=n_layers, dim_feedforward=dim_feedforward)
        super().__init__(cfg, dropout, device, precision, max_seqs, max_frames)


class EendEdaModel(_EdaBase):
    """eend_eda/models.py:465-652."""

    def __init__(self, n_speakers, in_size, n_heads, n_units, n_layers, dim_feedforward=2048, dropout=0.5,
                 diar_weight: float = 1.0, attractor_weight: float = 1.0, encoder_type="transformer",
                 eda_type="lstm", *, device=None, precision: str = "fp32", max_seqs: int = 8,
                 max_frames: int = 2000):
        if encoder_type not in ("transformer", "conformer"):
            raise NotImplementedError(f"encoder_type not support {encoder_type}!!!")
        if eda_type != "lstm":
            raise NotImplementedError(f"eda_type not support {eda_type}!!!")
        self.n_speakers = n_speakers
        cfg = EDAConfig(model_type="EendEda", n_speakers=n_speakers, in_size=in_size, n_heads=n_heads,
                        n_units=n_units, n_layers=n_layers, dim_feedforward=dim_feedforward,
                        encoder_type=encoder_type)
        super().__init__(cfg, dropout, device, precision, max_seqs, max_frames)
