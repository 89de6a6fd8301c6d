"""OnlineTransformerDADiarization — drop-in for speaker_diarization/fs_eend/fs_eend.py:20-96
(inference surface: constructor, load_state_dict, test).

test(src, ilens, max_nspks) runs in libsdiar (HIP, gfx950): BatchNorm-folded
input Linear + LayerNorm, causal transformer encoder, look-ahead Conv1d, L2
norm, the shared fusion-layer attractor decoder on the (T, C) token grid and
the per-frame emb·attractorᵀ scores.  stream(chunk) returns an FsEendStream that
produces the same scores chunk by chunk from per-layer K/V histories (every
chunk's kernels replayed as one hipGraph).  FS-EEND does not shard (causal
full-history attention): multi-GPU runs are replicas, one
recording per GPU.
"""
from __future__ import annotations

import ctypes
from typing import List

import numpy as np
import torch

from .. import _lib
from ..weights import FSEENDConfig, unwrap_checkpoint


class OnlineTransformerDADiarization:
    def __init__(self, n_speakers, in_size, n_units, n_heads, enc_n_layers, dec_n_layers, dropout, has_mask,
                 max_seqlen, dec_dim_feedforward, conv_delay=9, mask_delay=0, decom_kernel_size=64, *,
                 device=None, precision: str = "fp32", max_seqs: int = 1, max_frames: int = None,
                 max_nspks: int = 6):
        if precision not in ("bf16", "fp32", "bf16x3"):
            raise ValueError(f"precision must be bf16, fp32 or bf16x3, got {precision}")
        self.cfg = FSEENDConfig(n_speakers=n_speakers, in_size=in_size, n_units=n_units, n_heads=n_heads,
                                enc_n_layers=enc_n_layers, dec_n_layers=dec_n_layers, dropout=dropout,
                                has_mask=has_mask, max_seqlen=max_seqlen, dec_dim_feedforward=dec_dim_feedforward,
                                conv_delay=conv_delay, mask_delay=mask_delay)
        self.n_speakers = n_speakers
        self.precision = precision
        self.max_seqs = max_seqs
        self.max_frames = max_frames or max_seqlen
        self.max_nspks = max_nspks
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise ValueError("FS-EEND (MI355X backend) runs on a HIP device only")
        self._h = None

    def load_state_dict(self, state_dict, strict: bool = True):
        """Accepts the module state_dict or the Lightning checkpoint layout
        ({"state_dict": {"model.<key>": ...}}, fs_eend/train.py:183-191)."""
        if not strict:
            raise ValueError("strict=False is not supported by the MI355X backend")
        c = self.cfg
        conf = _lib.FseendConfig(in_size=c.in_size, n_units=c.n_units, n_heads=c.n_heads, enc_n_layers=c.enc_n_layers,
                                 enc_dim_feedforward=c.enc_dim_feedforward, dec_n_layers=c.dec_n_layers,
                                 dec_dim_feedforward=c.dec_dim_feedforward, conv_delay=c.conv_delay,
                                 mask_delay=c.mask_delay, has_mask=int(bool(c.has_mask)), max_seqs=self.max_seqs,
                                 max_frames=self.max_frames, max_nspks=self.max_nspks,
                                 precision={"fp32": 0, "bf16": 1, "bf16x3": 2}[self.precision])
        h = _lib.create_handle("fseend", conf, _lib.host_state(unwrap_checkpoint(state_dict)))
        self._release()
        self._h = h
        self.in_ld = _lib.load().sd_fseend_input_stride(h)
        return self

    def _release(self):
        if self._h is not None:
            _lib.load().sd_fseend_destroy(self._h)
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
            raise ValueError("FS-EEND (MI355X backend) runs on a HIP device only")
        return self

    def device_bytes(self) -> int:
        return int(_lib.load().sd_fseend_device_bytes(self._h)) if self._h is not None else 0

    def test_device(self, feats, ilens: List[int], max_nspks: int = 6, want_emb: bool = True,
                    want_attractors: bool = True):
        """Device-level call on a padded (S, T, ld) feature tensor; returns the padded
        (preds (S,T,C), emb (S,T,D) | None, attractors (S,T,C,D) | None)."""
        if self._h is None:
            raise RuntimeError("load_state_dict() must be called before test()")
        S, T, ld = feats.shape
        D = self.cfg.n_units
        dev = self.device
        preds = torch.empty(S, T, max_nspks, device=dev, dtype=torch.float32)
        emb = torch.empty(S, T, D, device=dev, dtype=torch.float32) if want_emb else None
        att = torch.empty(S, T, max_nspks, D, device=dev, dtype=torch.float32) if want_attractors else None
        lens = (ctypes_int_array(ilens))
        _lib.call("sd_fseend_test", self._h, _lib.ptr(feats.contiguous()), ld, S, T, lens, max_nspks,
                  _lib.ptr(preds), _lib.ptr(emb), _lib.ptr(att), _lib.stream_ptr(dev))
        return preds, emb, att

    def test(self, src, ilens, max_nspks=6):
        """fs_eend.py:79-96: list of (T_i, in_size) -> (preds [(T_i, C)], emb [(T_i, D)],
        attractors [(T_i, C, D)])."""
        ilens = [int(n) for n in ilens]
        S, T = len(src), max(int(x.shape[0]) for x in src)
        buf = torch.full((S, T, self.in_ld), -1.0, device=self.device, dtype=torch.float32)   # pad_sequence(-1)
        for i, x in enumerate(src):
            buf[i, : x.shape[0], : self.cfg.in_size] = x.to(self.device, torch.float32)
        buf[:, :, self.cfg.in_size:] = 0.0
        preds, emb, att = self.test_device(buf, ilens, max_nspks)
        return ([preds[i, : ilens[i]] for i in range(S)], [emb[i, : ilens[i]] for i in range(S)],
                [att[i, : ilens[i]] for i in range(S)])


    def stream(self, chunk: int = 1, max_frames: int = None, max_nspks: int = 6, use_graph: bool = True):
        """Streaming counterpart of test() for one recording: push feature rows as they arrive,
        receive each frame's (max_nspks) scores once its 9-frame look-ahead is available."""
        if self._h is None:
            raise RuntimeError("load_state_dict() must be called before stream()")
        return FsEendStream(self, chunk, max_frames or self.max_frames, max_nspks, use_graph)


class FsEendStream:
    """Chunked FS-EEND scoring (libsdiar sd_fseend_stream_*).  push(x) accepts any number of
    (n, in_size) rows (buffered into chunks of `chunk` frames) and returns the (m, C) scores of
    the frames that became final; flush() ends the input and returns the rest.  Concatenated,
    the outputs equal test([x_all], [T])[0][0] (fs_eend.py:79-96)."""

    def __init__(self, model: "OnlineTransformerDADiarization", chunk: int, max_frames: int, max_nspks: int,
                 use_graph: bool):
        self.model = model
        self.chunk = int(chunk)
        self.C = int(max_nspks)
        self.max_frames = int(max_frames)
        self.device = model.device
        h = ctypes.c_void_p()
        _lib.call("sd_fseend_stream_create", model._h, self.chunk, self.max_frames, self.C, int(bool(use_graph)),
                  ctypes.byref(h))
        self._s = h
        self._pending = torch.zeros(0, model.cfg.in_size, device=self.device)
        self._buf = torch.zeros(self.chunk, model.in_ld, device=self.device, dtype=torch.float32)
        # one push emits at most ceil((chunk + 9) / chunk) chunks; flush up to ceil(9 / chunk) + 1
        self._out = torch.empty((self.chunk + 9) * 2 + self.chunk, self.C, device=self.device, dtype=torch.float32)

    def device_bytes(self) -> int:
        return int(_lib.load().sd_fseend_stream_device_bytes(self._s))

    def debug_counters(self) -> np.ndarray:
        """The device block-merge counters (decode attention per (slot, head), then the slot block's),
        read after the stream drains; each is 0 between launches."""
        n = ctypes.c_int()
        buf = (ctypes.c_uint * 256)()
        _lib.call("sd_fseend_stream_debug_counters", self._s, buf, 256, ctypes.byref(n), _lib.stream_ptr(self.device))
        return np.array(buf[: min(n.value, 256)], dtype=np.uint32)

    def _push_rows(self, rows) -> torch.Tensor:
        n = int(rows.shape[0])
        self._buf.zero_()
        self._buf[:n, : self.model.cfg.in_size] = rows
        cnt = ctypes.c_int()
        _lib.call("sd_fseend_stream_push", self._s, _lib.ptr(self._buf), self.model.in_ld, n, _lib.ptr(self._out),
                  self._out.shape[0], ctypes.byref(cnt), _lib.stream_ptr(self.device))
        return self._out[: cnt.value].clone()

    def push(self, x) -> torch.Tensor:
        x = x.to(self.device, torch.float32).reshape(-1, self.model.cfg.in_size)
        data = torch.cat([self._pending, x], 0)
        outs = []
        full = data.shape[0] // self.chunk * self.chunk
        for i in range(0, full, self.chunk):
            outs.append(self._push_rows(data[i : i + self.chunk]))
        self._pending = data[full:]
        return torch.cat(outs, 0) if outs else self._out[:0].clone()

    def set_audio(self, sample_rate: int = 8000, frame_size: int = 200, frame_shift: int = 80,
                  context_size: int = 7, subsampling: int = 10):
        """Take raw audio from now on (push_audio): the FS-EEND frontend of fs_eend/dataset.py:217-223
        (transform 'logmel23', sr hardcoded 8000) + splice + subsample, incrementally on the device
        inside each chunk's captured graph.  Valid on a fresh or reset() stream."""
        from ..feature import _mel_device
        n_fft = 1 << (frame_size - 1).bit_length()
        self._fb = _mel_device(sample_rate, n_fft, self.device)
        _lib.call("sd_fseend_stream_set_audio", self._s, _lib.ptr(self._fb), self._fb.shape[0], frame_size,
                  frame_shift, context_size, subsampling)
        self._hop_rows = frame_shift * subsampling       # samples per model frame
        self._audio = True
        return self

    def _ensure_out(self, rows: int):
        if self._out.shape[0] < rows:
            self._out = torch.empty(rows, self.C, device=self.device, dtype=torch.float32)

    def push_audio(self, samples) -> torch.Tensor:
        """samples: 1-D float32 audio at the frontend's rate (any length, e.g. 640 = 80 ms) ->
        the (m, C) scores of the frames that became final."""
        if not getattr(self, "_audio", False):
            raise RuntimeError("push_audio: call set_audio() first")
        x = samples.to(self.device, torch.float32).reshape(-1).contiguous()
        self._ensure_out(x.numel() // self._hop_rows + 2 * (self.chunk + 10))
        cnt = ctypes.c_int()
        _lib.call("sd_fseend_stream_push_audio", self._s, _lib.ptr(x) if x.numel() else None, x.numel(),
                  _lib.ptr(self._out), self._out.shape[0], ctypes.byref(cnt), _lib.stream_ptr(self.device))
        return self._out[: cnt.value].clone()

    def flush(self) -> torch.Tensor:
        outs = []
        if self._pending.shape[0] > 0:
            outs.append(self._push_rows(self._pending))
            self._pending = self._pending[:0]
        self._ensure_out(4 * (self.chunk + 10))
        cnt = ctypes.c_int()
        _lib.call("sd_fseend_stream_flush", self._s, _lib.ptr(self._out), self._out.shape[0], ctypes.byref(cnt),
                  _lib.stream_ptr(self.device))
        outs.append(self._out[: cnt.value].clone())
        return torch.cat(outs, 0)

    def reset(self):
        """Back to an empty stream taking feature rows (set_audio() again for audio)."""
        self._pending = self._pending[:0]
        self._audio = False
        _lib.call("sd_fseend_stream_reset", self._s, _lib.stream_ptr(self.device))

    def close(self):
        if getattr(self, "_s", None) is not None:
            _lib.load().sd_fseend_stream_destroy(self._s)
        self._s = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def ctypes_int_array(vals):
    import ctypes
    return (ctypes.c_int * len(vals))(*vals)
