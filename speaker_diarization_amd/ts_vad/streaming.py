"""TSVADModel of egs/alimeeting/ts_vad2_streaming/model.py — chunk-streaming decode on gfx950.

Same constructor inputs (TSVADStreamingConfig mirrors the streaming TSVADConfig fields the
decode reads), same state_dict keys (strict load), and the reference's streaming entry points:
`forward_chunk_by_chunk(xs, target_speech, labels, decoding_chunk_size, num_decoding_left_chunks)`
and its `forward_chunk_by_chunk_temp1` alias (the one `infer_debug` calls with
simulate_streaming, model.py:951-975), both B = 1 like the reference (`forward_chunk` asserts
it, :720).  libsdiar decodes the whole window in one call: the KV caches of the reference's
chunk loop become block-causal attention masks (include/sdiar.h, sd_tsvad_stream_*).
`forward_windows` decodes a batch of independent windows in one call (what infer.py's window
loop does one window at a time, infer_debug batch 1).
"""
from __future__ import annotations

import ctypes

import numpy as np

from .. import _lib
from ..weights import TSVADStreamingConfig, unwrap_checkpoint


class TSVADStreamingModel:
    def __init__(self, cfg: TSVADStreamingConfig = None, device=None, precision: str = "bf16",
                 max_labels: int = 400, max_windows: int = 1):
        import torch
        self.cfg = cfg or TSVADStreamingConfig()
        if precision not in ("bf16", "fp32"):
            raise ValueError(f"precision must be bf16 or fp32, got {precision}")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise ValueError("TSVADStreamingModel (MI355X backend) runs on a HIP device only")
        self.precision, self.max_labels, self.max_windows = precision, max_labels, max_windows
        self.max_num_speaker = self.cfg.max_num_speaker
        self.subsampling_rate = 4   # Subsampling4 (model.py:1318)
        c = self.cfg
        conf = _lib.TsvadStreamConfig(
            max_num_speaker=c.max_num_speaker, max_labels=max_labels, precision=1 if precision == "bf16" else 0,
            num_transformer_layer=c.num_transformer_layer, num_attention_head=c.num_attention_head,
            transformer_embed_dim=c.transformer_embed_dim, transformer_ffn_embed_dim=c.transformer_ffn_embed_dim,
            speaker_embed_dim=c.speaker_embed_dim, max_windows=max_windows)
        h = ctypes.c_void_p()
        _lib.call("sd_tsvad_stream_create", ctypes.byref(conf), ctypes.byref(h))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib._lib is not None:
            _lib.load().sd_tsvad_stream_destroy(h)
            self._h = None

    def load_state_dict(self, state_dict, strict: bool = True):
        import torch
        if not strict:
            raise ValueError("the MI355X backend only supports strict=True loading")
        state_dict = unwrap_checkpoint(state_dict)
        with torch.device("cpu"):
            for k, v in state_dict.items():
                t = torch.as_tensor(np.asarray(v.cpu() if hasattr(v, "cpu") else v)).to(torch.float32).contiguous()
                shape = (ctypes.c_int64 * max(t.dim(), 1))(*t.shape)
                _lib.call("sd_tsvad_stream_set_param", self._h, k.encode(), ctypes.c_void_p(t.data_ptr()), shape,
                          t.dim())
        _lib.call("sd_tsvad_stream_finalize", self._h)
        return self

    def eval(self):
        return self

    @property
    def device_bytes(self) -> int:
        return int(_lib.load().sd_tsvad_stream_device_bytes(self._h))

    def forward_chunk_by_chunk(self, xs, target_speech, labels, decoding_chunk_size: int = 0,
                               num_decoding_left_chunks: int = -1, out=None):
        """xs (1, T, 80) fbank, target_speech (1, NS, 192), labels (1, NS, T_lab) (only its length
        is read) -> logits (1, NS, T_lab) (model.py:368-461 / 594-655)."""
        import torch
        assert decoding_chunk_size > 0
        assert xs.size(0) == 1, "chunk streaming decodes one window at a time (model.py:720)"
        T_lab = labels if isinstance(labels, int) else labels.size(-1)
        n = self.subsampling_rate * T_lab
        x = xs[0].to(self.device, torch.float32)
        if x.shape[0] != n:   # F.pad to 4 x labels (a negative gap trims), model.py:614-618
            x = torch.nn.functional.pad(x.t(), (0, n - x.shape[0])).t()
        x = x.contiguous()
        ts = target_speech[0].to(self.device, torch.float32).contiguous()
        assert ts.shape == (self.max_num_speaker, self.cfg.speaker_embed_dim)
        if out is None:
            out = torch.empty(1, self.max_num_speaker, T_lab, device=self.device, dtype=torch.float32)
        _lib.call("sd_tsvad_stream_forward", self._h, _lib.ptr(x), _lib.ptr(ts), 1, T_lab, int(decoding_chunk_size),
                  int(num_decoding_left_chunks), _lib.ptr(out), _lib.stream_ptr(self.device))
        return out

    def forward_windows(self, xs, target_speech, T_lab: int, decoding_chunk_size: int,
                        num_decoding_left_chunks: int = -1, out=None):
        """B windows at once: xs (B, 4 * T_lab, 80) fbank on the device, target_speech (B, NS, 192)
        -> logits (B, NS, T_lab); window b equals forward_chunk_by_chunk on window b alone."""
        import torch
        B = xs.shape[0]
        assert decoding_chunk_size > 0
        assert xs.shape[1:] == (self.subsampling_rate * T_lab, 80), xs.shape
        assert target_speech.shape == (B, self.max_num_speaker, self.cfg.speaker_embed_dim)
        assert xs.device == self.device and xs.dtype == torch.float32 and xs.is_contiguous()
        ts = target_speech.to(self.device, torch.float32).contiguous()
        if out is None:
            out = torch.empty(B, self.max_num_speaker, T_lab, device=self.device, dtype=torch.float32)
        _lib.call("sd_tsvad_stream_forward", self._h, _lib.ptr(xs), _lib.ptr(ts), B, T_lab, int(decoding_chunk_size),
                  int(num_decoding_left_chunks), _lib.ptr(out), _lib.stream_ptr(self.device))
        return out

    forward_chunk_by_chunk_temp1 = forward_chunk_by_chunk


class StreamingWindowDecoder:
    """Adapter that lets ts_vad.pipeline.TSVADPipeline (window plan, device fbank + window CMN,
    overlap average) drive the chunk-streaming model: the streaming recipe's decode
    (run_ts_vad2_streaming.sh: rs_len 10, segment_shift 1, decoding_chunk_size 25,
    num_decoding_left_chunks -1; infer.py window loop -> infer_debug -> forward_chunk_by_chunk_temp1).
    The recipe decodes one window per batch (run_ts_vad2_streaming.sh:74 batch_size=1; forward_chunk
    asserts B == 1, model.py:720), so every window is decoded at its own length: the adapter sets
    `reference_batch_size = 1` and TSVADPipeline then fuses only consecutive windows of identical
    length into one sd_tsvad_stream_forward call (a tail window is never padded with another
    window's frames, which would turn its partial last chunk into a full one).  Each window's fbank
    is padded / trimmed to 4 x labels (model.py:614-618)."""

    reference_batch_size = 1

    def __init__(self, model: TSVADStreamingModel, decoding_chunk_size: int = 25, num_decoding_left_chunks: int = -1,
                 rs_len: int = 10, label_rate: int = 25, sample_rate: int = 16000):
        from types import SimpleNamespace
        self.model = model
        self.cfg = SimpleNamespace(rs_len=rs_len, label_rate=label_rate, sample_rate=sample_rate)
        self.max_batch = model.max_windows
        self.max_num_speaker = model.max_num_speaker
        self.device = model.device
        self.chunk, self.left = decoding_chunk_size, num_decoding_left_chunks

    def forward(self, ref, ts, T_lab: int, check: bool = True, out=None):
        """check: accepted for TSVADModel's signature; the streaming model has no LSTM to report."""
        import torch
        n = self.model.subsampling_rate * T_lab
        if ref.shape[1] != n:
            ref = torch.nn.functional.pad(ref, (0, 0, 0, n - ref.shape[1]))
        return self.model.forward_windows(ref.contiguous(), ts, T_lab, self.chunk, self.left, out=out)
