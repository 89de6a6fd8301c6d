"""TSVADModel — drop-in for egs/alimeeting/ts_vad2/model.py:179 (inference).

Same constructor inputs (TSVADConfig + data config), same state_dict keys,
same forward(ref_speech, target_speech, labels, num_updates) -> logits
(B, max_num_speaker, T_label) and infer(...) -> (result, res_dict) surface.
The forward runs entirely in libsdiar (HIP, gfx950); this class only moves
state_dict tensors across the C ABI and wraps device pointers.
"""
from __future__ import annotations

import ctypes
from collections import defaultdict

import numpy as np

from .. import _lib
from ..weights import TSVADConfig, unwrap_checkpoint


def fbank_frames(rs_len: int, sample_rate: int = 16000) -> int:
    n = rs_len * sample_rate
    return 1 + (n - 400) // 160


class TSVADModel:
    def __init__(self, cfg: TSVADConfig = None, task_cfg=None, device=None, precision: str = "bf16",
                 max_batch: int = 64):
        import torch
        self.cfg = cfg or TSVADConfig()
        if task_cfg is not None:   # mirror of TSVADDataConfig fields the model reads
            for k in ("rs_len", "max_num_speaker", "label_rate", "sample_rate"):
                if hasattr(task_cfg, k):
                    setattr(self.cfg, k, getattr(task_cfg, k))
        assert self.cfg.label_rate == 25, f"self.label_rate is {self.cfg.label_rate} not support!"
        if precision not in ("bf16", "fp32", "bf16x3"):
            raise ValueError(f"precision must be bf16, fp32 or bf16x3, got {precision}")
        self.precision = precision
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise ValueError("TSVADModel (MI355X backend) runs on a HIP device only")
        self.max_batch = max_batch
        self.max_num_speaker = self.cfg.max_num_speaker
        self.max_fbank = fbank_frames(self.cfg.rs_len, self.cfg.sample_rate)
        self._h = None
        self._create()

    # ------------------------------------------------------------------ handle
    def _create(self):
        c = self.cfg
        conf = _lib.TsvadConfig(
            variant=c.variant, max_num_speaker=c.max_num_speaker, rs_len=c.rs_len, max_batch=self.max_batch,
            max_fbank_frames=self.max_fbank, precision={"fp32": 0, "bf16": 1, "bf16x3": 2}[self.precision],
            num_transformer_layer=c.num_transformer_layer, num_attention_head=c.num_attention_head,
            transformer_embed_dim=c.transformer_embed_dim,
            transformer_ffn_embed_dim=c.transformer_ffn_embed_dim, speaker_embed_dim=c.speaker_embed_dim)
        h = ctypes.c_void_p()
        _lib.call("sd_tsvad_create", ctypes.byref(conf), ctypes.byref(h))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib._lib is not None:
            _lib.load().sd_tsvad_destroy(h)
            self._h = None

    def load_state_dict(self, state_dict, strict: bool = True):
        """Strict load (missing/unexpected keys raise RuntimeError like torch)."""
        import torch
        if not strict:
            raise ValueError("the MI355X backend only supports strict=True loading")
        state_dict = unwrap_checkpoint(state_dict)
        with torch.device("cpu"):
            for k, v in state_dict.items():
                t = torch.as_tensor(np.asarray(v.cpu() if hasattr(v, "cpu") else v)).to(torch.float32).contiguous()
                shape = (ctypes.c_int64 * max(t.dim(), 1))(*t.shape)
                _lib.call("sd_tsvad_set_param", self._h, k.encode(), ctypes.c_void_p(t.data_ptr()), shape, t.dim())
        _lib.call("sd_tsvad_finalize", self._h)
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
        return int(_lib.load().sd_tsvad_device_bytes(self._h))

    # ------------------------------------------------------------------ forward
    def forward(self, ref_speech, target_speech, labels, num_updates: int = 0, out=None, check: bool = True,
                forward_batch: int = 0, _force: int = 0):
        """ref_speech (B, T_fb, 80), target_speech (B, NS, 192), labels (B, NS, T) (only
        labels.size(-1) is read, model.py:681/770) -> logits (B, NS, T).  check: wait for the
        stream and raise RuntimeError in this call if the BiLSTM's persistent recurrence lost
        co-residency (its logits are NaN); check=False defers that to status().
        forward_batch: windows per reference forward call when this call covers several of them (the
        pipeline's fused device batches): the scope of BatchNorm1D's NaN bypass (model.py:161-171).  0: this
        call is one batch.  A call of more than max_batch windows runs as several device forwards cut at
        reference-batch boundaries; a reference batch wider than max_batch is cut into device forwards that
        each learn (`_force`) whether a non-finite input sits anywhere in that batch, so the bypass keeps the
        reference's scope."""
        import torch
        B, T_fb, F = ref_speech.shape
        T_lab = labels if isinstance(labels, int) else labels.size(-1)
        assert F == 80, "CAM++ expects 80-dim fbank"
        ref = ref_speech.to(self.device, torch.float32).contiguous()
        ts = target_speech.to(self.device, torch.float32).contiguous()
        assert ts.shape == (B, self.max_num_speaker, self.cfg.speaker_embed_dim)
        if out is None:
            out = torch.empty(B, self.max_num_speaker, T_lab, device=self.device, dtype=torch.float32)
        G = forward_batch if forward_batch > 0 else B
        if B > self.max_batch:
            if G <= self.max_batch:      # whole reference batches per device forward
                step = self.max_batch // G * G
                for s in range(0, B, step):
                    e = min(B, s + step)
                    self.forward(ref[s:e], ts[s:e], T_lab, out=out[s:e], check=False, forward_batch=G)
            else:                        # a reference batch spans device forwards: its non-finite flags up front
                for g0 in range(0, B, G):
                    g1 = min(B, g0 + G)
                    force = 3 if not bool(torch.isfinite(ref[g0:g1]).all()) else 0
                    if self.cfg.variant == 0 and not bool(torch.isfinite(ts[g0:g1]).all()):
                        force |= 2
                    for s in range(g0, g1, self.max_batch):
                        e = min(g1, s + self.max_batch)
                        self.forward(ref[s:e], ts[s:e], T_lab, out=out[s:e], check=False, _force=force)
            if check:
                self.status()
            return out
        _lib.call("sd_tsvad_forward_batched", self._h, _lib.ptr(ref), _lib.ptr(ts), B, T_fb, T_lab,
                  int(forward_batch), int(_force), _lib.ptr(out), _lib.stream_ptr(self.device))
        if check:
            self.status()
        return out

    def status(self):
        """sd_tsvad_status: wait for the device stream, raise RuntimeError if a persistent LSTM
        recurrence of the forwards enqueued so far timed out."""
        _lib.call("sd_tsvad_status", self._h, _lib.stream_ptr(self.device))

    __call__ = forward

    # ------------------------------------------------------------------ infer (model.py:923-970)
    def infer(self, ref_speech, target_speech, labels, labels_len, num_updates: int = 0, file_path=None,
              speaker_ids=None, start=None):
        import torch
        outs = self.forward(ref_speech, target_speech, labels, num_updates)
        outs_prob = torch.sigmoid(outs).cpu().numpy()
        logits = outs.cpu().numpy().astype(np.float64)
        lab = labels.cpu().numpy().astype(np.float64)
        lens = np.asarray(labels_len.cpu() if hasattr(labels_len, "cpu") else labels_len)
        loss = 0.0
        for i in range(len(lens)):
            x, y = logits[i, :, : lens[i]], lab[i, :, : lens[i]]
            loss += np.mean(np.maximum(x, 0) - x * y + np.log1p(np.exp(-np.abs(x))))
        result = {"losses": {"diar": loss / len(lens)}}
        mi, fa, cf, acc, der = calc_diarization_result(outs_prob.transpose((0, 2, 1)),
                                                        lab.transpose(0, 2, 1), lens)
        result.update(labels_len=labels_len, DER=der, ACC=acc, MI=mi, FA=fa, CF=cf)
        res_dict = defaultdict(lambda: defaultdict(list))
        B = outs_prob.shape[0]
        for b in range(B):
            n = max(speaker_ids[b])
            for t in range(int(lens[b])):
                for i in range(n):
                    res_dict[str(file_path[b]) + "-" + str(speaker_ids[b][i])][start[b] + t].append(outs_prob[b, i, t])
        return result, res_dict


def calc_diarization_error(pred, label, length):
    """model.py:973-1015 (EEND-style frame error counts), numpy."""
    batch_size, max_len, num_output = label.shape
    mask = np.zeros((batch_size, max_len, num_output))
    for i in range(batch_size):
        mask[i, : length[i], :] = 1
    label_np = label.astype(int) * mask
    pred_np = (pred > 0.5).astype(int) * mask
    n_ref = np.sum(label_np, axis=2)
    n_sys = np.sum(pred_np, axis=2)
    speech_scored = float(np.sum(n_ref > 0))
    speech_miss = float(np.sum(np.logical_and(n_ref > 0, n_sys == 0)))
    speech_falarm = float(np.sum(np.logical_and(n_ref == 0, n_sys > 0)))
    speaker_scored = float(np.sum(n_ref))
    speaker_miss = float(np.sum(np.maximum(n_ref - n_sys, 0)))
    speaker_falarm = float(np.sum(np.maximum(n_sys - n_ref, 0)))
    n_map = np.sum(np.logical_and(label_np == 1, pred_np == 1), axis=2)
    speaker_error = float(np.sum(np.minimum(n_ref, n_sys) - n_map))
    correct = float(1.0 * np.sum((label_np == pred_np) * mask) / num_output)
    num_frames = np.sum(length)
    return (correct, num_frames, speech_scored, speech_miss, speech_falarm, speaker_scored, speaker_miss,
            speaker_falarm, speaker_error)


def calc_diarization_result(outs_prob, labels, labels_len):
    """model.py:1018-1048."""
    (correct, num_frames, speech_scored, speech_miss, speech_falarm, speaker_scored, speaker_miss,
     speaker_falarm, speaker_error) = calc_diarization_error(outs_prob, labels, labels_len)
    if speech_scored == 0 or speaker_scored == 0:
        return 0, 0, 0, 0, 0
    return (speaker_miss / speaker_scored, speaker_falarm / speaker_scored, speaker_error / speaker_scored,
            correct / num_frames, (speaker_miss + speaker_falarm + speaker_error) / speaker_scored)
