"""SSNDModel — drop-in for egs/alimeeting/ssnd/ssnd_model.py:372-900 (inference).

Same constructor arguments (the ones inference reads), same state_dict keys (strict load), and
the reference's inference entry points: `infer(feats, speaker_embs) -> (vad_pred, emb_pred)`
(:752-776), `offline_diarization(feats, threshold)` (:778-800) and `online_infer(blocks, l_c,
l_r, t1, t2)` (:802-897).  The forward (CAM++ extractor, Conformer encoder, speaker-query
cross-attention DetectionDecoder, RepresentationDecoder) runs in libsdiar (sd_ssnd_*, HIP on
gfx950); this class moves state_dict tensors across the C ABI, wraps device pointers and keeps
the reference's host-side bookkeeping (speaker buffer of online_infer).
"""
from __future__ import annotations

import ctypes

import numpy as np

from .. import _lib
from ..weights import SSNDConfig, unwrap_checkpoint


class SSNDModel:
    def __init__(self, speaker_pretrain_model_path=None, extractor_model_type="CAM++_wo_gsp", feat_dim=80,
                 emb_dim=256, q_det_aux_dim=256, q_rep_aux_dim=256, d_model=256, nhead=8, d_ff=512,
                 num_layers=4, max_speakers=4, vad_out_len=100, pos_emb_dim=256, max_seq_len=1000,
                 n_all_speakers=1000, training=False, device=None, precision: str = "fp32", max_batch: int = 8,
                 **_unused_training_args):
        import torch
        if extractor_model_type != "CAM++_wo_gsp":
            raise ValueError(f"the MI355X SSND backend builds extractor CAM++_wo_gsp, got {extractor_model_type}")
        if precision not in ("bf16", "fp32"):
            raise ValueError(f"precision must be bf16 or fp32, got {precision}")
        self.cfg = SSNDConfig(feat_dim=feat_dim, emb_dim=emb_dim, q_det_aux_dim=q_det_aux_dim,
                              q_rep_aux_dim=q_rep_aux_dim, d_model=d_model, nhead=nhead, d_ff=d_ff,
                              num_layers=num_layers, max_speakers=max_speakers, vad_out_len=vad_out_len,
                              pos_emb_dim=pos_emb_dim, max_seq_len=max_seq_len, n_all_speakers=n_all_speakers)
        self.device = torch.device(device) if device is not None and str(device) != "cpu" else \
            torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise ValueError("SSNDModel (MI355X backend) runs on a HIP device only")
        self.precision, self.max_batch = precision, max_batch
        self.max_speakers, self.emb_dim, self.d_model = max_speakers, emb_dim, d_model
        # a block of vad_out_len label frames = 4 * vad_out_len fbank frames (CAM++ /2, down conv /2)
        self.block_frames = 4 * vad_out_len
        c = self.cfg
        conf = _lib.SsndConfig(max_batch=max_batch, max_fbank_frames=self.block_frames, max_speakers=max_speakers,
                               feat_dim=feat_dim, emb_dim=emb_dim, q_det_aux_dim=q_det_aux_dim,
                               q_rep_aux_dim=q_rep_aux_dim, d_model=d_model, nhead=nhead, d_ff=d_ff,
                               num_layers=num_layers, vad_out_len=vad_out_len, pos_emb_dim=pos_emb_dim,
                               max_seq_len=max_seq_len, n_all_speakers=n_all_speakers,
                               conformer_kernel=c.conformer_kernel, precision=1 if precision == "bf16" else 0)
        h = ctypes.c_void_p()
        _lib.call("sd_ssnd_create", ctypes.byref(conf), ctypes.byref(h))
        self._h = h
        self.E_all = self.e_pse = self.e_non = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib._lib is not None:
            _lib.load().sd_ssnd_destroy(h)
            self._h = None

    def load_state_dict(self, state_dict, strict: bool = True):
        import torch
        if not strict:
            raise ValueError("the MI355X backend only supports strict=True loading")
        state_dict = unwrap_checkpoint(state_dict, kind="ssnd")
        with torch.device("cpu"):
            for k, v in state_dict.items():
                t = torch.as_tensor(np.asarray(v.cpu() if hasattr(v, "cpu") else v)).to(torch.float32).contiguous()
                shape = (ctypes.c_int64 * max(t.dim(), 1))(*t.shape)
                _lib.call("sd_ssnd_set_param", self._h, k.encode(), ctypes.c_void_p(t.data_ptr()), shape, t.dim())
                if k in ("E_all", "e_pse", "e_non"):
                    setattr(self, k, t.to(self.device))
        _lib.call("sd_ssnd_finalize", self._h)
        return self

    def eval(self):
        return self

    @property
    def device_bytes(self) -> int:
        return int(_lib.load().sd_ssnd_device_bytes(self._h))

    # ------------------------------------------------------------------ inference
    def infer(self, feats, speaker_embs):
        """feats (B, T_fb, 80) fbank blocks, speaker_embs (B, N, emb_dim) -> vad_pred (B, N, T) pre-sigmoid,
        emb_pred (B, N, emb_dim) (ssnd_model.py:752-776)."""
        import torch
        x = feats.to(self.device, torch.float32).contiguous()
        spk = speaker_embs.to(self.device, torch.float32).contiguous()
        B, T_fb, F = x.shape
        N = self.max_speakers
        assert F == 80 and spk.shape == (B, N, self.emb_dim), (x.shape, spk.shape)
        T = self.cfg.vad_out_len
        vad = torch.empty(B, N, T, device=self.device, dtype=torch.float32)
        emb = torch.empty(B, N, self.emb_dim, device=self.device, dtype=torch.float32)
        for s in range(0, B, self.max_batch):
            e = min(B, s + self.max_batch)
            _lib.call("sd_ssnd_infer", self._h, _lib.ptr(x[s:e]), _lib.ptr(spk[s:e]), e - s, T_fb, _lib.ptr(vad[s:e]),
                      _lib.ptr(emb[s:e]), _lib.stream_ptr(self.device))
        return vad, emb

    def decode(self, enc_out, x_fea, speaker_embs):
        """The decoders alone on given encoder / extractor outputs (infer after :763)."""
        import torch
        enc = enc_out.to(self.device, torch.float32).contiguous()
        x = x_fea.to(self.device, torch.float32).contiguous()
        spk = speaker_embs.to(self.device, torch.float32).contiguous()
        B, T, _ = enc.shape
        N = self.max_speakers
        vad = torch.empty(B, N, T, device=self.device, dtype=torch.float32)
        emb = torch.empty(B, N, self.emb_dim, device=self.device, dtype=torch.float32)
        for s in range(0, B, self.max_batch):
            e = min(B, s + self.max_batch)
            _lib.call("sd_ssnd_decode", self._h, _lib.ptr(enc[s:e]), _lib.ptr(x[s:e]), _lib.ptr(spk[s:e]), e - s, T,
                      _lib.ptr(vad[s:e]), _lib.ptr(emb[s:e]), _lib.stream_ptr(self.device))
        return vad, emb

    def offline_diarization(self, feats, threshold=0.5):
        """ssnd_model.py:778-800: E_all[:N] as the speaker embeddings of every block ->
        ((N, T) 0/1 labels, (N, T) probabilities) for a (1, T_fb, 80) or (T_fb, 80) block."""
        import torch
        if feats.ndim == 2:
            feats = feats.unsqueeze(0)
        B = feats.shape[0]
        spk = self.E_all[: self.max_speakers].unsqueeze(0).expand(B, self.max_speakers, self.emb_dim)
        vad, _ = self.infer(feats, spk)
        prob = torch.sigmoid(vad)
        return (prob > threshold).long().squeeze(0), prob.squeeze(0)

    def online_infer(self, blocks, l_c, l_r, t1=0.5, t2=0.5, device=None):
        """ssnd_model.py:802-897 (the paper's block-wise online loop): per block, the pseudo speaker
        plus the weighted-mean embeddings of the speakers registered so far (padded with e_non) are
        the queries; the block's last l_c (+ l_r right context) frames are emitted per speaker and
        the embedding buffer is updated with weights v = mean VAD probability.  Returns
        {spk_id: np.ndarray of frame probabilities}."""
        import torch
        dia, buf = {}, {}
        num_frames = 0
        S, N = self.emb_dim, self.max_speakers
        e_pse, e_non = self.e_pse.squeeze(0), self.e_non.squeeze(0)
        dev = self.device
        pse_id = 0
        for block in blocks:
            if not torch.is_tensor(block):
                block = torch.tensor(np.asarray(block), dtype=torch.float32)
            block = block.to(dev, torch.float32)
            emb_list, spk_list = [e_pse], [pse_id]
            for spk_id in buf:
                e_sum = torch.zeros(S, device=dev)
                w_sum = 0.0
                for e, w in buf[spk_id]:
                    e_sum += e * w
                    w_sum += w
                emb_list.append(e_sum / w_sum if w_sum > 0 else e_non)
                spk_list.append(spk_id)
            while len(emb_list) < N:
                emb_list.append(e_non)
                spk_list.append(-1)
            emb_t = torch.stack(emb_list).unsqueeze(0)
            vad, spk_pred = self.infer(block.unsqueeze(0), emb_t)
            prob = torch.sigmoid(vad)[0]
            y_pse, e_pse_new = prob[0], spk_pred[0, 0]
            v_pse = y_pse.mean().item()
            cur = y_pse[-(l_c + l_r):-l_r] if l_r > 0 else y_pse[-l_c:]
            if pse_id not in dia:
                dia[pse_id] = torch.zeros(num_frames)
            dia[pse_id] = torch.cat([dia[pse_id], cur.cpu()])
            if v_pse > t1:
                buf[pse_id] = [(e_pse_new.detach(), v_pse)]
            for n in range(1, N):
                if spk_list[n] == -1:
                    continue
                y_n, e_n = prob[n], spk_pred[0, n]
                v_n = y_n.mean().item()
                cur_n = y_n[-(l_c + l_r):-l_r] if l_r > 0 else y_n[-l_c:]
                if spk_list[n] not in dia:
                    dia[spk_list[n]] = torch.zeros(num_frames)
                dia[spk_list[n]] = torch.cat([dia[spk_list[n]], cur_n.cpu()])
                if v_n > t2:
                    buf.setdefault(spk_list[n], []).append((e_n.detach(), v_n))
            num_frames += l_c
        return {k: v.numpy() for k, v in dia.items()}
