"""EEND-EDA inference restated on CPU — TEST INFRASTRUCTURE ONLY (oracle / cpu_baseline).

Frontend (speaker_diarization/feature.py):
  stft      feature.py:155-184  -> librosa.stft(n_fft, win_length, hop, hann, center=True)
  transform feature.py:64-73    -> 'logmel23_mn': log10(max(|Y|^2 · mel^T, 1e-10)) - mean
  splice    feature.py:130-152  -> zero-padded ±context frames
  subsample infer_eda.py:97-98  -> Y[::subsampling]
librosa 0.10.2 (requirements.txt:13) is not installed here: `librosa_stft` and
`slaney_mel` restate its published algorithms (constant/zero centre padding,
periodic Hann zero-padded to n_fft, Slaney mel scale with area normalisation) —
parity unpinned for those two functions; the glue around them is pinned by the
golden produced from the reference feature.py with these two injected.

Model (speaker_diarization/eend_eda):
  forward_embedding models.py:213-234 (TransformerEda) / 515-538 (EendEda)
  LstmEncoderDedecoderAttractor.forward encoder_decoder_attractor.py:19-59
  infer models.py:297-347 (TransformerEda) / 601-652 (EendEda)
  chunking infer_eda.py:21-28, 92-121
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from .tsvad_ref import conformer, lstm, transformer_layer


# ----------------------------------------------------------------------------- librosa 0.10.2
def hann_periodic(n: int) -> np.ndarray:
    """scipy.signal.get_window('hann', n, fftbins=True)."""
    k = np.arange(n, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * k / n)


def librosa_stft(y: np.ndarray, n_fft: int, hop_length: int, win_length: int) -> np.ndarray:
    """librosa.stft(y, n_fft, hop_length, win_length, window='hann', center=True,
    pad_mode='constant') -> (1 + n_fft//2, n_frames) complex128 for float64 y."""
    y = np.asarray(y, dtype=np.float64)
    win = np.zeros(n_fft)
    lpad = (n_fft - win_length) // 2
    win[lpad:lpad + win_length] = hann_periodic(win_length)
    yp = np.pad(y, (n_fft // 2, n_fft // 2), mode="constant")
    n_frames = 1 + (len(yp) - n_fft) // hop_length
    idx = np.arange(n_fft)[None, :] + hop_length * np.arange(n_frames)[:, None]
    return np.fft.rfft(yp[idx] * win[None, :], axis=1).T


def _hz_to_mel(f):
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-30) / min_log_hz) / logstep, mels)


def _mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)


def slaney_mel(sr: float, n_fft: int, n_mels: int, fmin: float = 0.0, fmax: float = None) -> np.ndarray:
    """librosa.filters.mel(sr=sr, n_fft=n_fft, n_mels=n_mels) (htk=False, norm='slaney',
    dtype float32): (n_mels, 1 + n_fft//2)."""
    fmax = sr / 2.0 if fmax is None else fmax
    weights = np.zeros((n_mels, 1 + n_fft // 2), dtype=np.float32)
    fftfreqs = np.fft.rfftfreq(n=n_fft, d=1.0 / sr)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fftfreqs[None, :]
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, None]
    return weights


# ----------------------------------------------------------------------------- feature.py
def stft(data, frame_size=400, frame_shift=160):
    """feature.stft: n_fft = next pow2 of frame_size; drops the last frame when
    len(data) % frame_shift == 0 (feature.py:176-184)."""
    fft_size = 1 << (frame_size - 1).bit_length()
    Y = librosa_stft(data, fft_size, frame_shift, frame_size).T
    return Y[:-1] if len(data) % frame_shift == 0 else Y


def transform_logmel23_mn(Y, sample_rate=16000):
    """feature.transform(Y, 'logmel23_mn') (feature.py:64-73): float64 math, float32 out."""
    Y = np.abs(Y)
    n_fft = 2 * (Y.shape[1] - 1)
    mel = slaney_mel(sample_rate, n_fft, 23)
    Y = np.dot(Y ** 2, mel.T)
    Y = np.log10(np.maximum(Y, 1e-10))
    Y = Y - np.mean(Y, axis=0)
    return Y.astype(np.float32)


def transform_logmel23(Y, sample_rate=8000):
    """feature.transform(Y, 'logmel23') (feature.py:56-63), used by FS-EEND."""
    Y = np.abs(Y)
    n_fft = 2 * (Y.shape[1] - 1)
    mel = slaney_mel(sample_rate, n_fft, 23)
    Y = np.log10(np.maximum(np.dot(Y ** 2, mel.T), 1e-10))
    return Y.astype(np.float32)


def splice(Y, context_size=0):
    """feature.splice (feature.py:130-152): row t = Y_pad[t : t + 2c + 1] flattened."""
    Yp = np.pad(Y, [(context_size, context_size), (0, 0)], "constant")
    T, D = Y.shape
    idx = np.arange(T)[:, None] + np.arange(2 * context_size + 1)[None, :]
    return Yp[idx].reshape(T, D * (2 * context_size + 1))


def features(wav, sample_rate=16000, frame_size=400, frame_shift=160, context_size=7, subsampling=10,
             transform="logmel23_mn"):
    """infer_eda.py:94-98: stft -> transform -> splice -> [::subsampling]."""
    Y = stft(wav, frame_size, frame_shift)
    if transform == "logmel23_mn":
        Y = transform_logmel23_mn(Y, sample_rate)
    elif transform == "logmel23":
        Y = transform_logmel23(Y, sample_rate)
    else:
        raise ValueError("Unknown transform_type: %s" % transform)
    return splice(Y, context_size)[::subsampling]


def gen_chunk_indices(data_len, chunk_size):
    """infer_eda.py:21-28."""
    start = 0
    while start < data_len:
        yield start, min(data_len, start + chunk_size)
        start += chunk_size


# ----------------------------------------------------------------------------- model
def _prefixes(variant):
    return ("encoder.", "encoder_norm.", "transformer_encoder.layers.") if variant == 0 else \
        ("linear.", "linear_norm.", "encoder.layers.")


@torch.no_grad()
def embedding(sd, cfg, src):
    """forward_embedding up to emb (before the shuffle): src list of (T_i, in) ->
    (B, T, E), padding_value -1 and no key mask for the transformer variants
    (models.py:216-225); the conformer variant masks keys by ilens (529-531)."""
    ilens = [x.shape[0] for x in src]
    x = torch.nn.utils.rnn.pad_sequence(list(src), padding_value=-1, batch_first=True).float()
    inp, norm, layers = _prefixes(cfg.variant)
    x = F.linear(x, sd[inp + "weight"], sd[inp + "bias"])
    x = F.layer_norm(x, (cfg.n_units,), sd[norm + "weight"], sd[norm + "bias"], 1e-5)
    if cfg.variant in (0, 1):
        x = x.transpose(0, 1)
        for i in range(cfg.n_layers):
            x = transformer_layer(x, sd, f"{layers}{i}.", cfg.n_heads)
        return x.transpose(0, 1), ilens
    return conformer(x, torch.tensor(ilens), sd, "encoder.", num_layers=cfg.n_layers, nh=cfg.n_heads,
                     group_norm=False), ilens


@torch.no_grad()
def attractors(sd, emb_shuffled, ilens, max_n_speakers=15):
    """LstmEncoderDedecoderAttractor.forward (encoder_decoder_attractor.py:42-59)."""
    B = emb_shuffled.shape[0]
    E = emb_shuffled.shape[2]
    _, (h, c) = lstm(emb_shuffled, sd, "eda.encoder.", bidirectional=False, lengths=ilens)
    zeros = torch.zeros(B, max_n_speakers, E)
    att, _ = lstm(zeros, sd, "eda.decoder.", bidirectional=False, h0=h, c0=c)
    probs = torch.sigmoid(F.linear(att, sd["eda.linear.weight"], sd["eda.linear.bias"])[..., 0])
    return att, probs


@torch.no_grad()
def infer_full(sd, cfg, src, perms, max_n_speakers=15):
    """Everything of infer() before speaker selection: returns (act (B,T,max_n-1)
    sigmoid activities, probs (B, max_n)).  perms[i]: the torch.randperm(ilens[i])
    drawn by forward_embedding for batch element i (models.py:229-233)."""
    emb, ilens = embedding(sd, cfg, src)
    sh = emb.clone()
    for i, p in enumerate(perms):
        sh[i, : ilens[i]] = emb[i, torch.as_tensor(p, dtype=torch.long)]
    att, probs = attractors(sd, sh, ilens, max_n_speakers)
    pred = torch.bmm(emb, att[:, :-1, :].permute(0, 2, 1))
    return torch.sigmoid(pred), probs


def select(act, probs, variant, infer_num_speakers=None, attractor_threshold=0.5):
    """Speaker selection of infer() (models.py:334-346 / 639-651), per batch element.
    TransformerEda with infer_num_speakers indexes the 14 columns with the order of
    the 15 probs (IndexError when the last attractor ranks in the top n)."""
    out = []
    for p, y in zip(probs, act):
        if infer_num_speakers is not None:
            if variant == 0:
                order = torch.sort(torch.as_tensor(p), descending=True)[1]
                out.append(y[:, order[:infer_num_speakers]])
            else:
                out.append(y[:, :infer_num_speakers])
        elif attractor_threshold is not None:
            silence = np.where(np.asarray(p) < attractor_threshold)[0]
            n_spk = silence[0] if silence.size else None
            out.append(y[:, :n_spk])
    return out


def chunk_perms(ilens, generator=None):
    """The per-chunk randperm draws in call order (CPU default generator)."""
    return [torch.randperm(n, generator=generator) for n in ilens]
