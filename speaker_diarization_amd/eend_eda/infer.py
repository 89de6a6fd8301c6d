"""Recording-level EEND-EDA inference — eend_eda/infer_eda.py:92-124 on MI355X.

Reference loop per recording: features on the CPU (librosa), then one
model.infer([chunk]) per 2000-frame chunk, sequentially, each drawing one
torch.randperm.  Here: the features of the whole recording are computed on the
GPU in one pass, the permutations are drawn on the host in chunk order (the
same CPU-generator stream the reference consumes), and all equal-length chunks
run as one batched device forward (chunks are independent: no state crosses
chunk boundaries, infer_eda.py:99-113).  Multi-GPU: every rank computes the
cheap frontend over the whole recording (the per-recording mean needs all
frames), forwards its contiguous share of the chunks, and the activities are
all-gathered (RCCL over xGMI).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from ..feature import eend_features, get_input_dim


@dataclass
class EdaInferArgs:
    """infer.py argument defaults (eend_eda/infer.py:11-45) for the C1/C3 recipes."""
    num_speakers: Optional[int] = 2
    input_transform: str = "logmel23_mn"
    label_delay: int = 0
    chunk_size: int = 2000
    context_size: int = 7
    subsampling: int = 10
    sampling_rate: int = 16000
    frame_size: int = 400
    frame_shift: int = 160
    attractor_threshold: float = 0.5
    max_n_speakers: int = 15


def gen_chunk_indices(data_len: int, chunk_size: int):
    """infer_eda.py:21-28."""
    start = 0
    while start < data_len:
        yield start, min(data_len, start + chunk_size)
        start += chunk_size


def chunk_groups(chunks, max_seqs: int):
    """Consecutive equal-length chunks batched up to max_seqs per device forward."""
    groups = []
    for i, (s, e) in enumerate(chunks):
        if groups and groups[-1][2] == e - s and i - groups[-1][0] < max_seqs:
            groups[-1][1] = i + 1
        else:
            groups.append([i, i + 1, e - s])
    return [tuple(g) for g in groups]


def shard_chunks(n_chunks: int, world: int, rank: int):
    per, rem = divmod(n_chunks, world)
    c0 = rank * per + min(rank, rem)
    return c0, c0 + per + (1 if rank < rem else 0)


def recording_features(model, wav, args: EdaInferArgs):
    if get_input_dim(args.frame_size, args.context_size, args.input_transform) != model.cfg.in_size:
        raise RuntimeError("feature dimension does not match the model in_size")
    return eend_features(wav, args.sampling_rate, args.frame_size, args.frame_shift, args.input_transform,
                         args.context_size, args.subsampling, ld=model.in_ld)


def chunk_activities(model, feats, args: EdaInferArgs, perms, c0: int = 0, c1: Optional[int] = None):
    """Device forward of chunks [c0, c1): returns (list of (act (T_c, n_att-1) CUDA),
    probs (n, n_att) CPU)."""
    import torch
    chunks = list(gen_chunk_indices(feats.shape[0], args.chunk_size))
    c1 = len(chunks) if c1 is None else c1
    acts, probs = [], []
    sub = chunks[c0:c1]
    for g0, g1, T in chunk_groups(sub, model.max_seqs):
        s0 = sub[g0][0]
        x = feats[s0: s0 + (g1 - g0) * T].view(g1 - g0, T, feats.shape[1])
        key_len = [T] * (g1 - g0) if model.cfg.variant == 2 else None
        a, p = model.forward_infer(x, [T] * (g1 - g0), perms[c0 + g0: c0 + g1], args.max_n_speakers,
                                   key_len=key_len, check=False)
        acts.extend(a[i] for i in range(g1 - g0))
        probs.append(p)
    if sub:
        model.status()        # one wait for every group: a lost LSTM co-residency raises here
    return acts, (torch.cat(probs).cpu() if probs else torch.zeros(0, args.max_n_speakers))


def chunk_outputs(model, wav, args: EdaInferArgs = EdaInferArgs(), group=None):
    """Device half of infer_eda.py:99-113: features, every chunk's forward (one randperm draw
    per chunk, in order) and, with N ranks, the all-gather.  Returns (acts, probs, lens):
    per-chunk (T_c, max_n - 1) CUDA activities, (n_chunks, max_n) CPU attractor probs."""
    import torch
    import torch.distributed as dist

    feats = recording_features(model, wav, args)
    chunks = list(gen_chunk_indices(feats.shape[0], args.chunk_size))
    perms = [torch.randperm(e - s) for s, e in chunks]          # one draw per chunk, in order
    world = dist.get_world_size(group) if (group is not None or dist.is_initialized()) else 1
    if world == 1:
        acts, probs = chunk_activities(model, feats, args, perms)
    else:
        rank = dist.get_rank(group)
        c0, c1 = shard_chunks(len(chunks), world, rank)
        local, lprobs = chunk_activities(model, feats, args, perms, c0, c1)
        acts, probs = gather_chunks(local, lprobs, chunks, args, world, group, device=feats.device)
    return acts, probs, [e - s for s, e in chunks]


def select_chunks(model, acts, probs, lens, args: EdaInferArgs = EdaInferArgs()) -> List[np.ndarray]:
    """Host half: model.infer's speaker selection per chunk (models.py:334-346 / 639-651,
    including TransformerEda's IndexError quirk) -> out_chunks."""
    out_chunks = []
    for c, a in enumerate(acts):
        y = model.select(a[None], probs[c: c + 1], [lens[c]], args.num_speakers, args.attractor_threshold)[0]
        out_chunks.append(y.cpu().numpy())
    return out_chunks


def infer_chunks(model, wav, args: EdaInferArgs = EdaInferArgs(), group=None) -> List[np.ndarray]:
    """The per-chunk loop of infer_eda.py:99-113: wav (1-D float32 CUDA tensor) ->
    out_chunks, one (T_c, n_spk) float32 array per 2000-frame chunk, in chunk order."""
    acts, probs, lens = chunk_outputs(model, wav, args, group)
    return select_chunks(model, acts, probs, lens, args)


def stitch(out_chunks: List[np.ndarray], args: EdaInferArgs = EdaInferArgs()) -> np.ndarray:
    """infer_eda.py:115-121: np.vstack of the chunk outputs (raises ValueError, as the
    reference does, when threshold-mode chunks selected different speaker counts), then
    the label-delay shift."""
    from scipy.ndimage import shift
    outdata = np.vstack(out_chunks)
    if args.label_delay != 0:
        outdata = shift(outdata, (-args.label_delay, 0))
    return outdata


def infer_recording(model, wav, args: EdaInferArgs = EdaInferArgs(), group=None) -> np.ndarray:
    """wav: 1-D float32 CUDA tensor -> T_hat (T, n_spk) float32, the array infer_eda.py
    writes to <recid>.h5 (:115-124)."""
    return stitch(infer_chunks(model, wav, args, group), args)


def gather_chunks(local: List, lprobs, chunks, args: EdaInferArgs, world: int, group=None, device=None):
    """All-gather of per-chunk activities + attractor probabilities in chunk order.
    `device` is where the gather buffer lives (the rank's GPU; a rank may own no chunk
    when world > n_chunks, so it cannot be taken from `local`)."""
    import torch
    import torch.distributed as dist
    if device is None:
        device = local[0].device if local else torch.device("cuda", torch.cuda.current_device())
    dev = torch.device(device)
    na = args.max_n_speakers
    ranges = [shard_chunks(len(chunks), world, r) for r in range(world)]
    maxn = max(b - a for a, b in ranges)
    T = args.chunk_size
    buf = torch.zeros(maxn, T, na - 1 + 1, device=dev, dtype=torch.float32)
    for i, a in enumerate(local):
        buf[i, : a.shape[0], : na - 1] = a
        buf[i, :na, na - 1] = lprobs[i].to(dev)      # probs ride in the spare column
    allg = torch.empty(world * maxn, T, na, device=dev, dtype=torch.float32)
    dist.all_gather_into_tensor(allg, buf, group=group)
    acts, probs = [], []
    for r, (a, b) in enumerate(ranges):
        for i in range(b - a):
            c = a + i
            n = chunks[c][1] - chunks[c][0]
            acts.append(allg[r * maxn + i, :n, : na - 1])
            probs.append(allg[r * maxn + i, :na, na - 1].cpu())
    return acts, torch.stack(probs)
