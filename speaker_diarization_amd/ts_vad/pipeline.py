"""Meeting-level TS-VAD inference on MI355X: wav in HBM -> per-speaker posteriors.

Replaces the loop of ts_vad2/infer.py:216-285 (DataLoader of windows -> fbank on
CPU -> model.infer -> res_dict) with: one fbank pass over the meeting (HIP) ->
per-batch window CMN/pad (HIP) -> TSVADModel forward (HIP) -> window logits
kept in HBM -> sigmoid + overlap average in window order (HIP).  Multi-GPU:
windows are sharded by contiguous batch ranges (one process per GPU); the only
exchange is an all-gather of the per-window logits (RCCL over xGMI).
"""
from __future__ import annotations

import numpy as np

from .. import _lib
from ..frontend import kaldi_fbank, window_cmn
from .model import TSVADModel
from .windows import WindowPlan, plan_windows, shard_batches


_DEV_CACHE = {}


def _plan_i32(plan: WindowPlan, name: str, arr, dev, w0: int = 0, w1: int = None):
    """Device int32 copy of a plan array, cached per (plan, slice, device): a pageable H2D copy per step
    would block the host until the GPU drains the stream and leave the GPU idle while Python re-enqueues."""
    import torch
    key = (plan.n_labels, plan.rs_len, plan.segment_shift, plan.label_rate, plan.sample_rate, name, w0, w1, str(dev))
    t = _DEV_CACHE.get(key)
    if t is None:
        if len(_DEV_CACHE) > 256:
            _DEV_CACHE.clear()
        t = torch.from_numpy(np.ascontiguousarray(arr).astype(np.int32)).to(dev)
        _DEV_CACHE[key] = t
    return t


def _ts_block(ts, dev, NS: int, B: int):
    """(B, NS, E) contiguous copy of the meeting's target-speaker embeddings (every window of a meeting takes the
    same speakers).  Not cached: a cache keyed by the tensor's address served a freed-and-reused allocation's
    stale rows in a later call (tests/test_gpu_shard.py, round 5)."""
    import torch
    return ts.to(dev, torch.float32).reshape(1, NS, -1).expand(B, -1, -1).contiguous()


class TSVADPipeline:
    def __init__(self, model: TSVADModel, segment_shift: int = 1, batch_size: int = 64):
        self.model = model
        self.cfg = model.cfg
        self.segment_shift = segment_shift
        # a model that fixes the reference batch (the streaming decoder: batch 1) overrides it
        batch_size = getattr(model, "reference_batch_size", batch_size)
        self.batch_size = min(batch_size, model.max_batch)
        # a device batch fuses whole reference batches: BatchNorm1D's NaN bypass keeps the reference scope
        self._fwd_kw = {"forward_batch": self.batch_size} if isinstance(model, TSVADModel) else {}

    def plan(self, n_labels: int) -> WindowPlan:
        """The meeting's window plan, built once per label count (the host work between two steps: the
        plan, its fbank counts and the batch grouping are pure functions of n_labels)."""
        cache = self.__dict__.setdefault("_plans", {})
        p = cache.get(n_labels)
        if p is None:
            if len(cache) > 64:
                cache.clear()
            p = cache[n_labels] = plan_windows(n_labels, self.cfg.rs_len, self.segment_shift, self.cfg.label_rate,
                                               self.cfg.sample_rate)
        return p

    def window_logits(self, wav, ts, plan: WindowPlan, w0: int = 0, w1: int = None, out=None, check: bool = True):
        """Logits of windows [w0, w1) -> (w1-w0, NS, chunk) (cols >= window len unused).
        wav: (n_samples,) CUDA float32 covering at least those windows' audio.  check: wait for the stream and
        raise if a persistent recurrence lost co-residency (posteriors() checks once, after its average)."""
        import torch
        dev = self.model.device
        w1 = plan.n_win if w1 is None else w1
        NS, chunk = self.model.max_num_speaker, plan.chunk
        if out is None:
            out = torch.empty(w1 - w0, NS, chunk, device=dev, dtype=torch.float32)
        if w1 <= w0:
            return out
        # every host-side step (plan slices, device tables, the per-batch target-speaker block) comes before the
        # first launch, so the fbank -> window CMN -> forward launches reach the GPU back to back (round 4's
        # trace: 0.59 ms of idle GPU between the fbank and the first window CMN)
        spl = plan.samples_per_label
        s0 = int(plan.starts[w0]) * spl
        s1 = min(wav.numel(), int(plan.ends[w1 - 1]) * spl)
        f0 = int(plan.fbank_start[w0])
        fstart = _plan_i32(plan, "fstart", plan.fbank_start[w0:w1] - f0, dev, w0, w1)
        fn = _plan_i32(plan, "fn", plan.fbank_n[w0:w1], dev, w0, w1)
        batches = self.device_batches(plan, w0, w1)
        ts_all = _ts_block(ts, dev, NS, max(b1 - b0 for b0, b1, _, _ in batches))
        feats = kaldi_fbank(wav[s0:s1])
        for b0, b1, T_out, T_lab in batches:
            ref = window_cmn(feats, fstart[b0 - w0:b1 - w0], fn[b0 - w0:b1 - w0], T_out)
            dst = out[b0 - w0:b1 - w0]
            if T_lab == chunk:           # whole rows: the forward writes straight into the output
                self.model.forward(ref, ts_all[: b1 - b0], T_lab, out=dst, check=False, **self._fwd_kw)
            else:
                dst[:, :, :T_lab] = self.model.forward(ref, ts_all[: b1 - b0], T_lab, check=False, **self._fwd_kw)
                dst[:, :, T_lab:] = 0.0
        if check:
            self._check()
        return out

    def _check(self):
        status = getattr(self.model, "status", None)
        if status is not None:
            status()          # one wait per call: a lost LSTM co-residency raises here

    def device_batches(self, plan: WindowPlan, w0: int, w1: int):
        """Reference batches (batch_size windows, zero-padded to their own max length,
        ts_vad_dataset.py:664-701) of [w0, w1); consecutive batches with the same
        padded shape are fused into one device launch of up to model.max_batch
        windows — identical inputs per window, fewer and larger kernels."""
        key = ("_batches", self.batch_size, self.model.max_batch, w0, w1)
        hit = plan.__dict__.get(key)
        if hit is not None:
            return list(hit)
        groups = []
        for b0 in range(w0, w1, self.batch_size):
            b1 = min(w1, b0 + self.batch_size)
            key = (int(plan.fbank_n[b0:b1].max()), int(plan.lens[b0:b1].max()))
            if groups and groups[-1][2:] == key and b1 - groups[-1][0] <= self.model.max_batch:
                groups[-1] = (groups[-1][0], b1) + key
            else:
                groups.append((b0, b1) + key)
        plan.__dict__[("_batches", self.batch_size, self.model.max_batch, w0, w1)] = tuple(groups)
        return groups

    @staticmethod
    def mean_probs(probs, plan: WindowPlan):
        """(n_win, NS, chunk) probabilities -> (NS, n_labels): infer.py:90-94's np.mean over each
        frame's list of window values, bit-identical (sd_overlap_mean)."""
        import torch
        dev = probs.device
        NS = probs.shape[1]
        out = torch.empty(NS, plan.n_labels, device=dev, dtype=torch.float32)
        st = _plan_i32(plan, "starts", plan.starts, dev)
        ln = _plan_i32(plan, "lens", plan.lens, dev)
        _lib.call("sd_overlap_mean", _lib.ptr(probs.contiguous()), plan.n_win, NS, probs.shape[2],
                  _lib.ptr(st), _lib.ptr(ln), plan.dis, plan.chunk, plan.n_labels, _lib.ptr(out),
                  _lib.stream_ptr(dev))
        return out

    @staticmethod
    def average(logits, plan: WindowPlan):
        """(n_win, NS, chunk) logits -> (NS, n_labels) posteriors (sigmoid + overlap mean)."""
        import torch
        dev = logits.device
        NS = logits.shape[1]
        out = torch.empty(NS, plan.n_labels, device=dev, dtype=torch.float32)
        st = _plan_i32(plan, "starts", plan.starts, dev)
        ln = _plan_i32(plan, "lens", plan.lens, dev)
        _lib.call("sd_overlap_average", _lib.ptr(logits.contiguous()), plan.n_win, NS, logits.shape[2],
                  _lib.ptr(st), _lib.ptr(ln), plan.dis, plan.chunk, plan.n_labels, _lib.ptr(out),
                  _lib.stream_ptr(dev))
        return out

    def posteriors(self, wav, ts, n_labels: int = None, group=None):
        """wav: (n_samples,) CUDA float32 in [-1,1); ts: (NS, 192) target-speaker
        embeddings (zeros for absent speakers, ts_vad_dataset.py:507-510).
        Returns (NS, n_labels) frame posteriors at 25 Hz."""
        import torch
        import torch.distributed as dist
        spl = self.cfg.sample_rate // self.cfg.label_rate
        if n_labels is None:
            n_labels = wav.numel() // spl
        plan = self.plan(n_labels)
        world = dist.get_world_size(group) if (group is not None or dist.is_initialized()) else 1
        if world == 1:
            post = self.average(self.window_logits(wav, ts, plan, check=False), plan)
            self._check()      # after the average is enqueued: no idle GPU between the forward and it
            return post
        rank = dist.get_rank(group)
        w0, w1 = shard_batches(plan, self.batch_size, world, rank)
        local = self.window_logits(wav, ts, plan, w0, w1)
        logits = gather_windows(local, plan, self.batch_size, world, group)
        return self.average(logits, plan)


def gather_windows(local, plan: WindowPlan, batch_size: int, world: int, group=None):
    """All-gather of per-rank window logits (RCCL over xGMI); re-assembled in
    global window order from the deterministic shard table."""
    import torch
    import torch.distributed as dist
    ranges = [shard_batches(plan, batch_size, world, r) for r in range(world)]
    maxn = max(b - a for a, b in ranges)
    pad = torch.zeros(maxn, *local.shape[1:], device=local.device, dtype=local.dtype)
    pad[: local.shape[0]] = local
    if local.is_cuda and dist.get_backend(group) == "gloo":
        # gloo gathers host tensors: stage through host memory (RCCL, the multi-GPU backend, gathers in HBM)
        allg = torch.empty(world * maxn, *local.shape[1:], dtype=local.dtype)
        dist.all_gather_into_tensor(allg, pad.cpu(), group=group)
        allg = allg.to(local.device)
    else:
        allg = torch.empty(world * maxn, *local.shape[1:], device=local.device, dtype=local.dtype)
        dist.all_gather_into_tensor(allg, pad, group=group)
    parts = [allg[r * maxn: r * maxn + (b - a)] for r, (a, b) in enumerate(ranges)]
    return torch.cat(parts, 0)
