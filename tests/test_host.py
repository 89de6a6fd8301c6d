"""CPU-side checks: the C-ABI library loads and exports include/sdiar.h, host
logic (window planning, sharding, postprocess) matches the reference semantics."""
import ctypes
import os
import re

import numpy as np
import pytest

from speaker_diarization_amd import _lib
from speaker_diarization_amd.ts_vad import postprocess as pp
from speaker_diarization_amd.ts_vad.windows import plan_windows, shard_batches

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    src = open(os.path.join(REPO, "include", "sdiar.h")).read()
    return sorted(set(re.findall(r"\b(sd_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_lib.EXPORTED)
    assert lib.sd_version() == 1


def test_create_rejects_bad_config_without_gpu():
    cfg = _lib.TsvadConfig(variant=7, max_num_speaker=4, rs_len=4, max_batch=1, max_fbank_frames=398,
                           precision=0, num_transformer_layer=2, num_attention_head=4,
                           transformer_embed_dim=384, transformer_ffn_embed_dim=1536, speaker_embed_dim=192)
    h = ctypes.c_void_p()
    with pytest.raises(ValueError, match="variant"):
        _lib.call("sd_tsvad_create", ctypes.byref(cfg), ctypes.byref(h))


def test_plan_matches_oracle_plan():
    from oracle.pipeline_ref import plan
    for n, rs, sh in [(15000, 6, 1), (15001, 4, 1), (90000, 4, 1), (37, 6, 1), (1000, 4, 2)]:
        p = plan_windows(n, rs, sh)
        assert list(zip(p.starts.tolist(), p.ends.tolist())) == plan(n, rs, sh)
    p = plan_windows(15000, 6, 1)
    assert p.n_win == 600 and p.lens.max() == 150 and p.lens.min() == 25
    assert (p.fbank_n[p.lens == 150] == 598).all()
    assert (p.fbank_start == p.starts * 4).all()


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_shards_partition_on_batch_grid(world):
    p = plan_windows(90000, 4, 1)
    rngs = [shard_batches(p, 64, world, r) for r in range(world)]
    covered = []
    for a, b in rngs:
        assert a % 64 == 0
        covered.extend(range(a, b))
    assert covered == list(range(p.n_win))


def _zeros_to_ones_literal(inputs, min_silence, threshold, frame_len):
    # behaviour of ts_vad2/infer.py:27-47 written as an explicit state machine
    out, run = [], 0
    thr = int(min_silence // frame_len)
    for v in inputs:
        if v >= threshold:
            out += ([0] if run > thr else [1]) * run
            run = 0
            out.append(1)
        else:
            run += 1
    out += ([0] if run > thr else [1]) * run
    return out


def test_postprocess_run_filters():
    rng = np.random.default_rng(0)
    for _ in range(50):
        x = rng.uniform(0, 1, rng.integers(1, 200)).astype(np.float32)
        for thr in (0.3, 0.5):
            assert pp.change_zeros_to_ones(x, 0.32, thr, 0.04) == _zeros_to_ones_literal(x, 0.32, thr, 0.04)
    assert pp.change_zeros_to_ones([1, 0, 0, 1], 0.32, 0.5, 0.04) == [1, 1, 1, 1]
    # 0.32 // 0.04 == 8.0: silences of <= 8 frames are filled, 9 are kept
    assert pp.change_zeros_to_ones([1] + [0] * 8 + [1], 0.32, 0.5, 0.04) == [1] * 10
    assert pp.change_zeros_to_ones([1] + [0] * 9 + [1], 0.32, 0.5, 0.04) == [1] + [0] * 9 + [1]
    assert pp.change_ones_to_zeros([0, 1, 1, 0], 0.0, 0.5, 0.04) == [0, 1, 1, 0]


def test_rttm_segments_format():
    lines = pp.segments_to_rttm("m1", "2", [1, 1, 0, 0, 1, 1, 1], 0.04)
    assert lines[0] == "SPEAKER m1 1 0.000 0.080 <NA> <NA> 2 <NA> <NA>\n"
    # reference convention: after a silence the start is taken at the frame before (infer.py:114)
    assert lines[1] == "SPEAKER m1 1 0.120 0.120 <NA> <NA> 2 <NA> <NA>\n"


def test_host_postprocess_matches_reference_loop():
    """posteriors_to_rttm (host path) == the literal infer.py loop, line for line."""
    from oracle import postprocess_ref
    rng = np.random.default_rng(4)
    for T in (1, 30, 2000):
        x = np.clip(1 / (1 + np.exp(-np.cumsum(rng.normal(0, 0.1, (3, T)), 1))), 0, 1).astype(np.float32)
        x[0, ::7] = np.float32(0.35)   # exactly on a float32 threshold
        post = {f"m{T}-{s}": x[s] for s in range(3)}
        for kw in ({}, dict(min_speech=0.2, med_filter=5)):
            assert pp.posteriors_to_rttm(post, **kw) == postprocess_ref.rttm_lines(post, **kw)
