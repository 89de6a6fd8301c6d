"""Goldens captured from the reference's own TS-VAD output stage (run here only).

1. ``postprocess_*.npz`` — ``egs/alimeeting/ts_vad2/infer.py`` ``postprocess(res_dict, args)``
   (:72-163) imported from /root/reference with stubs for lhotse / tqdm / tensorboard
   (SURVEY Appendix A), run on seeded res_dicts: per-frame lists of float32 window
   probabilities (1-6 values, so the np.mean of :90-94 is exercised; ``postprocess_win12``: the
   lists a 12-s window / 1-s shift plan builds, 1-12 values per frame in window order, so numpy's
   8-accumulator pairwise summation inside np.mean is exercised too), values placed exactly
   on the float32 thresholds, 1-frame speech runs, silences of exactly min_silence // frame_len
   frames, tracks starting with speech, tracks of 1 and 22 frames (below / at the medfilt
   width) and two meetings.  Stored: the res_dict (flattened), the ten ``res_rttm_<thr>``
   files byte for byte and the ``der_result`` lines md-eval.pl printed against a reference
   RTTM written from the same seeds.
2. ``tsvad_infer.npz`` — ``egs/alimeeting/ts_vad2/model.py`` ``TSVADModel.infer`` (:923-970)
   on a batch of windows with partial lengths and absent speakers: the result dict (loss, DER,
   ACC, MI, FA, CF) and the res_dict, for the CAM++/transformer model with seeded weights.

    python tests/golden/make_postprocess_golden.py     (needs /root/reference and perl)
"""
import argparse
import os
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import REF, REPO, _stub, install_stubs, tsvad_inputs  # noqa: E402

TS_DIR = os.path.join(REF, "egs/alimeeting/ts_vad2")
SCTK = os.path.join(REF, "egs/alimeeting/SCTK-2.4.12")
THRESHOLDS = (0.2, 0.3, 0.35, 0.4, 0.45, 0.5, 0.55, 0.6, 0.7, 0.8)

# name: (seed, meetings, speakers, frames per meeting, windows covering a frame (max))
POSTPROCESS_CASES = {
    "postprocess_smooth": (11, 2, 4, 1500, 6),
    "postprocess_edges": (12, 1, 3, 400, 4),
    "postprocess_tiny": (13, 2, 2, 22, 3),
    "postprocess_win12": (14, 1, 4, 1500, 12),      # window layout: rs_len 12 s, shift 1 s
}
WINDOW_CASES = {"postprocess_win12": (12, 1)}        # name: (rs_len s, segment_shift s)


def _import_infer():
    import torch  # noqa: F401
    install_stubs()
    for n in ("lhotse", "lhotse.dataset", "lhotse.dataset.sampling"):
        _stub(n)
    _stub("lhotse.dataset.sampling.base", CutSampler=object)
    _stub("tqdm", tqdm=lambda x, **k: x)
    import torch.utils
    tb = _stub("torch.utils.tensorboard", SummaryWriter=object)
    torch.utils.tensorboard = tb
    sys.path.insert(0, TS_DIR)
    for mod in ("infer", "model", "checkpoint", "utils", "build_datasets", "ts_vad_dataset"):
        sys.modules.pop(mod, None)
    import infer as ref_infer
    return ref_infer


def _track(rng, T, kind, w_max):
    """Per-frame lists of float32 probabilities for one (meeting, speaker) track."""
    if kind == "smooth":
        x = np.cumsum(rng.standard_normal(T)) * 0.25
        p = 1 / (1 + np.exp(-(x - x.mean())))
    else:
        p = rng.random(T)
        # exact float32 threshold values, 1-frame runs, silences of 6/7/8/9 frames
        for thr in THRESHOLDS:
            p[rng.integers(0, T, size=max(1, T // 40))] = np.float32(thr)
        for _ in range(max(1, T // 60)):
            s = int(rng.integers(0, max(1, T - 12)))
            n = int(rng.integers(6, 10))
            p[s:s + n] = 0.05
            if s + n < T:
                p[s + n] = 0.95
    lists = []
    for t in range(T):
        k = int(rng.integers(1, w_max + 1))
        base = np.float32(p[t])
        vals = [base] + [np.float32(np.clip(base + rng.normal(0, 0.02), 0, 1)) for _ in range(k - 1)]
        lists.append([np.float32(v) for v in vals])
    return lists


def window_probs(name):
    """(n_win, NS, chunk) float32 window probabilities + window starts/lens of a WINDOW_CASES
    plan (ts_vad_dataset.py:242-271 at inference: windows every shift, partial tails kept)."""
    seed, n_meet, n_spk, T, _ = POSTPROCESS_CASES[name]
    rs, shift = WINDOW_CASES[name]
    chunk, dis = 25 * rs, 25 * shift
    starts = np.arange(0, T, dis)
    ends = np.minimum(starts + chunk, T)
    rng = np.random.default_rng(seed)
    base = np.stack([1 / (1 + np.exp(-np.cumsum(rng.standard_normal(T)) * 0.25)) for _ in range(n_spk)])
    probs = np.zeros((len(starts), n_spk, chunk), np.float32)
    for w, (s0, e0) in enumerate(zip(starts, ends)):
        probs[w, :, : e0 - s0] = np.clip(base[:, s0:e0] + rng.normal(0, 0.05, (n_spk, e0 - s0)), 0, 1)
    return probs, starts.astype(np.int64), (ends - starts).astype(np.int64)


def make_res_dict(name):
    seed, n_meet, n_spk, T, w_max = POSTPROCESS_CASES[name]
    if name in WINDOW_CASES:        # what TSVADModel.infer appends, window by window (model.py:960-966)
        probs, starts, lens = window_probs(name)
        res = {f"R00_M00-{s}": [[] for _ in range(T)] for s in range(1, n_spk + 1)}
        for w in range(len(starts)):
            for t in range(int(lens[w])):
                for i in range(n_spk):
                    res[f"R00_M00-{i + 1}"][int(starts[w]) + t].append(np.float32(probs[w, i, t]))
        return res
    rng = np.random.default_rng(seed)
    kind = "smooth" if name.endswith("smooth") else "edges"
    res = {}
    for m in range(n_meet):
        for s in range(1, n_spk + 1):
            res[f"R{m:02d}_M{m:02d}-{s}"] = _track(rng, T + 7 * m, kind, w_max)
    return res


def ref_rttm(res, seed):
    """A reference RTTM over the same recordings (random turns), for md-eval."""
    rng = np.random.default_rng(seed + 100)
    lines = []
    for key in sorted(res):
        name, spk = key.rsplit("-", 1)
        T = len(res[key]) * 0.04
        t = 0.0
        while t < T:
            d = float(rng.uniform(0.5, 4.0))
            if rng.random() < 0.5:
                lines.append(f"SPEAKER {name} 1 {t:.2f} {min(d, T - t):.2f} <NA> <NA> {spk} <NA> <NA>\n")
            t += d
    return lines


def run_postprocess(name, ref_infer):
    from collections import defaultdict
    res = make_res_dict(name)
    seed = POSTPROCESS_CASES[name][0]
    tmp = tempfile.mkdtemp(prefix="sdiar_pp_")
    try:
        rttm_dir = os.path.join(tmp, "ref")
        os.makedirs(rttm_dir)
        with open(os.path.join(rttm_dir, "ref.rttm"), "w") as f:
            f.writelines(ref_rttm(res, seed))
        res_dict = defaultdict(lambda: defaultdict(list))
        for key, lists in res.items():
            for t, vals in enumerate(lists):
                res_dict[key][t] = list(vals)
        args = argparse.Namespace(results_path=tmp, split="Eval", label_rate=25, rttm_name="ref.rttm",
                                  med_filter=21, min_silence=0.32, min_speech=0.0, sctk_tool_path=SCTK,
                                  collar=0.25, rttm_dir=rttm_dir)
        import contextlib
        import io
        with contextlib.redirect_stdout(io.StringIO()):
            ref_infer.postprocess(res_dict, args)
        eval_dir = os.path.join(tmp, "Eval")
        rttms = [open(os.path.join(eval_dir, f"res_rttm_{thr}")).read() for thr in THRESHOLDS]
        der = open(os.path.join(eval_dir, "der_result")).read()
        ref_lines = open(os.path.join(rttm_dir, "ref.rttm")).read()
    finally:
        shutil.rmtree(tmp)
    keys = sorted(res)
    counts = [np.array([len(v) for v in res[k]], np.int64) for k in keys]
    vals = [np.array([x for v in res[k] for x in v], np.float32) for k in keys]
    out = dict(keys=np.array(keys), thresholds=np.array(THRESHOLDS), rttm=np.array(rttms), der_result=np.array(der),
               ref_rttm=np.array(ref_lines), key_order=np.array(list(res)))
    for i in range(len(keys)):
        out[f"counts_{i}"] = counts[i]
        out[f"values_{i}"] = vals[i]
        # np.mean of every frame's list: the function infer.py:93 calls, on the same lists
        out[f"means_{i}"] = np.array([np.mean(v) for v in res[keys[i]]], np.float32)
    if name in WINDOW_CASES:
        out["win_probs"], out["win_starts"], out["win_lens"] = window_probs(name)
        out["win_geometry"] = np.array(WINDOW_CASES[name], np.int64)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
    print(name, len(keys), "tracks", [len(r.splitlines()) for r in rttms], "RTTM lines")


def load_res_dict(npz):
    """tests: the res_dict stored by run_postprocess -> {key: [[float32, ...] per frame]}."""
    g = np.load(npz)
    res = {}
    for i, k in enumerate(g["keys"]):
        c, v = g[f"counts_{i}"], g[f"values_{i}"]
        off = np.concatenate([[0], np.cumsum(c)])
        res[str(k)] = [list(v[off[t]:off[t + 1]]) for t in range(len(c))]
    order = [str(k) for k in g["key_order"]]
    return {k: res[k] for k in order}


# ----------------------------------------------------------------------------- TSVADModel.infer
INFER_CASE = dict(B=4, T_fb=398, n_lab=100, lens=[100, 100, 63, 17], spk=[[1, 2, 3, 4], [1, 2, 3, 4],
                  [1, 2, -1, -1], [1, 2, 3, -1]], starts=[0, 25, 50, 75], files=["R0001_M0001", "R0001_M0001",
                  "R0001_M0001", "R0002_M0002"], iseed=2024, wseed=780, lseed=2025)


def infer_labels():
    c = INFER_CASE
    rng = np.random.default_rng(c["lseed"])
    lab = (rng.random((c["B"], 4, c["n_lab"])) < 0.35).astype(np.float32)
    for b, ids in enumerate(c["spk"]):
        for i, s in enumerate(ids):
            if s < 0:
                lab[b, i] = 0
        lab[b, :, c["lens"][b]:] = 0
    return lab


def make_infer():
    import torch
    from speaker_diarization_amd.weights import TSVADConfig, tsvad_state_dict, to_torch
    c = INFER_CASE
    install_stubs()
    sys.path.insert(0, TS_DIR)
    for mod in ("model", "cam_pplus_wespeaker", "build_datasets", "ts_vad_dataset"):
        sys.modules.pop(mod, None)
    import model as ref_model
    ref_model.TSVADModel.load_speaker_encoder = lambda self, *a, **k: None
    dcfg = ref_model.TSVADDataConfig()
    dcfg.rs_len = 4
    torch.manual_seed(0)
    m = ref_model.TSVADModel(cfg=ref_model.TSVADConfig(), task_cfg=dcfg)
    m.eval()
    m.load_state_dict(to_torch(tsvad_state_dict(TSVADConfig(rs_len=4), seed=c["wseed"])), strict=True)
    x, ts = tsvad_inputs(c["B"], c["T_fb"], c["n_lab"], seed=c["iseed"])
    labels = torch.from_numpy(infer_labels())
    lens = torch.tensor(c["lens"])
    with torch.no_grad():
        result, res_dict = m.infer(torch.from_numpy(x), torch.from_numpy(ts), labels, lens, file_path=c["files"],
                                   speaker_ids=c["spk"], start=c["starts"])
    keys = list(res_dict)
    out = dict(keys=np.array(keys), loss=np.float64(float(result["losses"]["diar"])),
               metrics=np.array([result[k] for k in ("DER", "ACC", "MI", "FA", "CF")], np.float64))
    for i, k in enumerate(keys):
        frames = sorted(res_dict[k])
        out[f"frames_{i}"] = np.array(frames, np.int64)
        out[f"counts_{i}"] = np.array([len(res_dict[k][t]) for t in frames], np.int64)
        out[f"values_{i}"] = np.array([v for t in frames for v in res_dict[k][t]], np.float32)
        # insertion order of the frames (dict order is part of the surface postprocess sorts)
        out[f"order_{i}"] = np.array(list(res_dict[k]), np.int64)
    np.savez_compressed(os.path.join(HERE, "tsvad_infer.npz"), **out)
    print("tsvad_infer", keys, out["metrics"], out["loss"])
    sys.path.remove(TS_DIR)


if __name__ == "__main__":
    import torch
    torch.set_num_threads(8)
    names = sys.argv[1:] or (list(POSTPROCESS_CASES) + ["tsvad_infer"])
    ref_infer = None
    for n in names:
        if n == "tsvad_infer":
            make_infer()
        else:
            ref_infer = ref_infer or _import_infer()
            run_postprocess(n, ref_infer)
