#!/usr/bin/env python3
"""Diarized frames/sec (10 ms hop) of the MI355X TS-VAD path — BASELINE.json metric.

Default workload (N=1): config C2 — AliMeeting-shaped 10-min 4-speaker meeting
(synthetic 16 kHz audio, seeded random weights of the reference architecture),
TS-VAD CAM++_ots_vad + 6-layer Conformer + BiLSTM (ots_vad_style v1), rs_len 6 s,
segment_shift 1 s, 64 windows per batch, bf16 MFMA.  One step = the whole hot
path over one meeting: wav already in HBM -> kaldi fbank -> window CMN -> model
-> sigmoid + overlap-average posteriors (NS, 25 Hz frames).

N GPUs (`--gpus N`: bench.py starts N ranks itself, or runs under the driver's
torchrun; one process per GPU, RCCL): BASELINE C4 — one fixed 60-min 4-speaker
meeting, TS-VAD CAM++ + transformer, rs_len 4 — as STRONG scaling: its windows are
sharded by contiguous ranges of the global 64-window batch grid, each rank runs the
sub-span fbank + its windows, and the per-window logits are all-gathered (the only
exchange) before the ordered overlap average.  The N=1 line carries the same
meeting's 1-GPU time (`c4_60min_ms`), so every point of the series reads against
one workload.  `--workload c2 --gpus N` runs the headline model on that meeting;
`--scaling weak` gives N x 10-min meetings.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import statistics
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

WORKLOADS = {
    "c2": dict(variant=1, rs_len=6, minutes=10.0, desc="C2: AliMeeting-shaped 4-spk meeting, TS-VAD "
               "CAM++_ots_vad + 6-layer Conformer + BiLSTM (ots_vad_style v1), rs_len 6 s, shift 1 s"),
    "c4": dict(variant=0, rs_len=4, minutes=60.0, strong=True,
               desc="C4: 4-spk long-form meeting, TS-VAD CAM++ + transformer (default TSVADConfig), "
                    "rs_len 4 s, shift 1 s"),
    # secondary workloads (EEND family); not the BASELINE headline line
    "c1": dict(kind="eda", model_type="TransformerEda", layers=2, n_spk=2, minutes=10.0, num_speakers=2,
               desc="C1: 2-spk 16 kHz recording, EEND-EDA TransformerEda 2-layer (infer_eda.py: logmel23_mn, "
                    "context 7, subsampling 10, 2000-frame chunks), num_speakers 2"),
    "c3": dict(kind="eda", model_type="EendEda", layers=4, n_spk=4, minutes=10.0, num_speakers=None,
               desc="C3: 4-spk 16 kHz recording, EEND-EDA EendEda 4-layer transformer, attractor-threshold "
                    "speaker counting"),
    "c5": dict(kind="fseend", n_spk=3, minutes=10.0,
               desc="C5: 8 kHz recording, FS-EEND (4-layer causal encoder, shared 2x fusion decoder, "
                    "logmel23, 100 ms frames), whole recording per test() call; replicas only"),
    "emb": dict(kind="embed", n_spk=4, minutes=10.0,
                desc="Target-speaker embeddings: CAM++ (CAMPPLUS_COMMON, 192-d) over 4 speakers' enrollment "
                     "audio (2.5 min each, 16 kHz), extract_embed 6 s chunks every 1 s, batch 96 "
                     "(generate_chunk_speaker_embedding_from_modelscope_for_diarization.py); replicas only"),
    "tss": dict(kind="tsvad_stream", n_spk=4, minutes=10.0, chunk=25, left=-1,
                desc="Chunk-streaming TS-VAD (ts_vad2_streaming, run_ts_vad2_streaming.sh decode: rs_len 10 s, "
                     "segment_shift 1 s, decoding_chunk_size 25 (1 s), num_decoding_left_chunks -1, "
                     "simulate_streaming), 4 speakers, every window decoded at its own length, 256 windows "
                     "per device call; replicas only"),
    "c5s": dict(kind="fseend_stream", n_spk=3, minutes=10.0, chunk=1,
                desc="C5 latency mode: FS-EEND fed 8 kHz audio in 80 ms pushes (640 samples); each model frame "
                     "(100 ms) runs its STFT/logmel/splice and the causal encoder as one captured hipGraph, "
                     "per-layer K/V histories, scores final 9 frames later; host waits for every push; "
                     "replicas only"),
}

# dense TFLOP/s (MI355X_MICROARCH.md); bf16x3 = the bf16 peak over its 3 MFMAs per fp32-equivalent product
PEAKS = {"bf16": 2500.0, "f32": 157.3, "bf16x3": 2500.0 / 3}
HBM_PEAK = 8000.0                        # GB/s
ATTN_KERNELS = ("mha_block", "attention_bf16", "attention_bf16x3", "attention_f32")   # fused block first (C2)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one process per GPU); without an external launcher bench.py starts them itself")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default=None, choices=sorted(WORKLOADS) + ["dist_check"],
                    help="default: c2 on one GPU, c4 (the 60-min strong-scaling meeting) on N > 1; "
                         "dist_check = CPU/gloo launcher self-test (no GPU)")
    ap.add_argument("--no-c4-ref", action="store_true",
                    help="N=1 C2 line: skip the 1-GPU time of the C4 60-min meeting the N>1 lines run")
    ap.add_argument("--minutes", type=float, default=None,
                    help="weak scaling: meeting minutes per GPU; strong scaling: total meeting minutes")
    ap.add_argument("--scaling", default=None, choices=["weak", "strong"],
                    help="default: strong (fixed 60-min meeting) when WORLD_SIZE > 1, else one 10-min meeting")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32", "bf16x3"])
    ap.add_argument("--batch", type=int, default=64, help="reference batch (windows, zero-pad unit)")
    ap.add_argument("--device-batch", type=int, default=640, help="windows per device launch (a 10-min meeting in one launch)")
    ap.add_argument("--cpu-seconds", type=float, default=24.0, help="CPU-baseline budget (3 timed runs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--chunk", type=int, default=None, help="c5s: model frames per streaming push")
    ap.add_argument("--no-graph", action="store_true", help="c5s: direct launches instead of hipGraph replay")
    ap.add_argument("--feature-rows", action="store_true", help="c5s: push precomputed feature rows (model only)")
    ap.add_argument("--push-samples", type=int, default=640, help="c5s: audio samples per push (640 = 80 ms)")
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------- host facts
def _cgroup_cpus():
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, int(int(q) / int(p)))
    except Exception:
        return None


def host_threads():
    """Threads for the CPU baseline: every host core this process may use (BASELINE.md §2:
    os.cpu_count()), capped by the cgroup CPU quota and OMP_NUM_THREADS (the GPU box
    grants one GPU's job a 16-CPU share of a much larger machine)."""
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except Exception:
        pass
    cg = _cgroup_cpus()
    if cg:
        n = min(n, cg)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return n


def host_info(threads):
    model = platform.processor() or ""
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for ln in out.splitlines():
            if ln.startswith("Model name:"):
                model = ln.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    try:
        nproc = int(subprocess.run(["nproc"], capture_output=True, text=True, timeout=10).stdout.strip())
    except Exception:
        nproc = None
    return {"cores": threads, "nproc": nproc, "os_cpu_count": os.cpu_count(), "cgroup_cpus": _cgroup_cpus(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "cpu_model": model}


def median3(fn):
    """one warm-up run (done by the caller), then the median of 3."""
    ts = []
    out = None
    for _ in range(3):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts), ts, out


# ----------------------------------------------------------------------------- rooflines
def roofline_of(name, st, traffic=None):
    """Roofline of one kernel from the live HIP-event timer: the bound is the roof the
    kernel's algorithmic work sits closer to (max(flops/peak_flops,
    bytes/peak_bw) over the measured time), and `achieved` is quoted in that roof's unit."""
    secs = st["ms"] * 1e-3
    # f32 MFMA peak for exact-f32 kernels; the bf16 peak / 3 for bf16x3 kernels (their flops are the fp32
    # products; each costs three bf16 MFMA products); else bf16
    dt = "f32" if name.endswith("f32") else "bf16x3" if name.endswith("bf16x3") else "bf16"
    tf = st["flops"] / secs / 1e12 if st["flops"] > 0 else 0.0
    gbs = st["bytes"] / secs / 1e9
    f_mfma, f_hbm = tf / PEAKS[dt], gbs / HBM_PEAK
    common = dict(traffic=traffic, kernel=name, launches=st["launches"],
                  avg_launch_ms=round(st["ms"] / st["launches"], 4),
                  flops_per_launch=st["flops"] / st["launches"],
                  algorithmic_bytes_per_launch=round(st["bytes"] / st["launches"]),
                  mfma_frac=round(f_mfma, 4), hbm_frac=round(f_hbm, 4))
    if f_mfma >= f_hbm:
        return dict(bound="mfma", achieved=round(tf, 2), peak=PEAKS[dt], unit="TFLOP/s", frac=round(f_mfma, 4),
                    **common)
    return dict(bound="hbm", achieved=round(gbs, 1), peak=HBM_PEAK, unit="GB/s", frac=round(f_hbm, 4), **common)


def pmc_traffic(workload, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py), or None."""
    pmc = os.path.join(HERE, "profiles", "pmc_traffic.json")
    if not os.path.exists(pmc):
        return None
    try:
        return json.load(open(pmc)).get(workload, {}).get(kernel)
    except (OSError, ValueError):
        return None


def live_kernels(step):
    """One extra step under the libsdiar HIP-event timer (events on the launch stream)."""
    import torch
    from speaker_diarization_amd import _lib
    lib = _lib.load()
    lib.sd_prof_reset()
    lib.sd_prof_enable(1)
    step()
    torch.cuda.synchronize()
    lib.sd_prof_enable(0)
    kernels = _lib.prof_stats()
    lib.sd_prof_reset()
    return kernels


def lstm_handoff_floor_us(steps=4000, probe="sd_probe_lstm_handoff"):
    """Measured exchange floor of the persistent LSTM recurrence: sd_probe_lstm_handoff runs the
    recurrence's own 4-workgroup hand-off protocol (poll, h-fragment loads, publish) with no gate
    arithmetic; sd_probe_lstm_granule the same exchange on the guide's data-tagged 8-byte granules
    (the hardware's hand-off price); us per step (median of 3 launches)."""
    import ctypes
    import torch
    from speaker_diarization_amd import _lib
    v = ctypes.c_float()
    runs = []
    for _ in range(3):
        _lib.call(probe, steps, ctypes.byref(v), _lib.stream_ptr())
        runs.append(v.value)
    torch.cuda.synchronize()
    return float(np.median(runs))


def latency_roofline_of(name, st, floor_us, granule_us=None):
    """Latency-model roofline of a sequential kernel: `achieved` = its time per dependent
    step (live HIP-event time / steps it counted), `peak` = the measured per-step floor of the mechanism
    the steps wait on; frac = peak / achieved (1.0 = at the floor)."""
    us = st["ms"] * 1000.0 / st["steps"]
    r = roofline_of(name, st)
    return dict(bound="latency", achieved=round(us, 4), peak=round(floor_us, 4), unit="us/step",
                frac=round(floor_us / us, 4), traffic=None, kernel=name, launches=st["launches"],
                steps_per_launch=round(st["steps"] / st["launches"], 1), avg_launch_ms=round(st["ms"] / st["launches"], 4),
                floor="sd_probe_lstm_handoff: the recurrence's 4-workgroup h exchange alone, us per step",
                # the guide's data-tagged granule transport on the same exchange (round 5): measured SLOWER than
                # the counter protocol (4.3 vs 2.0 us per step), so the counter probe stays the binding floor
                granule_probe_us=None if granule_us is None else round(granule_us, 4),
                mfma_frac=r["mfma_frac"], hbm_frac=r["hbm_frac"])


def kernel_report(kernels, workload, ms_per_step, precision):
    """roofline (dominant single kernel), attention_roofline, whole-step work and a
    per-kernel table, all from the live timer.  A dominant kernel that counts sequential steps (the
    LSTM recurrence of C1 / C3) gets the latency model instead of a flop / byte roof."""
    if not kernels:
        return {}
    dom = max(kernels, key=lambda k: kernels[k]["ms"])
    if kernels[dom].get("steps", 0) > 0 and dom == "lstm_recurrence":
        out = {"roofline": latency_roofline_of(dom, kernels[dom], lstm_handoff_floor_us(),
                                               lstm_handoff_floor_us(probe="sd_probe_lstm_granule"))}
    else:
        out = {"roofline": roofline_of(dom, kernels[dom], pmc_traffic(workload, dom))}
    att = [k for k in ATTN_KERNELS if k in kernels]
    if att:
        out["attention_roofline"] = roofline_of(att[0], kernels[att[0]], pmc_traffic(workload, att[0]))
    flops = sum(v["flops"] for v in kernels.values())
    byts = sum(v["bytes"] for v in kernels.values())
    kms = sum(v["ms"] for v in kernels.values())
    dt = {"fp32": "f32", "bf16x3": "bf16x3"}.get(precision, "bf16")
    s = ms_per_step * 1e-3
    out["step_work"] = {"algorithmic_gflop_per_step": round(flops / 1e9, 2),
                        "algorithmic_gb_per_step": round(byts / 1e9, 3),
                        "kernel_ms_per_step": round(kms, 3), "ms_per_step": round(ms_per_step, 3),
                        "achieved_tflops": round(flops / s / 1e12, 1), "mfma_frac": round(flops / s / 1e12 / PEAKS[dt], 4),
                        "achieved_gbs": round(byts / s / 1e9, 1), "hbm_frac": round(byts / s / 1e9 / HBM_PEAK, 4)}
    tab = {}
    for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["ms"])[:24]:
        r = roofline_of(k, v)
        tab[k] = {"share": round(v["ms"] / kms, 3), "ms": round(v["ms"], 3), "launches": v["launches"],
                  "bound": r["bound"], "frac": r["frac"]}
    out["kernels"] = tab
    return out


# ----------------------------------------------------------------------------- distributed helpers
def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """`bench.py --gpus N` with no external launcher: start N fresh child processes of this
    script, one per GPU, with the torchrun environment (RANK, LOCAL_RANK, WORLD_SIZE,
    MASTER_ADDR/PORT) — the reference's own multi-process pattern is torchrun
    --nproc_per_node (egs/magicdata-ramc/tests/test_ddp.sh:3).  This parent never touches
    the GPU (no torch import), so nothing GPU-initialised is forked or exec'd.  If a rank
    fails, the others are stopped (they would wait in a collective) and its code is returned."""
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in procs:           # our own children, by handle
                    q.terminate()
        time.sleep(0.05)
    return rc


def dist_setup(backend="nccl"):
    """One process per GPU from the torchrun environment (the driver's launcher or
    launch_ranks); backend "nccl" is RCCL on ROCm.  backend "gloo" is the CPU self-test."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend == "gloo":
        dev = torch.device("cpu")
        if world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("nccl", device_id=dev)
    if world > 1:
        world = dist.get_world_size()
    return world, rank, dev


def ranks_joined(world, dev):
    """Every rank's id, all-gathered over the job's backend (RCCL on the GPU path): the
    line's proof that N ranks joined the collective the data path uses."""
    if world == 1:
        return [0]
    import torch
    import torch.distributed as dist
    gdev = torch.device("cpu") if dist.get_backend() == "gloo" else dev   # gloo gathers host tensors
    mine = torch.tensor([dist.get_rank()], device=gdev, dtype=torch.int64)
    allr = torch.empty(world, device=gdev, dtype=torch.int64)
    dist.all_gather_into_tensor(allr, mine)
    return [int(x) for x in allr.cpu()]


def _sync(dev):
    import torch
    if dev.type == "cuda":
        torch.cuda.synchronize()


def timed(step, warmup, steps, world, dev):
    """W untimed warm-up steps, then exactly K steps bracketed by barrier + synchronize on
    both sides; max over ranks."""
    import torch
    import torch.distributed as dist
    for _ in range(warmup):
        step()
    _sync(dev)
    if world > 1:
        dist.barrier()
    _sync(dev)
    t0 = time.perf_counter()
    out = None
    for _ in range(steps):
        out = step()
    _sync(dev)
    if world > 1:
        dist.barrier()
    _sync(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, out


def main_dist_check(a):
    """CPU self-test of the launcher (tests/test_bench_launcher.py): the same rank setup,
    timing and line as the TS-VAD strong-scaling path, with gloo instead of RCCL and the
    device forward replaced by seeded window logits, so no GPU is needed.  Each rank takes its
    contiguous share of the C4 60-min meeting's 64-window batch grid; the all-gather of
    ts_vad/pipeline.py re-assembles the global window order, which every rank checks."""
    import torch
    from speaker_diarization_amd.ts_vad.pipeline import gather_windows
    from speaker_diarization_amd.ts_vad.windows import plan_windows, shard_batches
    world, rank, dev = dist_setup("gloo")
    joined = ranks_joined(world, dev)
    plan = plan_windows(60 * 60 * 25, 4, 1)
    g = torch.Generator().manual_seed(777)
    full = torch.randn(plan.n_win, 4, plan.chunk, generator=g)
    w0, w1 = shard_batches(plan, a.batch, world, rank)

    def step():
        local = full[w0:w1].clone()
        return gather_windows(local, plan, a.batch, world) if world > 1 else local
    elapsed, got = timed(step, a.warmup, a.steps, world, dev)
    ok = bool(torch.equal(got, full))
    if rank == 0:
        print(json.dumps({"metric": "launcher self-test (window-logit all-gather)", "value": round(
            plan.n_win * a.steps / elapsed, 1), "unit": "windows/s", "n_gpus": world, "rccl_ranks": None,
            "ranks_joined": joined, "backend": "gloo", "gather_matches_global_order": ok,
            "shard": [w0, w1], "n_win": plan.n_win, "steps": a.steps, "warmup": a.warmup}))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


# ----------------------------------------------------------------------------- TS-VAD (C2 / C4)
def cpu_baseline(cfg, sd_np, meeting, ts, budget_s):
    """The CPU oracle (PyTorch-CPU restatement of the reference inference loop,
    parity-pinned by tests/golden) on a bounded sample of the same meeting, BASELINE.md §2
    protocol: all usable host cores, 1 warm-up + median of 3, model-only (wav -> posteriors)
    and end-to-end (-> RTTM text at the 10 recipe thresholds, oracle/postprocess_ref.py)."""
    import torch
    from oracle.pipeline_ref import meeting_posteriors
    from oracle.postprocess_ref import rttm_lines
    from speaker_diarization_amd.weights import to_torch
    threads = host_threads()
    torch.set_num_threads(threads)
    sd = to_torch(sd_np)
    n_lab = meeting.labels.shape[1]
    probe = 8
    t0 = time.perf_counter()      # the warm-up run also sizes the sample
    meeting_posteriors(sd, cfg, meeting.wav, ts, n_lab, shift=1, batch_size=probe, max_windows=probe)
    per_win = (time.perf_counter() - t0) / probe
    n = int(max(probe, min(320, budget_s / 3.0 / max(per_win, 1e-6))))
    n = max(probe, (n // probe) * probe)
    post = {}

    def model_only():
        post["p"] = meeting_posteriors(sd, cfg, meeting.wav, ts, n_lab, shift=1, batch_size=min(64, n),
                                       max_windows=n)
    t_model, runs, _ = median3(model_only)
    span = n * 100 // 4   # label frames fully covered by the sample's windows (1 window per second)
    keys = {f"{meeting.name}-{i + 1}": post["p"][i, :span] for i in range(4)}
    t_post, _, _ = median3(lambda: rttm_lines(keys))
    frames = n * 100          # each window advances the meeting by segment_shift (1 s) = 100 frames
    info = host_info(threads)
    return dict(value=round(frames / t_model, 2), unit="frames/s", kind="port",
                end_to_end_value=round(frames / (t_model + t_post), 2),
                sample=f"first {n} windows ({n} s of meeting, fp32, batch {min(64, n)}) of the same meeting "
                       f"through oracle/pipeline_ref.py (+ oracle/postprocess_ref.py for end-to-end) on "
                       f"{threads} host threads; 1 warm-up + median of 3 runs "
                       f"({', '.join('%.2f' % r for r in runs)} s model-only, {t_post:.3f} s RTTM)",
                **info), post["p"], n


def variant_posteriors(job, a, dev, sd_np, precision):
    """The job's meeting through a second model holding a weight variant (numpy posteriors)."""
    import torch
    from speaker_diarization_amd.ts_vad.model import TSVADModel
    from speaker_diarization_amd.ts_vad.pipeline import TSVADPipeline
    from speaker_diarization_amd.weights import to_torch
    m = TSVADModel(job["cfg"], device=dev, precision=precision,
                   max_batch=max(a.batch, a.device_batch) if precision == a.precision else a.batch)
    m.load_state_dict(to_torch(sd_np))
    p = TSVADPipeline(m, segment_shift=1, batch_size=a.batch).posteriors(job["wav"], job["ts"], job["n_lab"])
    out = p.cpu().numpy()
    del m
    torch.cuda.empty_cache()
    return out


def variant_der(job, a, dev, meeting, n_win):
    """DER parity that can fail (round-5 verdict item 1): the same span on the 'dynamic' weight variant
    (weights.py dynamic_weights: gsp_fc and the BiLSTM input centred and scaled upstream, fc x4, so the
    activations move with the frame and 99 % of the posteriors sit in [0.2, 0.8]), GPU fp32, GPU bf16x3 and GPU
    in the line's precision against the fp32 CPU oracle.  fp32 and bf16x3 are the gate; on this variant bf16 as
    a number format moves the DER by more than 0.1 whichever stage computes in it (tests/bf16_der_emulation.py,
    DESIGN.md §6 round-6 item 1), so the bf16 figures measure that, not a kernel difference."""
    import torch
    from oracle.pipeline_ref import meeting_posteriors
    from speaker_diarization_amd.weights import to_torch, tsvad_state_dict
    sd = tsvad_state_dict(job["cfg"], seed=777, dynamic=True)
    torch.set_num_threads(host_threads())
    cpu_post = meeting_posteriors(to_torch(sd), job["cfg"], meeting.wav, job["ts_np"], job["n_lab"], shift=1,
                                  batch_size=min(64, n_win), max_windows=n_win)
    out = {}
    for prec in dict.fromkeys(("fp32", "bf16x3", a.precision)):
        g = variant_posteriors(job, a, dev, sd, prec)
        d = der_parity(meeting, g, cpu_post, float(n_win))
        d.pop("note", None)
        d["posterior_parity"] = posterior_parity(g, cpu_post, n_win * 25)
        out[prec] = d
    out["note"] = ("fp32 and bf16x3 (fp32-equivalent split-bf16 GEMMs) are the gate (|dDER| <= 0.1 at every "
                   "threshold on a non-degenerate table); bf16 on this variant measures the number format's effect "
                   "(tests/bf16_der_emulation.py), not parity")
    return out


def der_parity(meeting, gpu_post, cpu_post, span_s, n_real=4, label_rate=25, gpu_fp32=None):
    """The '+ DER' half of the metric: md-eval DER (collar 0.25, ts_vad2/infer.py:136-151) of the
    GPU path and of the CPU reference path over the same span (the first span_s seconds, which
    every window of the CPU sample covers exactly as in the full plan), against the synthetic
    meeting's reference RTTM, at the recipe's thresholds."""
    from oracle.postprocess_ref import rttm_lines
    from speaker_diarization_amd import der as der_mod
    from speaker_diarization_amd.ts_vad.postprocess import THRESHOLDS, posteriors_to_rttm_gpu
    import torch
    T = int(span_s * label_rate)
    keys = [f"{meeting.name}-{i + 1}" for i in range(n_real)]

    def dv(x):   # the GPU RTTM writer takes device posteriors
        return torch.from_numpy(np.ascontiguousarray(x, np.float32)).cuda() if isinstance(x, np.ndarray) else x
    gpu_rttm = posteriors_to_rttm_gpu(keys, dv(gpu_post[:n_real, :T]))
    cpu_rttm = rttm_lines({k: cpu_post[i, :T] for i, k in enumerate(keys)})
    ref = [f"SPEAKER {meeting.name} 1 {s:.3f} {min(e, span_s) - s:.3f} <NA> <NA> {spk + 1} <NA> <NA>\n"
           for spk, s, e in sorted(meeting.segments, key=lambda x: (x[1], x[0])) if s < span_s]
    ref = der_mod.read_rttm(ref)
    f32_rttm = posteriors_to_rttm_gpu(keys, dv(gpu_fp32[:n_real, :T])) if gpu_fp32 is not None else None
    table, t32 = {}, {}
    for thr in THRESHOLDS:
        g = der_mod.md_eval(ref, der_mod.read_rttm(gpu_rttm[thr]), collar=0.25).der
        c = der_mod.md_eval(ref, der_mod.read_rttm(cpu_rttm[thr]), collar=0.25).der
        table[thr] = (round(g, 2), round(c, 2))
        if f32_rttm is not None:
            t32[thr] = round(der_mod.md_eval(ref, der_mod.read_rttm(f32_rttm[thr]), collar=0.25).der, 2)
    diffs = [abs(g - c) for g, c in table.values()]
    out = {"span_s": span_s, "collar": 0.25, "threshold": 0.5, "gpu": table[0.5][0], "cpu_reference": table[0.5][1],
           "max_abs_diff_over_thresholds": round(max(diffs), 3),
           "per_threshold_gpu_cpu": {str(k): v for k, v in table.items()},
           "note": "seeded random weights: absolute DER is meaningless, the GPU-vs-reference difference is the check"}
    if t32:
        out["fp32_per_threshold"] = {str(k): v for k, v in t32.items()}
        out["fp32_max_abs_diff_over_thresholds"] = round(max(abs(t32[k] - table[k][1]) for k in t32), 3)
    return out


def tsvad_job(wl, a, world, dev, total_min):
    """Model, pipeline and synthetic meeting of a TS-VAD workload (C2 / C4)."""
    import torch
    from speaker_diarization_amd.synth import make_meeting, speaker_embeddings
    from speaker_diarization_amd.ts_vad.model import TSVADModel
    from speaker_diarization_amd.ts_vad.pipeline import TSVADPipeline
    from speaker_diarization_amd.weights import TSVADConfig, to_torch, tsvad_state_dict
    cfg = TSVADConfig(rs_len=wl["rs_len"]) if wl["variant"] == 0 else TSVADConfig.ots_vad_v1(rs_len=wl["rs_len"])
    sd_np = tsvad_state_dict(cfg, seed=777)
    model = TSVADModel(cfg, device=dev, precision=a.precision, max_batch=max(a.batch, a.device_batch))
    model.load_state_dict(to_torch(sd_np))
    pipe = TSVADPipeline(model, segment_shift=1, batch_size=a.batch)
    meeting = make_meeting(total_min * 60.0, n_spk=4, seed=777)
    ts_np = speaker_embeddings(4, seed=777)
    job = dict(cfg=cfg, sd_np=sd_np, model=model, pipe=pipe, meeting=meeting, ts_np=ts_np,
               wav=torch.from_numpy(meeting.wav).to(dev), ts=torch.from_numpy(ts_np).to(dev),
               n_lab=meeting.labels.shape[1], frames=meeting.wav.size // 160)
    job["step"] = lambda: pipe.posteriors(job["wav"], job["ts"], job["n_lab"])
    return job


def c4_reference(a, dev):
    """The N>1 lines' workload (BASELINE C4: CAM++ + transformer, rs_len 4, one fixed 60-min
    meeting) timed on this one GPU, so the scaling series reads against one workload."""
    wl = WORKLOADS["c4"]
    job = tsvad_job(wl, a, 1, dev, 60.0)
    steps = max(1, min(a.steps, 3))
    elapsed, _ = timed(job["step"], 1, steps, 1, dev)
    out = {"workload": wl["desc"], "meeting_minutes": 60.0, "windows": job["pipe"].plan(job["n_lab"]).n_win,
           "steps": steps, "warmup": 1, "ms_per_step": round(elapsed / steps * 1e3, 3),
           "value": round(job["frames"] * steps / elapsed, 1), "unit": "frames/s",
           "note": "same meeting, model and window grid as the --gpus N > 1 lines (strong scaling)"}
    del job
    return out


def posterior_parity(gpu_post, cpu_post, span_frames, n_real=4, med_filter=21):
    """Posterior-level parity of the product path against the fp32 CPU oracle over the span
    the CPU sample covers exactly: max / mean |diff| of the averaged posteriors, and per recipe
    threshold the frames whose speech decision differs — on the raw posteriors and after the
    reference's medfilt(21) (ts_vad2/infer.py:90-100, scipy.signal.medfilt as the reference)."""
    from scipy.signal import medfilt
    from speaker_diarization_amd.ts_vad.postprocess import THRESHOLDS
    g = np.asarray(gpu_post[:n_real, :span_frames], np.float32)
    c = np.asarray(cpu_post[:n_real, :span_frames], np.float32)
    d = np.abs(g.astype(np.float64) - c)
    gm = np.stack([medfilt(x, med_filter) for x in g])
    cm = np.stack([medfilt(x, med_filter) for x in c])
    return {"frames_compared": int(g.size), "tracks": n_real, "span_label_frames": int(span_frames),
            "max_abs_diff": float(d.max()), "mean_abs_diff": float(d.mean()),
            "decision_flips_raw": {str(t): int(((g > t) != (c > t)).sum()) for t in THRESHOLDS},
            "decision_flips_medfilt": {str(t): int(((gm > t) != (cm > t)).sum()) for t in THRESHOLDS},
            "reference": "oracle/pipeline_ref.py (ts_vad2/infer.py:216-285 restated, fp32 torch-CPU)"}


def main(a, wl):
    from speaker_diarization_amd.ts_vad.postprocess import posteriors_to_rttm_gpu

    world, rank, dev = dist_setup()
    joined = ranks_joined(world, dev)
    scaling = a.scaling or ("strong" if (world > 1 or wl.get("strong")) else "weak")
    if scaling == "strong":
        total_min = a.minutes if a.minutes is not None else 60.0
    else:
        total_min = (a.minutes if a.minutes is not None else wl["minutes"]) * world
    job = tsvad_job(wl, a, world, dev, total_min)
    pipe, meeting, step = job["pipe"], job["meeting"], job["step"]
    frames_per_step = job["frames"]     # 10 ms frames of the whole meeting

    elapsed, post = timed(step, a.warmup, a.steps, world, dev)
    ms_per_step = elapsed / a.steps * 1000.0
    value = frames_per_step * a.steps / elapsed

    # End-to-end (wav in HBM -> RTTM text at the 10 recipe thresholds): median of 3.
    keys = [f"{meeting.name}-{i + 1}" for i in range(4)]

    def e2e():
        p = pipe.posteriors(job["wav"], job["ts"], job["n_lab"])
        return posteriors_to_rttm_gpu(keys, p) if rank == 0 else None
    e2e()
    t_e2e, _, _ = median3(e2e)

    kernels = None if a.no_kernel_timing else live_kernels(step)

    cpu, der, parity = None, None, None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu, cpu_post, n_cpu = cpu_baseline(job["cfg"], job["sd_np"], meeting, job["ts_np"], a.cpu_seconds)
        der = der_parity(meeting, post, cpu_post, float(n_cpu))
        parity = posterior_parity(post.cpu().numpy(), cpu_post, n_cpu * 25)
        der["dynamic"] = variant_der(job, a, dev, meeting, n_cpu)
    c4 = None
    if world == 1 and a.workload == "c2" and not a.no_c4_ref:
        c4 = c4_reference(a, dev)

    if rank == 0:
        plan = pipe.plan(job["n_lab"])
        line = {
            "metric": "diarized frames/sec (10 ms hop)",
            "value": round(value, 1),
            "unit": "frames/s",
            "n_gpus": world,
            "rccl_ranks": joined if world > 1 else None,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": a.precision,
            "data": "synthetic 16 kHz 4-speaker meeting (speaker_diarization_amd/synth.py), seeded random "
                    "weights of the reference architecture",
            "config": {"workload": wl["desc"], "meeting_minutes": total_min,
                       "minutes_per_gpu": round(total_min / world, 3), "windows": plan.n_win,
                       "global_batch": a.batch, "device_batch": max(a.batch, a.device_batch),
                       "parallelism": (f"window-shard x{world} on the 64-window batch grid + RCCL all-gather of "
                                       f"window logits" if world > 1 else "1 GPU")},
            "end_to_end": {"ms_per_step": round(t_e2e * 1e3, 3), "value": round(frames_per_step / t_e2e, 1),
                           "what": "wav in HBM -> posteriors -> GPU medfilt/threshold/run-length -> RTTM lines "
                                   "(10 thresholds), median of 3"},
        }
        if c4 is not None:
            line["c4_60min_ms"] = c4["ms_per_step"]
            line["c4_60min"] = c4
        line.update(kernel_report(kernels, a.workload, ms_per_step, a.precision))
        line["cpu_baseline"] = cpu
        line["parity"] = parity
        line["der"] = der
        if cpu:
            line["speedup_vs_cpu"] = round(value / cpu["value"], 1)
            line["end_to_end"]["speedup_vs_cpu"] = round(frames_per_step / t_e2e / cpu["end_to_end_value"], 1)
        print(json.dumps(line))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


# ----------------------------------------------------------------------------- EEND family
def eda_cpu_baseline(wl, meeting, sd_np, num_speakers):
    """oracle/eend_ref.py (infer_eda.py:92-124 restated, fp32) over the whole recording."""
    import torch
    from oracle import eend_ref
    from speaker_diarization_amd.weights import EDAConfig, to_torch
    threads = host_threads()
    torch.set_num_threads(threads)
    cfg = EDAConfig(model_type=wl["model_type"], n_speakers=wl["n_spk"], n_layers=wl["layers"])
    sd = to_torch(sd_np)
    wav = meeting.wav.astype(np.float64)

    def run():
        Y = eend_ref.features(wav)
        outs = []
        g = torch.Generator().manual_seed(777)
        for s, e in eend_ref.gen_chunk_indices(len(Y), 2000):
            src = [torch.from_numpy(np.ascontiguousarray(Y[s:e], np.float32))]
            act, probs = eend_ref.infer_full(sd, cfg, src, eend_ref.chunk_perms([e - s], g))
            try:
                outs.append(eend_ref.select(act, probs, cfg.variant, num_speakers)[0])
            except IndexError:        # the reference's top-n quirk; the forward has run
                pass
        return outs
    run()
    t, runs, _ = median3(run)
    frames = meeting.wav.size // 160
    return dict(value=round(frames / t, 2), unit="frames/s", kind="port",
                sample=f"the whole {meeting.wav.size / 16000 / 60:.0f}-min recording through oracle/eend_ref.py "
                       f"(librosa-restated frontend + encoder + EDA LSTMs, fp32) on {threads} threads; 1 warm-up "
                       f"+ median of 3 ({', '.join('%.2f' % r for r in runs)} s)", **host_info(threads))


def fseend_cpu_baseline(meeting, sd_np, budget_s):
    """oracle/fseend_ref.py test() over the whole recording (one call, as fs_eend/model.py:198)."""
    import torch
    from oracle import eend_ref, fseend_ref
    from speaker_diarization_amd.weights import FSEENDConfig, to_torch
    threads = host_threads()
    torch.set_num_threads(threads)
    cfg = FSEENDConfig()
    sd = to_torch(sd_np)
    Y = eend_ref.features(meeting.wav.astype(np.float64), 8000, 200, 80, 7, 10, "logmel23")
    T = len(Y)
    x = torch.from_numpy(np.ascontiguousarray(Y[:T], np.float32))[None]

    def run():
        with torch.no_grad():
            return fseend_ref.fseend_test(sd, cfg, x, [T], 6)
    run()
    t, runs, _ = median3(run)
    return dict(value=round(T * 10 / t, 2), unit="frames/s", kind="port",
                sample=f"the whole recording ({T} model frames, {T / 10:.0f} s) through oracle/fseend_ref.py test() (fp32, "
                       f"{threads} threads); 1 warm-up + median of 3 ({', '.join('%.2f' % r for r in runs)} s)",
                **host_info(threads))


def embed_cpu_baseline(wavs, sd_np, budget_s):
    """oracle/tsvad_ref.extract_embed (FBank povey + CAM++ + stats pooling) on the first
    speaker's enrollment audio, truncated to a bounded number of 6-s chunks."""
    import torch
    from oracle.tsvad_ref import extract_embed
    from speaker_diarization_amd.weights import to_torch
    threads = host_threads()
    torch.set_num_threads(threads)
    sd = to_torch(sd_np)
    w = wavs[0].cpu().numpy().astype(np.float64)
    n_sec = 6 + 23      # 24 chunks of 6 s every 1 s
    w = w[: n_sec * 16000 + 1]

    def run():
        with torch.no_grad():
            return extract_embed(sd, w, batch_size=96)
    run()
    t, runs, out = median3(run)
    return dict(value=round((len(w) // 160) / t, 2), unit="frames/s", kind="port",
                sample=f"{out.shape[0]} chunks (first {n_sec} s of one speaker's audio) through oracle/tsvad_ref.py "
                       f"extract_embed (fp32, {threads} threads); 1 warm-up + median of 3 "
                       f"({', '.join('%.2f' % r for r in runs)} s)", **host_info(threads))


def main_eend(a, wl):
    """EEND-EDA (c1/c3), FS-EEND (c5), embeddings and streaming TS-VAD: wav in HBM ->
    frontend -> model -> activities.  Multi-GPU: EEND-EDA shards chunks (all-gather of
    activities); the others run replicas."""
    import torch
    from speaker_diarization_amd.synth import make_meeting

    world, rank, dev = dist_setup()
    minutes = a.minutes if a.minutes is not None else wl["minutes"]
    kind = wl["kind"]
    prec = a.precision
    cpu_fn = None
    parity_fn = None
    extra = {}
    if kind == "eda":
        from speaker_diarization_amd.eend_eda.infer import EdaInferArgs, chunk_outputs, select_chunks, stitch
        from speaker_diarization_amd.eend_eda.models import EendEdaModel, TransformerEdaModel
        from speaker_diarization_amd.weights import EDAConfig, eda_state_dict, to_torch
        total_s = minutes * 60.0 * world          # weak scaling: chunks of an N x longer recording
        meeting = make_meeting(total_s, n_spk=wl["n_spk"], seed=777)
        torch.manual_seed(777)
        kw = dict(n_speakers=wl["n_spk"], in_size=345, n_heads=4, n_units=256, n_layers=wl["layers"],
                  precision=prec, max_seqs=32, max_frames=2000)
        m = TransformerEdaModel(**kw) if wl["model_type"] == "TransformerEda" else EendEdaModel(**kw)
        cfg = EDAConfig(model_type=wl["model_type"], n_speakers=wl["n_spk"], n_layers=wl["layers"])
        iargs = EdaInferArgs(num_speakers=wl["num_speakers"])
        wav = torch.from_numpy(meeting.wav.astype(np.float32)).to(dev)
        sd_np = eda_state_dict(cfg, seed=777)
        m.load_state_dict(to_torch(sd_np))

        def step():      # infer_eda.py:99-113, device half: frontend + every chunk's forward
            return chunk_outputs(m, wav, iargs)
        frames = meeting.wav.size // 160

        def cpu_fn():
            return eda_cpu_baseline(wl, meeting, sd_np, wl["num_speakers"])

        def parity_fn():
            return eda_oracle_parity(m, wav, meeting, sd_np, wl, iargs)

        def after(outs):
            """Speaker selection + the h5 stitch (infer_eda.py:112-121) on the timed run's outputs,
            outside the timed region (host indexing of the activities).  With seeded random weights
            the reference's own selection can fail — TransformerEda's top-n indexes the 15th
            attractor (models.py:337-339), threshold-mode chunks disagree on the speaker count (the
            np.vstack) — exactly as the reference would; the outcome is reported, not hidden."""
            try:
                extra["T_hat"] = list(stitch(select_chunks(m, *outs, iargs), iargs).shape)
            except IndexError as e:
                extra["T_hat"] = "IndexError in the reference's TransformerEda top-n selection: %s" % e
            except ValueError as e:
                extra["T_hat"] = "np.vstack ValueError (threshold-mode speaker counts differ): %s" % str(e)[:80]
    elif kind == "embed":
        from speaker_diarization_amd.ts_vad.embedding import CAMPPlus, extract_embed
        from speaker_diarization_amd.weights import campplus_state_dict, to_torch
        per = minutes * 60.0 / wl["n_spk"]
        wavs = [torch.from_numpy(make_meeting(per, n_spk=1, seed=900 + 10 * rank + i).wav.astype(np.float32)).to(dev)
                for i in range(wl["n_spk"])]
        m = CAMPPlus(feat_dim=80, embedding_size=192, device=dev, precision=prec, max_batch=96)
        sd_np = campplus_state_dict(777, 192)
        m.load_state_dict(to_torch(sd_np))

        def step():
            return [extract_embed(w, m, batch_size=96) for w in wavs]
        frames = sum(w.numel() for w in wavs) // 160 * world

        def cpu_fn():
            return embed_cpu_baseline(wavs, sd_np, a.cpu_seconds)
    elif kind == "tsvad_stream":
        from speaker_diarization_amd.synth import speaker_embeddings
        from speaker_diarization_amd.ts_vad.pipeline import TSVADPipeline
        from speaker_diarization_amd.ts_vad.streaming import StreamingWindowDecoder, TSVADStreamingModel
        from speaker_diarization_amd.weights import TSVADStreamingConfig, to_torch, tsvad_streaming_state_dict
        meeting = make_meeting(minutes * 60.0, n_spk=wl["n_spk"], seed=777 + rank)
        n_dev = int(os.environ.get("SDIAR_TSS_WINDOWS", "256"))   # windows per device call
        m = TSVADStreamingModel(device=dev, precision=prec, max_labels=250, max_windows=n_dev)
        m.load_state_dict(to_torch(tsvad_streaming_state_dict(TSVADStreamingConfig(), seed=777)))
        pipe = TSVADPipeline(StreamingWindowDecoder(m, wl["chunk"], wl["left"]), segment_shift=1, batch_size=64)
        wav = torch.from_numpy(meeting.wav.astype(np.float32)).to(dev)
        ts = torch.from_numpy(speaker_embeddings(4, seed=777)).to(dev)
        plan = pipe.plan(wav.numel() // 640)

        def step():   # replicas: every rank decodes its own meeting
            return pipe.average(pipe.window_logits(wav, ts, plan), plan)
        frames = meeting.wav.size // 160 * world

        def cpu_fn():
            return tss_cpu_baseline(meeting, plan, wl)
    else:
        from speaker_diarization_amd.feature import eend_features
        from speaker_diarization_amd.fs_eend.model import OnlineTransformerDADiarization
        from speaker_diarization_amd.weights import FSEENDConfig, fseend_state_dict, to_torch
        total_s = minutes * 60.0                   # replicas: every rank its own recording
        meeting = make_meeting(total_s, n_spk=wl["n_spk"], seed=777 + rank, sample_rate=8000)
        n_sub = -(-((meeting.wav.size // 80)) // 10) + 1
        m = OnlineTransformerDADiarization(None, 345, 256, 4, 4, 2, 0.1, True, 10000, 2048, precision=prec,
                                           max_seqs=1, max_frames=max(n_sub, 16), max_nspks=6)
        sd_np = fseend_state_dict(FSEENDConfig(), seed=777)
        m.load_state_dict(to_torch(sd_np))
        wav = torch.from_numpy(meeting.wav.astype(np.float32)).to(dev)

        def step():
            f = eend_features(wav, 8000, 200, 80, "logmel23", 7, 10, ld=m.in_ld)
            return m.test_device(f[None], [f.shape[0]], 6, want_emb=False, want_attractors=False)
        frames = meeting.wav.size // 80 * world

        def cpu_fn():
            return fseend_cpu_baseline(meeting, sd_np, a.cpu_seconds)

        def parity_fn():
            return fseend_oracle_parity(meeting, sd_np, step()[0][0], frames=1000)
    elapsed, out = timed(step, a.warmup, a.steps, world, dev)
    if kind == "eda":
        after(out)
    ms_per_step = elapsed / a.steps * 1000.0
    kernels = None if a.no_kernel_timing else live_kernels(step)
    if rank == 0:
        line = {"metric": "diarized frames/sec (10 ms hop)", "value": round(frames * a.steps / elapsed, 1),
                "unit": "frames/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": prec,
                "data": "synthetic recording (speaker_diarization_amd/synth.py), seeded random weights",
                "config": {"workload": wl["desc"], "minutes_per_gpu": minutes,
                           "parallelism": ("chunk-shard x%d + RCCL all-gather" % world if kind == "eda" else
                                           "replicas x%d" % world) if world > 1 else "1 GPU"}}
        line.update(extra)
        line.update(kernel_report(kernels, a.workload, ms_per_step, prec))
        if world == 1 and not a.no_cpu_baseline:
            line["cpu_baseline"] = cpu_fn()
            line["speedup_vs_cpu"] = round(line["value"] / line["cpu_baseline"]["value"], 1)
            if parity_fn is not None:
                line["parity"] = parity_fn()
        print(json.dumps(line))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def eda_oracle_parity(m, wav, meeting, sd_np, wl, iargs, n_chunks=2):
    """EEND-EDA activities and attractor probabilities of the product path vs the fp32 CPU oracle
    (oracle/eend_ref.py: infer_eda.py:92-124 restated) on the first n_chunks 2000-frame chunks, both driven
    by the SAME per-chunk randperm draws (the frame shuffle decides the attractors, models.py:229-233):
    max / mean |diff| over all (max_n - 1) attractor columns and the decisions (> 0.5, make_rttm's
    threshold) that differ."""
    import torch
    from oracle import eend_ref
    from speaker_diarization_amd.eend_eda.infer import chunk_activities, gen_chunk_indices, recording_features
    from speaker_diarization_amd.weights import EDAConfig, to_torch
    torch.set_num_threads(host_threads())
    cfg = EDAConfig(model_type=wl["model_type"], n_speakers=wl["n_spk"], n_layers=wl["layers"])
    feats = recording_features(m, wav, iargs)
    chunks = list(gen_chunk_indices(feats.shape[0], iargs.chunk_size))[:n_chunks]
    g = torch.Generator().manual_seed(777)
    perms = [torch.randperm(e - s, generator=g) for s, e in chunks]
    acts, probs = chunk_activities(m, feats, iargs, perms, 0, len(chunks))
    Y = eend_ref.features(meeting.wav.astype(np.float64))
    dmax, dsum, cnt, flips, pmax = 0.0, 0.0, 0, 0, 0.0
    for c, (s, e) in enumerate(chunks):
        src = [torch.from_numpy(np.ascontiguousarray(Y[s:e], np.float32))]
        act_ref, probs_ref = eend_ref.infer_full(to_torch(sd_np), cfg, src, [perms[c]])
        a = acts[c].cpu().numpy().astype(np.float64)
        r = act_ref[0].numpy().astype(np.float64)
        d = np.abs(a - r)
        dmax, dsum, cnt = max(dmax, float(d.max())), dsum + float(d.sum()), cnt + d.size
        flips += int(((a > 0.5) != (r > 0.5)).sum())
        pmax = max(pmax, float(np.abs(probs[c].numpy() - np.asarray(probs_ref[0])).max()))
    return {"chunks_compared": len(chunks), "frames_compared": int(sum(e - s for s, e in chunks)),
            "max_abs_diff": dmax, "mean_abs_diff": dsum / max(cnt, 1), "decision_flips_at_0.5": flips,
            "decisions": cnt, "attractor_prob_max_abs_diff": pmax,
            "reference": "oracle/eend_ref.py infer_full (fp32 torch-CPU, librosa-restated frontend), same randperms"}


def tss_cpu_baseline(meeting, plan, wl, n_win=8):
    """The reference's streaming decode on the host: oracle/tsvad_stream_ref.py (the literal
    forward_chunk_by_chunk_temp1 cache loop, one window per call like infer_debug) over the
    first n_win windows of the same meeting (window fbank + CMN, oracle/fbank_ref.py), fp32,
    all usable host threads, 1 warm-up + median of 3.  Meeting frames/s = windows/s x
    (meeting frames / windows)."""
    import torch
    from oracle.fbank_ref import window_fbank
    from oracle.tsvad_stream_ref import forward_chunk_by_chunk
    from speaker_diarization_amd.synth import speaker_embeddings
    from speaker_diarization_amd.weights import TSVADStreamingConfig, to_torch, tsvad_streaming_state_dict
    threads = host_threads()
    torch.set_num_threads(threads)
    sd = to_torch(tsvad_streaming_state_dict(TSVADStreamingConfig(), seed=777))
    ts = torch.from_numpy(speaker_embeddings(4, seed=777))[None]
    spl = plan.samples_per_label
    wins = [(torch.from_numpy(window_fbank(meeting.wav[int(plan.starts[w]) * spl:int(plan.ends[w]) * spl]))[None],
             int(plan.lens[w])) for w in range(min(n_win, plan.n_win))]

    def run():
        with torch.no_grad():
            for f, n in wins:
                forward_chunk_by_chunk(sd, f, ts, n, wl["chunk"], wl["left"])
    run()
    t, runs, _ = median3(run)
    frames_per_win = (meeting.wav.size // 160) / plan.n_win
    return dict(value=round(len(wins) * frames_per_win / t, 2), unit="frames/s", kind="port",
                sample="first %d windows (10 s each) of the same meeting through oracle/tsvad_stream_ref.py "
                       "(literal chunk loop with KV caches, fp32, %d host threads); 1 warm-up + median of 3 (%s s)"
                       % (len(wins), threads, ", ".join("%.2f" % r for r in runs)), **host_info(threads))


def main_stream(a, wl):
    """C5 latency mode: one recording per GPU streamed through the C ABI as it would arrive live.
    Default: raw 8 kHz audio in BASELINE C5's 80 ms pushes (640 samples, sd_fseend_stream_push_audio):
    each model frame's STFT / logmel / splice (fs_eend/dataset.py:217-223, feature.py:130-184) runs inside
    the encoder chunk's captured hipGraph; a push returns 0 or 1 final frame (a model frame is 100 ms, its
    score is final 9 frames later).  `--feature-rows` pushes precomputed feature rows instead (model only).
    Every push is synchronised, as a live caller waiting for its scores would be.  value = 10 ms frames/s
    of the streamed recording (N replicas: summed); per-push latency percentiles alongside."""
    import ctypes
    import torch
    from speaker_diarization_amd import _lib
    from speaker_diarization_amd.feature import _mel_device, eend_features
    from speaker_diarization_amd.fs_eend.model import OnlineTransformerDADiarization
    from speaker_diarization_amd.synth import make_meeting
    from speaker_diarization_amd.weights import FSEENDConfig, fseend_state_dict, to_torch

    world, rank, dev = dist_setup()
    minutes = a.minutes if a.minutes is not None else wl["minutes"]
    chunk = a.chunk or wl["chunk"]
    audio = not a.feature_rows
    meeting = make_meeting(minutes * 60.0, n_spk=wl["n_spk"], seed=777 + rank, sample_rate=8000)
    wav = torch.from_numpy(meeting.wav.astype(np.float32)).to(dev)
    sd_np = fseend_state_dict(FSEENDConfig(), seed=777)
    m = OnlineTransformerDADiarization(None, 345, 256, 4, 4, 2, 0.1, True, 10000, 2048, precision=a.precision,
                                       max_seqs=1, max_frames=64, max_nspks=6)
    m.load_state_dict(to_torch(sd_np))
    feats = eend_features(wav, 8000, 200, 80, "logmel23", 7, 10, ld=m.in_ld).contiguous()
    T = feats.shape[0]
    lib = _lib.load()
    s = ctypes.c_void_p()
    _lib.call("sd_fseend_stream_create", m._h, chunk, T + chunk, 6, 0 if a.no_graph else 1, ctypes.byref(s))
    preds = torch.empty(T + 64, 6, device=dev)
    sp = _lib.stream_ptr(dev)
    cnt = ctypes.c_int()
    base, row_bytes = feats.data_ptr(), m.in_ld * 4
    fb = _mel_device(8000, 256, dev)
    push_samples = a.push_samples
    lat = []

    def step(record):
        lib.sd_fseend_stream_reset(s, sp)
        out = 0
        if audio:
            _lib.call("sd_fseend_stream_set_audio", s, fb.data_ptr(), 23, 200, 80, 7, 10)
            n = wav.numel()
            for i in range(0, n, push_samples):
                k = min(push_samples, n - i)
                t0 = time.perf_counter()
                _lib.check(lib.sd_fseend_stream_push_audio(s, wav.data_ptr() + 4 * i, k, preds.data_ptr() + out * 24,
                                                           preds.shape[0] - out, ctypes.byref(cnt), sp))
                torch.cuda.synchronize()
                if record:
                    lat.append(time.perf_counter() - t0)
                out += cnt.value
        else:
            for i in range(0, T, chunk):
                n = min(chunk, T - i)
                t0 = time.perf_counter()
                _lib.check(lib.sd_fseend_stream_push(s, base + i * row_bytes, m.in_ld, n, preds.data_ptr() + out * 24,
                                                     preds.shape[0] - out, ctypes.byref(cnt), sp))
                torch.cuda.synchronize()
                if record:
                    lat.append(time.perf_counter() - t0)
                out += cnt.value
        _lib.check(lib.sd_fseend_stream_flush(s, preds.data_ptr() + out * 24, preds.shape[0] - out,
                                              ctypes.byref(cnt), sp))
        torch.cuda.synchronize()
        assert out + cnt.value == T, (out, cnt.value, T)

    def stats():
        e, d, ne, nd = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int(), ctypes.c_int()
        _lib.call("sd_fseend_stream_stats", s, ctypes.byref(e), ctypes.byref(d), ctypes.byref(ne), ctypes.byref(nd))
        return e.value, d.value, ne.value, nd.value

    for _ in range(a.warmup):
        step(False)
    st0 = stats()
    elapsed, _ = timed(lambda: step(True), 0, a.steps, world, dev)
    st1 = stats()
    lat[:] = lat[-(len(lat) // a.steps) * a.steps:]   # timed steps only
    # every step streams the whole recording from reset: a push attends over (T + 1) / 2 history rows on average
    latency_model = stream_latency_model(sd_np, st0, st1, len(lat), float(np.percentile(np.array(lat) * 1e6, 50)),
                                         audio, a.precision, kv=dict(rows=(T + 1) / 2, enc_layers=4, dec_layers=2,
                                                                     slots=6, d=256)) if a.steps else None
    # parity of this very run: against the whole-recording GPU test() on the same features, and against
    # the fp32 CPU oracle (oracle/fseend_ref.py test() on oracle/eend_ref.py features) over the first frames
    Tc = min(T, 2000)
    m2 = OnlineTransformerDADiarization(None, 345, 256, 4, 4, 2, 0.1, True, 10000, 2048, precision=a.precision,
                                        max_seqs=1, max_frames=Tc, max_nspks=6)
    m2.load_state_dict(to_torch(sd_np))
    full, _, _ = m2.test_device(feats[None, :Tc], [Tc], 6, want_emb=False, want_attractors=False)
    nc = Tc - 9 if Tc < T else Tc     # the truncated reference sees no look-ahead for its last 9 frames
    err = float((full[0, :nc] - preds[:nc]).abs().max())
    parity = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        parity = fseend_oracle_parity(meeting, sd_np, preds[:T], frames=min(T, 1000))
    lib.sd_fseend_stream_destroy(s)
    L = np.array(lat) * 1e3
    frames = meeting.wav.size // 80 * world
    if rank == 0:
        unit_ms = push_samples / 8.0 if audio else chunk * 100
        line = {"metric": "diarized frames/sec (10 ms hop)", "value": round(frames * a.steps / elapsed, 1),
                "unit": "frames/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                "ms_per_step": round(elapsed / a.steps * 1000.0, 3), "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": a.precision,
                "data": "synthetic 8 kHz recording (speaker_diarization_amd/synth.py), seeded random weights",
                "config": {"workload": wl["desc"], "minutes_per_gpu": minutes, "input": "audio" if audio else
                           "feature rows", "push_audio_ms": unit_ms, "push_samples": push_samples if audio else None,
                           "chunk_frames": chunk, "model_frames": T, "pushes_per_step": len(L) // max(a.steps, 1),
                           "hipgraph": not a.no_graph,
                           "parallelism": "replicas x%d" % world if world > 1 else "1 GPU"},
                "latency_ms": {"per": "push of %.0f ms of audio incl. frontend" % unit_ms if audio else
                               "push of %d model frame(s), model only" % chunk,
                               "p50": round(float(np.percentile(L, 50)), 4),
                               "p90": round(float(np.percentile(L, 90)), 4),
                               "p99": round(float(np.percentile(L, 99)), 4),
                               "max": round(float(L.max()), 4), "mean": round(float(L.mean()), 4)},
                "real_time_factor": round(float(L.mean()) / unit_ms, 5),
                "roofline": latency_model,
                "max_abs_diff_vs_test": err, "parity": parity}
        if rank == 0 and world == 1 and not a.no_cpu_baseline:
            line["cpu_baseline"] = fseend_cpu_baseline(meeting, sd_np, a.cpu_seconds)
            line["speedup_vs_cpu"] = round(line["value"] / line["cpu_baseline"]["value"], 1)
        print(json.dumps(line))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def kernel_boundary_us(n=200, reps=20):
    """Measured cost of one dependent kernel boundary inside a replayed hipGraph: a captured chain of n
    trivial dependent kernels (1-element in-place adds), replayed `reps` times; device time per kernel."""
    import torch
    x = torch.zeros(1, device="cuda")
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        for _ in range(3):
            x.add_(1.0)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                x.add_(1.0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.replay()
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / (n * reps)


def stream_latency_model(sd_np, st0, st1, pushes, p50_us, audio, precision, kv=None):
    """C5 latency roofline (SURVEY §8(d) latency model): a push cannot finish faster than its chain of
    dependent device operations: (graph nodes run per push + the per-push copies) x the measured kernel
    boundary, plus the bytes those chunk runs must read / HBM peak: the weights, and the K|V history rows
    each attention scores (encoder: one sequence per layer; decoder: `slots` sequences per application;
    2 * d values per row, `rows` = the mean history length over the timed pushes).  achieved = p50 per push
    (host wall, incl. the graph launch and the synchronisation); frac = floor / achieved."""
    enc_runs, dec_runs = st1[0] - st0[0], st1[1] - st0[1]
    ne, nd = st1[2], st1[3]
    esz = 2 if precision == "bf16" else 4
    groups = {}
    for k, v in sd_np.items():
        if k.endswith("num_batches_tracked"):
            continue
        groups[k.split(".")[0]] = groups.get(k.split(".")[0], 0) + int(np.asarray(v).size)
    enc_bytes = groups.get("enc", 0) * esz
    dec_bytes = (groups.get("cnn", 0) + 2 * groups.get("dec", 0)) * esz   # the fusion layer runs twice
    per_push_nodes = (enc_runs * ne + dec_runs * nd) / max(pushes, 1)
    per_push_copies = 1.0 + dec_runs / max(pushes, 1)     # the samples' copy, each emitted frame's copy
    b_us = kernel_boundary_us()
    bytes_per_push = (enc_runs * enc_bytes + dec_runs * dec_bytes) / max(pushes, 1)
    kv_bytes = 0.0
    if kv:
        row = 2 * kv["d"] * esz * kv["rows"]
        kv_bytes = (enc_runs * kv["enc_layers"] * row + dec_runs * kv["dec_layers"] * kv["slots"] * row) / max(pushes, 1)
    bytes_per_push += kv_bytes
    floor = (per_push_nodes + per_push_copies) * b_us + bytes_per_push / (HBM_PEAK * 1e9) * 1e6
    return dict(bound="latency", achieved=round(p50_us, 2), peak=round(floor, 2), unit="us/push",
                frac=round(floor / p50_us, 4), traffic=None,
                model={"encoder_runs_per_push": round(enc_runs / max(pushes, 1), 4),
                       "decoder_runs_per_push": round(dec_runs / max(pushes, 1), 4),
                       "encoder_graph_nodes": ne, "decoder_graph_nodes": nd,
                       "device_ops_per_push": round(per_push_nodes + per_push_copies, 2),
                       "kernel_boundary_us": round(b_us, 3),
                       "weight_bytes_per_push": int(bytes_per_push - kv_bytes),
                       "kv_history_bytes_per_push": int(kv_bytes),
                       "input": "audio" if audio else "feature rows",
                       "floor": "(graph nodes + copies per push) x measured dependent-kernel boundary "
                                "(replayed hipGraph of trivial kernels) + (weight + K|V history bytes) per push "
                                "/ 8 TB/s"})


def fseend_oracle_parity(meeting, sd_np, gpu_scores, frames=1000):
    """FS-EEND scores (fs_eend.py:79-96; activity = score > 0, i.e. sigmoid > 0.5, loss.py:214) of the
    product path vs the fp32 CPU oracle (oracle/eend_ref.py frontend + oracle/fseend_ref.py test()) on the
    first `frames` model frames of the same recording (the oracle sees only those frames, so its last 9
    lack their look-ahead and are not compared)."""
    import torch
    from oracle import eend_ref, fseend_ref
    from speaker_diarization_amd.weights import FSEENDConfig, to_torch
    torch.set_num_threads(host_threads())
    Y = eend_ref.features(meeting.wav[: frames * 800 + 700].astype(np.float64), 8000, 200, 80, 7, 10, "logmel23")
    Tn = min(frames, len(Y))
    x = torch.from_numpy(np.ascontiguousarray(Y[:Tn], np.float32))[None]
    with torch.no_grad():
        ro = fseend_ref.fseend_test(to_torch(sd_np), FSEENDConfig(), x, [Tn], 6)[0][0].numpy()
    n = Tn - 9
    g = gpu_scores[:n].float().cpu().numpy()
    c = ro[:n]
    d = np.abs(g.astype(np.float64) - c)
    return {"frames_compared": int(n), "slots": int(g.shape[1]), "max_abs_diff": float(d.max()),
            "mean_abs_diff": float(d.mean()), "decision_flips_at_0": int(((g > 0) != (c > 0)).sum()),
            "decisions": int(g.size), "reference": "oracle/fseend_ref.py test() on oracle/eend_ref.py features, fp32"}


if __name__ == "__main__":
    _a = parse()
    if _a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no external launcher: start the N ranks here (this process never touches the GPU)
        sys.exit(launch_ranks(_a.gpus, sys.argv[1:]))
    _world = int(os.environ.get("WORLD_SIZE", "1"))
    if _world != _a.gpus:
        print(f"[bench] --gpus {_a.gpus} but the launcher started {_world} ranks; using {_world}", file=sys.stderr)
    if _a.workload is None:
        _a.workload = "c4" if _world > 1 else "c2"
    if _a.workload == "dist_check":
        main_dist_check(_a)
        sys.exit(0)
    _wl = WORKLOADS[_a.workload]
    if _wl.get("kind") == "fseend_stream":
        main_stream(_a, _wl)
    elif _wl.get("kind") in ("eda", "fseend", "embed", "tsvad_stream"):
        main_eend(_a, _wl)
    else:
        main(_a, _wl)
