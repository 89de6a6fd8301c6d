"""Microbenchmark of the encoder GEMM shapes through sd_op_gemm_bf16 (the C2 conformer linears:
M = 640 windows x 4 speakers x 150 frames = 384000 rows... 360000 in the bench plan).
Prints per-shape kernel time from HIP events; run under rocprofv3 for counters.

    python tools/gemm_micro.py [--reps 10] [--shapes 384x512,1152x384]
"""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from speaker_diarization_amd import _lib
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--M", type=int, default=360000)
    ap.add_argument("--shapes", default="384x512,1152x384,512x384,384x384,768x384")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    for sh in a.shapes.split(","):
        N, K = (int(v) for v in sh.split("x"))
        x = (torch.randn(a.M, K, device=dev) * 0.5).to(torch.bfloat16)
        w = torch.randn(N, K, device=dev) / K ** 0.5
        out = torch.empty(a.M, N, device=dev, dtype=torch.bfloat16)
        st = _lib.stream_ptr(dev)
        args = (_lib.ptr(x), a.M, K, K, 0, _lib.ptr(w), N, None, None, None, None, 0, _lib.ptr(out), N, st)
        _lib.call("sd_op_gemm_bf16", *args)
        torch.cuda.synchronize()
        lib.sd_prof_reset()
        lib.sd_prof_enable(1)
        for _ in range(a.reps):
            _lib.call("sd_op_gemm_bf16", *args)
        torch.cuda.synchronize()
        lib.sd_prof_enable(0)
        stats = _lib.prof_stats()
        lib.sd_prof_reset()
        ms = sum(v["ms"] for k, v in stats.items() if "gemm" in k) / a.reps
        flops = 2.0 * a.M * N * K
        byts = 2.0 * a.M * (K + N)
        print(f"N={N:5d} K={K:4d}: {ms * 1e3:8.1f} us  {flops / ms / 1e9:7.1f} TF/s  {byts / ms / 1e6:7.1f} GB/s "
              f"({', '.join(sorted(stats))})", flush=True)
        # correctness over the whole output (bf16 inputs, fp32 accumulate, bf16 store)
        ref = x.float() @ w.to(torch.bfloat16).float().t()
        err = (out.float() - ref).abs().max().item()
        tol = 0.02 * ref.abs().max().item() + 1e-2
        print(f"    max|err| = {err:.3e} (tol {tol:.3e})", flush=True)
        assert err < tol, err
        del ref


if __name__ == "__main__":
    main()
