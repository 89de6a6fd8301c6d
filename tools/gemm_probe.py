"""GEMM probe: time conv_gemm's bf16 path (sd_op_linear, precision 2) on given shapes.

    python tools/gemm_probe.py 153600x512x384 38400x2048x1536 ...
Prints per-shape kernel time (HIP events inside libsdiar) and TF/s / GB/s.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from speaker_diarization_amd import _lib  # noqa: E402


def probe(M, N, K, reps=10, act=0):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(M + N + K)   # the same operands in every process (A/B hashes)
    x = torch.randn(M, K, device=dev, generator=g)
    w = torch.randn(N, K, device=dev, generator=g) / K ** 0.5
    b = torch.randn(N, device=dev, generator=g)
    out = torch.empty(M, N, device=dev)
    st = _lib.stream_ptr(dev)
    lib = _lib.load()
    _lib.call("sd_op_linear", _lib.ptr(x), M, K, _lib.ptr(w), _lib.ptr(b), N, act, _lib.ptr(out), 2, st)
    torch.cuda.synchronize()
    lib.sd_prof_reset()
    lib.sd_prof_enable(1)
    for _ in range(reps):
        _lib.call("sd_op_linear", _lib.ptr(x), M, K, _lib.ptr(w), _lib.ptr(b), N, act, _lib.ptr(out), 2, st)
    torch.cuda.synchronize()
    lib.sd_prof_enable(0)
    s = _lib.prof_stats()
    import hashlib
    print("out sha256", hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16], flush=True)
    for key, g in s.items():   # keyed by the GEMM path that ran (gemm_ring, gemm_dma, ...)
        if not key.startswith("gemm") or not g["launches"]:
            continue
        us = g["ms"] / g["launches"] * 1e3
        tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
        gbs = (M * K * 2 + N * K * 2 + M * N * 4) / (us * 1e-6) / 1e9
        print(f"{key} M={M:7d} N={N:5d} K={K:5d}: {us:8.1f} us  {tf:7.1f} TF/s  {gbs:7.0f} GB/s (A bf16 + W + out f32)",
              flush=True)
    if os.environ.get("GEMM_PROBE_TORCH"):
        # the library GEMM (hipBLASLt through torch) on the same shape, bf16 in, bf16 / fp32 out
        xb, wb = x.bfloat16(), w.bfloat16()
        for name, fn in (("torch bf16-out", lambda: torch.addmm(b.bfloat16(), xb, wb.t())),
                         ("torch f32-out", lambda: torch.mm(xb, wb.t(), out_dtype=torch.float32))):
            try:
                fn()
            except Exception as e:  # out_dtype may be unsupported on this build
                print(name, "unavailable:", type(e).__name__, str(e)[:80], flush=True)
                continue
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / reps * 1e3
            print(f"{name} M={M:7d} N={N:5d} K={K:5d}: {us:8.1f} us  {2.0 * M * N * K / (us * 1e-6) / 1e12:7.1f} TF/s",
                  flush=True)


if __name__ == "__main__":
    shapes = sys.argv[1:] or ["153600x512x384", "153600x384x512", "153600x1152x384", "38400x2048x1536",
                              "153600x384x384"]
    for s in shapes:
        M, N, K = (int(v) for v in s.split("x"))
        probe(M, N, K)
