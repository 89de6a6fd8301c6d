"""Attention kernel timing on FS-EEND shapes: run under rocprofv3 --kernel-trace --stats and read the
attn_long_kernel rows (the fp32<->bf16 conversions of the C-ABI op show up as their own kernels).
    rocprofv3 --kernel-trace --stats -d gpurun_out/ab -o ab -- python tools/attn_bench.py"""
import sys
import torch
sys.path.insert(0, '.')
from speaker_diarization_amd import _lib  # noqa: E402

dev = torch.device('cuda', 0)
st = _lib.stream_ptr(dev)
# (label, S, T, D, nh, causal): S = 1 is the encoder launch, S = 6 the decoder's per-slot time attention
CASES = [c for c in [("enc", 1, 6000, 256, 4, 1), ("dec", 6, 6000, 256, 4, 1)] if len(sys.argv) < 2 or c[0] in sys.argv[1:]]
for label, S, T, D, nh, causal in CASES:
    qkv = torch.randn(S * T, 3 * D, device=dev)
    out = torch.empty(S * T, D, device=dev)
    for _ in range(10):
        _lib.call("sd_op_attention", qkv.data_ptr(), S, T, D, nh, causal, 0, None, out.data_ptr(), 2, st)
    torch.cuda.synchronize()
    fl = 4.0 * S * nh * T * T * (D // nh) * (0.5 if causal else 1.0)
    print(f"{label}: S={S} T={T} D={D} nh={nh} causal={causal}: {fl / 1e9:.2f} GFLOP per launch")
