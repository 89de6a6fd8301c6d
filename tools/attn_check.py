"""Max-abs error of sd_op_attention (bf16 path) vs torch fp32 on a few shapes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from speaker_diarization_amd import _lib  # noqa: E402


def ref_attn(qkv, S, T, D, nh, causal):
    q, k, v = qkv.view(S, T, 3, nh, D // nh).permute(2, 0, 3, 1, 4)
    return F.scaled_dot_product_attention(q, k, v, is_causal=bool(causal)).permute(0, 2, 1, 3).reshape(S * T, D)


for S, T, D, nh, causal in [(2, 157, 256, 4, 0), (2, 150, 384, 8, 0), (40, 6, 256, 4, 0), (2, 64, 256, 4, 0),
                            (2, 32, 384, 8, 0), (2, 16, 256, 4, 0)]:
    g = torch.Generator().manual_seed(T)
    qkv = torch.randn(S * T, 3 * D, generator=g)
    ref = ref_attn(qkv, S, T, D, nh, causal)
    dev = torch.device("cuda", 0)
    out = torch.empty(S * T, D, device=dev)
    _lib.call("sd_op_attention", qkv.to(dev).data_ptr(), S, T, D, nh, causal, 0, None, out.data_ptr(), 2,
              _lib.stream_ptr(dev))
    torch.cuda.synchronize()
    err = (out.cpu() - ref).abs()
    print(S, T, D, nh, causal, "max", float(err.max()), "mean", float(err.mean()), "argmax row",
          int(err.max(1).values.argmax()) % T)
