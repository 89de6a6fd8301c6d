"""Print per-kernel (and per-GEMM-shape with SDIAR_PROF_DETAIL=1) timing of one pipeline step.
    python tools/kernel_table.py [variant 0|1] [minutes] [precision bf16|fp32|bf16x3]"""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))   # the repo root
import torch
from speaker_diarization_amd import _lib
from speaker_diarization_amd.synth import make_meeting, speaker_embeddings
from speaker_diarization_amd.ts_vad.model import TSVADModel
from speaker_diarization_amd.ts_vad.pipeline import TSVADPipeline
from speaker_diarization_amd.weights import TSVADConfig, to_torch, tsvad_state_dict

variant = int(sys.argv[1]) if len(sys.argv) > 1 else 1
minutes = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
precision = sys.argv[3] if len(sys.argv) > 3 else "bf16"
cfg = TSVADConfig(rs_len=4) if variant == 0 else TSVADConfig.ots_vad_v1(rs_len=6)
dev = torch.device("cuda", 0)
m = TSVADModel(cfg, device=dev, precision=precision, max_batch=int(os.environ.get("SDIAR_MAX_BATCH", "640")))
m.load_state_dict(to_torch(tsvad_state_dict(cfg, seed=777)))
pipe = TSVADPipeline(m, 1, 64)
mt = make_meeting(minutes * 60, 4, seed=777)
wav = torch.from_numpy(mt.wav).to(dev)
ts = torch.from_numpy(speaker_embeddings(4)).to(dev)
pipe.posteriors(wav, ts); torch.cuda.synchronize()
lib = _lib.load(); lib.sd_prof_reset(); lib.sd_prof_enable(1)
pipe.posteriors(wav, ts); torch.cuda.synchronize()
lib.sd_prof_enable(0)
st = _lib.prof_stats()
tot = sum(v["ms"] for v in st.values())
print(f"total kernel ms {tot:.2f}")
for k, v in sorted(st.items(), key=lambda kv: -kv[1]["ms"]):
    tf = v["flops"] / (v["ms"] * 1e-3) / 1e12 if v["ms"] else 0
    gbs = v["bytes"] / (v["ms"] * 1e-3) / 1e9 if v["ms"] else 0
    print(f"{v['ms']:8.2f} ms {100*v['ms']/tot:5.1f}% n={v['launches']:5d} {tf:7.1f} TF/s {gbs:7.0f} GB/s  {k}")
