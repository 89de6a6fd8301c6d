// Encoder layers shared by the TS-VAD, EEND-EDA and EEND runners:
// nn.TransformerEncoderLayer (post-LN, ReLU) and torchaudio's ConformerLayer,
// with their state_dict loaders.  Activations are channel-last token streams
// (S*T, E); the residual stream X stays fp32, GEMM-only intermediates are bf16
// in bf16 mode.
#pragma once
#include <string>
#include <vector>
#include "kernels.h"
#include "params.h"

namespace sd {

// Activation tensors: fp32, or bf16 bits when the flag is set.
struct Tens {
  void* p;
  bool bf;
};
inline Tens act_at(const Tens& a, int64_t elems) {
  return Tens{static_cast<char*>(a.p) + elems * (a.bf ? 2 : 4), a.bf};
}

// Linear on a row-major activation: out (M, w.N) with row stride ldo.
ConvGemmArgs lin(Tens A, int M, int lda, const PackedW& w, const float* bias, Tens out, int ldo);

struct ConvL {
  PackedW w;
  const float* alpha = nullptr;
  const float* beta = nullptr;
  const float* pre_s = nullptr;
  const float* pre_h = nullptr;
};

struct TransformerL {     // nn.TransformerEncoderLayer, post-LN, ReLU FFN
  PackedW in_proj, out_proj, l1, l2;
  const float *in_b, *out_b, *b1, *b2, *n1g, *n1b, *n2g, *n2b;
};

struct ConformerL {       // torchaudio.models.conformer.ConformerLayer (conv after attention)
  const float *f1_lng, *f1_lnb, *f1_b1, *f1_b2;
  PackedW f1_w1, f1_w2;
  const float *at_lng, *at_lnb, *in_b, *out_b;
  PackedW in_proj, out_proj;
  const float *cv_lng, *cv_lnb, *pw1_b, *dw_w, *dw_b, *gn_g, *gn_b, *pw2_b;
  bool group_norm = true;  // false: BatchNorm1d folded into dw_w / dw_b, SiLU fused into the dwconv
  PackedW pw1, pw2;
  const float *f2_lng, *f2_lnb, *f2_b1, *f2_b2;
  PackedW f2_w1, f2_w2;
  const float *fin_g, *fin_b;
  // rowprog.hip pieces (bf16 mode, D 384): ffn1 / ffn2 (W1 | ½W2), out_proj, pointwise_conv2
  const void *rp_f1 = nullptr, *rp_f2 = nullptr, *rp_out = nullptr, *rp_pw2 = nullptr;
  const float *rp_f1_b1 = nullptr, *rp_f2_b1 = nullptr;   // up-projection biases with the LN shift folded in
  int rp_hidden = 0;
};

// Reads reference state_dict entries (strict: every key it touches is marked used).
struct LayerLoader {
  ParamStore& ps;
  DeviceArena& arena;
  bool bf16;
  const float* up(const std::string& key);
  PackedW packed(const std::string& key, float mult = 1.f);
  ConvL linear(const std::string& prefix, float mult = 1.f);   // weight + required bias
  TransformerL transformer(const std::string& prefix);
  ConformerL conformer(const std::string& prefix, bool group_norm);
};

// Scratch for one encoder layer over up to `rows` tokens.
struct EncoderWork {
  float* Y;        // rows * E (fp32)
  float* QKV;      // rows * 3E
  float* AO;       // rows * E
  float* H;        // rows * max(ffn, 2E)
  float* partial;  // S * cdiv(E, 64) * 2
  bool bf16;
  // Split-K FFN down-projections allowed (their split count depends on the row count, so a model whose
  // rows are sharded over ranks — TS-VAD windows, bit-identical for any world size — leaves this off).
  bool split_k = false;
};

// X: (S*T, E) fp32, updated in place.  key_len: device int32 (S) or nullptr.
// causal: key j visible to query i iff j <= i + causal_delay (fs_eend.py:168-171 mask).
// X = LN(X + pd) for the FFN down-projection pd (split-K into slabs in hbuf's upper half when that pays).
void ffn_down_add_ln(const ConvGemmArgs& pd, void* hbuf, float* X, const float* g, const float* b, bool bf,
                     uint16_t* xb, hipStream_t st, bool split_k);
// bf16 mode leaves bf16(X) in w.AO on return; xb_in: it is there on entry too (consecutive layers).
void run_transformer(const TransformerL& L, float* X, int S, int T, int E, int nh, const int* key_len,
                     const EncoderWork& w, hipStream_t st, int causal = 0, int causal_delay = 0,
                     bool xb_in = false);
void run_conformer(const ConformerL& L, float* X, int S, int T, int E, int nh, int kernel,
                   const int* key_len, const EncoderWork& w, hipStream_t st);
// All layers of a torchaudio Conformer; runs the per-token parts as rowprog.hip programs when every
// layer has its pieces (bf16, D 384), else run_conformer per layer.
// TS-VAD speaker streams around a fused (row-program) conformer stack: the first program builds its input
// rows [ts | mix] on load (no build_speaker_input pass) and the last writes bf16 rows straight into the
// speakers-to-channels layout (no speakers_to_channels pass, no fp32 output).  Only with
// conformer_stack_fused() true.
struct SpeakerStreams {
  const float* ts = nullptr;    // (B*NS, 192)
  const float* mix = nullptr;   // (B, Tmix, ldmix), columns 0..191
  int ldmix = 0, Tmix = 0, NS = 0;
  void* out = nullptr;          // bf16 (B, T, NS*E)
};
bool conformer_stack_fused(const std::vector<ConformerL>& Ls, int E, bool bf16);
void run_conformer_stack(const std::vector<ConformerL>& Ls, float* X, int S, int T, int E, int nh, int kernel,
                         const int* key_len, const EncoderWork& w, hipStream_t st,
                         const SpeakerStreams* io = nullptr);

}  // namespace sd
