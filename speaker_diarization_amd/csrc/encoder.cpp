// Shared encoder layers (see encoder.h).
#include "encoder.h"

#include <algorithm>
#include <cmath>

namespace sd {

ConvGemmArgs lin(Tens A, int M, int lda, const PackedW& w, const float* bias, Tens out, int ldo) {
  ConvGemmArgs p = linear_args(A.p, M, w.K, lda, w.w, w.N, out.p, ldo);
  p.a_bf16 = A.bf;
  p.out_bf16 = out.bf;
  p.beta = bias;
  return p;
}

const float* LayerLoader::up(const std::string& key) { return arena.upload(ps.get(key).data); }

PackedW LayerLoader::packed(const std::string& key, float mult) {
  int N, Cin, kh, kw;
  auto w = ps.pack(key, N, Cin, kh, kw, mult);
  return upload_packed(arena, w, N, Cin, kh, kw, bf16);
}

ConvL LayerLoader::linear(const std::string& prefix, float mult) {
  ConvL L;
  L.w = packed(prefix + ".weight", mult);
  // nn.Linear / Conv1d(bias=True): the bias key is required (strict load).
  std::vector<float> b = ps.get(prefix + ".bias").data;
  for (auto& v : b) v *= mult;
  L.beta = arena.upload(b);
  return L;
}

TransformerL LayerLoader::transformer(const std::string& p) {
  // torch/nn/modules/transformer.py TransformerEncoderLayer; nn.MultiheadAttention
  // keeps its packed projection as in_proj_weight / in_proj_bias.
  TransformerL L;
  L.in_proj = packed(p + ".self_attn.in_proj_weight");
  L.in_b = up(p + ".self_attn.in_proj_bias");
  ConvL o = linear(p + ".self_attn.out_proj");
  L.out_proj = o.w; L.out_b = o.beta;
  ConvL l1 = linear(p + ".linear1");
  L.l1 = l1.w; L.b1 = l1.beta;
  ConvL l2 = linear(p + ".linear2");
  L.l2 = l2.w; L.b2 = l2.beta;
  L.n1g = up(p + ".norm1.weight");
  L.n1b = up(p + ".norm1.bias");
  L.n2g = up(p + ".norm2.weight");
  L.n2b = up(p + ".norm2.bias");
  return L;
}

ConformerL LayerLoader::conformer(const std::string& p, bool group_norm) {
  // torchaudio/models/conformer.py (2.5.1): ffn1 -> self-attn -> conv module -> ffn2 -> LN.
  ConformerL L;
  L.group_norm = group_norm;
  // ffn: sequential.0 LayerNorm, .1 Linear, .2 SiLU, .4 Linear; residual x*0.5 folded into .4 (exact).
  L.f1_lng = up(p + ".ffn1.sequential.0.weight"); L.f1_lnb = up(p + ".ffn1.sequential.0.bias");
  { ConvL a = linear(p + ".ffn1.sequential.1"); L.f1_w1 = a.w; L.f1_b1 = a.beta; }
  { ConvL a = linear(p + ".ffn1.sequential.4", 0.5f); L.f1_w2 = a.w; L.f1_b2 = a.beta; }
  L.at_lng = up(p + ".self_attn_layer_norm.weight"); L.at_lnb = up(p + ".self_attn_layer_norm.bias");
  L.in_proj = packed(p + ".self_attn.in_proj_weight");
  L.in_b = up(p + ".self_attn.in_proj_bias");
  { ConvL a = linear(p + ".self_attn.out_proj"); L.out_proj = a.w; L.out_b = a.beta; }
  L.cv_lng = up(p + ".conv_module.layer_norm.weight"); L.cv_lnb = up(p + ".conv_module.layer_norm.bias");
  {
    // pointwise_conv1 (2C out) with its rows interleaved [16 values | 16 gates] so a GEMM
    // tile holds each channel's value and gate together (GLU epilogue / glu_dwconv).
    int N, Cin, kh, kw;
    const std::vector<float> w = ps.pack(p + ".conv_module.sequential.0.weight", N, Cin, kh, kw);
    const std::vector<float>& b = ps.get(p + ".conv_module.sequential.0.bias").data;
    SD_CHECK(N % 32 == 0 && (int)b.size() == N, kErrParam, "conv_module.sequential.0 shape");
    const int C = N / 2;
    const size_t K = w.size() / N;
    std::vector<float> wp(w.size()), bp(N);
    for (int r = 0; r < N; ++r) {
      const int r2 = glu_interleave_row(r, C);
      std::copy(w.begin() + r * K, w.begin() + (r + 1) * K, wp.begin() + r2 * K);
      bp[r2] = b[r];
    }
    L.pw1 = upload_packed(arena, wp, N, Cin, kh, kw, bf16);
    L.pw1_b = arena.upload(bp);
  }
  {
    const HostTensor& dw = ps.get(p + ".conv_module.sequential.2.weight");  // (C, 1, k)
    SD_CHECK(dw.shape.size() == 3 && dw.shape[1] == 1, kErrParam, "depthwise conv weight shape");
    std::vector<float> w = dw.data, b = ps.get(p + ".conv_module.sequential.2.bias").data;
    if (group_norm) {
      L.gn_g = up(p + ".conv_module.sequential.3.weight");
      L.gn_b = up(p + ".conv_module.sequential.3.bias");
    } else {
      // eval BatchNorm1d after the depthwise conv: fold into its weight/bias.
      std::vector<float> s, h;
      ps.bn_fold(p + ".conv_module.sequential.3", s, h);
      const int64_t C = dw.shape[0], k = dw.shape[2];
      for (int64_t c = 0; c < C; ++c) {
        for (int64_t j = 0; j < k; ++j) w[c * k + j] *= s[c];
        b[c] = b[c] * s[c] + h[c];
      }
      L.gn_g = L.gn_b = nullptr;
    }
    L.dw_w = arena.upload(w);
    L.dw_b = arena.upload(b);
  }
  { ConvL a = linear(p + ".conv_module.sequential.5"); L.pw2 = a.w; L.pw2_b = a.beta; }
  L.f2_lng = up(p + ".ffn2.sequential.0.weight"); L.f2_lnb = up(p + ".ffn2.sequential.0.bias");
  { ConvL a = linear(p + ".ffn2.sequential.1"); L.f2_w1 = a.w; L.f2_b1 = a.beta; }
  { ConvL a = linear(p + ".ffn2.sequential.4", 0.5f); L.f2_w2 = a.w; L.f2_b2 = a.beta; }
  L.fin_g = up(p + ".final_layer_norm.weight"); L.fin_b = up(p + ".final_layer_norm.bias");
  if (bf16 && rowprog_supported(L.out_proj.N, L.f1_w1.N, true) && L.f2_w1.N == L.f1_w1.N &&
      L.pw2.N == L.out_proj.N && L.pw2.K == L.out_proj.N) {
    auto put = [&](const std::vector<uint16_t>& h) {
      void* d = arena.alloc(h.size() * 2);
      SD_HIP(hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice));
      return static_cast<const void*>(d);
    };
    auto w32 = [&](const std::string& key, float mult) {
      int N, Cin, kh, kw;
      return ps.pack(key, N, Cin, kh, kw, mult);
    };
    const int E = L.out_proj.N, Hd = L.f1_w1.N;
    L.rp_hidden = Hd;
    for (int f = 1; f <= 2; ++f) {
      const std::string q = p + ".ffn" + std::to_string(f) + ".sequential.";
      std::vector<float> b1;
      const void* w = put(rowprog_pack_ffn(w32(q + "1.weight", 1.f), w32(q + "4.weight", 0.5f), Hd, ps.get(q + "0.weight").data,
                                           ps.get(q + "0.bias").data, ps.get(q + "1.bias").data, b1));
      (f == 1 ? L.rp_f1 : L.rp_f2) = w;
      (f == 1 ? L.rp_f1_b1 : L.rp_f2_b1) = arena.upload(b1);
    }
    L.rp_out = put(rowprog_pack_pre(w32(p + ".self_attn.out_proj.weight", 1.f), E, E));
    L.rp_pw2 = put(rowprog_pack_pre(w32(p + ".conv_module.sequential.5.weight", 1.f), E, E));
  }
  return L;
}

void ffn_down_add_ln(const ConvGemmArgs& pd, void* hbuf, float* X, const float* g, const float* b, bool bf,
                     uint16_t* xb, hipStream_t st, bool split_k) {
  // X = LN(X + FFN-down(h)).  Short-M, long-K shapes (M 6000, K 2048) run split-K into fp32 slabs that the
  // LayerNorm sums; the slabs live in the hidden buffer's unused upper half (the bf16 hidden layer takes
  // rows * K * 2 of its rows * K * 4 bytes).
  const int rows = pd.B * pd.Ho * pd.Wo, E = pd.N;
  const int ks = bf && split_k ? gemm_splitk_count(pd) : 1;
  if (ks > 1 && (int64_t)ks * E * 4 <= (int64_t)pd.K * 2 && pd.K % 8 == 0) {
    float* slabs = reinterpret_cast<float*>(static_cast<uint16_t*>(hbuf) + (int64_t)rows * pd.K);
    conv_gemm_splitk(pd, ks, slabs, st);
    add_layernorm(X, slabs, false, rows, E, g, b, 1e-5f, false, X, false, st, xb, ks);
    return;
  }
  conv_gemm(pd, bf, st);
  add_layernorm(X, pd.out, bf, rows, E, g, b, 1e-5f, false, X, false, st, xb);
}

void run_transformer(const TransformerL& L, float* X, int S, int T, int E, int nh, const int* key_len,
                     const EncoderWork& w, hipStream_t st, int causal, int causal_delay, bool xb_in) {
  // nn.TransformerEncoderLayer, post-LN: X = LN1(X + SA(X)); X = LN2(X + FFN(X)).
  // X is the fp32 residual stream; the sub-block outputs t (bf16 in bf16 mode) are added
  // inside the LayerNorm kernel, so every GEMM epilogue only stores.  In bf16 mode both LNs also
  // write bf16(X) into AO (dead between the out-projection and the next attention), the A operand
  // of the GEMMs that read X: the bf16 GEMM paths take bf16 A (an fp32 A is rounded the same way
  // inside the slow register-staged kernel).  xb_in: AO already holds bf16(X) (the previous layer).
  const int rows = S * T;
  const bool bf = w.bf16;
  const Tens x{X, false}, t{w.Y, bf}, qkv{w.QKV, bf}, ao{w.AO, bf}, h{w.H, bf};
  uint16_t* xb = bf ? reinterpret_cast<uint16_t*>(w.AO) : nullptr;
  const Tens xa = bf ? Tens{xb, true} : x;
  conv_gemm(lin(bf && xb_in ? xa : x, rows, E, L.in_proj, L.in_b, qkv, 3 * E), bf, st);
  AttnArgs a;
  a.qkv = qkv.p; a.io_bf16 = bf; a.S = S; a.T = T; a.D = E; a.nh = nh; a.ld_qkv = 3 * E;
  a.out = ao.p; a.ldo = E; a.scale = 1.f / std::sqrt((float)(E / nh));
  a.key_len = key_len;
  a.causal = causal;
  a.causal_delay = causal_delay;
  attention(a, bf, st);
  conv_gemm(lin(ao, rows, E, L.out_proj, L.out_b, t, E), bf, st);
  add_layernorm(X, t.p, bf, rows, E, L.n1g, L.n1b, 1e-5f, false, X, false, st, xb);
  ConvGemmArgs p = lin(xa, rows, E, L.l1, L.b1, h, L.l1.N);
  p.act = kActRelu;
  conv_gemm(p, bf, st);
  ffn_down_add_ln(lin(h, rows, L.l1.N, L.l2, L.b2, t, E), w.H, X, L.n2g, L.n2b, bf, xb, st, w.split_k);
}

void run_conformer(const ConformerL& L, float* X, int S, int T, int E, int nh, int kernel,
                   const int* key_len, const EncoderWork& w, hipStream_t st) {
  // torchaudio ConformerLayer (pre-LN): X fp32 residual stream.  Each sub-block's output t
  // (into the LN-output buffer, which is dead by then) is added to X by the NEXT
  // LayerNorm (add_layernorm writes X += t and y = LN(X)); the last one is the final LN.
  const int rows = S * T;
  const bool bf = w.bf16;
  const Tens y{w.Y, bf}, qkv{w.QKV, bf}, ao{w.AO, bf}, h{w.H, bf};
  auto ffn_body = [&](const PackedW& w1, const float* b1, const PackedW& w2, const float* b2) {
    ConvGemmArgs p = lin(y, rows, E, w1, b1, h, w1.N);
    p.act = kActSilu;
    conv_gemm(p, bf, st);
    conv_gemm(lin(h, rows, w1.N, w2, b2, y, E), bf, st);   // weights pre-scaled by 0.5
  };
  // ffn1
  layernorm(X, rows, E, E, L.f1_lng, L.f1_lnb, 1e-5f, y.p, E, bf, st);
  ffn_body(L.f1_w1, L.f1_b1, L.f1_w2, L.f1_b2);
  // self attention block (key_padding_mask from lengths)
  if (mha_block_supported(E, nh, T, bf)) {
    // in-projection + attention in one launch (mha_block.hip) on the LayerNorm'd rows
    add_layernorm(X, y.p, bf, rows, E, L.at_lng, L.at_lnb, 1e-5f, true, y.p, bf, st);
    MhaBlockArgs m;
    m.y = y.p;
    m.ln_g = L.at_lng; m.ln_b = L.at_lnb; m.eps = 1e-5f;
    m.W = L.in_proj.w; m.bias = L.in_b; m.out = ao.p; m.ldo = E;
    m.S = S; m.T = T; m.D = E; m.nh = nh; m.scale = 1.f / std::sqrt((float)(E / nh)); m.key_len = key_len;
    mha_block(m, st);
  } else {
    add_layernorm(X, y.p, bf, rows, E, L.at_lng, L.at_lnb, 1e-5f, true, y.p, bf, st);
    conv_gemm(lin(y, rows, E, L.in_proj, L.in_b, qkv, 3 * E), bf, st);
    AttnArgs a;
    a.qkv = qkv.p; a.io_bf16 = bf; a.S = S; a.T = T; a.D = E; a.nh = nh; a.ld_qkv = 3 * E;
    a.out = ao.p; a.ldo = E; a.scale = 1.f / std::sqrt((float)(E / nh));
    a.key_len = key_len;
    attention(a, bf, st);
  }
  conv_gemm(lin(ao, rows, E, L.out_proj, L.out_b, y, E), bf, st);
  // convolution module (no padding mask in torchaudio's conv module)
  add_layernorm(X, y.p, bf, rows, E, L.cv_lng, L.cv_lnb, 1e-5f, true, y.p, bf, st);
  // pointwise_conv1 + GLU: fused into the streaming GEMM's epilogue when it runs (bf16),
  // otherwise applied by the depthwise-conv kernel on load.
  ConvGemmArgs p1 = lin(y, rows, E, L.pw1, L.pw1_b, h, E);
  p1.glu = 1;
  const bool glu_epi = bf && gemm_stream_supported(p1);
  if (!glu_epi) {
    p1 = lin(y, rows, E, L.pw1, L.pw1_b, h, 2 * E);
  }
  conv_gemm(p1, bf, st);
  glu_dwconv(h.p, S, T, E, L.dw_w, L.dw_b, kernel, ao.p, L.group_norm ? w.partial : nullptr, !L.group_norm,
             !glu_epi, bf, st);
  if (L.group_norm) groupnorm_silu(ao.p, S, T, E, w.partial, L.gn_g, L.gn_b, 1e-5f, bf, st);
  conv_gemm(lin(ao, rows, E, L.pw2, L.pw2_b, y, E), bf, st);
  // ffn2 + final LayerNorm
  add_layernorm(X, y.p, bf, rows, E, L.f2_lng, L.f2_lnb, 1e-5f, true, y.p, bf, st);
  ffn_body(L.f2_w1, L.f2_b1, L.f2_w2, L.f2_b2);
  add_layernorm(X, y.p, bf, rows, E, L.fin_g, L.fin_b, 1e-5f, false, X, false, st);
}

bool conformer_stack_fused(const std::vector<ConformerL>& Ls, int E, bool bf16) {
  bool fused = bf16 && !Ls.empty() && E == 384;
  for (const ConformerL& L : Ls) fused = fused && L.rp_f1 && rowprog_supported(E, L.rp_hidden, true);
  return fused;
}

void run_conformer_stack(const std::vector<ConformerL>& Ls, float* X, int S, int T, int E, int nh, int kernel,
                         const int* key_len, const EncoderWork& w, hipStream_t st, const SpeakerStreams* io) {
  const bool fused = conformer_stack_fused(Ls, E, w.bf16);
  SD_CHECK(!io || fused, kErrInvalid, "run_conformer_stack: speaker streams need the fused stack");
  if (!fused) {
    for (const ConformerL& L : Ls) run_conformer(L, X, S, T, E, nh, kernel, key_len, w, st);
    return;
  }
  // Per layer: [ffn1 + attn-LN] (first layer only; later layers get it from the previous program) ->
  // attention on y -> [out_proj + residual + conv-LN] -> pw1/GLU -> dwconv (-> GroupNorm+SiLU) ->
  // [pw2 + residual + ffn2 + final LN (+ next layer's ffn1 + attn-LN)].  X stays the fp32 residual stream.
  const int rows = S * T;
  const Tens y{w.Y, true}, qkv{w.QKV, true}, ao{w.AO, true}, h{w.H, true};
  // the residual stream between the row programs in their MFMA-tiled layout (kernels.h RowProgArgs::x_tiled);
  // the caller sees X row-major (or only the speaker-layout output); so does mha_block's attention output and
  // the attention LayerNorm's rows (y of the FFN programs), which go only to mha_block
  const int tiled = rows % 16 == 0;
  const int tiled_a = tiled && mha_block_supported(E, nh, T, true);
  const int tiled_y = tiled_a;
  auto ffn = [](const ConformerL& L, bool second) {
    RowFfnArgs f;
    f.w = second ? L.rp_f2 : L.rp_f1;
    f.hidden = L.rp_hidden;
    f.b1 = second ? L.rp_f2_b1 : L.rp_f1_b1;
    f.b2 = second ? L.f2_b2 : L.f1_b2;
    if (second) { f.post_g = L.fin_g; f.post_b = L.fin_b; }
    return f;
  };
  {
    RowProgArgs r;
    r.X = X; r.Xo = X; r.M = rows;
    if (io) {
      r.X = nullptr; r.x_ts = io->ts; r.x_mix = io->mix; r.x_ldmix = io->ldmix; r.x_Tmix = io->Tmix;
      r.x_NS = io->NS; r.T_seq = T;
    }
    r.n_ffn = 1; r.ffn[0] = ffn(Ls[0], false);
    r.y = y.p; r.y_g = Ls[0].at_lng; r.y_b = Ls[0].at_lnb;
    r.xo_tiled = tiled;
    r.y_tiled = tiled_y;
    rowprog(r, "rowprog_ffn", st);
  }
  for (size_t li = 0; li < Ls.size(); ++li) {
    const ConformerL& L = Ls[li];
    if (mha_block_supported(E, nh, T, true)) {
      MhaBlockArgs m;
      m.y = y.p;
      m.ln_g = L.at_lng; m.ln_b = L.at_lnb; m.eps = 1e-5f;
      m.W = L.in_proj.w; m.bias = L.in_b; m.out = ao.p; m.ldo = E;
      m.S = S; m.T = T; m.D = E; m.nh = nh; m.scale = 1.f / std::sqrt((float)(E / nh)); m.key_len = key_len;
      m.out_tiled = tiled_a;   // read only by the out-projection program below
      m.y_tiled = tiled_y;
      mha_block(m, st);
    } else {
      conv_gemm(lin(y, rows, E, L.in_proj, L.in_b, qkv, 3 * E), true, st);
      AttnArgs a;
      a.qkv = qkv.p; a.io_bf16 = true; a.S = S; a.T = T; a.D = E; a.nh = nh; a.ld_qkv = 3 * E;
      a.out = ao.p; a.ldo = E; a.scale = 1.f / std::sqrt((float)(E / nh));
      a.key_len = key_len;
      attention(a, true, st);
    }
    // pw1 (+ GLU) reads the conv-LN rows the out-projection program writes: tiled when the register-A GEMM
    // takes it
    ConvGemmArgs p1 = lin(y, rows, E, L.pw1, L.pw1_b, h, E);
    p1.glu = 1;
    const bool glu_epi = gemm_stream_supported(p1);
    if (!glu_epi) p1 = lin(y, rows, E, L.pw1, L.pw1_b, h, 2 * E);
    p1.a_tiled = tiled && gemm_areg_supported(p1);
    {
      RowProgArgs r;
      r.X = X; r.Xo = X; r.M = rows;
      r.A = ao.p; r.w0 = L.rp_out; r.b0 = L.out_b;
      r.y = y.p; r.y_g = L.cv_lng; r.y_b = L.cv_lnb;
      r.x_tiled = r.xo_tiled = tiled;
      r.a_tiled = tiled_a;
      r.y_tiled = p1.a_tiled;
      rowprog(r, "rowprog_out", st);
    }
    {
      conv_gemm(p1, true, st);
      glu_dwconv(h.p, S, T, E, L.dw_w, L.dw_b, kernel, ao.p, L.group_norm ? w.partial : nullptr, !L.group_norm,
                 !glu_epi, true, st);
    }
    {
      RowProgArgs r;
      r.X = X; r.Xo = X; r.M = rows;
      r.A = ao.p; r.w0 = L.rp_pw2; r.b0 = L.pw2_b;
      if (L.group_norm) {   // GroupNorm + SiLU applied by the program as it loads A (no separate pass)
        r.gn_partial = w.partial; r.gn_nblk = (E + 63) / 64; r.gn_T = T; r.gn_g = L.gn_g; r.gn_b = L.gn_b;
      }
      r.n_ffn = 1; r.ffn[0] = ffn(L, true);
      r.x_tiled = tiled;
      if (li + 1 < Ls.size()) {
        const ConformerL& Ln = Ls[li + 1];
        r.n_ffn = 2; r.ffn[1] = ffn(Ln, false);
        r.y = y.p; r.y_g = Ln.at_lng; r.y_b = Ln.at_lnb;
        r.xo_tiled = tiled;
        r.y_tiled = tiled_y;
      } else if (io) {
        r.Xo = nullptr; r.yt = io->out; r.yt_NS = io->NS; r.T_seq = T;
      }   // else: the stack's output X, row-major (in place over the tiled input: a tile is read whole first)
      rowprog(r, "rowprog_pw2_ffn", st);
    }
  }
}

}  // namespace sd
