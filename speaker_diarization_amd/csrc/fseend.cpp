// Native FS-EEND forward on gfx950 (OnlineTransformerDADiarization.test, fs_eend.py:79-96).
//
//   feats (S, T, 352) -> BatchNorm1d(345) folded into Linear(345->D) -> LayerNorm      :178-199
//   -> enc_n_layers x TransformerEncoderLayer, causal mask (key j <= i + mask_delay)    :163-171, 200
//   -> zero rows past each length, Conv1d(D, D, 2*delay+1, pad 9) -> emb / |emb|         :82-87
//   -> decoder init convert(cat(emb, slot PE)) = emb·W_embᵀ + (pe_c·W_peᵀ + b)           :125-131, 234-240
//   -> dec_n_layers x the ONE fusion layer on the (T, C) token grid:                    :456-478
//        time attention per slot (causal, token stride C) + LN11,
//        slot attention per frame (C tokens) + LN21, FFN + LN22
//   -> preds[t, c] = emb[t]·att[t,c] / |att[t,c]|                                       :88-90
#include "fseend.h"

#include <algorithm>
#include <cmath>

namespace sd {

void FsEendModel::finalize() {
  SD_CHECK(!finalized_, kErrState, "finalize called twice");
  const int D = cfg_.n_units;
  SD_CHECK(D % cfg_.n_heads == 0, kErrInvalid, "n_units must be divisible by n_heads");
  LayerLoader ld{ps_, arena_, cfg_.bf16};
  // BatchNorm1d (eval) folded into the first Linear: W' = W*s, b' = b + W·h (double on the host).
  {
    const HostTensor& w = ps_.get("enc.encoder.weight");
    SD_CHECK(w.shape.size() == 2 && w.shape[0] == D && w.shape[1] == cfg_.in_size, kErrParam,
             "size mismatch for enc.encoder.weight");
    std::vector<float> s, h;
    ps_.bn_fold("enc.bn", s, h);
    const std::vector<float>& b = ps_.get("enc.encoder.bias").data;
    in_ld_ = (cfg_.in_size + 7) / 8 * 8;
    std::vector<float> wp((size_t)D * in_ld_, 0.f), bp(D);
    for (int n = 0; n < D; ++n) {
      double acc = b[n];
      for (int k = 0; k < cfg_.in_size; ++k) {
        const float wv = w.data[(size_t)n * cfg_.in_size + k];
        wp[(size_t)n * in_ld_ + k] = wv * s[k];
        acc += (double)wv * h[k];
      }
      bp[n] = (float)acc;
    }
    in_.w = upload_packed(arena_, wp, D, in_ld_, 1, 1, cfg_.bf16);
    in_.beta = arena_.upload(bp);
  }
  norm_g_ = ld.up("enc.encoder_norm.weight");
  norm_b_ = ld.up("enc.encoder_norm.bias");
  for (int i = 0; i < cfg_.enc_n_layers; ++i)
    enc_.push_back(ld.transformer("enc.transformer_encoder.layers." + std::to_string(i)));
  // cnn
  {
    const HostTensor& cw = ps_.get("cnn.weight");
    SD_CHECK(cw.shape.size() == 3 && cw.shape[2] == 2 * cfg_.conv_delay + 1, kErrParam, "cnn.weight shape");
    cnn_.w = ld.packed("cnn.weight");
    cnn_.beta = ld.up("cnn.bias");
  }
  // Decoder: the unused input projection of MaskedTransformerDecoderModel (:110-111) is
  // still part of the state_dict.
  for (const char* k : {"dec.encoder.weight", "dec.encoder.bias", "dec.encoder_norm.weight", "dec.encoder_norm.bias"})
    ps_.mark(k);
  {
    const HostTensor& cw = ps_.get("dec.convert.weight");  // (D, 2D)
    SD_CHECK(cw.shape.size() == 2 && cw.shape[0] == D && cw.shape[1] == 2 * D, kErrParam,
             "size mismatch for dec.convert.weight");
    const std::vector<float>& cb = ps_.get("dec.convert.bias").data;
    const HostTensor& pe = ps_.get("dec.pos_enc.pe");      // (1, max_len, D)
    SD_CHECK(pe.shape.size() == 3 && pe.shape[2] == D && pe.shape[1] >= cfg_.max_nspks, kErrParam,
             "dec.pos_enc.pe shape");
    std::vector<float> we((size_t)D * D), sb((size_t)cfg_.max_nspks * D);
    for (int n = 0; n < D; ++n)
      for (int k = 0; k < D; ++k) we[(size_t)n * D + k] = cw.data[(size_t)n * 2 * D + k];
    for (int c = 0; c < cfg_.max_nspks; ++c)
      for (int n = 0; n < D; ++n) {
        double acc = cb[n];
        for (int k = 0; k < D; ++k)
          acc += (double)cw.data[(size_t)n * 2 * D + D + k] * pe.data[(size_t)c * D + k];
        sb[(size_t)c * D + n] = (float)acc;
      }
    conv_emb_ = upload_packed(arena_, we, D, D, 1, 1, cfg_.bf16);
    slot_bias_ = arena_.upload(sb);
  }
  // The shared fusion layer: torch's load_state_dict copies every index into the one
  // module, so the LAST index's tensors are the ones in effect.
  for (int i = 0; i + 1 < cfg_.dec_n_layers; ++i) {
    const std::string p = "dec.attractor_decoder." + std::to_string(i) + ".";
    for (const char* k : {"self_attn1.in_proj_weight", "self_attn1.in_proj_bias", "self_attn1.out_proj.weight",
                          "self_attn1.out_proj.bias", "self_attn2.in_proj_weight", "self_attn2.in_proj_bias",
                          "self_attn2.out_proj.weight", "self_attn2.out_proj.bias", "linear1.weight", "linear1.bias",
                          "linear2.weight", "linear2.bias", "norm11.weight", "norm11.bias", "norm12.weight",
                          "norm12.bias", "norm21.weight", "norm21.bias", "norm22.weight", "norm22.bias"}) {
      SD_CHECK(ps_.has(p + k), kErrParam, "Missing key(s) in state_dict: \"" + p + k + "\"");
      ps_.mark(p + k);
    }
  }
  {
    const std::string p = "dec.attractor_decoder." + std::to_string(cfg_.dec_n_layers - 1) + ".";
    fus_.in1 = ld.packed(p + "self_attn1.in_proj_weight");
    fus_.in1_b = ld.up(p + "self_attn1.in_proj_bias");
    { ConvL o = ld.linear(p + "self_attn1.out_proj"); fus_.out1 = o.w; fus_.out1_b = o.beta; }
    fus_.in2 = ld.packed(p + "self_attn2.in_proj_weight");
    fus_.in2_b = ld.up(p + "self_attn2.in_proj_bias");
    { ConvL o = ld.linear(p + "self_attn2.out_proj"); fus_.out2 = o.w; fus_.out2_b = o.beta; }
    { ConvL o = ld.linear(p + "linear1"); fus_.l1 = o.w; fus_.b1 = o.beta; }
    { ConvL o = ld.linear(p + "linear2"); fus_.l2 = o.w; fus_.b2 = o.beta; }
    fus_.n11g = ld.up(p + "norm11.weight"); fus_.n11b = ld.up(p + "norm11.bias");
    ps_.mark(p + "norm12.weight"); ps_.mark(p + "norm12.bias");   // constructed, unused (:461-462)
    fus_.n21g = ld.up(p + "norm21.weight"); fus_.n21b = ld.up(p + "norm21.bias");
    fus_.n22g = ld.up(p + "norm22.weight"); fus_.n22b = ld.up(p + "norm22.bias");
  }
  auto extra = ps_.unused();
  if (!extra.empty()) {
    std::string msg = "Unexpected key(s) in state_dict:";
    for (size_t i = 0; i < extra.size() && i < 8; ++i) msg += " \"" + extra[i] + "\"";
    throw Error{kErrParam, msg};
  }
  const int64_t rows = (int64_t)cfg_.max_seqs * cfg_.max_frames;
  const int64_t grid = rows * cfg_.max_nspks;
  X_ = ws(rows * D);
  Y_ = ws(rows * D);
  EMB_ = ws(rows * D);
  G_ = ws(rows * D);
  A_ = ws(grid * D);
  A2_ = ws(grid * D);
  QKV_ = ws(grid * 3 * D);
  AO_ = ws(grid * D);
  H_ = ws(std::max(grid * cfg_.dec_ffn, rows * (int64_t)cfg_.enc_ffn));
  finalized_ = true;
}

void FsEendModel::run_fusion(float* A, int S, int T, int C, hipStream_t st) {
  // TransformerEncoderFusionLayer.forward, norm_first=False (fs_eend.py:456-478) on rows (s, t, c).
  const int D = cfg_.n_units, nh = cfg_.n_heads;
  const int64_t n = (int64_t)S * T * C;
  const bool bf = cfg_.bf16;
  const Tens t{A2_, bf}, qkv{QKV_, bf}, ao{AO_, bf}, h{H_, bf};
  // bf16 mode: the GEMMs read bf16(A), which every LayerNorm also writes into AO (dead between the
  // out-projection and the next attention); the caller leaves it there before the first layer.
  uint16_t* ab = bf ? reinterpret_cast<uint16_t*>(AO_) : nullptr;
  const Tens a = bf ? Tens{ab, true} : Tens{A, false};
  const float scale = 1.f / std::sqrt((float)(D / nh));
  // (1) attention over time within each slot, causal
  conv_gemm(lin(a, (int)n, D, fus_.in1, fus_.in1_b, qkv, 3 * D), bf, st);
  {
    AttnArgs t;
    t.qkv = qkv.p; t.io_bf16 = bf; t.S = S * C; t.T = T; t.D = D; t.nh = nh; t.ld_qkv = 3 * D;
    t.out = ao.p; t.ldo = D; t.scale = scale;
    t.causal = 1; t.causal_delay = cfg_.mask_delay;
    t.seq_inner = C; t.seq_outer = (int64_t)T * C; t.seq_inner_stride = 1; t.tok_stride = C;
    attention(t, bf, st);
  }
  conv_gemm(lin(ao, (int)n, D, fus_.out1, fus_.out1_b, t, D), bf, st);
  add_layernorm(A, t.p, bf, (int)n, D, fus_.n11g, fus_.n11b, 1e-5f, false, A, false, st, ab);
  // (2) attention over the C slots of each frame, no mask
  conv_gemm(lin(a, (int)n, D, fus_.in2, fus_.in2_b, qkv, 3 * D), bf, st);
  {
    AttnArgs s;
    s.qkv = qkv.p; s.io_bf16 = bf; s.S = S * T; s.T = C; s.D = D; s.nh = nh; s.ld_qkv = 3 * D;
    s.out = ao.p; s.ldo = D; s.scale = scale;
    attention(s, bf, st);
  }
  conv_gemm(lin(ao, (int)n, D, fus_.out2, fus_.out2_b, t, D), bf, st);
  add_layernorm(A, t.p, bf, (int)n, D, fus_.n21g, fus_.n21b, 1e-5f, false, A, false, st, ab);
  // (3) feed-forward
  ConvGemmArgs p = lin(a, (int)n, D, fus_.l1, fus_.b1, h, fus_.l1.N);
  p.act = kActRelu;
  conv_gemm(p, bf, st);
  ffn_down_add_ln(lin(h, (int)n, fus_.l1.N, fus_.l2, fus_.b2, t, D), H_, A, fus_.n22g, fus_.n22b, bf, ab, st, true);
}

void FsEendModel::forward(const float* feats, int ld_in, int S, int T, const int* lengths, int C, float* preds,
                          float* emb_out, float* att_out, hipStream_t st) {
  SD_CHECK(finalized_, kErrState, "model not finalized");
  SD_CHECK(S >= 1 && S <= cfg_.max_seqs, kErrInvalid, "sequences exceed max_seqs");
  SD_CHECK(T >= 1 && T <= cfg_.max_frames, kErrInvalid, "frames exceed max_frames");
  SD_CHECK(C >= 1 && C <= cfg_.max_nspks, kErrInvalid, "max_nspks exceeds the configured maximum");
  SD_CHECK(ld_in >= in_ld_ && ld_in % 4 == 0, kErrInvalid, "feature row stride must be >= in_ld and % 4");
  const int D = cfg_.n_units, rows = S * T;
  const bool bf = cfg_.bf16;
  const EncoderWork w{Y_, QKV_, AO_, H_, nullptr, bf, true};   // replicas only: split-K allowed
  // Encoder
  conv_gemm(lin(Tens{const_cast<float*>(feats), false}, rows, ld_in, in_.w, in_.beta, Tens{Y_, false}, D), bf, st);
  layernorm(Y_, rows, D, D, norm_g_, norm_b_, 1e-5f, X_, D, false, st, bf ? reinterpret_cast<uint16_t*>(AO_) : nullptr);
  for (const auto& L : enc_)
    run_transformer(L, X_, S, T, D, cfg_.n_heads, nullptr, w, st, cfg_.has_mask, cfg_.mask_delay, true);
  // emb[:ilen] re-padded with zeros (:83-84), then the look-ahead conv (:85)
  for (int s = 0; s < S; ++s) {
    const int len = lengths ? lengths[s] : T;
    SD_CHECK(len >= 1 && len <= T, kErrInvalid, "sequence length out of range");
    if (len < T) {
      zero_fill(X_ + ((int64_t)s * T + len) * D, (size_t)(T - len) * D * sizeof(float), st);
      if (bf)   // the encoder's last LayerNorm left bf16(X) in AO_: the conv reads that copy
        zero_fill(reinterpret_cast<uint16_t*>(AO_) + ((int64_t)s * T + len) * D, (size_t)(T - len) * D * sizeof(uint16_t), st);
    }
  }
  int ks = 1;
  {
    ConvGemmArgs p;
    p.A = bf ? static_cast<const void*>(AO_) : X_; p.a_bf16 = bf; p.B = S; p.H = 1; p.W = T; p.Cin = D; p.lda = D; p.a_coff = 0;
    p.kh = 1; p.kw = cnn_.w.kw; p.sh = 1; p.sw = 1; p.ph = 0; p.pw = 9; p.dh = 1; p.dw = 1;
    p.Ho = 1; p.Wo = T + 18 - (cnn_.w.kw - 1);
    SD_CHECK(p.Wo == T, kErrInvalid, "cnn padding 9 requires conv_delay 9 (fs_eend.py:41)");
    p.Wt = cnn_.w.w; p.N = D; p.K = cnn_.w.K;
    p.beta = cnn_.beta;
    p.out = Y_; p.out_bf16 = false;
    p.o_sb = (int64_t)T * D; p.o_sh = 0; p.o_sw = D; p.o_sn = 1;
    // 19 taps x 256 = K 4864 over M = frames: split-K into fp32 slabs in the (now idle) hidden buffer,
    // summed by the L2 normalisation that consumes the conv output
    ks = bf ? gemm_splitk_count(p) : 1;
    if (ks > 1 && ks * D <= cfg_.enc_ffn) conv_gemm_splitk(p, ks, H_, st);
    else {
      ks = 1;
      conv_gemm(p, bf, st);
    }
  }
  float* emb = emb_out ? emb_out : EMB_;
  row_l2norm(ks > 1 ? H_ : Y_, rows, D, emb, st, ks);
  // Decoder
  conv_gemm(lin(Tens{emb, false}, rows, D, conv_emb_, nullptr, Tens{G_, false}, D), bf, st);
  float* A = att_out ? att_out : A_;
  slot_init(G_, rows, C, D, slot_bias_, A, st);
  if (bf) f32_to_bf16(A, (int64_t)rows * C * D, AO_, st);   // run_fusion's bf16(A) operand
  for (int i = 0; i < cfg_.dec_n_layers; ++i) run_fusion(A, S, T, C, st);
  slot_scores(emb, A, rows, C, D, preds, att_out != nullptr, st);
}

}  // namespace sd
