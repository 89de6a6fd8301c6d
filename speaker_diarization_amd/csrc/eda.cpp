// Native EEND-EDA forward on gfx950.
//
//   feats (S, T, 352) -> Linear(345->E) + LayerNorm        models.py:222-224 / 522-523
//   -> L x TransformerEncoderLayer (post-LN, ffn 2048)      models.py:226 / 525 (no key mask)
//      or torchaudio Conformer (BatchNorm conv module)      models.py:527-528 (key mask = ilens)
//   -> emb; shuffled copy emb[randperm(len)]                models.py:229-233 / 532-536
//   -> EDA: encoder LSTM over the shuffled frames (packed lengths) -> (h, c)
//      decoder LSTM over max_n_speakers zero inputs from (h, c)      encoder_decoder_attractor.py:42-50
//   -> probs = sigmoid(linear(att)), act = sigmoid(emb · att[:-1]ᵀ)  :53-58, models.py:324-331
// Speaker selection (sort / first-n / threshold) is host logic on the 15 probs.
#include "eda.h"

#include <algorithm>
#include <cstring>

namespace sd {

void EdaModel::finalize() {
  SD_CHECK(!finalized_, kErrState, "finalize called twice");
  SD_CHECK(cfg_.variant >= 0 && cfg_.variant <= 3, kErrInvalid, "unknown EDA model variant");
  const int E = cfg_.n_units;
  SD_CHECK(E % cfg_.n_heads == 0, kErrInvalid, "n_units must be divisible by n_heads");
  LayerLoader ld{ps_, arena_, cfg_.bf16};
  const bool plain = cfg_.variant == 3;
  const std::string inp = (cfg_.variant == 0 || plain) ? "encoder" : "linear";
  const std::string norm = (cfg_.variant == 0 || plain) ? "encoder_norm" : "linear_norm";
  {
    const HostTensor& w = ps_.get(inp + ".weight");
    SD_CHECK(w.shape.size() == 2 && w.shape[0] == E && w.shape[1] == cfg_.in_size, kErrParam,
             "size mismatch for " + inp + ".weight");
    in_ld_ = (cfg_.in_size + kEdaInPad - 1) / kEdaInPad * kEdaInPad;
    std::vector<float> wp((size_t)E * in_ld_, 0.f);
    for (int n = 0; n < E; ++n)
      std::copy(w.data.begin() + (size_t)n * cfg_.in_size, w.data.begin() + (size_t)(n + 1) * cfg_.in_size,
                wp.begin() + (size_t)n * in_ld_);
    in_.w = upload_packed(arena_, wp, E, in_ld_, 1, 1, cfg_.bf16);
    in_.beta = ld.up(inp + ".bias");
  }
  norm_g_ = ld.up(norm + ".weight");
  norm_b_ = ld.up(norm + ".bias");
  for (int i = 0; i < cfg_.n_layers; ++i) {
    if (cfg_.variant == 0 || plain)
      tfm_.push_back(ld.transformer("transformer_encoder.layers." + std::to_string(i)));
    else if (cfg_.variant == 1)
      tfm_.push_back(ld.transformer("encoder.layers." + std::to_string(i)));
    else
      conf_.push_back(ld.conformer("encoder.conformer_layers." + std::to_string(i), false));
  }
  auto lstm = [&](const std::string& p, const float** b, const float** hh) {
    const HostTensor& wh = ps_.get(p + "weight_hh_l0");
    SD_CHECK(wh.shape.size() == 2 && wh.shape[0] == 4 * E && wh.shape[1] == E, kErrParam,
             "size mismatch for " + p + "weight_hh_l0");
    const HostTensor& bi = ps_.get(p + "bias_ih_l0");
    const HostTensor& bh = ps_.get(p + "bias_hh_l0");
    std::vector<float> bias(bi.data.size());
    for (size_t i = 0; i < bias.size(); ++i) bias[i] = bi.data[i] + bh.data[i];
    *b = arena_.upload(bias);
    *hh = arena_.upload(wh.data);
    // bf16 mode: a bf16 copy feeds the group-persistent recurrence kernel (lstm.hip).  fp32 handles also keep
    // hi = bf16(W) and lo = bf16(W - hi) for the bf16x3 mode's split recurrence (exact fp32 mode uses neither).
    (hh == &enc_hh_ ? enc_hh_bf_ : dec_hh_bf_) = upload_packed(arena_, wh.data, 4 * E, E, 1, 1, true).w;
    if (!cfg_.bf16) (hh == &enc_hh_ ? enc_hh_lo_ : dec_hh_lo_) = upload_bf16_lo(arena_, wh.data);
  };
  if (plain) {
    dec_ = ld.linear("decoder");
    SD_CHECK(dec_.w.N == cfg_.n_speakers, kErrParam, "size mismatch for decoder.weight");
  } else {
    enc_ih_ = ld.packed("eda.encoder.weight_ih_l0");
    lstm("eda.encoder.", &enc_b_, &enc_hh_);
    // The decoder's inputs are zeros (encoder_decoder_attractor.py:50): W_ih never contributes.
    ps_.mark("eda.decoder.weight_ih_l0");
    lstm("eda.decoder.", &dec_b_, &dec_hh_);
    lin_w_ = ld.up("eda.linear.weight");
    lin_b_ = ld.up("eda.linear.bias");
  }
  auto extra = ps_.unused();
  if (!extra.empty()) {
    std::string msg = "Unexpected key(s) in state_dict:";
    for (size_t i = 0; i < extra.size() && i < 8; ++i) msg += " \"" + extra[i] + "\"";
    throw Error{kErrParam, msg};
  }
  // Workspace.
  const int64_t rows = (int64_t)cfg_.max_seqs * cfg_.max_frames;
  X_ = ws(rows * E);
  Y_ = ws(rows * E);
  QKV_ = ws(rows * 3 * E);
  AO_ = ws(rows * E);
  H_ = ws(rows * std::max(cfg_.dim_feedforward, 2 * E));
  partial_ = ws((int64_t)cfg_.max_seqs * ((E + 63) / 64) * 2);
  G_ = ws(rows * 4 * E);
  Gd_ = ws((int64_t)cfg_.max_seqs * cfg_.max_n_speakers * 4 * E);
  att_ = ws((int64_t)cfg_.max_seqs * cfg_.max_n_speakers * E);
  hT_ = ws((int64_t)cfg_.max_seqs * E);
  cT_ = ws((int64_t)cfg_.max_seqs * E);
  lstm_work_ = ws(lstm_work_floats(cfg_.max_seqs, E, 1));
  finalized_ = true;
}

void EdaModel::forward(const float* feats, int ld_in, int S, int T, const int* lengths, const int* key_len,
                       const int* perm, float* probs, float* act, hipStream_t st) {
  SD_CHECK(finalized_, kErrState, "model not finalized");
  lstm_err_.raise_if_set();   // an earlier forward's report nobody collected with sd_eda_status
  SD_CHECK(S >= 1 && S <= cfg_.max_seqs, kErrInvalid, "sequences exceed max_seqs");
  SD_CHECK(T >= 1 && T <= cfg_.max_frames, kErrInvalid, "frames exceed max_frames");
  SD_CHECK(ld_in >= in_ld_ && ld_in % 4 == 0, kErrInvalid, "feature row stride must be >= in_ld and % 4");
  const bool plain = cfg_.variant == 3;
  SD_CHECK(plain || (lengths && perm), kErrInvalid, "lengths and perm are required");
  const int E = cfg_.n_units, rows = S * T, NA = cfg_.max_n_speakers;
  const bool bf = cfg_.bf16;
  // No split-K: its split count depends on the batched M (chunks per forward x T), and EDA chunks are
  // sharded over ranks with activities bit-identical for any world size (test_eda_chunk_shards_bit_identical).
  const EncoderWork w{Y_, QKV_, AO_, H_, partial_, bf, false};
  // Linear + LayerNorm
  conv_gemm(lin(Tens{const_cast<float*>(feats), false}, rows, ld_in, in_.w, in_.beta, Tens{Y_, false}, E), bf, st);
  layernorm(Y_, rows, E, E, norm_g_, norm_b_, 1e-5f, X_, E, false, st);
  // bf16(X) for the first layer's in-projection (later layers get it from the LayerNorms): see tsvad.cpp
  if (bf && !tfm_.empty()) f32_to_bf16(X_, (int64_t)rows * E, AO_, st);
  for (size_t i = 0; i < tfm_.size(); ++i)
    run_transformer(tfm_[i], X_, S, T, E, cfg_.n_heads, key_len, w, st, 0, 0, bf || i > 0);
  run_conformer_stack(conf_, X_, S, T, E, cfg_.n_heads, 31, key_len, w, st);
  if (plain) {   // eend/models.py:97-99: decoder Linear, activation=sigmoid (eend_infer.py:69)
    ConvGemmArgs p = lin(Tens{X_, false}, rows, E, dec_.w, dec_.beta, Tens{act, false}, cfg_.n_speakers);
    p.act = kActSigmoid;
    conv_gemm(p, bf, st);
    return;
  }
  // EDA: shuffle -> encoder LSTM (packed) -> decoder LSTM from (h, c)
  gather_rows(X_, S, T, E, perm, lengths, Y_, st);
  conv_gemm(lin(Tens{Y_, false}, rows, E, enc_ih_, enc_b_, Tens{G_, false}, 4 * E), bf, st);
  // bf16: the bf16 recurrence; bf16x3 (precision 2): the split recurrence; fp32: the exact-f32 step kernel
  const bool x3 = !bf && gemm_x3();
  lstm_recurrence(G_, S, T, E, 1, enc_hh_, lengths, nullptr, nullptr, nullptr, 0, hT_, cT_, lstm_work_, st,
                  bf || x3 ? enc_hh_bf_ : nullptr, lstm_err_.get(0), x3 ? enc_hh_lo_ : nullptr);
  fill_rows(dec_b_, 4 * E, S * NA, Gd_, st);
  lstm_recurrence(Gd_, S, NA, E, 1, dec_hh_, nullptr, hT_, cT_, att_, E, nullptr, nullptr, lstm_work_, st,
                  bf || x3 ? dec_hh_bf_ : nullptr, lstm_err_.get(1), x3 ? dec_hh_lo_ : nullptr);
  attractor_scores(X_, S, T, E, att_, NA, lin_w_, lin_b_, probs, act, st);
}

}  // namespace sd
