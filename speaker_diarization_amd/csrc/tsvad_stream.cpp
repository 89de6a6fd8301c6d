// Chunk-streaming TS-VAD forward on gfx950 (see tsvad_stream.h).
//
//   window fbank (4 T_lab, 80), chunks of 4C frames
//     -> CAM++ get_time_out + speech_down_or_up, batched over the chunks   model.py:1321-1366
//     -> per speaker: [ts | mix] * sqrt(E) + pe[offset - cache_len ..]      model.py:767-777
//        -> 2 pre-LN layers, block-causal attention (chunk, left)          model.py:779-823
//     -> channels j*E + f -> backend_down over each chunk alone            model.py:833-849
//     -> 2 pre-LN layers, block-causal attention -> fc                     model.py:855-882
#include "tsvad_stream.h"

#include <cmath>
#include <functional>

namespace sd {

WenetLayerL TsvadStreamModel::load_layer(const std::string& p) {
  WenetLayerL L;
  const int E = cfg_.embed_dim;
  std::vector<float> w, b;
  for (const char* n : {"linear_q", "linear_k", "linear_v"}) {
    const HostTensor& wt = ps_.get(p + "self_attn." + n + ".weight");
    const HostTensor& bt = ps_.get(p + "self_attn." + n + ".bias");
    SD_CHECK(wt.numel() == (int64_t)E * E && bt.numel() == E, kErrParam, p + "self_attn." + n + " shape");
    w.insert(w.end(), wt.data.begin(), wt.data.end());
    b.insert(b.end(), bt.data.begin(), bt.data.end());
  }
  L.qkv = upload_packed(arena_, w, 3 * E, E, 1, 1, cfg_.bf16);
  L.qkv_b = arena_.upload(b);
  LayerLoader ld{ps_, arena_, cfg_.bf16};
  L.out = ld.packed(p + "self_attn.linear_out.weight");
  L.out_b = ld.up(p + "self_attn.linear_out.bias");
  L.w1 = ld.packed(p + "feed_forward.w_1.weight");
  L.b1 = ld.up(p + "feed_forward.w_1.bias");
  L.w2 = ld.packed(p + "feed_forward.w_2.weight");
  L.b2 = ld.up(p + "feed_forward.w_2.bias");
  SD_CHECK(L.w1.N == cfg_.ffn_dim && L.w2.K == cfg_.ffn_dim, kErrParam, p + "feed_forward width != ffn_dim");
  L.n1g = ld.up(p + "norm1.weight");
  L.n1b = ld.up(p + "norm1.bias");
  L.n2g = ld.up(p + "norm2.weight");
  L.n2b = ld.up(p + "norm2.bias");
  return L;
}

void TsvadStreamModel::finalize() {
  SD_CHECK(!finalized_, kErrState, "finalize called twice");
  SD_CHECK(cfg_.speaker_embed_dim * 2 == cfg_.embed_dim, kErrInvalid,
           "transformer_embed_dim must be 2 * speaker_embed_dim (cat of ts and mix embeddings)");
  const std::string se = "embed.speech_encoder.";
  cam_.load(ps_, arena_, se, cfg_.bf16);
  // CAMPPlus(embedding_size=odim) also holds the pooled head (unused on get_time_out).
  for (const char* k : {"xvector.dense.linear.weight", "xvector.dense.nonlinear.batchnorm.running_mean",
                        "xvector.dense.nonlinear.batchnorm.running_var"})
    ps_.mark(se + k);
  down_ = load_conv_bn(ps_, arena_, cfg_.bf16, "embed.speech_down_or_up.0.weight", "embed.speech_down_or_up.1.bn",
                       "embed.speech_down_or_up.0.bias");
  down_.pre_s = cam_.out_s();
  down_.pre_h = cam_.out_h();
  for (int i = 0; i < cfg_.num_transformer_layer; ++i) {
    single_.push_back(load_layer("single_backend." + std::to_string(i) + "."));
    multi_.push_back(load_layer("multi_backend." + std::to_string(i) + "."));
  }
  backend_down_ = load_conv_bn(ps_, arena_, cfg_.bf16, "backend_down.0.weight", "backend_down.1.bn",
                               "backend_down.0.bias");
  {
    const HostTensor& pe = ps_.get("pos_encoder.pe");
    SD_CHECK(pe.shape.size() == 3 && pe.shape[0] == 1 && pe.shape[2] == cfg_.embed_dim, kErrParam,
             "pos_encoder.pe must be (1, max_len, transformer_embed_dim)");
    pe_len_ = (int)pe.shape[1];
    pe_ = arena_.upload(pe.data);
  }
  fc_ = LayerLoader{ps_, arena_, cfg_.bf16}.linear("fc");
  auto extra = ps_.unused();
  if (!extra.empty()) {
    std::string msg = "Unexpected key(s) in state_dict:";
    for (size_t i = 0; i < extra.size() && i < 8; ++i) msg += " \"" + extra[i] + "\"";
    throw Error{kErrParam, msg};
  }
  // CAM++ workspace by total frames: a window's chunks hold 4 * T_lab fbank frames in all, and
  // the trunk's buffers scale with items x frames (see CamTrunk::alloc).
  const int64_t Tm = (int64_t)cfg_.max_windows * cfg_.max_labels, NS = cfg_.max_num_speaker, E = cfg_.embed_dim;
  cam_.alloc(arena_, (int)Tm, 6);
  const int64_t rows = NS * Tm;
  mix_ = ws(Tm * cfg_.speaker_embed_dim);
  X_ = ws(rows * E);
  Y_ = ws(rows * E);
  QKV_ = ws(rows * 3 * E);
  AO_ = ws(rows * E);
  T1_ = ws(rows * E);
  H_ = ws(rows * cfg_.ffn_dim);
  X2_ = ws(Tm * NS * E);
  finalized_ = true;
}

void TsvadStreamModel::run_layers(const std::vector<WenetLayerL>& Ls, float* X, int S, int T, int chunk, int left,
                                  hipStream_t st) {
  const bool bf = cfg_.bf16;
  const int E = cfg_.embed_dim, nh = cfg_.num_attention_head;
  const int rows = S * T;
  const float eps = 1e-5f;
  const Tens y{Y_, bf}, qkv{QKV_, bf}, ao{AO_, bf}, t1{T1_, bf}, h{H_, bf};
  layernorm(X, rows, E, E, Ls[0].n1g, Ls[0].n1b, eps, Y_, E, bf, st);           // norm1 of layer 0
  for (size_t i = 0; i < Ls.size(); ++i) {
    const WenetLayerL& L = Ls[i];
    conv_gemm(lin(y, rows, E, L.qkv, L.qkv_b, qkv, 3 * E), bf, st);
    AttnArgs a;
    a.qkv = QKV_; a.io_bf16 = bf; a.S = S; a.T = T; a.D = E; a.nh = nh; a.ld_qkv = 3 * E;
    a.out = AO_; a.ldo = E; a.scale = 1.f / std::sqrt((float)(E / nh));
    a.chunk = chunk; a.left = left;
    attention(a, bf, st);
    conv_gemm(lin(ao, rows, E, L.out, L.out_b, t1, E), bf, st);
    add_layernorm(X, T1_, bf, rows, E, L.n2g, L.n2b, eps, true, Y_, bf, st);     // x += attn; y = norm2(x)
    ConvGemmArgs f1 = lin(y, rows, E, L.w1, L.b1, h, cfg_.ffn_dim);
    f1.act = kActRelu;
    conv_gemm(f1, bf, st);
    conv_gemm(lin(h, rows, cfg_.ffn_dim, L.w2, L.b2, t1, E), bf, st);
    // x += ffn, fused with the next layer's norm1 (the last layer's LN output is unused)
    const WenetLayerL& nx = i + 1 < Ls.size() ? Ls[i + 1] : L;
    add_layernorm(X, T1_, bf, rows, E, nx.n1g, nx.n1b, eps, true, Y_, bf, st);
  }
}

void TsvadStreamModel::forward(const float* feats, const float* ts, int B, int T_lab, int chunk, int left,
                               float* logits, hipStream_t st) {
  SD_CHECK(finalized_, kErrState, "model not finalized");
  cam_.raise_if_set();   // an earlier call's cam_dense report
  SD_CHECK(B >= 1 && B <= cfg_.max_windows, kErrInvalid, "windows per call exceed max_windows");
  SD_CHECK(T_lab >= 1 && T_lab <= cfg_.max_labels, kErrInvalid, "label frames exceed max_labels");
  SD_CHECK(chunk >= 1, kErrInvalid, "decoding_chunk_size must be >= 1");
  const bool bf = cfg_.bf16;
  const int E = cfg_.embed_dim, SE = cfg_.speaker_embed_dim, NS = cfg_.max_num_speaker;
  // positional-encoding rows used: start(c) + C <= T_lab + C
  SD_CHECK(T_lab + chunk <= pe_len_, kErrShape, "window longer than pos_encoder max_len");
  const int n_full = T_lab / chunk, tail = T_lab % chunk;
  // Chunk runs: windows are contiguous, so without a tail every window's chunks form one run of
  // B * n_full equal chunks; with a tail, each window's full chunks and its tail are separate runs.
  // ---- embed: CAM++ (get_time_out) + speech_down_or_up per chunk (chunk c of the window holds
  // fbank rows 4Cc .. 4C(c+1) and label rows Cc .. C(c+1))
  auto embed = [&](int64_t lab0, int nb, int C) {
    const Tens x4 = cam_.forward(feats + lab0 * 4 * 80, nb, 4 * C, st);
    ConvGemmArgs p = cam_conv1d(x4, nb, CamTrunk::out_frames(4 * C), CamTrunk::kChannels, down_, 2, 2, 1,
                                Tens{mix_ + lab0 * SE, false}, SE);
    p.act = kActRelu;
    SD_CHECK(p.Wo == C, kErrShape, "label and ref_speech(mix speech) diff");
    conv_gemm(p, bf, st);
  };
  // ---- backend_down over each chunk alone (zero padding at the chunk edges)
  auto down = [&](int64_t lab0, int nb, int C) {
    ConvGemmArgs p = cam_conv1d(act_at(Tens{X2_, bf}, lab0 * NS * E), nb, C, NS * E, backend_down_, 1, 2, 1,
                                Tens{X_ + lab0 * E, false}, E);
    p.act = kActRelu;
    conv_gemm(p, bf, st);
  };
  auto per_chunk_runs = [&](const std::function<void(int64_t, int, int)>& f) {
    if (!tail) {
      f(0, B * n_full, chunk);
      return;
    }
    for (int b = 0; b < B; ++b) {
      const int64_t w0 = (int64_t)b * T_lab;
      if (n_full) f(w0, n_full, chunk);
      f(w0 + (int64_t)n_full * chunk, 1, tail);
    }
  };
  per_chunk_runs(embed);
  // ---- per-speaker encoder over S = B * NS sequences of T_lab tokens
  build_stream_input(ts, mix_, B, T_lab, NS, SE, std::sqrt((float)E), pe_, chunk, left, X_, st);
  run_layers(single_, X_, B * NS, T_lab, chunk, left, st);
  speakers_to_channels(X_, B, NS, T_lab, E, X2_, bf, st);
  per_chunk_runs(down);
  // ---- multi-speaker encoder (no positional encoding: model.py:853-858) + fc
  run_layers(multi_, X_, B, T_lab, chunk, left, st);
  ConvGemmArgs f = cam_conv1d(Tens{X_, false}, B, T_lab, E, fc_, 1, 0, 1, Tens{logits, false}, 1);
  f.o_sb = (int64_t)NS * T_lab; f.o_sw = 1; f.o_sn = T_lab;
  conv_gemm(f, bf, st);
}

}  // namespace sd
