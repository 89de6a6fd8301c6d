// Native TS-VAD forward (egs/alimeeting/ts_vad2/model.py) on gfx950.
//
//   ref_speech fbank (B, T_fb, 80)
//     -> CAM++ FCM head + xvector[:-2]       cam_pplus_wespeaker.py:271-399
//     -> speech_down_or_up conv+BN+ReLU      model.py:385-395 / 406-416
//   variant 0 (forward_common, model.py:758-897):
//     -> [ts_embed | mix] + PE, 2-layer transformer per speaker (batched over speakers)
//     -> backend_down conv(1536->384, k5)+BN+ReLU -> PE -> 2-layer transformer -> fc
//   variant 1 (forward_common_ots_vad, model.py:669-756):
//     -> GSP + gsp_fc -> [ts_embed | mix] -> 6-layer Conformer per speaker
//     -> BiLSTM(1536 -> 2x256) -> fc
//   -> logits (B, NS, T_lab)
// All activations are fp32 channel-last; every contraction is conv_gemm (bf16 or
// exact-f32 MFMA), eval BatchNorms are folded into GEMM prologues/epilogues.
#include "tsvad.h"

#include <cmath>

namespace sd {

namespace {

ConvGemmArgs conv1d(Tens in, int B, int T, int lda, const ConvL& L, int stride, int pad, int dil, Tens out,
                    int ldo) {
  ConvGemmArgs p;
  p.A = in.p; p.a_bf16 = in.bf; p.B = B; p.H = 1; p.W = T; p.Cin = L.w.Cin; p.lda = lda; p.a_coff = 0;
  p.kh = 1; p.kw = L.w.kw; p.sh = 1; p.sw = stride; p.ph = 0; p.pw = pad; p.dh = 1; p.dw = dil;
  p.Ho = 1;
  p.Wo = (T + 2 * pad - dil * (L.w.kw - 1) - 1) / stride + 1;
  p.Wt = L.w.w; p.N = L.w.N; p.K = L.w.K;
  p.pre_scale = L.pre_s; p.pre_shift = L.pre_h;
  p.alpha = L.alpha; p.beta = L.beta;
  p.out = out.p; p.out_bf16 = out.bf;
  p.o_sb = (int64_t)p.Wo * ldo; p.o_sh = 0; p.o_sw = ldo; p.o_sn = 1;
  return p;
}

ConvGemmArgs conv2d(Tens in, int B, int H, int W, const ConvL& L, int sh, int sw, int ph, int pw, Tens out) {
  ConvGemmArgs p;
  p.A = in.p; p.a_bf16 = in.bf; p.B = B; p.H = H; p.W = W; p.Cin = L.w.Cin; p.lda = L.w.Cin; p.a_coff = 0;
  p.kh = L.w.kh; p.kw = L.w.kw; p.sh = sh; p.sw = sw; p.ph = ph; p.pw = pw; p.dh = 1; p.dw = 1;
  p.Ho = (H + 2 * ph - L.w.kh) / sh + 1;
  p.Wo = (W + 2 * pw - L.w.kw) / sw + 1;
  p.Wt = L.w.w; p.N = L.w.N; p.K = L.w.K;
  p.pre_scale = L.pre_s; p.pre_shift = L.pre_h;
  p.alpha = L.alpha; p.beta = L.beta;
  p.out = out.p; p.out_bf16 = out.bf;
  p.o_sb = (int64_t)p.Ho * p.Wo * p.N; p.o_sh = (int64_t)p.Wo * p.N; p.o_sw = p.N; p.o_sn = 1;
  return p;
}

}  // namespace

ConvL TsvadModel::conv_bn(const std::string& wname, const std::string& bn, const std::string& bias) {
  ConvL L;
  int N, Cin, kh, kw;
  auto w = ps_.pack(wname, N, Cin, kh, kw);
  L.w = upload_packed(arena_, w, N, Cin, kh, kw, cfg_.bf16);
  if (!bn.empty()) {
    std::vector<float> s, h;
    ps_.bn_fold(bn, s, h, bias);
    L.alpha = arena_.upload(s);
    L.beta = arena_.upload(h);
  } else if (!bias.empty()) {
    L.beta = arena_.upload(ps_.get(bias).data);
  }
  return L;
}

void TsvadModel::finalize() {
  SD_CHECK(!finalized_, kErrState, "finalize called twice");
  SD_CHECK(cfg_.speaker_embed_dim * 2 == cfg_.embed_dim, kErrInvalid,
           "proj_layer (speaker_embed_dim*2 != transformer_embed_dim) is not supported");
  const std::string se = "speech_encoder.";
  // ---- FCM head (cam_pplus_wespeaker.py:271-308)
  {
    const HostTensor& w = ps_.get(se + "head.conv1.weight");
    SD_CHECK(w.numel() == 32 * 9, kErrParam, "head.conv1.weight must be (32,1,3,3)");
    fcm_conv1_.pre_s = arena_.upload(w.data);  // raw 32x9 weights for the direct stem kernel
    std::vector<float> s, h;
    ps_.bn_fold(se + "head.bn1", s, h);
    fcm_conv1_.alpha = arena_.upload(s);
    fcm_conv1_.beta = arena_.upload(h);
  }
  for (int layer = 1; layer <= 2; ++layer)
    for (int blk = 0; blk < 2; ++blk) {
      std::string p = se + "head.layer" + std::to_string(layer) + "." + std::to_string(blk) + ".";
      ResBlock rb;
      rb.stride = blk == 0 ? 2 : 1;
      rb.c1 = conv_bn(p + "conv1.weight", p + "bn1");
      rb.c2 = conv_bn(p + "conv2.weight", p + "bn2");
      rb.has_sc = ps_.has(p + "shortcut.0.weight");
      if (rb.has_sc) rb.sc = conv_bn(p + "shortcut.0.weight", p + "shortcut.1");
      fcm_blocks_.push_back(rb);
    }
  fcm_conv2_ = conv_bn(se + "head.conv2.weight", se + "head.bn2");
  // ---- xvector (cam_pplus_wespeaker.py:330-372)
  tdnn_ = conv_bn(se + "xvector.tdnn.linear.weight", se + "xvector.tdnn.nonlinear.batchnorm");
  const int nlayers[3] = {12, 24, 16};
  const int dils[3] = {1, 2, 2};
  dense_.resize(3);
  for (int b = 0; b < 3; ++b) {
    for (int i = 0; i < nlayers[b]; ++i) {
      std::string p = se + "xvector.block" + std::to_string(b + 1) + ".tdnnd" + std::to_string(i + 1) + ".";
      DenseL d;
      d.dil = dils[b];
      d.bottleneck = conv_bn(p + "linear1.weight", p + "nonlinear2.batchnorm");
      std::vector<float> s, h;
      ps_.bn_fold(p + "nonlinear1.batchnorm", s, h);
      d.bottleneck.pre_s = arena_.upload(s);
      d.bottleneck.pre_h = arena_.upload(h);
      d.local = conv_bn(p + "cam_layer.linear_local.weight", "",
                        ps_.has(p + "cam_layer.linear_local.bias") ? p + "cam_layer.linear_local.bias" : "");
      const HostTensor& w1 = ps_.get(p + "cam_layer.linear1.weight");
      const HostTensor& w2 = ps_.get(p + "cam_layer.linear2.weight");
      d.c1 = (int)w1.shape[0];
      d.c2 = (int)w2.shape[0];
      d.c1w = arena_.upload(w1.data);
      d.c1b = arena_.upload(ps_.get(p + "cam_layer.linear1.bias").data);
      d.c2w = arena_.upload(w2.data);
      d.c2b = arena_.upload(ps_.get(p + "cam_layer.linear2.bias").data);
      dense_[b].push_back(d);
    }
    std::string p = se + "xvector.transit" + std::to_string(b + 1) + ".";
    ConvL t = conv_bn(p + "linear.weight", "", ps_.has(p + "linear.bias") ? p + "linear.bias" : "");
    std::vector<float> s, h;
    ps_.bn_fold(p + "nonlinear.batchnorm", s, h);
    t.pre_s = arena_.upload(s);
    t.pre_h = arena_.upload(h);
    transit_.push_back(t);
  }
  {
    std::vector<float> s, h;
    ps_.bn_fold(se + "xvector.out_nonlinear.batchnorm", s, h);
    out_nl_s_ = arena_.upload(s);
    out_nl_h_ = arena_.upload(h);
  }
  // The pooled embedding head (stats + dense) is not on the get_time_out path.
  for (const char* k : {"xvector.dense.linear.weight", "xvector.dense.nonlinear.batchnorm.running_mean",
                        "xvector.dense.nonlinear.batchnorm.running_var"})
    ps_.mark(se + k);
  // ---- speech_down_or_up (model.py:385-395)
  down_ = conv_bn("speech_down_or_up.0.weight", "speech_down_or_up.1.bn", "speech_down_or_up.0.bias");
  down_.pre_s = out_nl_s_;
  down_.pre_h = out_nl_h_;

  if (cfg_.variant == 0) {
    const HostTensor& pe = ps_.get("pos_encoder.pe");
    SD_CHECK(pe.shape.size() == 3 && pe.shape[2] == cfg_.embed_dim, kErrParam, "pos_encoder.pe shape");
    pe_len_ = (int)pe.shape[0];
    pe_ = arena_.upload(pe.data);
    for (int i = 0; i < cfg_.num_transformer_layer; ++i) {
      single_.push_back(loader().transformer("single_backend.layers." + std::to_string(i)));
      multi_.push_back(loader().transformer("multi_backend.layers." + std::to_string(i)));
    }
    backend_down_ = conv_bn("backend_down.0.weight", "backend_down.1.bn", "backend_down.0.bias");
    fc_ = loader().linear("fc");
  } else {
    gsp_w_ = arena_.upload(ps_.get("gsp_fc.weight").data);
    gsp_b_ = arena_.upload(ps_.get("gsp_fc.bias").data);
    for (int i = 0; i < cfg_.conformer_layers; ++i)
      conf_.push_back(loader().conformer("single_backend.conformer_layers." + std::to_string(i), true));
    // BiLSTM: stack both directions' W_ih, fold b_ih + b_hh.
    const int H = cfg_.lstm_hidden;
    std::vector<float> wih, bias, whh;
    for (const char* sfx : {"", "_reverse"}) {
      const HostTensor& wi = ps_.get(std::string("multi_backend.weight_ih_l0") + sfx);
      const HostTensor& wh = ps_.get(std::string("multi_backend.weight_hh_l0") + sfx);
      const HostTensor& bi = ps_.get(std::string("multi_backend.bias_ih_l0") + sfx);
      const HostTensor& bh = ps_.get(std::string("multi_backend.bias_hh_l0") + sfx);
      SD_CHECK(wh.shape[0] == 4 * H && wh.shape[1] == H, kErrParam, "weight_hh shape");
      wih.insert(wih.end(), wi.data.begin(), wi.data.end());
      whh.insert(whh.end(), wh.data.begin(), wh.data.end());
      for (int64_t i = 0; i < bi.numel(); ++i) bias.push_back(bi.data[i] + bh.data[i]);
    }
    const HostTensor& wi0 = ps_.get("multi_backend.weight_ih_l0");
    lstm_ih_ = upload_packed(arena_, wih, 8 * H, (int)wi0.shape[1], 1, 1, cfg_.bf16);
    lstm_b_ = arena_.upload(bias);
    lstm_hh_ = arena_.upload(whh);
    if (cfg_.bf16) lstm_hh_bf_ = upload_packed(arena_, whh, 2 * 4 * H, H, 1, 1, true).w;
    fc_ = loader().linear("fc");
  }
  auto extra = ps_.unused();
  if (!extra.empty()) {
    std::string msg = "Unexpected key(s) in state_dict:";
    for (size_t i = 0; i < extra.size() && i < 8; ++i) msg += " \"" + extra[i] + "\"";
    throw Error{kErrParam, msg};
  }
  alloc_workspace();
  finalized_ = true;
}

void TsvadModel::alloc_workspace() {
  const int64_t Bm = cfg_.max_batch, Tf = cfg_.max_fbank_frames;
  const int64_t T2 = (Tf - 1) / 2 + 1, T3 = (T2 - 1) / 2 + 1;
  const int64_t Tl = std::max<int64_t>(T3 + 3, (int64_t)cfg_.rs_len * 25);
  const int64_t NS = cfg_.max_num_speaker, E = cfg_.embed_dim;
  fcmA_ = ws(Bm * 80 * Tf * 32);
  fcmB_ = ws(Bm * 80 * Tf * 32);
  fcmC_ = ws(Bm * 40 * Tf * 32);
  x0_ = ws(Bm * Tf * 320);
  d_[0] = ws(Bm * T2 * 512);
  d_[1] = ws(Bm * T2 * 1024);
  d_[2] = ws(Bm * T2 * 1024);
  x4_ = ws(Bm * T2 * 512);
  tmp_ = ws(Bm * T2 * 128);
  gate_ = ws(Bm * ((T2 + 99) / 100) * 32);
  mix_ = ws(Bm * T3 * cfg_.speaker_embed_dim);
  mixg_ = ws(Bm * T3 * cfg_.speaker_embed_dim);
  const int64_t rows = Bm * NS * Tl;
  X_ = ws(rows * E);
  Y_ = ws(rows * E);
  QKV_ = ws(rows * 3 * E);
  AO_ = ws(rows * E);
  H_ = ws(rows * std::max<int64_t>({(int64_t)cfg_.ffn_dim, 2 * E, (int64_t)cfg_.conformer_ffn}));
  X2_ = ws(rows * E);
  partial_ = ws(Bm * NS * ((E + 63) / 64) * 2);
  lstm_work_ = ws(3 * 2 * Bm * cfg_.lstm_hidden);
}

void TsvadModel::forward(const float* ref, const float* ts, int B, int Tf, int Tl, float* logits,
                         hipStream_t st) {
  SD_CHECK(finalized_, kErrState, "model not finalized");
  SD_CHECK(B >= 1 && B <= cfg_.max_batch, kErrInvalid, "batch exceeds max_batch");
  SD_CHECK(Tf >= 8 && Tf <= cfg_.max_fbank_frames, kErrInvalid, "fbank frames exceed max_fbank_frames");
  const bool bf = cfg_.bf16;   // bf16 mode: CAM++ activations stored as bf16
  const int F = 80;
  // ---------------- FCM head (cam_pplus_wespeaker.py:271-308), NHWC (B, F, T, 32)
  fcm_conv1(ref, B, Tf, F, fcm_conv1_.pre_s, fcm_conv1_.alpha, fcm_conv1_.beta, fcmA_, bf, st);
  // layer1.0: A(80) -> B(40); shortcut A -> C(40); conv2 B -> A(40) + C
  // layer1.1: A -> B; conv2 B -> C + A
  // layer2.0: C(40) -> A(20); shortcut C -> B(20); conv2 A -> C(20) + B
  // layer2.1: C -> A; conv2 A -> B + C
  float* cur = fcmA_;
  int H = F;
  float* bufs[3] = {fcmA_, fcmB_, fcmC_};
  for (size_t i = 0; i < fcm_blocks_.size(); ++i) {
    const ResBlock& rb = fcm_blocks_[i];
    float* others[2];
    int k = 0;
    for (float* b : bufs) if (b != cur) others[k++] = b;
    float* t1 = others[0];
    float* t2 = others[1];
    ConvGemmArgs p = conv2d(Tens{cur, bf}, B, H, Tf, rb.c1, rb.stride, 1, 1, 1, Tens{t1, bf});
    p.act = kActRelu;
    conv_gemm(p, bf, st);
    const int Ho = p.Ho;
    const float* res = cur;
    float* outb;
    if (rb.has_sc) {
      conv_gemm(conv2d(Tens{cur, bf}, B, H, Tf, rb.sc, rb.stride, 1, 0, 0, Tens{t2, bf}), bf, st);
      res = t2;
      outb = cur;   // input no longer needed
    } else {
      outb = t2;
    }
    ConvGemmArgs r = conv2d(Tens{t1, bf}, B, Ho, Tf, rb.c2, 1, 1, 1, 1, Tens{outb, bf});
    r.res = res; r.res_bf16 = bf; r.res_ld = 32;
    r.act = kActRelu;
    conv_gemm(r, bf, st);
    cur = outb;
    H = Ho;
  }
  {
    // head.conv2 (stride (2,1)) + bn2 + relu, stored as (B, T, C*F') with channel c*F'+f.
    ConvGemmArgs p = conv2d(Tens{cur, bf}, B, H, Tf, fcm_conv2_, 2, 1, 1, 1, Tens{x0_, bf});
    p.act = kActRelu;
    const int Fo = p.Ho;
    SD_CHECK(Fo * 32 == 320, kErrShape, "FCM output width mismatch");
    p.o_sb = (int64_t)Tf * 320; p.o_sh = 1; p.o_sw = 320; p.o_sn = Fo;
    conv_gemm(p, bf, st);
  }
  // ---------------- xvector: TDNN + dense blocks + transits (channel-last (B, T, C))
  const int T2 = (Tf - 1) / 2 + 1;
  const int ctot[3] = {512, 1024, 1024};
  {
    ConvGemmArgs p = conv1d(Tens{x0_, bf}, B, Tf, 320, tdnn_, 2, 2, 1, Tens{d_[0], bf}, ctot[0]);
    p.act = kActRelu;
    SD_CHECK(p.Wo == T2, kErrShape, "tdnn output length");
    conv_gemm(p, bf, st);
  }
  int cin = 128;
  for (int b = 0; b < 3; ++b) {
    const Tens D{d_[b], bf};
    const int ld = ctot[b];
    for (const DenseL& L : dense_[b]) {
      SD_CHECK(L.bottleneck.w.Cin == cin, kErrParam, "dense layer input width");
      ConvGemmArgs p = conv1d(D, B, T2, ld, L.bottleneck, 1, 0, 1, Tens{tmp_, bf}, 128);
      p.act = kActRelu;
      conv_gemm(p, bf, st);
      cam_context(tmp_, bf, B, T2, 128, 128, 100, L.c1w, L.c1b, L.c1, L.c2w, L.c2b, L.c2, gate_, st);
      ConvGemmArgs q = conv1d(Tens{tmp_, bf}, B, T2, 128, L.local, 1, L.dil, L.dil, act_at(D, cin), ld);
      q.gate = gate_; q.gate_seg = 100; q.gate_nseg = (T2 + 99) / 100;
      conv_gemm(q, bf, st);
      cin += L.local.w.N;
    }
    SD_CHECK(cin == ld, kErrShape, "dense block width");
    const Tens dst{b < 2 ? d_[b + 1] : x4_, bf};
    const int ldo = b < 2 ? ctot[b + 1] : 512;
    conv_gemm(conv1d(D, B, T2, ld, transit_[b], 1, 0, 1, dst, ldo), bf, st);
    cin = transit_[b].w.N;
  }
  // ---------------- speech_down_or_up (out_nonlinear BN-ReLU fused as prologue), fp32 out
  const int E = cfg_.embed_dim, SE = cfg_.speaker_embed_dim, NS = cfg_.max_num_speaker;
  ConvGemmArgs pd = conv1d(Tens{x4_, bf}, B, T2, 512, down_, 2, 2, 1, Tens{mix_, false}, SE);
  pd.act = kActRelu;
  const int T3 = pd.Wo;
  conv_gemm(pd, bf, st);
  const int S = B * NS;
  if (cfg_.variant == 0) {
    SD_CHECK(T3 - Tl <= 2 && T3 - Tl >= -1, kErrShape,
             "label and ref_speech(mix speech) diff: " + std::to_string(T3 - Tl));
    SD_CHECK(Tl <= pe_len_, kErrShape, "label length exceeds positional-encoding max_len");
    // Per-speaker encoder over S = B*NS sequences (model.py:869-879).
    build_speaker_input(ts, mix_, SE, T3, B, NS, Tl, SE, pe_, X_, st);
    for (const auto& L : single_) run_transformer(L, X_, S, Tl, E, cfg_.num_attention_head, nullptr, enc_work(), st);
    speakers_to_channels(X_, B, NS, Tl, E, X2_, bf, st);
    ConvGemmArgs p = conv1d(Tens{X2_, bf}, B, Tl, NS * E, backend_down_, 1, 2, 1, Tens{X_, false}, E);
    p.act = kActRelu;
    conv_gemm(p, bf, st);
    add_pe(X_, B * Tl, Tl, E, E, pe_, st);
    for (const auto& L : multi_) run_transformer(L, X_, B, Tl, E, cfg_.num_attention_head, nullptr, enc_work(), st);
    ConvGemmArgs f = conv1d(Tens{X_, false}, B, Tl, E, fc_, 1, 0, 1, Tens{logits, false}, 1);
    f.o_sb = (int64_t)NS * Tl; f.o_sw = 1; f.o_sn = Tl;
    conv_gemm(f, bf, st);
  } else {
    SD_CHECK(std::abs(T3 - Tl) <= 3, kErrShape,
             "label and ref_speech(mix speech) diff: " + std::to_string(T3 - Tl));
    gsp_fc(mix_, B * T3, SE, SE, gsp_w_, gsp_b_, SE, mixg_, SE, st);
    build_speaker_input(ts, mixg_, SE, T3, B, NS, Tl, SE, nullptr, X_, st);
    for (const auto& L : conf_)
      run_conformer(L, X_, S, Tl, E, cfg_.conformer_heads, cfg_.conformer_kernel, nullptr, enc_work(), st);
    speakers_to_channels(X_, B, NS, Tl, E, X2_, bf, st);
    const int Hh = cfg_.lstm_hidden;
    conv_gemm(lin(Tens{X2_, bf}, B * Tl, NS * E, lstm_ih_, lstm_b_, Tens{H_, false}, 8 * Hh), bf, st);
    lstm_recurrence(H_, B, Tl, Hh, 2, lstm_hh_, nullptr, nullptr, nullptr, Y_, 2 * Hh, nullptr,
                    nullptr, lstm_work_, st, lstm_hh_bf_);
    ConvGemmArgs f = conv1d(Tens{Y_, false}, B, Tl, 2 * Hh, fc_, 1, 0, 1, Tens{logits, false}, 1);
    f.o_sb = (int64_t)NS * Tl; f.o_sw = 1; f.o_sn = Tl;
    conv_gemm(f, bf, st);
  }
}

}  // namespace sd
