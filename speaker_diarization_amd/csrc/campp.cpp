// CAM++ trunk and the pooled embedding head on gfx950 (see campp.h).
//
//   fbank (B, T, 80)
//     -> FCM: conv3x3+BN+ReLU, 2x2 BasicResBlocks, conv3x3 s(2,1)+BN+ReLU   :271-308
//     -> TDNN k5 s2 + BN + ReLU                                             :330-345
//     -> 3 CAM dense blocks (12/24/16 layers, growth 32) + transits         :346-372
//   CamppModel adds out_nonlinear BN-ReLU -> StatsPool -> dense + BN      :374-386
// Activations are channel-last; every contraction is conv_gemm with the eval
// BatchNorms folded into prologues/epilogues.
#include "campp.h"

namespace sd {

namespace {

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

ConvGemmArgs cam_conv1d(Tens in, int B, int T, int lda, const ConvL& L, int stride, int pad, int dil, Tens out,
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

ConvL load_conv_bn(ParamStore& ps, DeviceArena& arena, bool bf16, const std::string& wname, const std::string& bn,
                   const std::string& bias) {
  ConvL L;
  int N, Cin, kh, kw;
  auto w = ps.pack(wname, N, Cin, kh, kw);
  L.w = upload_packed(arena, w, N, Cin, kh, kw, bf16);
  if (!bn.empty()) {
    std::vector<float> s, h;
    ps.bn_fold(bn, s, h, bias);
    L.alpha = arena.upload(s);
    L.beta = arena.upload(h);
  } else if (!bias.empty()) {
    L.beta = arena.upload(ps.get(bias).data);
  }
  return L;
}

// ------------------------------------------------------------------------------ CamTrunk
void CamTrunk::load(ParamStore& ps, DeviceArena& arena, const std::string& pre, bool bf16) {
  bf16_ = bf16;
  auto conv_bn = [&](const std::string& w, const std::string& bn, const std::string& bias = "") {
    return load_conv_bn(ps, arena, bf16, w, bn, bias);
  };
  // ---- FCM head (cam_pplus_wespeaker.py:271-308)
  {
    const HostTensor& w = ps.get(pre + "head.conv1.weight");
    SD_CHECK(w.numel() == 32 * 9, kErrParam, "head.conv1.weight must be (32,1,3,3)");
    fcm_conv1_.pre_s = arena.upload(w.data);  // raw 32x9 weights for the direct stem kernel
    std::vector<float> s, h;
    ps.bn_fold(pre + "head.bn1", s, h);
    fcm_conv1_.alpha = arena.upload(s);
    fcm_conv1_.beta = arena.upload(h);
  }
  for (int layer = 1; layer <= 2; ++layer)
    for (int blk = 0; blk < 2; ++blk) {
      std::string p = pre + "head.layer" + std::to_string(layer) + "." + std::to_string(blk) + ".";
      ResBlock rb;
      rb.stride = blk == 0 ? 2 : 1;
      rb.c1 = conv_bn(p + "conv1.weight", p + "bn1");
      rb.c2 = conv_bn(p + "conv2.weight", p + "bn2");
      rb.has_sc = ps.has(p + "shortcut.0.weight");
      if (rb.has_sc) rb.sc = conv_bn(p + "shortcut.0.weight", p + "shortcut.1");
      fcm_blocks_.push_back(rb);
    }
  fcm_conv2_ = conv_bn(pre + "head.conv2.weight", pre + "head.bn2");
  // ---- xvector (cam_pplus_wespeaker.py:330-372)
  tdnn_ = conv_bn(pre + "xvector.tdnn.linear.weight", pre + "xvector.tdnn.nonlinear.batchnorm");
  const int nlayers[3] = {12, 24, 16};
  const int dils[3] = {1, 2, 2};
  dense_.assign(3, {});
  for (int b = 0; b < 3; ++b) {
    for (int i = 0; i < nlayers[b]; ++i) {
      std::string p = pre + "xvector.block" + std::to_string(b + 1) + ".tdnnd" + std::to_string(i + 1) + ".";
      DenseL d;
      d.dil = dils[b];
      d.bottleneck = conv_bn(p + "linear1.weight", p + "nonlinear2.batchnorm");
      std::vector<float> s, h;
      ps.bn_fold(p + "nonlinear1.batchnorm", s, h);
      d.bottleneck.pre_s = arena.upload(s);
      d.bottleneck.pre_h = arena.upload(h);
      d.local = conv_bn(p + "cam_layer.linear_local.weight", "",
                        ps.has(p + "cam_layer.linear_local.bias") ? p + "cam_layer.linear_local.bias" : "");
      const HostTensor& w1 = ps.get(p + "cam_layer.linear1.weight");
      const HostTensor& w2 = ps.get(p + "cam_layer.linear2.weight");
      d.c1 = (int)w1.shape[0];
      d.c2 = (int)w2.shape[0];
      d.c1w = arena.upload(w1.data);
      d.c1b = arena.upload(ps.get(p + "cam_layer.linear1.bias").data);
      d.c2w = arena.upload(w2.data);
      d.c2b = arena.upload(ps.get(p + "cam_layer.linear2.bias").data);
      dense_[b].push_back(d);
    }
    std::string p = pre + "xvector.transit" + std::to_string(b + 1) + ".";
    ConvL t = conv_bn(p + "linear.weight", "", ps.has(p + "linear.bias") ? p + "linear.bias" : "");
    std::vector<float> s, h;
    ps.bn_fold(p + "nonlinear.batchnorm", s, h);
    t.pre_s = arena.upload(s);
    t.pre_h = arena.upload(h);
    transit_.push_back(t);
  }
  SD_CHECK(transit_.back().w.N == kChannels, kErrParam, "transit3 must produce 512 channels");
  std::vector<float> s, h;
  ps.bn_fold(pre + "xvector.out_nonlinear.batchnorm", s, h);
  out_s_ = arena.upload(s);
  out_h_ = arena.upload(h);
}

void CamTrunk::alloc(DeviceArena& a, int max_batch, int max_frames) {
  const int64_t Bm = max_batch, Tf = max_frames, T2 = out_frames(max_frames);
  fcmA_ = ws(a, Bm * 80 * Tf * 32);
  fcmB_ = ws(a, Bm * 80 * Tf * 32);
  fcmC_ = ws(a, Bm * 40 * Tf * 32);
  x0_ = ws(a, Bm * Tf * 320);
  d_[0] = ws(a, Bm * T2 * 512);
  d_[1] = ws(a, Bm * T2 * 1024);
  d_[2] = ws(a, Bm * T2 * 1024);
  x4_ = ws(a, Bm * T2 * 512);
  tmp_ = ws(a, Bm * T2 * 128);
  gate_ = ws(a, Bm * ((T2 + 99) / 100) * 32);
  dense_rec_ = a.alloc(cam_dense_record_bytes(max_batch));
  dense_cnt_ = static_cast<unsigned*>(a.alloc(cam_dense_counter_bytes(max_batch)));
  SD_HIP(hipMemset(dense_cnt_, 0, cam_dense_counter_bytes(max_batch)));
}

Tens CamTrunk::forward(const float* fbank, int B, int Tf, hipStream_t st, int b0) const {
  const bool bf = bf16_;   // bf16 mode: CAM++ activations stored as bf16
  const int F = 80;
  // Windows [b0, b0 + B) of a larger batch: every workspace map is addressed from its window-b0 slice (the
  // FCM buffers with their largest row count as the per-window stride), so two slices of one batch can run
  // concurrently on two streams and leave the full-batch layout behind.
  const int64_t esz = bf ? 2 : 4, T2w = out_frames(Tf);
  auto sl = [&](float* p, int64_t per, int64_t bytes) {
    return reinterpret_cast<float*>(reinterpret_cast<char*>(p) + b0 * per * bytes);
  };
  const float* ref = fbank + (int64_t)b0 * Tf * F;
  float* const fcmA = sl(fcmA_, 80LL * Tf * 32, esz);
  float* const fcmB = sl(fcmB_, 80LL * Tf * 32, esz);
  float* const fcmC = sl(fcmC_, 40LL * Tf * 32, esz);
  float* const x0 = sl(x0_, (int64_t)Tf * 320, esz);
  float* const dd[3] = {sl(d_[0], T2w * 512, esz), sl(d_[1], T2w * 1024, esz), sl(d_[2], T2w * 1024, esz)};
  float* const x4 = sl(x4_, T2w * kChannels, esz);
  float* const tmp = sl(tmp_, T2w * 128, esz);
  float* const gate = sl(gate_, ((T2w + 99) / 100) * 32, 4);
  // per-window records / counters: the two slices' launches never share one
  void* const dense_rec = static_cast<char*>(dense_rec_) + cam_dense_record_bytes(b0);
  unsigned* const dense_cnt = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(dense_cnt_) + cam_dense_counter_bytes(b0));
  // ---------------- FCM head (cam_pplus_wespeaker.py:271-308), NHWC (B, F, T, 32)
  // layer1.0: A(80) -> B(40); shortcut A -> C(40); conv2 B -> A(40) + C
  // layer1.1: A -> B; conv2 B -> C + A
  // layer2.0: C(40) -> A(20); shortcut C -> B(20); conv2 A -> C(20) + B
  // layer2.1: C -> A; conv2 A -> B + C
  // bf16: layer1.0's conv1 computes the stem (head.conv1 + bn1 + relu) from the fbank in LDS, and the two
  // strided blocks' shortcuts ride on their conv1's centre tap (fcm_conv.hip FcmFuse).
  float* cur = fcmA;
  int H = F;
  float* bufs[3] = {fcmA, fcmB, fcmC};
  bool stem_done = false;
  for (size_t i = 0; i < fcm_blocks_.size(); ++i) {
    const ResBlock& rb = fcm_blocks_[i];
    float* others[2];
    int k = 0;
    for (float* b : bufs) if (b != cur) others[k++] = b;
    float* t1 = others[0];
    float* t2 = others[1];
    ConvGemmArgs p = conv2d(Tens{cur, bf}, B, H, Tf, rb.c1, rb.stride, 1, 1, 1, Tens{t1, bf});
    p.act = kActRelu;
    FcmFuse fu;
    if (rb.has_sc) {
      fu.sc_w = rb.sc.w.w; fu.sc_alpha = rb.sc.alpha; fu.sc_beta = rb.sc.beta; fu.sc_out = t2;
    }
    if (i == 0) {
      fu.fbank = ref; fu.fb_F = F;
      fu.stem_w = fcm_conv1_.pre_s; fu.stem_alpha = fcm_conv1_.alpha; fu.stem_beta = fcm_conv1_.beta;
    }
    const bool fused = bf && rb.has_sc && rb.sc.w.N == 32 && rb.sc.w.K == 32 && fcm_fused_supported(p, fu);
    if (i == 0 && !fused) {
      fcm_conv1(ref, B, Tf, F, fcm_conv1_.pre_s, fcm_conv1_.alpha, fcm_conv1_.beta, fcmA, bf, st);
      stem_done = true;
    }
    SD_CHECK(i != 0 || fused || stem_done, kErrInvalid, "FCM stem not computed");
    if (fused) conv_fcm3x3_fused(p, fu, st);
    else conv_gemm(p, bf, st);
    const int Ho = p.Ho;
    const float* res = cur;
    float* outb;
    if (rb.has_sc) {
      if (!fused) conv_gemm(conv2d(Tens{cur, bf}, B, H, Tf, rb.sc, rb.stride, 1, 0, 0, Tens{t2, bf}), bf, st);
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
    ConvGemmArgs p = conv2d(Tens{cur, bf}, B, H, Tf, fcm_conv2_, 2, 1, 1, 1, Tens{x0, bf});
    p.act = kActRelu;
    const int Fo = p.Ho;
    SD_CHECK(Fo * 32 == 320, kErrShape, "FCM output width mismatch");
    p.o_sb = (int64_t)Tf * 320; p.o_sh = 1; p.o_sw = 320; p.o_sn = Fo;
    conv_gemm(p, bf, st);
  }
  // ---------------- xvector: TDNN + dense blocks + transits (channel-last (B, T, C))
  const int T2 = out_frames(Tf);
  const int ctot[3] = {512, 1024, 1024};
  {
    ConvGemmArgs p = cam_conv1d(Tens{x0, bf}, B, Tf, 320, tdnn_, 2, 2, 1, Tens{dd[0], bf}, ctot[0]);
    p.act = kActRelu;
    SD_CHECK(p.Wo == T2, kErrShape, "tdnn output length");
    conv_gemm(p, bf, st);
  }
  int cin = 128;
  for (int b = 0; b < 3; ++b) {
    const Tens D{dd[b], bf};
    const int ld = ctot[b];
    for (const DenseL& L : dense_[b]) {
      SD_CHECK(L.bottleneck.w.Cin == cin, kErrParam, "dense layer input width");
      if (cam_dense_supported(T2, cin, ld, L.bottleneck.w.N, L.c1, L.c2, L.local.w.N, L.local.w.kw, L.dil,
                                            100, bf)) {
        // the whole layer per item in one launch, the 128-channel bottleneck kept in LDS (cam_dense.hip)
        cam_dense(D.p, B, T2, ld, cin, L.dil, L.bottleneck.pre_s, L.bottleneck.pre_h, L.bottleneck.w.w,
                  L.bottleneck.alpha, L.bottleneck.beta, L.local.w.w, L.local.beta, L.c1w, L.c1b, L.c2w, L.c2b,
                  act_at(D, cin).p, dense_rec, dense_cnt, st, err_.get(0));
        cin += L.local.w.N;
        continue;
      }
      ConvGemmArgs p = cam_conv1d(D, B, T2, ld, L.bottleneck, 1, 0, 1, Tens{tmp, bf}, 128);
      p.act = kActRelu;
      conv_gemm(p, bf, st);
      if (cam_local_fused_supported(128, L.c1, L.c2, L.local.w.N, L.local.w.kw, L.dil, 100, ld, bf)) {
        // Small batches (the embedding extractor's 96 chunks): one launch per layer that also
        // computes the gate.  Large batches: the context kernel, then the conv kernel reading
        // only each segment's window rows (fewer bytes per workgroup, higher occupancy).
        if (B * ((T2 + 99) / 100) < 1024) {
          cam_local_fused(tmp, B, T2, L.dil, L.local.w.w, L.local.beta, L.c1w, L.c1b, L.c2w, L.c2b,
                          act_at(D, cin).p, ld, st);
        } else {
          cam_context(tmp, bf, B, T2, 128, 128, 100, L.c1w, L.c1b, L.c1, L.c2w, L.c2b, L.c2, gate, st);
          cam_local_conv(tmp, B, T2, L.dil, L.local.w.w, L.local.beta, gate, act_at(D, cin).p, ld, st);
        }
      } else {
        cam_context(tmp, bf, B, T2, 128, 128, 100, L.c1w, L.c1b, L.c1, L.c2w, L.c2b, L.c2, gate, st);
        ConvGemmArgs q = cam_conv1d(Tens{tmp, bf}, B, T2, 128, L.local, 1, L.dil, L.dil, act_at(D, cin), ld);
        q.gate = gate; q.gate_seg = 100; q.gate_nseg = (T2 + 99) / 100;
        conv_gemm(q, bf, st);
      }
      cin += L.local.w.N;
    }
    SD_CHECK(cin == ld, kErrShape, "dense block width");
    const Tens dst{b < 2 ? dd[b + 1] : x4, bf};
    const int ldo = b < 2 ? ctot[b + 1] : kChannels;
    conv_gemm(cam_conv1d(D, B, T2, ld, transit_[b], 1, 0, 1, dst, ldo), bf, st);
    cin = transit_[b].w.N;
  }
  return Tens{x4, bf};
}

// ------------------------------------------------------------------------------ CamppModel
void CamppModel::finalize() {
  SD_CHECK(!finalized_, kErrState, "finalize called twice");
  SD_CHECK(cfg_.feat_dim == 80, kErrInvalid, "CAM++ FCM head supports feat_dim 80 only");
  trunk_.load(ps_, arena_, "", cfg_.bf16);
  // xvector.dense (cam_pplus_wespeaker.py:219-233, 380-382): the pooled head is tiny
  // (B x 1024 x E), so it always runs on the exact-fp32 MFMA path.  Its BatchNorm is
  // affine=False ("batchnorm_", :22-23): a weight/bias key is unexpected, not a gamma/beta.
  for (const char* k : {"xvector.dense.nonlinear.batchnorm.weight", "xvector.dense.nonlinear.batchnorm.bias"})
    SD_CHECK(!ps_.has(k), kErrParam, std::string("Unexpected key(s) in state_dict: \"") + k + "\"");
  dense_ = load_conv_bn(ps_, arena_, false, "xvector.dense.linear.weight", "xvector.dense.nonlinear.batchnorm");
  SD_CHECK(dense_.w.Cin == 2 * CamTrunk::kChannels && dense_.w.kw == 1, kErrParam,
           "xvector.dense.linear.weight must be (E, 1024, 1)");
  SD_CHECK(dense_.w.N == cfg_.embedding_size, kErrParam, "xvector.dense.linear.weight rows != embedding_size");
  auto extra = ps_.unused();
  if (!extra.empty()) {
    std::string msg = "Unexpected key(s) in state_dict:";
    for (size_t i = 0; i < extra.size() && i < 8; ++i) msg += " \"" + extra[i] + "\"";
    throw Error{kErrParam, msg};
  }
  trunk_.alloc(arena_, cfg_.max_batch, cfg_.max_frames);
  stats_ = static_cast<float*>(arena_.alloc((size_t)cfg_.max_batch * 2 * CamTrunk::kChannels * sizeof(float)));
  finalized_ = true;
}

void CamppModel::forward(const float* fbank, int B, int Tf, float* emb, float* time_out, hipStream_t st) {
  SD_CHECK(finalized_, kErrState, "model not finalized");
  trunk_.raise_if_set();   // an earlier call's cam_dense report
  SD_CHECK(B >= 1 && B <= cfg_.max_batch, kErrInvalid, "batch exceeds max_batch");
  SD_CHECK(Tf >= 8 && Tf <= cfg_.max_frames, kErrInvalid, "fbank frames exceed max_frames");
  const Tens x4 = trunk_.forward(fbank, B, Tf, st);
  const int T2 = CamTrunk::out_frames(Tf), C = CamTrunk::kChannels;
  // out_nonlinear -> StatsPool (mean, unbiased std over time; :28-34) [+ the time-out map]
  stats_pool(x4.p, x4.bf, B, T2, C, trunk_.out_s(), trunk_.out_h(), emb ? stats_ : nullptr, time_out, st);
  if (!emb) return;
  // dense: Conv1d(1024 -> E, k1) on the (B, 1024) stats + BatchNorm1d(affine=False)
  ConvGemmArgs p = cam_conv1d(Tens{stats_, false}, B, 1, 2 * C, dense_, 1, 0, 1, Tens{emb, false},
                              cfg_.embedding_size);
  conv_gemm(p, false, st);
}

}  // namespace sd
