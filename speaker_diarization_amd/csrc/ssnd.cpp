// SSND block inference (see ssnd.h).
#include "ssnd.h"

#include <cmath>
#include <string>

namespace sd {

std::vector<SsndModel::DecL> SsndModel::load_decoder(const std::string& pre, int d_aux) {
  // SWDecoderBlockV2 weights (ssnd_model.py:224-244), exact fp32.  FqFusion/FkFusion divide the
  // Linear output by sqrt(d_model) (:209, :221): folded into the packed weight and bias.
  LayerLoader ld{ps_, arena_, false};
  const int D = cfg_.d_model;
  const float inv_s = 1.f / std::sqrt((float)D);
  std::vector<DecL> out;
  for (int i = 0; i < cfg_.num_layers; ++i) {
    const std::string p = pre + "layers." + std::to_string(i) + ".";
    DecL L;
    { ConvL a = ld.linear(p + "fq.linear", inv_s); L.fq = a.w; L.fq_b = a.beta; }
    { ConvL a = ld.linear(p + "fk.linear", inv_s); L.fk = a.w; L.fk_b = a.beta; }
    SD_CHECK(L.fq.K == d_aux && L.fq.N == D, kErrParam, p + "fq.linear.weight shape");
    SD_CHECK(L.fk.K == cfg_.pos_emb_dim && L.fk.N == D, kErrParam, p + "fk.linear.weight shape");
    {
      // cross attention: Q, K and V come from different tensors, so the packed in-projection is
      // split into its three (D, D) row blocks (nn.MultiheadAttention in_proj_weight layout).
      const HostTensor& w = ps_.get(p + "cross_attn.in_proj_weight");
      const HostTensor& b = ps_.get(p + "cross_attn.in_proj_bias");
      SD_CHECK(w.shape.size() == 2 && w.shape[0] == 3 * D && w.shape[1] == D && b.numel() == 3 * D, kErrParam,
               p + "cross_attn.in_proj_weight shape");
      PackedW* dst[3] = {&L.cq, &L.ck, &L.cv};
      const float** bd[3] = {&L.cq_b, &L.ck_b, &L.cv_b};
      for (int j = 0; j < 3; ++j) {
        std::vector<float> ws(w.data.begin() + (size_t)j * D * D, w.data.begin() + (size_t)(j + 1) * D * D);
        *dst[j] = upload_packed(arena_, ws, D, D, 1, 1, false);
        *bd[j] = arena_.upload(std::vector<float>(b.data.begin() + j * D, b.data.begin() + (j + 1) * D));
      }
    }
    { ConvL a = ld.linear(p + "cross_attn.out_proj"); L.co = a.w; L.co_b = a.beta; }
    L.sa_in = ld.packed(p + "self_attn.in_proj_weight");
    L.sa_in_b = ld.up(p + "self_attn.in_proj_bias");
    { ConvL a = ld.linear(p + "self_attn.out_proj"); L.so = a.w; L.so_b = a.beta; }
    { ConvL a = ld.linear(p + "ffn.0"); L.f1 = a.w; L.f1_b = a.beta; }
    { ConvL a = ld.linear(p + "ffn.3"); L.f2 = a.w; L.f2_b = a.beta; }
    SD_CHECK(L.f1.N == cfg_.d_ff, kErrParam, p + "ffn.0.weight rows != d_ff");
    L.n1g = ld.up(p + "norm1.weight"); L.n1b = ld.up(p + "norm1.bias");
    L.n2g = ld.up(p + "norm2.weight"); L.n2b = ld.up(p + "norm2.bias");
    L.n3g = ld.up(p + "norm3.weight"); L.n3b = ld.up(p + "norm3.bias");
    out.push_back(L);
  }
  return out;
}

void SsndModel::finalize() {
  SD_CHECK(!finalized_, kErrState, "finalize called twice");
  const SsndConfig& c = cfg_;
  SD_CHECK(c.feat_dim == 80, kErrInvalid, "CAM++ FCM head supports feat_dim 80 only");
  SD_CHECK(c.d_model % c.nhead == 0 && (c.d_model / c.nhead) % 4 == 0 && c.d_model / c.nhead <= 128, kErrInvalid,
           "d_model / nhead must be a multiple of 4 and <= 128");
  SD_CHECK(c.d_model % 64 == 0 && c.emb_dim % 64 == 0, kErrInvalid, "d_model and emb_dim must be multiples of 64");
  const bool bf = c.bf16;
  const int D = c.d_model, E = c.emb_dim, N = c.max_speakers;
  // ---- extractor (CAM++_wo_gsp)
  cam_.load(ps_, arena_, "extractor.speech_encoder.", bf);
  // CAMPPlusWithGSP keeps its (unused by forward) pooled head: consumed so strict loading accepts it.
  ps_.get("extractor.speech_encoder.xvector.dense.linear.weight");
  ps_.get("extractor.speech_encoder.xvector.dense.nonlinear.batchnorm.running_mean");
  ps_.get("extractor.speech_encoder.xvector.dense.nonlinear.batchnorm.running_var");
  LayerLoader ld{ps_, arena_, bf};
  out_proj_ = ld.linear("extractor.speech_encoder.output_proj");
  SD_CHECK(out_proj_.w.K == CamTrunk::kChannels && out_proj_.w.N == E, kErrParam, "output_proj must be (emb_dim, 512)");
  out_proj_.pre_s = cam_.out_s();   // xvector.out_nonlinear (BN-ReLU) as the GEMM prologue
  out_proj_.pre_h = cam_.out_h();
  down_ = load_conv_bn(ps_, arena_, bf, "extractor.speech_down_or_up.0.weight", "extractor.speech_down_or_up.1.bn",
                       "extractor.speech_down_or_up.0.bias");
  SD_CHECK(down_.w.kw == 5 && down_.w.Cin == E && down_.w.N == E, kErrParam, "speech_down_or_up.0 must be (E, E, 5)");
  // ---- encoder
  enc_in_ = ld.linear("encoder.input_proj");
  SD_CHECK(enc_in_.w.K == E && enc_in_.w.N == D, kErrParam, "encoder.input_proj shape");
  for (int i = 0; i < c.num_layers; ++i)
    conf_.push_back(ld.conformer("encoder.encoder.conformer_layers." + std::to_string(i), false));
  // ---- decoders (fp32)
  LayerLoader l32{ps_, arena_, false};
  det_ = load_decoder("det_decoder.", c.q_det_aux_dim);
  det_out_ = l32.linear("det_decoder.out_proj");
  SD_CHECK(det_out_.w.N == c.vad_out_len && det_out_.w.K == D, kErrParam, "det_decoder.out_proj must be (vad_out_len, D)");
  rep_ = load_decoder("rep_decoder.", c.q_rep_aux_dim);
  rep_in_ = l32.linear("rep_decoder.input_proj");
  SD_CHECK(rep_in_.w.K == E && rep_in_.w.N == D, kErrParam, "rep_decoder.input_proj shape");
  rep_out_ = l32.linear("rep_decoder.out_proj");
  SD_CHECK(rep_out_.w.K == D && rep_out_.w.N == E, kErrParam, "rep_decoder.out_proj shape");
  {
    // RepresentationDecoder query: xdec_proj(rep_query_emb.mean(-1)) depends on weights only
    // (:359-360 with x_dec = rep_query_emb expanded, :767): computed once here.
    const HostTensor& q = ps_.get("rep_query_emb");
    const HostTensor& w = ps_.get("rep_decoder.xdec_proj.weight");
    const HostTensor& b = ps_.get("rep_decoder.xdec_proj.bias");
    SD_CHECK(q.shape.size() == 2 && q.shape[0] == N && q.shape[1] == c.vad_out_len, kErrParam,
             "rep_query_emb must be (max_speakers, vad_out_len)");
    SD_CHECK(w.numel() == D && b.numel() == D, kErrParam, "rep_decoder.xdec_proj must be (d_model, 1)");
    std::vector<float> x((size_t)N * D);
    for (int n = 0; n < N; ++n) {
      float s = 0.f;
      for (int t = 0; t < c.vad_out_len; ++t) s += q.data[(size_t)n * c.vad_out_len + t];
      const float m = s / (float)c.vad_out_len;
      for (int j = 0; j < D; ++j) x[(size_t)n * D + j] = m * w.data[j] + b.data[j];
    }
    rep_xdec_ = arena_.upload(x);
    const HostTensor& qw = ps_.get("rep_decoder.qaux_proj.weight");
    SD_CHECK(qw.numel() == c.q_rep_aux_dim, kErrParam, "rep_decoder.qaux_proj must be (q_rep_aux_dim, 1)");
    qaux_w_ = arena_.upload(qw.data);
    qaux_b_ = ld.up("rep_decoder.qaux_proj.bias");
  }
  {
    const HostTensor& pe = ps_.get("pos_emb");
    SD_CHECK(pe.shape.size() == 3 && pe.shape[1] == c.max_seq_len && pe.shape[2] == c.pos_emb_dim, kErrParam,
             "pos_emb must be (1, max_seq_len, pos_emb_dim)");
    pos_ = arena_.upload(pe.data);
    const HostTensor& dq = ps_.get("det_query_emb");
    SD_CHECK(dq.shape.size() == 2 && dq.shape[0] == N && dq.shape[1] == D, kErrParam,
             "det_query_emb must be (max_speakers, d_model)");
    det_q_ = arena_.upload(dq.data);
    // Speaker tables read by the host-side offline / online drivers (ssnd_model.py:778-900).
    for (const char* k : {"E_all", "e_pse", "e_non"}) ps_.get(k);
  }
  auto extra = ps_.unused();
  if (!extra.empty()) {
    std::string msg = "Unexpected key(s) in state_dict:";
    for (size_t i = 0; i < extra.size() && i < 8; ++i) msg += " \"" + extra[i] + "\"";
    throw Error{kErrParam, msg};
  }
  // ---- workspace
  const int64_t Bm = c.max_batch;
  const int T2 = CamTrunk::out_frames(c.max_fbank_frames);
  const int64_t T = std::max(label_frames(c.max_fbank_frames), c.vad_out_len);
  cam_.alloc(arena_, c.max_batch, c.max_fbank_frames);
  xp_ = ws(Bm * T2 * E);
  x_ = ws(Bm * T * E);
  X_ = ws(Bm * T * D);
  Y_ = ws(Bm * T * D);
  QKV_ = ws(Bm * T * 3 * D);
  AO_ = ws(Bm * T * D);
  H_ = ws(Bm * T * std::max(c.d_ff, 2 * D));
  partial_ = ws(Bm * ((D + 63) / 64) * 2);
  pos_t_ = ws(Bm * T * c.pos_emb_dim);
  xdec_ = ws(Bm * N * D);
  qaux_ = ws(Bm * N * std::max({c.q_det_aux_dim, c.q_rep_aux_dim, E}));
  Qin_ = ws(Bm * N * D);
  Kin_ = ws(Bm * T * D);
  q_ = ws(Bm * N * 3 * D);
  k_ = ws(Bm * T * D);
  v_ = ws(Bm * T * D);
  ctx_ = ws(Bm * N * D);
  t1_ = ws(Bm * N * D);
  xa_ = ws(Bm * N * D);
  h_ = ws(Bm * N * c.d_ff);
  fea_ = ws(Bm * T * D);
  finalized_ = true;
}

void SsndModel::run_decoder(const std::vector<DecL>& Ls, float* xdec, const float* qaux, int d_aux, const float* fea,
                            int B, int T, hipStream_t st) {
  // SWDecoderBlockV2.forward (ssnd_model.py:246-272), eval: every tensor fp32.
  const int D = cfg_.d_model, N = cfg_.max_speakers, rq = B * N, rk = B * T, nh = cfg_.nhead;
  const float eps = 1e-5f;
  auto gemm = [&](const float* A, int M, int lda, const PackedW& w, const float* bias, float* out, int ldo,
                  const float* res = nullptr, int act = kActNone) {
    ConvGemmArgs p = lin(Tens{const_cast<float*>(A), false}, M, lda, w, bias, Tens{out, false}, ldo);
    if (res) { p.res = res; p.res_bf16 = false; p.res_ld = ldo; }
    p.act = act;
    conv_gemm(p, false, st);
  };
  auto attend = [&](const float* q, int ldq, int nq, const float* k, const float* v, int ldkv, int tk) {
    MhaSmallArgs a;
    a.q = q; a.ldq = ldq; a.q_bs = (int64_t)nq * ldq;
    a.k = k; a.ldk = ldkv; a.k_bs = (int64_t)tk * ldkv;
    a.v = v; a.ldv = ldkv; a.v_bs = (int64_t)tk * ldkv;
    a.o = ctx_; a.ldo = D; a.o_bs = (int64_t)nq * D;
    a.B = B; a.Nq = nq; a.Tk = tk; a.nh = nh; a.hd = D / nh;
    a.scale = 1.f / std::sqrt((float)(D / nh));
    mha_small(a, st);
  };
  for (const DecL& L : Ls) {
    gemm(qaux, rq, d_aux, L.fq, L.fq_b, Qin_, D, xdec);                  // Q = x_dec + Fq(q_aux)
    gemm(pos_t_, rk, cfg_.pos_emb_dim, L.fk, L.fk_b, Kin_, D, fea);      // K = x_fea + Fk(k_pos)
    gemm(Qin_, rq, D, L.cq, L.cq_b, q_, D);
    gemm(Kin_, rk, D, L.ck, L.ck_b, k_, D);
    gemm(fea, rk, D, L.cv, L.cv_b, v_, D);                               // V = x_fea
    attend(q_, D, N, k_, v_, D, T);
    gemm(ctx_, rq, D, L.co, L.co_b, t1_, D);
    add_layernorm(xdec, t1_, false, rq, D, L.n1g, L.n1b, eps, false, xa_, false, st);   // norm1(x_dec + x2)
    gemm(xa_, rq, D, L.sa_in, L.sa_in_b, q_, 3 * D);
    attend(q_, 3 * D, N, q_ + D, q_ + 2 * D, 3 * D, N);
    gemm(ctx_, rq, D, L.so, L.so_b, t1_, D);
    add_layernorm(xa_, t1_, false, rq, D, L.n2g, L.n2b, eps, false, xa_, false, st);    // norm2(x + x2)
    gemm(xa_, rq, D, L.f1, L.f1_b, h_, cfg_.d_ff, nullptr, kActRelu);
    gemm(h_, rq, cfg_.d_ff, L.f2, L.f2_b, t1_, D);
    add_layernorm(xa_, t1_, false, rq, D, L.n3g, L.n3b, eps, false, xdec, false, st);   // norm3(x + x2)
  }
}

void SsndModel::decode(const float* enc, const float* x, const float* spk, int B, int T, float* vad, float* emb,
                       hipStream_t st) {
  SD_CHECK(finalized_, kErrState, "model not finalized");
  SD_CHECK(B >= 1 && B <= cfg_.max_batch, kErrInvalid, "blocks exceed max_batch");
  SD_CHECK(T == cfg_.vad_out_len, kErrShape, "frames per block must equal vad_out_len (rep_query_emb.expand)");
  SD_CHECK(T <= cfg_.max_seq_len, kErrShape, "frames per block exceed the positional table");
  const int D = cfg_.d_model, E = cfg_.emb_dim, N = cfg_.max_speakers;
  tile_rows(pos_, T, cfg_.pos_emb_dim, pos_t_, B * T, st);              // pos_emb[:, :T].expand(B, ...)
  // DetectionDecoder: learnable queries, L2-normalised speaker embeddings as auxiliary queries.
  tile_rows(det_q_, N, D, xdec_, B * N, st);
  row_l2norm(spk, B * N, E, qaux_, st);
  run_decoder(det_, xdec_, qaux_, cfg_.q_det_aux_dim, enc, B, T, st);
  conv_gemm(lin(Tens{xdec_, false}, B * N, D, det_out_.w, det_out_.beta, Tens{vad, false}, cfg_.vad_out_len), false,
            st);
  // RepresentationDecoder on the extractor output, auxiliary query from sigmoid(vad_pred).
  conv_gemm(lin(Tens{const_cast<float*>(x), false}, B * T, E, rep_in_.w, rep_in_.beta, Tens{fea_, false}, D), false, st);
  tile_rows(rep_xdec_, N, D, xdec_, B * N, st);
  mean_sigmoid_affine(vad, B * N, T, cfg_.vad_out_len, qaux_w_, qaux_b_, cfg_.q_rep_aux_dim, qaux_, cfg_.q_rep_aux_dim,
                      st);
  run_decoder(rep_, xdec_, qaux_, cfg_.q_rep_aux_dim, fea_, B, T, st);
  conv_gemm(lin(Tens{xdec_, false}, B * N, D, rep_out_.w, rep_out_.beta, Tens{emb, false}, E), false, st);
}

void SsndModel::infer(const float* feats, const float* spk, int B, int Tf, float* vad, float* emb, hipStream_t st) {
  SD_CHECK(finalized_, kErrState, "model not finalized");
  cam_.raise_if_set();   // an earlier call's cam_dense report
  SD_CHECK(B >= 1 && B <= cfg_.max_batch, kErrInvalid, "blocks exceed max_batch");
  SD_CHECK(Tf >= 8 && Tf <= cfg_.max_fbank_frames, kErrInvalid, "fbank frames exceed max_fbank_frames");
  const bool bf = cfg_.bf16;
  const int D = cfg_.d_model, E = cfg_.emb_dim;
  const int T2 = CamTrunk::out_frames(Tf), T = label_frames(Tf);
  SD_CHECK(T == cfg_.vad_out_len, kErrShape, "a block must give vad_out_len label frames (4 fbank frames each)");
  // extractor: CAM++ trunk -> relu(out_nonlinear) -> output_proj -> Conv1d k5 s2 + BN + ReLU
  const Tens x4 = cam_.forward(feats, B, Tf, st);
  {
    ConvGemmArgs p = lin(x4, B * T2, CamTrunk::kChannels, out_proj_.w, out_proj_.beta, Tens{xp_, bf}, E);
    p.pre_scale = out_proj_.pre_s;
    p.pre_shift = out_proj_.pre_h;
    conv_gemm(p, bf, st);
  }
  {
    ConvGemmArgs p = cam_conv1d(Tens{xp_, bf}, B, T2, E, down_, 2, 2, 1, Tens{x_, false}, E);
    p.act = kActRelu;
    SD_CHECK(p.Wo == T, kErrShape, "speech_down_or_up output length");
    conv_gemm(p, bf, st);
  }
  // encoder: input_proj + Conformer (all frames valid: lengths = T, :191)
  conv_gemm(lin(Tens{x_, false}, B * T, E, enc_in_.w, enc_in_.beta, Tens{X_, false}, D), bf, st);
  const EncoderWork w{Y_, QKV_, AO_, H_, partial_, bf};
  run_conformer_stack(conf_, X_, B, T, D, cfg_.nhead, cfg_.conformer_kernel, nullptr, w, st);
  decode(X_, x_, spk, B, T, vad, emb, st);
}

}  // namespace sd
