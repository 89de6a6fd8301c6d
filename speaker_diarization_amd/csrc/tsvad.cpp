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
#include "prof.h"

#include <cmath>

namespace sd {

ConvL TsvadModel::conv_bn(const std::string& wname, const std::string& bn, const std::string& bias) {
  return load_conv_bn(ps_, arena_, cfg_.bf16, wname, bn, bias);
}

void TsvadModel::finalize() {
  SD_CHECK(!finalized_, kErrState, "finalize called twice");
  SD_CHECK(cfg_.speaker_embed_dim * 2 == cfg_.embed_dim, kErrInvalid,
           "proj_layer (speaker_embed_dim*2 != transformer_embed_dim) is not supported");
  const std::string se = "speech_encoder.";
  cam_.load(ps_, arena_, se, cfg_.bf16);   // cam_pplus_wespeaker.py:271-372
  // The pooled embedding head (stats + dense) is not on the get_time_out path.
  for (const char* k : {"xvector.dense.linear.weight", "xvector.dense.nonlinear.batchnorm.running_mean",
                        "xvector.dense.nonlinear.batchnorm.running_var"})
    ps_.mark(se + k);
  // ---- speech_down_or_up (model.py:385-395)
  // BatchNorm1D (model.py:161-171) is not folded into the conv: a batch holding a NaN skips it, so the conv
  // stores conv + bias and its consumer applies BN + ReLU, or ReLU alone for such a batch (BnRelu)
  auto bn_only = [&](const std::string& bn) {
    std::vector<float> sc, sh;
    ps_.bn_fold(bn, sc, sh);
    BnRelu r;
    r.a = arena_.upload(sc);
    r.b = arena_.upload(sh);
    return r;
  };
  down_ = conv_bn("speech_down_or_up.0.weight", "", "speech_down_or_up.0.bias");
  down_bn_ = bn_only("speech_down_or_up.1.bn");
  down_.pre_s = cam_.out_s();
  down_.pre_h = cam_.out_h();

  if (cfg_.variant == 0) {
    const HostTensor& pe = ps_.get("pos_encoder.pe");
    SD_CHECK(pe.shape.size() == 3 && pe.shape[2] == cfg_.embed_dim, kErrParam, "pos_encoder.pe shape");
    pe_len_ = (int)pe.shape[0];
    pe_ = arena_.upload(pe.data);
    for (int i = 0; i < cfg_.num_transformer_layer; ++i) {
      single_.push_back(loader().transformer("single_backend.layers." + std::to_string(i)));
      multi_.push_back(loader().transformer("multi_backend.layers." + std::to_string(i)));
    }
    backend_down_ = conv_bn("backend_down.0.weight", "", "backend_down.0.bias");
    backend_bn_ = bn_only("backend_down.1.bn");
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
    // bf16 copy for the bf16 recurrence; fp32 handles keep hi / lo for the bf16x3 mode's split recurrence
    lstm_hh_bf_ = upload_packed(arena_, whh, 2 * 4 * H, H, 1, 1, true).w;
    if (!cfg_.bf16) lstm_hh_lo_ = upload_bf16_lo(arena_, whh);
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
  cam_.alloc(arena_, cfg_.max_batch, cfg_.max_fbank_frames);
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
  lstm_work_ = ws(lstm_work_floats((int)Bm, cfg_.lstm_hidden, 2));
  nonfinite_ = static_cast<int*>(arena_.alloc(4 * (size_t)Bm * sizeof(int)));
}

TsvadModel::~TsvadModel() {
  if (ev_fork_) (void)hipEventDestroy(ev_fork_);
  if (ev_join_) (void)hipEventDestroy(ev_join_);
  if (side_) (void)hipStreamDestroy(side_);
}

void TsvadModel::forward_graph(const float* ref, const float* ts, int B, int Tf, int Tl, float* logits, int replays,
                               const char* dot, hipStream_t st) {
  SD_CHECK(replays >= 0, kErrInvalid, "forward_graph: replays < 0");
  hipStream_t cap = nullptr;
  SD_HIP(hipStreamCreateWithFlags(&cap, hipStreamNonBlocking));
  hipGraph_t g = nullptr;
  hipGraphExec_t ex = nullptr;
  try {
    SD_HIP(hipStreamSynchronize(st));
    SD_HIP(hipStreamBeginCapture(cap, hipStreamCaptureModeThreadLocal));
    try {
      forward(ref, ts, B, Tf, Tl, logits, cap);
    } catch (...) {
      hipGraph_t bad = nullptr;
      (void)hipStreamEndCapture(cap, &bad);
      if (bad) (void)hipGraphDestroy(bad);
      throw;
    }
    SD_HIP(hipStreamEndCapture(cap, &g));
    if (dot) SD_HIP(hipGraphDebugDotPrint(g, dot, 0));
    SD_HIP(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    for (int r = 0; r < replays; ++r) SD_HIP(hipGraphLaunch(ex, st));
    SD_HIP(hipStreamSynchronize(st));
  } catch (...) {
    if (ex) (void)hipGraphExecDestroy(ex);
    if (g) (void)hipGraphDestroy(g);
    (void)hipStreamDestroy(cap);
    throw;
  }
  (void)hipGraphExecDestroy(ex);
  (void)hipGraphDestroy(g);
  (void)hipStreamDestroy(cap);
}

void TsvadModel::debug_buffer(int which, void** ptr, int64_t* bytes) const {
  const int64_t Bm = cfg_.max_batch, T3 = ((CamTrunk::out_frames(cfg_.max_fbank_frames)) - 1) / 2 + 1;
  const int64_t Tl = std::max<int64_t>(T3 + 3, (int64_t)cfg_.rs_len * 25), E = cfg_.embed_dim, SE = cfg_.speaker_embed_dim;
  const int64_t NS = cfg_.max_num_speaker;
  switch (which) {
    case 0: *ptr = mix_; *bytes = Bm * T3 * SE * 4; break;
    case 1: *ptr = mixg_; *bytes = Bm * T3 * SE * 4; break;
    case 2: *ptr = X2_; *bytes = Bm * NS * Tl * E * 4; break;
    case 3: *ptr = H_; *bytes = Bm * NS * Tl * E * 4; break;
    case 4: *ptr = Y_; *bytes = Bm * NS * Tl * E * 4; break;
    default: throw Error{kErrInvalid, "debug_buffer: unknown buffer"};
  }
}

// Direct launches.  A hipGraph replay of this forward (forward_graph above) measured no faster on C2 (34.3 vs
// 34.4 ms per 10-min step in round 3: ~150 launches against a 34-ms GPU span).  Its round-3 replay divergence
// was root-caused in round 4: the captured hipMemsetAsync nodes that reset the BiLSTM's h/c state and exchange
// counters stopped taking effect from the second replay on, so the recurrence started from the previous
// replay's state.  Every forward now zeroes device state with zero_fill kernels, and replays are
// bit-identical to direct launches (tests/test_gpu_tsvad_graph.py).
void TsvadModel::forward(const float* ref, const float* ts, int B, int Tf, int Tl, float* logits,
                         hipStream_t st, int forward_batch, int force) {
  SD_CHECK(forward_batch >= 0 && force >= 0 && force <= 3, kErrInvalid, "forward: bad forward_batch / force");
  SD_CHECK(finalized_, kErrState, "model not finalized");
  SD_CHECK(B >= 1 && B <= cfg_.max_batch, kErrInvalid, "batch exceeds max_batch");
  SD_CHECK(Tf >= 8 && Tf <= cfg_.max_fbank_frames, kErrInvalid, "fbank frames exceed max_fbank_frames");
  // an earlier forward's LSTM report nobody collected with sd_tsvad_status
  lstm_err_.raise_if_set();
  cam_.raise_if_set();
  const bool bf = cfg_.bf16;
  // CAM++ up to transit3, (B, T2, 512).  Batches of more than one round of CUs run as two window slices on
  // two streams (bit-identical per window: every CAM++ kernel computes a window independently of the rest
  // of the batch); so does the fused conformer stack below.  SDIAR_CAM_ONE_STREAM: one launch sequence over
  // the whole batch.
  // Under the libsdiar kernel timer (bench.py's extra profiled step) the forward stays on one stream, so
  // each kernel's HIP-event time is its own and not shared with the other slice's kernels.
  static const bool one_stream_env = getenv("SDIAR_CAM_ONE_STREAM") != nullptr;
  const bool one_stream = one_stream_env || prof_enabled();
  const int E = cfg_.embed_dim, SE = cfg_.speaker_embed_dim, NS = cfg_.max_num_speaker;
  const int T2 = CamTrunk::out_frames(Tf);
  const bool two = !one_stream && B >= 384;
  if (two && !side_) {
    SD_HIP(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
    SD_HIP(hipEventCreateWithFlags(&ev_fork_, hipEventDisableTiming));
    SD_HIP(hipEventCreateWithFlags(&ev_join_, hipEventDisableTiming));
  }
  // ---------------- BatchNorm1D's NaN bypass: which windows hold a non-finite input, which reference forwards
  // (groups of forward_batch windows) therefore skip the BatchNorm (from the inputs alone, so first: the window
  // slices below then need nothing from each other until the LSTM)
  const int G = forward_batch > 0 ? forward_batch : B;
  int* win_fb = nonfinite_;
  int* win_ts = nonfinite_ + cfg_.max_batch;
  int* grp_sd = nonfinite_ + 2 * cfg_.max_batch;
  int* grp_bd = nonfinite_ + 3 * cfg_.max_batch;
  zero_fill(nonfinite_, 4 * (size_t)cfg_.max_batch * sizeof(int), st);
  nonfinite_windows(ref, B, (int64_t)Tf * 80, G, win_fb, grp_sd, grp_bd, st);
  nonfinite_windows(ts, B, (int64_t)NS * SE, G, win_ts, nullptr, cfg_.variant == 0 ? grp_bd : nullptr, st);
  if (force & 1) fill_u32(grp_sd, (size_t)cfg_.max_batch * sizeof(int), 1u, st);
  if (force & 3) fill_u32(grp_bd, (size_t)cfg_.max_batch * sizeof(int), 1u, st);
  BnRelu sd_bn = down_bn_, bd_bn = backend_bn_;
  sd_bn.grp = grp_sd; sd_bn.group = G;
  bd_bn.grp = grp_bd; bd_bn.group = G;
  // speech_down_or_up conv geometry (its output frame count T3)
  const int T3 = cam_conv1d(Tens{nullptr, bf}, 1, T2, CamTrunk::kChannels, down_, 2, 2, 1, Tens{mix_, false}, SE).Wo;
  const bool fused_v1 = cfg_.variant == 1 && SE == 192 && E == 2 * SE && conformer_stack_fused(conf_, E, bf);
  // v1 conformer stack over windows [b0, b0 + Bh): every buffer of the fused stack is addressed from the slice's
  // first row (bf16 y / qkv / ao / h, fp32 X, per-sequence GroupNorm partials, the speaker streams)
  auto conformer_slice = [&](int b0, int Bh, hipStream_t s) {
    const int64_t s0 = (int64_t)b0 * NS, r0 = s0 * Tl;
    auto at = [](float* p, int64_t bytes) { return reinterpret_cast<float*>(reinterpret_cast<char*>(p) + bytes); };
    EncoderWork w = enc_work();
    w.Y = at(Y_, r0 * E * 2);
    w.QKV = at(QKV_, r0 * 3 * E * 2);
    w.AO = at(AO_, r0 * E * 2);
    w.H = at(H_, r0 * 2 * E * 2);
    w.partial = partial_ + s0 * ((E + 63) / 64) * 2;
    SpeakerStreams io;
    io.ts = ts + s0 * SE; io.mix = mixg_ + (int64_t)b0 * T3 * SE; io.ldmix = SE; io.Tmix = T3; io.NS = NS;
    io.out = at(X2_, (int64_t)b0 * Tl * NS * E * 2);
    run_conformer_stack(conf_, X_ + r0 * E, Bh * NS, Tl, E, cfg_.conformer_heads, cfg_.conformer_kernel, nullptr, w,
                        s, &io);
  };
  if (fused_v1) SD_CHECK(std::abs(T3 - Tl) <= 3, kErrShape, "label and ref_speech(mix speech) diff: " + std::to_string(T3 - Tl));
  if (fused_v1 && two) {
    // Two window slices, each through the whole per-window part of the model on its own stream: CAM++ trunk,
    // speech_down conv, gsp_fc, conformer stack.  Nothing joins between the trunk and the conformer, so one
    // slice's HBM-bound CAM++ kernels overlap the other's MFMA-bound conformer programs (bit-identical per
    // window: every kernel up to the LSTM computes a window independently of the rest of the batch).
    const int B1 = B / 2;
    SD_HIP(hipEventRecord(ev_fork_, st));
    SD_HIP(hipStreamWaitEvent(side_, ev_fork_, 0));
    auto slice = [&](int b0, int Bh, hipStream_t s) {
      const Tens x4s = cam_.forward(ref, Bh, Tf, s, b0);
      float* mx = mix_ + (int64_t)b0 * T3 * SE;
      conv_gemm(cam_conv1d(x4s, Bh, T2, CamTrunk::kChannels, down_, 2, 2, 1, Tens{mx, false}, SE), bf, s);
      BnRelu sb = sd_bn;
      sb.win0 = b0;
      gsp_fc(mx, Bh * T3, SE, SE, gsp_w_, gsp_b_, SE, mixg_ + (int64_t)b0 * T3 * SE, SE, s, sb, T3);
      conformer_slice(b0, Bh, s);
    };
    slice(0, B1, st);
    slice(B1, B - B1, side_);
    SD_HIP(hipEventRecord(ev_join_, side_));
    SD_HIP(hipStreamWaitEvent(st, ev_join_, 0));
  } else {
  // CAM++ up to transit3, (B, T2, 512): two window slices on two streams for large batches (v0)
  Tens x4;
  if (two) {
    const int B1 = B / 2;
    SD_HIP(hipEventRecord(ev_fork_, st));
    SD_HIP(hipStreamWaitEvent(side_, ev_fork_, 0));
    x4 = cam_.forward(ref, B1, Tf, st, 0);
    (void)cam_.forward(ref, B - B1, Tf, side_, B1);
    SD_HIP(hipEventRecord(ev_join_, side_));
    SD_HIP(hipStreamWaitEvent(st, ev_join_, 0));
  } else {
    x4 = cam_.forward(ref, B, Tf, st);
  }
  // ---------------- speech_down_or_up conv (out_nonlinear BN-ReLU fused as prologue) + bias, fp32 out; its
  // BatchNorm1D + ReLU are applied by the consumer (gsp_fc / build_speaker_input)
  ConvGemmArgs pd = cam_conv1d(x4, B, T2, CamTrunk::kChannels, down_, 2, 2, 1, Tens{mix_, false}, SE);
  conv_gemm(pd, bf, st);
  const int S = B * NS;
  if (cfg_.variant == 0) {
    SD_CHECK(T3 - Tl <= 2 && T3 - Tl >= -1, kErrShape,
             "label and ref_speech(mix speech) diff: " + std::to_string(T3 - Tl));
    SD_CHECK(Tl <= pe_len_, kErrShape, "label length exceeds positional-encoding max_len");
    // Per-speaker encoder over S = B*NS sequences (model.py:869-879).
    build_speaker_input(ts, mix_, SE, T3, B, NS, Tl, SE, pe_, X_, st, sd_bn);
    // bf16(X) for the first layer's in-projection too (every later layer gets it from the LayerNorms): an
    // fp32 A operand would send that GEMM to the register-staged kernel (C4: 1.5 ms per 640 windows vs 0.3)
    if (bf) f32_to_bf16(X_, (int64_t)S * Tl * E, enc_work().AO, st);
    for (size_t i = 0; i < single_.size(); ++i)
      run_transformer(single_[i], X_, S, Tl, E, cfg_.num_attention_head, nullptr, enc_work(), st, 0, 0, bf || i > 0);
    speakers_to_channels(X_, B, NS, Tl, E, X2_, bf, st);
    ConvGemmArgs p = cam_conv1d(Tens{X2_, bf}, B, Tl, NS * E, backend_down_, 1, 2, 1, Tens{X_, false}, E);
    conv_gemm(p, bf, st);
    add_pe(X_, B * Tl, Tl, E, E, pe_, st, bd_bn);   // backend_down's BatchNorm1D + ReLU, then the PE
    if (bf) f32_to_bf16(X_, (int64_t)B * Tl * E, enc_work().AO, st);
    for (size_t i = 0; i < multi_.size(); ++i)
      run_transformer(multi_[i], X_, B, Tl, E, cfg_.num_attention_head, nullptr, enc_work(), st, 0, 0, bf || i > 0);
    ConvGemmArgs f = cam_conv1d(Tens{X_, false}, B, Tl, E, fc_, 1, 0, 1, Tens{logits, false}, 1);
    f.o_sb = (int64_t)NS * Tl; f.o_sw = 1; f.o_sn = Tl;
    conv_gemm(f, bf, st);
    poison_windows(logits, B, (int64_t)NS * Tl, win_fb, win_ts, st);
    return;
  }
  SD_CHECK(std::abs(T3 - Tl) <= 3, kErrShape, "label and ref_speech(mix speech) diff: " + std::to_string(T3 - Tl));
  gsp_fc(mix_, B * T3, SE, SE, gsp_w_, gsp_b_, SE, mixg_, SE, st, sd_bn, T3);
  if (fused_v1) {
    conformer_slice(0, B, st);
  } else {
    build_speaker_input(ts, mixg_, SE, T3, B, NS, Tl, SE, nullptr, X_, st);
    run_conformer_stack(conf_, X_, S, Tl, E, cfg_.conformer_heads, cfg_.conformer_kernel, nullptr, enc_work(), st);
    speakers_to_channels(X_, B, NS, Tl, E, X2_, bf, st);
  }
  }
  {
    const int Hh = cfg_.lstm_hidden;
    conv_gemm(lin(Tens{X2_, bf}, B * Tl, NS * E, lstm_ih_, lstm_b_, Tens{H_, false}, 8 * Hh), bf, st);
    // SDIAR_LSTM_FP32 (diagnostic, tools/parity_stages.py): the exact-fp32 recurrence in bf16 mode too
    static const bool lstm_fp32 = getenv("SDIAR_LSTM_FP32") != nullptr;
    const bool x3 = !bf && gemm_x3();   // bf16x3 (precision 2): the split recurrence; fp32: exact step kernel
    lstm_recurrence(H_, B, Tl, Hh, 2, lstm_hh_, nullptr, nullptr, nullptr, Y_, 2 * Hh, nullptr,
                    nullptr, lstm_work_, st, (bf && !lstm_fp32) || x3 ? lstm_hh_bf_ : nullptr, lstm_err_.get(0),
                    x3 ? lstm_hh_lo_ : nullptr);
    ConvGemmArgs f = cam_conv1d(Tens{Y_, false}, B, Tl, 2 * Hh, fc_, 1, 0, 1, Tens{logits, false}, 1);
    f.o_sb = (int64_t)NS * Tl; f.o_sw = 1; f.o_sn = Tl;
    conv_gemm(f, bf, st);
  }
  // a window whose fbank or target-speaker embeddings hold a NaN / Inf has NaN logits in the reference
  poison_windows(logits, B, (int64_t)NS * Tl, win_fb, win_ts, st);
}

}  // namespace sd
