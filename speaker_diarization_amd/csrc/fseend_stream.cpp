// Streaming FS-EEND runner (see fseend_stream.h).  The per-chunk kernel sequences
// mirror FsEendModel::forward / run_fusion (fseend.cpp) restricted to the chunk's rows,
// with every attention replaced by attn_decode against the K|V histories.
#include "fseend_stream.h"

#include <algorithm>
#include <cmath>

namespace sd {

FsEendStream::FsEendStream(FsEendModel& m, int chunk, int max_frames, int C, bool use_graph)
    : m_(m),
      c_(chunk),
      cap_(cdiv(max_frames, chunk) * chunk),
      C_(C),
      use_graph_(use_graph),
      bf_(m.cfg_.bf16),
      es_(m.cfg_.bf16 ? 2 : 4) {
  const FsEendConfig& cfg = m.cfg_;
  SD_CHECK(m.finalized(), kErrState, "model not finalized");
  SD_CHECK(cfg.has_mask == 1 && cfg.mask_delay == 0, kErrInvalid,
           "streaming needs the causal encoder (has_mask=True, mask_delay=0)");
  SD_CHECK(chunk >= 1 && chunk <= 32, kErrInvalid, "chunk must be 1..32 frames");
  SD_CHECK(max_frames >= 1, kErrInvalid, "max_frames must be positive");
  SD_CHECK(C >= 1 && C <= cfg.max_nspks, kErrInvalid, "max_nspks exceeds the configured maximum");
  SD_CHECK(cfg.conv_delay == 9, kErrInvalid, "cnn padding 9 requires conv_delay 9 (fs_eend.py:41)");
  const int D = cfg.n_units;
  SD_CHECK(D / cfg.n_heads == 64, kErrInvalid, "streaming attention needs head dim 64");
  const int64_t rd = (int64_t)c_ * C_;
  const int ffn = std::max(cfg.enc_ffn, cfg.dec_ffn);
  state_ = wsb<int>(4);
  F_ = wsb<float>((size_t)c_ * m.in_ld_);
  Y_ = wsb<float>((size_t)c_ * D);
  X_ = wsb<float>((size_t)c_ * D);
  W_ = wsb<float>((size_t)(c_ + 18) * D);
  Yc_ = wsb<float>((size_t)c_ * D);
  E_ = wsb<float>((size_t)c_ * D);
  G_ = wsb<float>((size_t)c_ * D);
  A_ = wsb<float>((size_t)rd * D);
  P_ = wsb<float>((size_t)rd);
  QKV_ = arena_.alloc(rd * 3 * D * es_);
  AO_ = arena_.alloc(rd * D * es_);
  T_ = arena_.alloc(rd * D * es_);
  H_ = arena_.alloc(rd * ffn * es_);
  n_blocks_ = attn_decode_blocks(cap_);
  ws_ = wsb<float>((size_t)C_ * cfg.n_heads * n_blocks_ * c_ * (2 + 64));
  for (int l = 0; l < cfg.enc_n_layers; ++l) kv_enc_.push_back(arena_.alloc((size_t)cap_ * 2 * D * es_));
  for (int a = 0; a < cfg.dec_n_layers; ++a) kv_dec_.push_back(arena_.alloc((size_t)cap_ * C_ * 2 * D * es_));
  hist_ = wsb<float>((size_t)cap_ * D);
  SD_HIP(hipMemset(F_, 0, (size_t)c_ * m.in_ld_ * sizeof(float)));
  SD_HIP(hipMemset(state_, 0, 4 * sizeof(int)));
  SD_HIP(hipStreamCreateWithFlags(&cap_st_, hipStreamNonBlocking));
}

FsEendStream::~FsEendStream() {
  for (int i = 0; i < 2; ++i) {
    if (exec_[i]) (void)hipGraphExecDestroy(exec_[i]);
    if (graph_[i]) (void)hipGraphDestroy(graph_[i]);
  }
  if (cap_st_) (void)hipStreamDestroy(cap_st_);
}

void FsEendStream::enc_chunk(hipStream_t st) {
  // MaskedTransformerEncoderModel.forward (fs_eend.py:178-204) on the chunk's c rows.
  const FsEendModel& m = m_;
  const int D = m.cfg_.n_units, nh = m.cfg_.n_heads, c = c_;
  const Tens x{X_, false}, qkv{QKV_, bf_}, ao{AO_, bf_}, t{T_, bf_}, h{H_, bf_};
  conv_gemm(lin(Tens{F_, false}, c, m.in_ld_, m.in_.w, m.in_.beta, Tens{Y_, false}, D), bf_, st);
  layernorm(Y_, c, D, D, m.norm_g_, m.norm_b_, 1e-5f, X_, D, false, st);
  for (size_t l = 0; l < m.enc_.size(); ++l) {
    const TransformerL& L = m.enc_[l];
    conv_gemm(lin(x, c, D, L.in_proj, L.in_b, qkv, 3 * D), bf_, st);
    kv_append(static_cast<char*>(QKV_) + D * es_, 3 * D * es_, c, 2 * D * es_, kv_enc_[l], 2 * D * es_, state_, 1,
              st);
    DecodeAttnArgs a;
    a.q = QKV_; a.q_tok = 3 * D;
    a.k = kv_enc_[l]; a.v = static_cast<char*>(kv_enc_[l]) + D * es_; a.kv_tok = 2 * D;
    a.out = AO_; a.o_tok = D;
    a.nseq = 1; a.nq = c; a.nh = nh; a.hd = D / nh; a.scale = 1.f / std::sqrt((float)(D / nh));
    a.pos = state_; a.delay = 0; a.max_keys = cap_; a.n_blocks = n_blocks_; a.ws = ws_; a.io_bf16 = bf_;
    attn_decode(a, st);
    conv_gemm(lin(ao, c, D, L.out_proj, L.out_b, t, D), bf_, st);
    add_layernorm(X_, T_, bf_, c, D, L.n1g, L.n1b, 1e-5f, false, X_, false, st);
    ConvGemmArgs p = lin(x, c, D, L.l1, L.b1, h, L.l1.N);
    p.act = kActRelu;
    conv_gemm(p, bf_, st);
    conv_gemm(lin(h, c, L.l1.N, L.l2, L.b2, t, D), bf_, st);
    add_layernorm(X_, T_, bf_, c, D, L.n2g, L.n2b, 1e-5f, false, X_, false, st);
  }
  kv_append(X_, D * 4, c, D * 4, hist_, D * 4, state_, 1, st);
  cursor_advance(state_ + 0, c, state_ + 1, st);
}

void FsEendStream::fusion_step(int app, hipStream_t st) {
  // TransformerEncoderFusionLayer.forward (fs_eend.py:456-478) on the chunk's (t, slot) rows.
  const FsEendModel& m = m_;
  const FusionL& f = m.fus_;
  const int D = m.cfg_.n_units, nh = m.cfg_.n_heads, C = C_;
  const int n = c_ * C;
  const Tens a{A_, false}, qkv{QKV_, bf_}, ao{AO_, bf_}, t{T_, bf_}, h{H_, bf_};
  const float scale = 1.f / std::sqrt((float)(D / nh));
  // (1) time attention per slot against this application's history (causal)
  conv_gemm(lin(a, n, D, f.in1, f.in1_b, qkv, 3 * D), bf_, st);
  kv_append(static_cast<char*>(QKV_) + D * es_, 3 * D * es_, n, 2 * D * es_, kv_dec_[app], 2 * D * es_, state_ + 2,
            C, st);
  {
    DecodeAttnArgs d;
    d.q = QKV_; d.q_tok = (int64_t)C * 3 * D; d.q_seq = 3 * D;
    d.k = kv_dec_[app]; d.v = static_cast<char*>(kv_dec_[app]) + D * es_;
    d.kv_tok = (int64_t)C * 2 * D; d.kv_seq = 2 * D;
    d.out = AO_; d.o_tok = (int64_t)C * D; d.o_seq = D;
    d.nseq = C; d.nq = c_; d.nh = nh; d.hd = D / nh; d.scale = scale;
    d.pos = state_ + 2; d.delay = 0; d.max_keys = cap_; d.n_blocks = n_blocks_; d.ws = ws_; d.io_bf16 = bf_;
    attn_decode(d, st);
  }
  conv_gemm(lin(ao, n, D, f.out1, f.out1_b, t, D), bf_, st);
  add_layernorm(A_, T_, bf_, n, D, f.n11g, f.n11b, 1e-5f, false, A_, false, st);
  // (2) attention over the C slots of each frame
  conv_gemm(lin(a, n, D, f.in2, f.in2_b, qkv, 3 * D), bf_, st);
  {
    AttnArgs s;
    s.qkv = QKV_; s.io_bf16 = bf_; s.S = c_; s.T = C; s.D = D; s.nh = nh; s.ld_qkv = 3 * D;
    s.out = AO_; s.ldo = D; s.scale = scale;
    attention(s, bf_, st);
  }
  conv_gemm(lin(ao, n, D, f.out2, f.out2_b, t, D), bf_, st);
  add_layernorm(A_, T_, bf_, n, D, f.n21g, f.n21b, 1e-5f, false, A_, false, st);
  // (3) feed-forward
  ConvGemmArgs p = lin(a, n, D, f.l1, f.b1, h, f.l1.N);
  p.act = kActRelu;
  conv_gemm(p, bf_, st);
  conv_gemm(lin(h, n, f.l1.N, f.l2, f.b2, t, D), bf_, st);
  add_layernorm(A_, T_, bf_, n, D, f.n22g, f.n22b, 1e-5f, false, A_, false, st);
}

void FsEendStream::dec_chunk(hipStream_t st) {
  // fs_eend.py:83-90 for frames [n_dec, n_dec + c): conv window, L2 norm, decoder, scores.
  const FsEendModel& m = m_;
  const int D = m.cfg_.n_units, c = c_;
  gather_window(hist_, D, state_ + 2, state_ + 1, 9, c + 18, W_, st);
  {
    ConvGemmArgs p;
    p.A = W_; p.a_bf16 = false; p.B = 1; p.H = 1; p.W = c + 18; p.Cin = D; p.lda = D; p.a_coff = 0;
    p.kh = 1; p.kw = m.cnn_.w.kw; p.sh = 1; p.sw = 1; p.ph = 0; p.pw = 0; p.dh = 1; p.dw = 1;
    p.Ho = 1; p.Wo = c;
    p.Wt = m.cnn_.w.w; p.N = D; p.K = m.cnn_.w.K;
    p.beta = m.cnn_.beta;
    p.out = Yc_; p.out_bf16 = false;
    p.o_sb = (int64_t)c * D; p.o_sh = 0; p.o_sw = D; p.o_sn = 1;
    conv_gemm(p, bf_, st);
  }
  row_l2norm(Yc_, c, D, E_, st);
  conv_gemm(lin(Tens{E_, false}, c, D, m.conv_emb_, nullptr, Tens{G_, false}, D), bf_, st);
  slot_init(G_, c, C_, D, m.slot_bias_, A_, st);
  for (int i = 0; i < m.cfg_.dec_n_layers; ++i) fusion_step(i, st);
  slot_scores(E_, A_, c, C_, D, P_, false, st);
  cursor_advance(state_ + 2, c, nullptr, st);
}

void FsEendStream::run(int which, hipStream_t st) {
  auto body = [&](hipStream_t s) {
    if (which == 0) enc_chunk(s);
    else dec_chunk(s);
  };
  if (!use_graph_ || !ran_direct_[which]) {
    // First call (or graphs off): direct launches, which also perform the launchers'
    // one-time setup (function attributes, CU counts) outside any capture.
    body(st);
    ran_direct_[which] = true;
    return;
  }
  if (!exec_[which]) {
    SD_HIP(hipStreamBeginCapture(cap_st_, hipStreamCaptureModeThreadLocal));
    try {
      body(cap_st_);
    } catch (...) {
      hipGraph_t g = nullptr;
      (void)hipStreamEndCapture(cap_st_, &g);
      if (g) (void)hipGraphDestroy(g);
      throw;
    }
    SD_HIP(hipStreamEndCapture(cap_st_, &graph_[which]));
    SD_HIP(hipGraphInstantiate(&exec_[which], graph_[which], nullptr, nullptr, 0));
  }
  SD_HIP(hipGraphLaunch(exec_[which], st));
}

int FsEendStream::emit(float* preds, int cap, int rows, hipStream_t st) {
  SD_CHECK(rows <= cap, kErrInvalid, "prediction buffer too small");
  SD_CHECK(preds || rows == 0, kErrInvalid, "null prediction buffer");
  if (rows > 0)
    SD_HIP(hipMemcpyAsync(preds, P_, (size_t)rows * C_ * sizeof(float), hipMemcpyDeviceToDevice, st));
  n_out_ += rows;
  return rows;
}

int FsEendStream::push(const float* feats, int ld, int n, float* preds, int cap, hipStream_t st) {
  SD_CHECK(!closed_, kErrState, "stream input already ended (partial chunk or flush); call reset()");
  SD_CHECK(n >= 1 && n <= c_, kErrInvalid, "push: 1..chunk frames");
  SD_CHECK(feats && ld >= m_.in_ld_, kErrInvalid, "push: feature row stride below the input stride");
  SD_CHECK(n_enc_ + c_ <= cap_, kErrInvalid, "stream exceeds max_frames");
  SD_HIP(hipMemcpy2DAsync(F_, (size_t)m_.in_ld_ * sizeof(float), feats, (size_t)ld * sizeof(float),
                          (size_t)m_.in_ld_ * sizeof(float), n, hipMemcpyDeviceToDevice, st));
  if (n < c_) SD_HIP(hipMemsetAsync(F_ + (size_t)n * m_.in_ld_, 0, (size_t)(c_ - n) * m_.in_ld_ * sizeof(float), st));
  run(0, st);
  n_enc_ += c_;
  n_valid_ = n_enc_ - c_ + n;
  if (n < c_) {
    closed_ = true;
    SD_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(state_ + 1), n_valid_, 1, st));
  }
  int out = 0;
  while (n_dec_ + c_ + 9 <= n_valid_) {
    run(1, st);
    n_dec_ += c_;
    out += emit(preds ? preds + (size_t)out * C_ : nullptr, cap - out, c_, st);
  }
  return out;
}

int FsEendStream::flush(float* preds, int cap, hipStream_t st) {
  closed_ = true;
  int out = 0;
  while (n_dec_ < n_valid_) {
    run(1, st);
    const int rows = std::min(c_, n_valid_ - n_dec_);
    n_dec_ += c_;
    out += emit(preds ? preds + (size_t)out * C_ : nullptr, cap - out, rows, st);
  }
  return out;
}

void FsEendStream::reset(hipStream_t st) {
  SD_HIP(hipMemsetAsync(state_, 0, 4 * sizeof(int), st));
  n_enc_ = n_valid_ = n_dec_ = n_out_ = 0;
  closed_ = false;
}

}  // namespace sd
