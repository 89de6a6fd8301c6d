// Streaming FS-EEND runner (see fseend_stream.h).  The per-chunk kernel sequences
// mirror FsEendModel::forward / run_fusion (fseend.cpp) restricted to the chunk's rows,
// with every attention replaced by attn_decode against the K|V histories.
#include "fseend_stream.h"

#include <algorithm>
#include <climits>
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
  X2_ = wsb<float>((size_t)c_ * D);
  W_ = wsb<float>((size_t)(c_ + 18) * D);
  Yc_ = wsb<float>((size_t)c_ * D);
  E_ = wsb<float>((size_t)c_ * D);
  G_ = wsb<float>((size_t)c_ * D);
  A_ = wsb<float>((size_t)rd * D);
  A2_ = wsb<float>((size_t)rd * D);
  P_ = wsb<float>((size_t)rd);
  QKV_ = arena_.alloc(rd * 3 * D * es_);
  AO_ = arena_.alloc(rd * D * es_);
  T_ = arena_.alloc(rd * D * es_);
  H_ = arena_.alloc(rd * ffn * es_);
  n_blocks_ = attn_decode_blocks(cap_);
  ws_ = wsb<float>((size_t)C_ * cfg.n_heads * n_blocks_ * c_ * (2 + 64));
  dcnt_ = wsb<unsigned>((size_t)C_ * cfg.n_heads);
  SD_HIP(hipMemset(dcnt_, 0, (size_t)C_ * cfg.n_heads * sizeof(unsigned)));
  sws_ = wsb<float>((size_t)cfg.n_heads * rd * D);
  scnt_ = wsb<unsigned>(1);
  SD_HIP(hipMemset(scnt_, 0, sizeof(unsigned)));
  fws_ = wsb<float>((size_t)128 * 8 * D);
  ows_ = wsb<float>((size_t)C_ * cfg.n_heads * c_ * D);
  ocnt_ = wsb<unsigned>((size_t)C_);
  SD_HIP(hipMemset(ocnt_, 0, (size_t)C_ * sizeof(unsigned)));
  fcnt_ = wsb<unsigned>(1);
  SD_HIP(hipMemset(fcnt_, 0, sizeof(unsigned)));
  for (int l = 0; l < cfg.enc_n_layers; ++l) kv_enc_.push_back(arena_.alloc((size_t)cap_ * 2 * D * es_));
  for (int a = 0; a < cfg.dec_n_layers; ++a) kv_dec_.push_back(arena_.alloc((size_t)cap_ * C_ * 2 * D * es_));
  hist_ = wsb<float>((size_t)cap_ * D);
  SD_HIP(hipMemset(F_, 0, (size_t)c_ * m.in_ld_ * sizeof(float)));
  SD_HIP(hipMemset(state_, 0, 4 * sizeof(int)));
  SD_HIP(hipStreamCreateWithFlags(&cap_st_, hipStreamNonBlocking));
}

FsEendStream::~FsEendStream() {
  for (int i = 0; i < 3; ++i) {
    if (exec_[i]) (void)hipGraphExecDestroy(exec_[i]);
    if (graph_[i]) (void)hipGraphDestroy(graph_[i]);
  }
  if (cap_st_) (void)hipStreamDestroy(cap_st_);
}

namespace {

// Post-LN residual handed to the next GEMM: its A rows are LN(x + t)*g + b, and the result
// becomes the residual stream `out` (x and out ping-pong).  t == nullptr: plain LN of x.
struct PendingLn {
  const float* x = nullptr;
  const void* t = nullptr;
  const float* g = nullptr;
  const float* b = nullptr;
  float* out = nullptr;
};

struct KvEpi {
  void* dst = nullptr;
  const int* cursor = nullptr;
  int mult = 1;
  int64_t ld = 0;   // elements
};

// Runs p, taking its A rows from `ln` when given and storing columns [D, 3D) to the K|V
// history when `kv` is given: fused into the skinny kernel when it applies, else
// add_layernorm / kv_append around a plain GEMM (same results).
void gemm_fused(ConvGemmArgs p, const PendingLn* ln, const KvEpi* kv, int D, bool bf, hipStream_t st) {
  const int M = p.B * p.Ho * p.Wo;
  ConvGemmArgs q = p;
  if (ln) {
    q.ln_x = ln->x; q.ln_t = ln->t; q.ln_t_bf16 = bf; q.ln_g = ln->g; q.ln_b = ln->b; q.ln_out = ln->out;
    q.A = ln->out; q.a_bf16 = false; q.lda = p.K;
  }
  if (kv) {
    q.kv_out = kv->dst; q.kv_cursor = kv->cursor; q.kv_mult = kv->mult; q.kv_col0 = D; q.kv_ld = kv->ld;
  }
  if ((ln || kv) && gemm_skinny_supported(q)) {
    conv_gemm(q, bf, st);
    return;
  }
  if (ln) {
    if (ln->t) add_layernorm(const_cast<float*>(ln->x), ln->t, bf, M, p.K, ln->g, ln->b, 1e-5f, false, ln->out, false, st);
    else layernorm(ln->x, M, p.K, p.K, ln->g, ln->b, 1e-5f, ln->out, p.K, false, st);
    p.A = ln->out; p.a_bf16 = false; p.lda = p.K;
  }
  conv_gemm(p, bf, st);
  if (kv) {
    const size_t es = bf ? 2 : 4;
    kv_append(static_cast<char*>(p.out) + D * es, p.o_sw * es, M, 2 * D * es, kv->dst, kv->ld * es, kv->cursor,
              kv->mult, st);
  }
}

}  // namespace

// linear1 -> relu -> linear2 of a transformer layer on n rows with the pending post-LN folded in: one stream_ffn_pair
// launch when it applies (else the two skinny GEMMs), the result in T_ either way
void FsEendStream::ffn(const PackedW& l1, const float* b1, const PackedW& l2, const float* b2, const float* ln_x,
                       const void* ln_t, const float* ln_g, const float* ln_b, float* ln_out, int n, hipStream_t st) {
  const int D = m_.cfg_.n_units;
  FfnPairArgs f;
  f.ln_x = ln_x; f.ln_t = ln_t; f.t_bf16 = bf_; f.ln_g = ln_g; f.ln_b = ln_b; f.ln_out = ln_out;
  f.w1 = l1.w; f.b1 = b1; f.w2 = l2.w; f.b2 = b2; f.w_bf16 = bf_;
  f.out = T_; f.out_bf16 = bf_; f.ws = fws_; f.cnt = fcnt_; f.n = n; f.D = D; f.F = l1.N;
  if (l1.K == D && l2.K == l1.N && l2.N == D && stream_ffn_pair(f, st)) return;
  const Tens h{H_, bf_}, t{T_, bf_};
  const PendingLn ln{ln_x, ln_t, ln_g, ln_b, ln_out};
  ConvGemmArgs p = lin(Tens{ln_out, false}, n, D, l1, b1, h, l1.N);
  p.act = kActRelu;
  gemm_fused(p, &ln, nullptr, D, bf_, st);
  conv_gemm(lin(h, n, l1.N, l2, b2, t, D), bf_, st);
}

void FsEendStream::enc_chunk(hipStream_t st) {
  // MaskedTransformerEncoderModel.forward (fs_eend.py:178-204) on the chunk's c rows.  Every
  // post-LN (norm1/norm2, fs_eend.py via nn.TransformerEncoderLayer) is applied while the
  // next GEMM stages its rows; the K|V halves of the in-projection go straight to the history.
  const FsEendModel& m = m_;
  const int D = m.cfg_.n_units, nh = m.cfg_.n_heads, c = c_;
  const Tens qkv{QKV_, bf_}, ao{AO_, bf_}, t{T_, bf_}, h{H_, bf_};
  if (audio_)   // the chunk's feature rows from the audio history, at the encoder cursor
    stream_frontend(aud_, aud_cap_, c, nfft_, hop_, fsz_, fb_, n_mels_, ctx_, sub_, state_, bound_, lm_, F_, m.in_ld_, st);
  conv_gemm(lin(Tens{F_, false}, c, m.in_ld_, m.in_.w, m.in_.beta, Tens{Y_, false}, D), bf_, st);
  float* xb[2] = {X_, X2_};
  int xi = 0;
  PendingLn ln{Y_, nullptr, m.norm_g_, m.norm_b_, xb[0]};   // encoder_norm (fs_eend.py:197)
  for (size_t l = 0; l < m.enc_.size(); ++l) {
    const TransformerL& L = m.enc_[l];
    const KvEpi kv{kv_enc_[l], state_, 1, 2 * D};
    gemm_fused(lin(Tens{xb[xi], false}, c, D, L.in_proj, L.in_b, qkv, 3 * D), &ln, &kv, D, bf_, st);
    DecodeAttnArgs a;
    a.q = QKV_; a.q_tok = 3 * D;
    a.k = kv_enc_[l]; a.v = static_cast<char*>(kv_enc_[l]) + D * es_; a.kv_tok = 2 * D;
    a.out = AO_; a.o_tok = D;
    a.nseq = 1; a.nq = c; a.nh = nh; a.hd = D / nh; a.scale = 1.f / std::sqrt((float)(D / nh));
    a.pos = state_; a.delay = 0; a.max_keys = cap_; a.n_blocks = n_blocks_; a.ws = ws_; a.io_bf16 = bf_; a.cnt = dcnt_;
    if (L.out_proj.K == D && L.out_proj.N == D) {   // the out-projection inside the attention's merge
      a.wo = L.out_proj.w; a.bo = L.out_b; a.o2 = T_; a.ws2 = ows_; a.cnt2 = ocnt_;
    }
    if (!attn_decode(a, st)) conv_gemm(lin(ao, c, D, L.out_proj, L.out_b, t, D), bf_, st);
    xi ^= 1;
    ffn(L.l1, L.b1, L.l2, L.b2, xb[xi ^ 1], T_, L.n1g, L.n1b, xb[xi], c, st);
    ln = PendingLn{xb[xi], T_, L.n2g, L.n2b, xb[xi ^ 1]};
    xi ^= 1;
  }
  // last norm2 -> encoder-output history row, cursor advance (encoder frames and valid frames)
  stream_enc_finish(ln.x, ln.t, bf_, ln.g, ln.b, 1e-5f, c, D, hist_, state_ + 0, state_ + 1, st);
}

void FsEendStream::dec_chunk(hipStream_t st) {
  // fs_eend.py:83-90 for frames [n_dec, n_dec + c): conv window, L2 norm, decoder
  // (MaskedTransformerDecoderModel.forward :125-134 with TransformerEncoderFusionLayer
  // :456-478 applied dec_n_layers times), scores.  Post-LNs fold into the next GEMM.
  const FsEendModel& m = m_;
  const FusionL& f = m.fus_;
  const int D = m.cfg_.n_units, nh = m.cfg_.n_heads, c = c_, C = C_;
  const int n = c * C;
  const Tens qkv{QKV_, bf_}, ao{AO_, bf_}, t{T_, bf_}, h{H_, bf_};
  const float scale = 1.f / std::sqrt((float)(D / nh));
  // The window gather, the embedding's L2 norm and the slot init run as the A prologues of the GEMMs that
  // consume them (gemm_skinny pro_mode 3 / 1 / 2: same values, three launches fewer) when the skinny path
  // takes the chunk (else they run as their own kernels).
  {
    ConvGemmArgs p;
    p.A = W_; p.a_bf16 = false; p.B = 1; p.H = 1; p.W = c + 18; p.Cin = D; p.lda = D; p.a_coff = 0;
    p.kh = 1; p.kw = m.cnn_.w.kw; p.sh = 1; p.sw = 1; p.ph = 0; p.pw = 0; p.dh = 1; p.dw = 1;
    p.Ho = 1; p.Wo = c;
    p.Wt = m.cnn_.w.w; p.N = D; p.K = m.cnn_.w.K;
    p.beta = m.cnn_.beta;
    p.out = Yc_; p.out_bf16 = false;
    p.o_sb = (int64_t)c * D; p.o_sh = 0; p.o_sw = D; p.o_sn = 1;
    ConvGemmArgs q = p;
    q.pro_mode = 3; q.ln_x = hist_; q.pro_cursor = state_ + 2; q.pro_nvalid = state_ + 1; q.pro_pad = 9;
    if (gemm_skinny_supported(q)) {
      conv_gemm_skinny(q, bf_, st);
    } else {
      gather_window(hist_, D, state_ + 2, state_ + 1, 9, c + 18, W_, st);
      conv_gemm(p, bf_, st);
    }
  }
  {
    ConvGemmArgs p = lin(Tens{E_, false}, c, D, m.conv_emb_, nullptr, Tens{G_, false}, D);
    ConvGemmArgs q = p;
    q.pro_mode = 1; q.ln_x = Yc_; q.ln_out = E_;
    if (gemm_skinny_supported(q)) {
      conv_gemm_skinny(q, bf_, st);
    } else {
      row_l2norm(Yc_, c, D, E_, st);
      conv_gemm(p, bf_, st);
    }
  }
  float* ab[2] = {A_, A2_};
  int ai = 0;
  PendingLn ln;
  bool pending = false;
  for (int app = 0; app < m.cfg_.dec_n_layers; ++app) {
    // (1) time attention per slot against this application's history (causal)
    const KvEpi kv{kv_dec_[app], state_ + 2, C, 2 * D};
    if (app == 0) {   // slot_init as the in-projection's A prologue (ab[0] = G rows + slot bias)
      ConvGemmArgs q = lin(Tens{ab[ai], false}, n, D, f.in1, f.in1_b, qkv, 3 * D);
      q.pro_mode = 2; q.ln_x = G_; q.pro_p = m.slot_bias_; q.pro_C = C; q.ln_out = ab[0];
      q.kv_out = kv.dst; q.kv_cursor = kv.cursor; q.kv_mult = kv.mult; q.kv_col0 = D; q.kv_ld = kv.ld;
      if (gemm_skinny_supported(q)) {
        conv_gemm_skinny(q, bf_, st);
      } else {
        slot_init(G_, c, C, D, m.slot_bias_, ab[0], st);
        gemm_fused(lin(Tens{ab[ai], false}, n, D, f.in1, f.in1_b, qkv, 3 * D), nullptr, &kv, D, bf_, st);
      }
    } else {
      gemm_fused(lin(Tens{ab[ai], false}, n, D, f.in1, f.in1_b, qkv, 3 * D), pending ? &ln : nullptr, &kv, D, bf_, st);
    }
    {
      DecodeAttnArgs d;
      d.q = QKV_; d.q_tok = (int64_t)C * 3 * D; d.q_seq = 3 * D;
      d.k = kv_dec_[app]; d.v = static_cast<char*>(kv_dec_[app]) + D * es_;
      d.kv_tok = (int64_t)C * 2 * D; d.kv_seq = 2 * D;
      d.out = AO_; d.o_tok = (int64_t)C * D; d.o_seq = D;
      d.nseq = C; d.nq = c; d.nh = nh; d.hd = D / nh; d.scale = scale;
      d.pos = state_ + 2; d.delay = 0; d.max_keys = cap_; d.n_blocks = n_blocks_; d.ws = ws_; d.io_bf16 = bf_; d.cnt = dcnt_;
      if (f.out1.K == D && f.out1.N == D) {
        d.wo = f.out1.w; d.bo = f.out1_b; d.o2 = T_; d.ws2 = ows_; d.cnt2 = ocnt_;
      }
      if (!attn_decode(d, st)) conv_gemm(lin(ao, n, D, f.out1, f.out1_b, t, D), bf_, st);
    }
    ln = PendingLn{ab[ai], T_, f.n11g, f.n11b, ab[ai ^ 1]};
    ai ^= 1;
    // (2) attention over the C slots of each frame: one launch (stream_slot_block) when the chunk is small
    SlotBlockArgs sb;
    sb.ln_x = ln.x; sb.ln_t = ln.t; sb.t_bf16 = bf_; sb.ln_g = ln.g; sb.ln_b = ln.b; sb.ln_out = ln.out;
    sb.w_in = f.in2.w; sb.b_in = f.in2_b; sb.w_out = f.out2.w; sb.b_out = f.out2_b; sb.w_bf16 = bf_;
    sb.out = T_; sb.out_bf16 = bf_; sb.ws = sws_; sb.cnt = scnt_;
    sb.c = c; sb.C = C; sb.D = D; sb.nh = nh; sb.scale = scale;
    if (!stream_slot_block(sb, st)) {
      gemm_fused(lin(Tens{ab[ai], false}, n, D, f.in2, f.in2_b, qkv, 3 * D), &ln, nullptr, D, bf_, st);
      AttnArgs s;
      s.qkv = QKV_; s.io_bf16 = bf_; s.S = c; s.T = C; s.D = D; s.nh = nh; s.ld_qkv = 3 * D;
      s.out = AO_; s.ldo = D; s.scale = scale;
      attention(s, bf_, st);
      conv_gemm(lin(ao, n, D, f.out2, f.out2_b, t, D), bf_, st);
    }
    ai ^= 1;
    // (3) feed-forward
    ffn(f.l1, f.b1, f.l2, f.b2, ab[ai ^ 1], T_, f.n21g, f.n21b, ab[ai], n, st);
    ln = PendingLn{ab[ai], T_, f.n22g, f.n22b, ab[ai ^ 1]};
    ai ^= 1;
    pending = true;
  }
  // last norm22 + slot scores + decoder cursor advance
  stream_dec_finish(ln.x, ln.t, bf_, ln.g, ln.b, 1e-5f, c, C, D, E_, P_, state_ + 2, st);
}

int FsEendStream::graph_nodes(int which) const {
  if (!graph_[which]) return 0;
  size_t n = 0;
  SD_HIP(hipGraphGetNodes(graph_[which], nullptr, &n));
  return (int)n;
}

void FsEendStream::run(int which, hipStream_t st) {
  if (which != 1) ++runs_[0];
  if (which != 0) ++runs_[1];
  auto body = [&](hipStream_t s) {
    if (which != 1) enc_chunk(s);
    if (which != 0) dec_chunk(s);
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
  SD_CHECK(!audio_, kErrState, "stream takes audio (push_audio); reset() it to push feature rows");
  SD_CHECK(!closed_, kErrState, "stream input already ended (partial chunk or flush); call reset()");
  SD_CHECK(n >= 1 && n <= c_, kErrInvalid, "push: 1..chunk frames");
  SD_CHECK(feats && ld >= m_.in_ld_, kErrInvalid, "push: feature row stride below the input stride");
  SD_CHECK(n_enc_ + c_ <= cap_, kErrInvalid, "stream exceeds max_frames");
  SD_HIP(hipMemcpy2DAsync(F_, (size_t)m_.in_ld_ * sizeof(float), feats, (size_t)ld * sizeof(float),
                          (size_t)m_.in_ld_ * sizeof(float), n, hipMemcpyDeviceToDevice, st));
  if (n < c_) SD_HIP(hipMemsetAsync(F_ + (size_t)n * m_.in_ld_, 0, (size_t)(c_ - n) * m_.in_ld_ * sizeof(float), st));
  run(0, st);
  return after_enc(n, preds, cap, st);
}

void FsEendStream::set_audio(const float* mel_fb, int n_mels, int frame_size, int frame_shift, int context, int sub) {
  SD_CHECK(n_enc_ == 0 && n_samp_ == 0 && !closed_, kErrState, "set_audio: call on a fresh or reset stream");
  SD_CHECK(mel_fb && n_mels >= 1 && frame_size >= 1 && frame_shift >= 1 && context >= 0 && sub >= 1, kErrInvalid,
           "set_audio: bad frontend geometry");
  SD_CHECK((2 * context + 1) * n_mels <= m_.in_ld_ && (2 * context + 1) * n_mels == m_.cfg_.in_size, kErrInvalid,
           "set_audio: spliced width does not match the model's in_size");
  const int nfft = 1 << (32 - __builtin_clz((unsigned)(frame_size - 1)));
  SD_CHECK(nfft == 256 || nfft == 512, kErrInvalid, "set_audio: n_fft must be 256 or 512");
  fb_ = mel_fb; n_mels_ = n_mels; fsz_ = frame_size; hop_ = frame_shift; nfft_ = nfft; ctx_ = context; sub_ = sub;
  if (!aud_) {
    aud_cap_ = (int64_t)cap_ * sub * frame_shift + nfft;
    aud_ = wsb<float>((size_t)aud_cap_);
    lm_ = wsb<double>((size_t)((c_ - 1) * sub + 2 * context + 1) * n_mels);
    bound_ = wsb<int>(2);
  }
  const int open_bound[2] = {INT_MAX, INT_MAX};
  SD_HIP(hipMemcpy(bound_, open_bound, sizeof(open_bound), hipMemcpyHostToDevice));
  // the encoder graphs now start with the frontend: capture them anew
  for (int i = 0; i < 3; i += 2) {
    if (exec_[i]) (void)hipGraphExecDestroy(exec_[i]);
    if (graph_[i]) (void)hipGraphDestroy(graph_[i]);
    exec_[i] = nullptr; graph_[i] = nullptr; ran_direct_[i] = false;
  }
  audio_ = true;
}

int FsEendStream::push_audio(const float* samples, int64_t n, float* preds, int cap, hipStream_t st) {
  SD_CHECK(audio_, kErrState, "push_audio: the stream has no audio frontend (set_audio)");
  SD_CHECK(!closed_, kErrState, "stream input already ended (flush); call reset()");
  SD_CHECK(n >= 0 && (samples || n == 0), kErrInvalid, "push_audio: bad sample buffer");
  SD_CHECK(n_samp_ + n <= aud_cap_ - nfft_, kErrInvalid, "stream exceeds max_frames");
  if (n > 0)
    SD_HIP(hipMemcpyAsync(aud_ + n_samp_, samples, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, st));
  n_samp_ += n;
  // STFT frame j is final once the last sample its window reads, j hop + reach - 1 (the window of
  // frame_size sits at (n_fft - frame_size) / 2 in the centred n_fft frame), has arrived — such frames are
  // frames of the input whatever its final length; model frame i once its last spliced frame i sub + context is
  const int64_t reach = (nfft_ - fsz_) / 2 + fsz_ - nfft_ / 2;
  const int64_t n_stft = n_samp_ >= reach ? (n_samp_ - reach) / hop_ + 1 : 0;
  const int64_t n_model = n_stft >= ctx_ + 1 ? (n_stft - ctx_ - 1) / sub_ + 1 : 0;
  int out = 0;
  while (n_model - n_enc_ >= c_) {
    SD_CHECK(n_enc_ + c_ <= cap_, kErrInvalid, "stream exceeds max_frames");
    // steady state: this encoder chunk makes exactly one decoder chunk ready -> both in one graph launch
    const int nv = n_enc_ + c_;
    if (n_dec_ + c_ + 9 <= nv && n_dec_ + 2 * c_ + 9 > nv) {
      run(2, st);
      n_enc_ = nv;
      n_valid_ = nv;
      n_dec_ += c_;
      out += emit(preds ? preds + (size_t)out * C_ : nullptr, cap - out, c_, st);
    } else {
      run(0, st);
      out += after_enc(c_, preds ? preds + (size_t)out * C_ : nullptr, cap - out, st);
    }
  }
  return out;
}

int FsEendStream::after_enc(int n, float* preds, int cap, hipStream_t st) {
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
  int out = 0;
  if (audio_ && !closed_) {
    // the input length is known now: feature.stft's frame count (the last frame dropped when the length
    // is a multiple of the hop, feature.py:176-184), [::sub] rows; the remaining chunks see zero samples
    // past the end and zero splice rows past the last frame, exactly as the whole-recording frontend
    const int64_t nf = n_samp_ < 1 ? 0 : 1 + n_samp_ / hop_ - (n_samp_ % hop_ == 0 ? 1 : 0);
    const int64_t n_rows = (nf + sub_ - 1) / sub_;
    const int b[2] = {(int)n_samp_, (int)nf};
    SD_HIP(hipMemcpyAsync(bound_, b, sizeof(b), hipMemcpyHostToDevice, st));
    SD_HIP(hipStreamSynchronize(st));   // b lives on this stack frame
    while (n_enc_ < n_rows) {
      SD_CHECK(n_enc_ + c_ <= cap_, kErrInvalid, "stream exceeds max_frames");
      const int n = (int)std::min<int64_t>(c_, n_rows - n_enc_);
      run(0, st);
      out += after_enc(n, preds ? preds + (size_t)out * C_ : nullptr, cap - out, st);
      if (n < c_) break;
    }
  }
  closed_ = true;
  while (n_dec_ < n_valid_) {
    run(1, st);
    const int rows = std::min(c_, n_valid_ - n_dec_);
    n_dec_ += c_;
    out += emit(preds ? preds + (size_t)out * C_ : nullptr, cap - out, rows, st);
  }
  return out;
}

int FsEendStream::debug_counters(unsigned* host, int cap, hipStream_t st) const {
  const int nd = C_ * m_.cfg_.n_heads;
  SD_HIP(hipStreamSynchronize(st));
  if (cap > 0) SD_HIP(hipMemcpy(host, dcnt_, (size_t)std::min(cap, nd) * sizeof(unsigned), hipMemcpyDeviceToHost));
  if (cap > nd) SD_HIP(hipMemcpy(host + nd, scnt_, sizeof(unsigned), hipMemcpyDeviceToHost));
  return nd + 1;
}

void FsEendStream::reset(hipStream_t st) {
  SD_HIP(hipMemsetAsync(state_, 0, 4 * sizeof(int), st));
  // the block-merge counters return to 0 after every complete launch (wrapping increment); zeroing them here
  // also clears what an interrupted launch may have left
  SD_HIP(hipMemsetAsync(dcnt_, 0, (size_t)C_ * m_.cfg_.n_heads * sizeof(unsigned), st));
  SD_HIP(hipMemsetAsync(scnt_, 0, sizeof(unsigned), st));
  SD_HIP(hipMemsetAsync(fcnt_, 0, sizeof(unsigned), st));
  SD_HIP(hipMemsetAsync(ocnt_, 0, (size_t)C_ * sizeof(unsigned), st));
  // wait for the chunks flush() / push*() enqueued: they read bound_ and replay the graphs destroyed below,
  // and set_audio() rewrites bound_ with a synchronous copy that is not ordered after a non-blocking st
  SD_HIP(hipStreamSynchronize(st));
  n_enc_ = n_valid_ = n_dec_ = n_out_ = 0;
  closed_ = false;
  if (audio_) {   // back to feature rows until set_audio() again (the next capture rebuilds the encoder graph)
    audio_ = false;
    n_samp_ = 0;
    for (int i = 0; i < 3; i += 2) {
      if (exec_[i]) (void)hipGraphExecDestroy(exec_[i]);
      if (graph_[i]) (void)hipGraphDestroy(graph_[i]);
      exec_[i] = nullptr; graph_[i] = nullptr; ran_direct_[i] = false;
    }
  }
}

}  // namespace sd
