// Launchers for the gfx950 kernels (internal C++ API; the C-ABI is in capi.cpp).
#pragma once
#include <type_traits>
#include <vector>
#include "common.h"

namespace sd {

// ---------------------------------------------------------------- conv_gemm
struct ConvGemmArgs {
  // Input activation, channel-last: element (b, h, w, c) at
  // A[((b*H + h)*W + w)*lda + a_coff + c]; fp32, or bf16 when a_bf16.
  const void* A = nullptr;
  bool a_bf16 = false;
  int B = 1, H = 1, W = 1, Cin = 0, lda = 0, a_coff = 0;
  // A (bf16, lda == K, M % 16 == 0) in the row programs' tiled fragment layout (RowProgArgs::a_tiled): only the
  // register-A GEMM takes it (conv_gemm refuses it otherwise)
  int a_tiled = 0;
  int Ho = 1, Wo = 1;
  int kh = 1, kw = 1, sh = 1, sw = 1, ph = 0, pw = 0, dh = 1, dw = 1;
  // Packed weights Wt[N][K] (bf16 bits or fp32), K = kh*kw*Cin, tap-major.
  const void* Wt = nullptr;
  int N = 0, K = 0;
  const float* pre_scale = nullptr;  // per input channel; a' = relu(a*s + h)
  const float* pre_shift = nullptr;
  const float* alpha = nullptr;      // per output channel scale
  const float* beta = nullptr;       // per output channel shift
  const void* res = nullptr;         // residual at the output's (m, n) address map, stride res_ld
  bool res_bf16 = false;
  int res_ld = 0;
  int act = kActNone;
  const float* gate = nullptr;       // gate[(b*gate_nseg + wo/gate_seg)*N + n]
  int gate_seg = 1, gate_nseg = 1;
  void* out = nullptr;               // out[b*o_sb + ho*o_sh + wo*o_sw + n*o_sn]
  bool out_bf16 = false;
  int64_t o_sb = 0, o_sh = 0, o_sw = 0, o_sn = 1;
  // GLU epilogue (streaming path only): the N GEMM columns are 32-wide groups [a 16 | gate 16]
  // (weights permuted by glu_interleave_rows); output channel g*16 + j = a * sigmoid(gate), N/2 wide.
  int glu = 0;
  // Skinny path only (gemm_skinny_supported; streaming FS-EEND).  LayerNorm prologue: the staged
  // A rows are LN(ln_x + ln_t)*ln_g + ln_b over K (ln_x fp32 rows of K, ln_t fp32/bf16 or null);
  // workgroup 0 also stores them to ln_out (the next residual stream; must not alias ln_x).
  const float* ln_x = nullptr;
  const void* ln_t = nullptr;
  bool ln_t_bf16 = false;
  const float* ln_g = nullptr;
  const float* ln_b = nullptr;
  float ln_eps = 1e-5f;
  float* ln_out = nullptr;
  // Other skinny-only A prologues (pro_mode; ln_g unset):
  //   1  rows of ln_x (fp32, K wide, K <= 512) scaled to unit L2 norm with row_l2norm's arithmetic;
  //      workgroup 0 stores them to ln_out
  //   2  row r of A = ln_x[r / pro_C] + pro_p[r % pro_C] (slot_init's sum); workgroup 0 stores them to ln_out
  //   3  the staged span (the rows a stride-1 1-D conv reads) = rows [*pro_cursor - pro_pad, ...) of ln_x
  //      (row stride lda), zero outside [0, *pro_nvalid) (gather_window's window; p.A unused)
  int pro_mode = 0;
  const float* pro_p = nullptr;
  int pro_C = 1, pro_pad = 0;
  const int* pro_cursor = nullptr;
  const int* pro_nvalid = nullptr;
  // K/V history epilogue: columns n >= kv_col0 are also stored (out dtype) at
  // kv_out[(*kv_cursor * kv_mult + m) * kv_ld + n - kv_col0].
  void* kv_out = nullptr;
  const int* kv_cursor = nullptr;
  int kv_mult = 1, kv_col0 = 0;
  int64_t kv_ld = 0;
  // Split-K (gemm_dma path only, via conv_gemm_splitk): blockIdx.y = split z sums k-tiles of its share of
  // K into fp32 slab z at out + z * split_stride (bias in slab 0 only; no act / alpha / residual).
  int ksplit = 1;
  int64_t split_stride = 0;
};
// Row order of a GLU projection (2C, K) -> groups of [16 value rows | their 16 gate rows].
inline int glu_interleave_row(int r, int C) {   // new row index of original row r
  const bool gate = r >= C;
  const int c = gate ? r - C : r;
  return (c / 16) * 32 + (gate ? 16 : 0) + c % 16;
}
void conv_gemm(const ConvGemmArgs& p, bool bf16, hipStream_t st);
// Arithmetic of conv_gemm's exact (non-bf16) path on this host thread: false = the exact-f32 MFMA
// (v_mfma_f32_16x16x4_f32); true = "bf16x3": each fp32 operand split into bf16 hi + lo, acc += hi·hi + hi·lo +
// lo·hi on v_mfma_f32_16x16x32_bf16 (fp32 accumulate; ~2^-16 relative per product, 5.3x the f32 MFMA rate).
// Handles created with precision 2 set it around their compute calls (capi.cpp, GemmX3Scope).
bool gemm_x3();
struct GemmX3Scope {
  explicit GemmX3Scope(bool on);
  ~GemmX3Scope();
  bool prev;
};
void conv_gemm_bf16(const ConvGemmArgs& p, hipStream_t st);   // bf16-MFMA production kernel
bool gemm_dma_supported(const ConvGemmArgs& p);               // bf16 A, no prologue, taps==1 or Cin%64==0
// Split-K: the split count worth using for p on the gemm_dma path (1 = none), and the launch writing
// ksplit fp32 row-major (M x N) slabs to `slabs` (the consumer sums them, e.g. add_layernorm's t_slabs).
int gemm_splitk_count(const ConvGemmArgs& p);
void conv_gemm_splitk(const ConvGemmArgs& p, int ksplit, float* slabs, hipStream_t st);
bool gemm_ring_supported(const ConvGemmArgs& p);             // bf16 A/out, taps==1, K<=1024, N>=96, tall M
void conv_gemm_ring(const ConvGemmArgs& p, hipStream_t st);
bool gemm_stream_supported(const ConvGemmArgs& p);            // bf16 A linear, K%64==0, K<=768, no res
void conv_gemm_stream(const ConvGemmArgs& p, hipStream_t st);
bool fcm_conv_supported(const ConvGemmArgs& p);               // bf16 3x3 32->32, pad 1, freq stride 1|2
void conv_fcm3x3(const ConvGemmArgs& p, hipStream_t st);
// CAM++ BasicResBlock entry conv (3x3, freq stride 2, bf16 NHWC out) with the block's 1x1 shortcut as a
// second output and/or the FCM stem (head.conv1 + BN + ReLU of the fbank) computed in LDS instead of
// read from HBM (p.A unused then; p.H = fb_F = 80, p.W = frames).
struct FcmFuse {
  const void* sc_w = nullptr;                 // packed bf16 Wt[32][32]
  const float *sc_alpha = nullptr, *sc_beta = nullptr;
  void* sc_out = nullptr;                     // bf16 NHWC (B, Ho, Wo, 32)
  const float* fbank = nullptr;               // (B, W, fb_F) fp32
  int fb_F = 0;
  const float *stem_w = nullptr, *stem_alpha = nullptr, *stem_beta = nullptr;   // 32x9 raw, folded BN
};
bool fcm_fused_supported(const ConvGemmArgs& p, const FcmFuse& f);
void conv_fcm3x3_fused(const ConvGemmArgs& p, const FcmFuse& f, hipStream_t st);
void conv_gemm_dma(const ConvGemmArgs& p, hipStream_t st);     // LDS-DMA fed variant
bool gemm_areg_supported(const ConvGemmArgs& p);             // bf16 A linear, K in {192,256,384}, N % 64 == 0, N >= 768
void conv_gemm_areg(const ConvGemmArgs& p, hipStream_t st);
bool gemm_skinny_supported(const ConvGemmArgs& p);            // <= 16 rows, linear or stride-1 1-D conv
void conv_gemm_skinny(const ConvGemmArgs& p, bool w_bf16, hipStream_t st);

// Output row (b, ho, wo) sits at linear row m = (b*Ho + ho)*Wo + wo, stride o_sw
// (strides of size-1 dimensions do not matter).
__host__ __device__ inline bool out_rows_linear(const ConvGemmArgs& p) {
  return (p.Ho == 1 || p.o_sh == (int64_t)p.Wo * p.o_sw) && (p.B == 1 || p.o_sb == (int64_t)p.Ho * p.Wo * p.o_sw);
}
// A 1x1 conv whose input row m is output row m (stride 1, no padding): a plain GEMM on A.
inline bool a_rows_linear(const ConvGemmArgs& p) {
  return p.kh * p.kw == 1 && p.sh == 1 && p.sw == 1 && p.ph == 0 && p.pw == 0 && p.H == p.Ho && p.W == p.Wo;
}

// Plain row-major linear layer helper: out[m*ldo + o_coff + n] = act(A[m*lda+k]·W[n][k] * alpha + beta (+res)).
ConvGemmArgs linear_args(const void* A, int M, int K, int lda, const void* Wt, int N,
                         void* out, int ldo);

// ---------------------------------------------------------------- fcm / cam++
// First FCM conv (Cin = 1, 3x3, pad 1) + folded BN + ReLU.  fbank (B, T, F) ->
// NHWC (B, F, T, 32).  cam_pplus_wespeaker.py:277-301.
void fcm_conv1(const float* fbank, int B, int T, int F, const float* w /*32x9*/,
               const float* alpha, const float* beta, void* out, bool out_bf16, hipStream_t st);

// CAMLayer context gate (cam_pplus_wespeaker.py:106-123):
// ctx[b,s,c] = mean_t x[b,t,c] + mean_{t in seg s} x[b,t,c];
// gate[b,s,:] = sigmoid(W2·relu(W1·ctx + b1) + b2).
void cam_context(const void* x, bool x_bf16, int B, int T, int C, int ldx, int seg_len,
                 const float* w1, const float* b1, int C1, const float* w2, const float* b2,
                 int C2, float* gate, hipStream_t st);
// CAM++ dense-layer tail fused (cam_fused.hip): context gate + linear_local k3 conv + gating
// for one bf16 bottleneck map x (B, T, 128) -> out (B, T, 32) at row stride ldo (bf16).
// One CAM++ dense layer (bottleneck BN-ReLU-1x1-BN-ReLU, CAMLayer context gate, k-3 local conv x gate) in
// one launch, h kept in LDS (cam_dense.hip); x: (B, T, ld) bf16 map whose channels [0, cin) are the
// input, out: its channel slice at cin.  bf16, T <= 320.  Items of more than 160 frames run as two
// workgroups that meet through `records` (cam_dense_record_bytes(B), 16-B aligned) and `counters`
// (cam_dense_counter_bytes(B), zeroed ONCE when allocated, then owned by the launches: never shared by
// launches that may run concurrently).
bool cam_dense_supported(int T, int cin, int ld, int bn, int C1, int C2, int N, int taps, int dil, int seg_len,
                         bool bf16);
size_t cam_dense_record_bytes(int B);
void cam_dense_set_probe(void* stamps);
void rowprog_set_probe(void* stamps);
// Graph-replay diagnostic (diag.hip): [memset(X, 0) -> kernel Y = X; X = 7] replayed `replays` times;
// bad_per_replay[r] = non-zero Y values after replay r (host array).
void graph_memset_probe(int n, int replays, bool fork, int* bad_per_replay, hipStream_t st);   // test-only phase stamps ([grid][16] u64), null = off
size_t cam_dense_counter_bytes(int B);
void cam_dense(const void* x, int B, int T, int ld, int cin, int dil, const float* s1, const float* h1,
               const void* wb, const float* a2, const float* b2, const void* wl, const float* bl, const float* w1,
               const float* c1, const float* w2, const float* c2, void* out, void* records, unsigned* counters,
               hipStream_t st, int* err = nullptr);   // err: device address of a PinnedFlags slot (lost exchange)
bool cam_local_fused_supported(int C, int C1, int C2, int N, int taps, int dil, int seg_len, int ldo, bool bf16);
void cam_local_fused(const void* x, int B, int T, int dil, const void* wt, const float* bias, const float* w1,
                     const float* b1, const float* w2, const float* b2, void* out, int ldo, hipStream_t st);
// The conv + gating half alone, gate (B, nseg, 32) from cam_context().
void cam_local_conv(const void* x, int B, int T, int dil, const void* wt, const float* bias, const float* gate,
                    void* out, int ldo, hipStream_t st);
// CAM++ out_nonlinear + StatsPool (cam_pplus_wespeaker.py:28-39, 372-379):
// v = relu(x * s + h) over x (B, T, C) channel-last (C % 64 == 0);
// stats (B, 2C) = [mean_t v | unbiased std_t v] (nullable); tout (B, T, C) = v (nullable).
void stats_pool(const void* x, bool x_bf16, int B, int T, int C, const float* s, const float* h,
                float* stats, float* tout, hipStream_t st);

// ---------------------------------------------------------------- norms
// y = LN(x) * g + b over the last dim D; rows of x at stride ldx, y at ldy.
// y may be bf16 (y_bf16); x is fp32 (the residual stream).
// y2 (optional, fp32 y only): a bf16 copy of y, the A operand of the GEMMs that read it.
void layernorm(const float* x, int rows, int D, int ldx, const float* g, const float* b,
               float eps, void* y, int ldy, bool y_bf16, hipStream_t st, uint16_t* y2 = nullptr);
// Residual add fused into LayerNorm: v = x + t (t fp32 or bf16, rows of D); write_x: x = v;
// y = LN(v) (y may alias x or t: each row is read completely before it is written).
// t_slabs > 1 (fp32 t only): t is the sum of t_slabs slabs t + i * rows * D (a split-K GEMM's partials).
void add_layernorm(float* x, const void* t, bool t_bf16, int rows, int D, const float* g, const float* b,
                   float eps, bool write_x, void* y, bool y_bf16, hipStream_t st, uint16_t* y2 = nullptr,
                   int t_slabs = 1);

// ---------------------------------------------------------------- attention
// Multi-head self-attention core on a packed in-projection output.
// qkv: (S*T, 3*D) row-major (q | k | v), heads of size hd = D/nh.
// out: (S*T, ldo) at column h*hd.  Optional causal mask (key > query + delay is
// masked) and per-sequence key lengths (keys >= len[s] masked).
struct AttnArgs {
  const void* qkv = nullptr;       // fp32, or bf16 when io_bf16 (also the output dtype)
  bool io_bf16 = false;
  int S = 0, T = 0, D = 0, nh = 0;
  int ld_qkv = 0;
  void* out = nullptr;
  int ldo = 0;
  float scale = 1.f;
  int causal = 0, causal_delay = 0;
  const int* key_len = nullptr;
  // Token t of sequence s lives at row (s / seq_inner) * seq_outer + (s % seq_inner) * seq_inner_stride
  // + t * tok_stride of qkv / out.  Defaults (seq_outer 0 -> T) give contiguous sequences; the FS-EEND
  // decoder runs its time attention over the slots of a (T, C) token grid with tok_stride C.
  // Chunk-streaming mask (ts_vad2_streaming forward_chunk_by_chunk with KV caches, expressed as
  // one forward): query i sees key j iff chunk(j) <= chunk(i) and, when left >= 0,
  // chunk(j) >= chunk(i) - left, with chunk(x) = x / chunk.  chunk 0: off.
  int chunk = 0, left = -1;
  int seq_inner = 1;
  int64_t seq_outer = 0;
  int seq_inner_stride = 0;
  int tok_stride = 1;
  // Test probe (sd_probe_attention_mask): mask_dump (T*T int32, zeroed) receives 1/2 = visible/masked
  // for each visited pair of seq 0, head 0.
  int* mask_dump = nullptr;
  int xcd_small = 0;   // set by the launcher: the small-grid XCD grouping of attn_long (attention.hip)
};
void attention(const AttnArgs& a, bool bf16, hipStream_t st);

// ---------------------------------------------------------------- mha_block.hip
// Conformer self-attention block in one launch (bf16, D 384, 8 heads, T <= 160): q|k|v = y · W_inᵀ + bias
// (y the LayerNorm'd bf16 rows, W_in packed bf16 (3D, D)), per head softmax(q kᵀ * scale) v -> out (S*T
// rows of stride ldo, bf16).  key_len (device int32 per sequence) optional.
struct MhaBlockArgs {
  const void* y = nullptr;   // bf16 rows, already LayerNorm'd (self_attn_layer_norm)
  const float* ln_g = nullptr;   // (informational: the norm the rows went through)
  const float* ln_b = nullptr;
  float eps = 1e-5f;
  const void* W = nullptr;
  const float* bias = nullptr;
  void* out = nullptr;
  int ldo = 0;
  int S = 0, T = 0, D = 0, nh = 0;
  float scale = 1.f;
  const int* key_len = nullptr;
  // out in the row programs' tiled A layout (RowProgArgs::a_tiled; needs S * T % 16 == 0, ldo == D) instead of
  // row-major rows of stride ldo
  int out_tiled = 0;
  int y_tiled = 0;   // y in that layout too (RowProgArgs::y_tiled)
};
bool mha_block_supported(int D, int nh, int T, bool bf16);


// ---------------------------------------------------------------- rowprog.hip
// Conformer per-token row program (bf16 weights, D 384): acc = X; [acc += A·W0ᵀ + b0];
// per FFN i: acc += W2·silu(W1·LN_i(acc) + b1) + b2 (the ½ folded into W2 / b2), [acc = LN_post_i(acc)];
// Xo = acc (may alias X); [y = LN_y(acc) bf16].  Weights packed by rowprog_pack_pre / rowprog_pack_ffn.
struct RowFfnArgs {
  const void* w = nullptr;     // rowprog_pack_ffn pieces (the FFN's LayerNorm affine folded in)
  int hidden = 0;
  const float *b1 = nullptr, *b2 = nullptr;   // b1 folded by rowprog_pack_ffn
  const float *post_g = nullptr, *post_b = nullptr;
};
struct RowProgArgs {
  const float* X = nullptr;
  float* Xo = nullptr;
  int M = 0;
  const void* A = nullptr;     // (M, 384) bf16 rows of the pre-GEMM
  const void* w0 = nullptr;    // rowprog_pack_pre pieces (384 x 384)
  const float* b0 = nullptr;
  int n_ffn = 0;
  RowFfnArgs ffn[2];
  const float *y_g = nullptr, *y_b = nullptr;
  void* y = nullptr;
  float eps = 1e-5f;
  // optional A transform of the pre-GEMM: A = silu(GroupNorm(A)) (one group per sequence of gn_T rows),
  // statistics from glu_dwconv's partial sums (gn_nblk pairs per sequence)
  const float* gn_partial = nullptr;
  int gn_nblk = 0, gn_T = 0;
  const float *gn_g = nullptr, *gn_b = nullptr;
  // optional X source instead of X: the TS-VAD per-speaker input rows [ts_embed | mix] built on load
  // (build_speaker_input_kernel's layout, no positional encoding): row (s = b*NS + spk, t) of T_seq
  // rows per sequence = ts[s][0..SE) | mix[b][t][0..SE) (zeros for t >= Tmix), SE = 192
  const float* x_ts = nullptr;
  const float* x_mix = nullptr;
  int x_ldmix = 0, x_Tmix = 0, x_NS = 0, T_seq = 0;
  // optional output: bf16(acc) in the speakers-to-channels layout (B, T_seq, NS * 384), row (b*NS + spk, t)
  // -> (b, t) columns spk*384 .. (speakers_to_channels); with Xo == nullptr the fp32 rows are not written
  void* yt = nullptr;
  int yt_NS = 0;
  // start offset of the odd workgroups, in s_sleep(64) units (set by rowprog()):
  // half the CUs run their epilogue store burst while the other half streams MFMAs
  int stagger = 0;
  // diagnostics (sd_debug_rowprog_probe): per wave, lane 0 accumulates s_memtime cycles of the tile's phases
  // into probe[(block * 8 + wave) * 8 + k] (k: 0 whole, 1 piece waits, 2 refill issue, 3 epilogue, 4 loads)
  unsigned long long* probe = nullptr;
  // X / Xo in the MFMA-tiled layout (M % 16 == 0): 16-row group g, feature f = 16 ft + 4 q + r of row 16 g + l at
  // float ((g * 24 + ft) * 64 + l + 16 q) * 4 + r -- each wave's 16 x 384 fp32 residual block is 24 contiguous
  // 1-KiB runs, one per load / store instruction (row-major it is 16 scattered 64-B pieces per instruction).  The
  // residual stream between row programs is private to them (run_conformer_stack), so it stays tiled in between.
  int x_tiled = 0, xo_tiled = 0;
  // A in the tiled layout of the pre-GEMM's B-operand fragments (M % 16 == 0): row 16 g + l, feature
  // f = 32 kk + 8 q + j at bf16 ((g * 12 + kk) * 64 + l + 16 q) * 8 + j, so fragment kk of a 16-row group is one
  // contiguous 1-KiB run (mha_block writes it with out_tiled)
  int a_tiled = 0;
  int y_tiled = 0;   // y written in the a_tiled layout (for mha_block, MhaBlockArgs::y_tiled)
};
bool rowprog_supported(int D, int hidden, bool bf16);
void rowprog(const RowProgArgs& a, const char* name, hipStream_t st);
// Host packers (bf16 MFMA fragment pieces): W0 (384, 384) row-major; W1 (hidden, 384), W2 (384, hidden).
std::vector<uint16_t> rowprog_pack_pre(const std::vector<float>& W, int N, int K);
// The FFN's LayerNorm (ln_g, ln_b) is folded: W1' = W1 diag(ln_g), b1_folded = W1 ln_b + b1.
std::vector<uint16_t> rowprog_pack_ffn(const std::vector<float>& W1, const std::vector<float>& W2, int hidden,
                                       const std::vector<float>& ln_g, const std::vector<float>& ln_b,
                                       const std::vector<float>& b1, std::vector<float>& b1_folded);
void mha_block(const MhaBlockArgs& a, hipStream_t st, int variant = -1);   // variant: tests (-1: the env's)

// ---------------------------------------------------------------- ssnd_ops.hip
// Multi-head attention core on separate fp32 q / k / v row sets (SSND decoder cross and self
// attention, ssnd_model.py:261-266): row i of batch b at ptr + b * bs + i * ld, head h at
// columns h*hd..; out (B, Nq) rows likewise.  key_len (device int32 per b) optional.
struct MhaSmallArgs {
  const float* q = nullptr; int ldq = 0; int64_t q_bs = 0;
  const float* k = nullptr; int ldk = 0; int64_t k_bs = 0;
  const float* v = nullptr; int ldv = 0; int64_t v_bs = 0;
  float* o = nullptr; int ldo = 0; int64_t o_bs = 0;
  int B = 0, Nq = 0, Tk = 0, nh = 0, hd = 0;
  float scale = 1.f;
  const int* key_len = nullptr;
};
void mha_small(const MhaSmallArgs& a, hipStream_t st);
// dst row r = src row r % src_rows (D floats per row).
void tile_rows(const float* src, int src_rows, int D, float* dst, int dst_rows, hipStream_t st);
// out[r, j] = mean_t sigmoid(x[r, t]) * w[j] + b[j], t < T, j < N.
void mean_sigmoid_affine(const float* x, int rows, int T, int ldx, const float* w, const float* b, int N, float* out,
                         int ldo, hipStream_t st);

// Stream-ordered zeroing of `bytes` (4-byte words) as a kernel: every forward uses it instead of
// hipMemsetAsync so that a captured forward holds no memset node (ops.hip).
void zero_fill(void* p, size_t bytes, hipStream_t st);
void fill_u32(void* p, size_t bytes, uint32_t value, hipStream_t st);   // the same with any 32-bit word

// ---------------------------------------------------------------- ts-vad glue
// BatchNorm1D + ReLU applied by the consumer of a conv output x = conv + bias (model.py:161-171, used at :255
// and :393): v = relu(a[c] x + b[c]), or v = relu(x) for every window of a reference forward (a group of
// `group` consecutive windows) whose BN input held a non-finite value: BatchNorm1D skips its BatchNorm for the
// WHOLE batch then.  a == null: v = x (no BN here).  grp: per-group flags (nonfinite_windows) or null.
struct BnRelu {
  const float* a = nullptr;
  const float* b = nullptr;
  const int* grp = nullptr;
  int group = 1;
  int win0 = 0;   // the kernel's window 0 is window win0 of the batch (a window slice): group (w + win0) / group
};
// Non-finite scan of per-window inputs x (B windows of per_win floats, 16-B aligned rows): win[w] |= 1 and
// grp_a[w / group] |= 1, grp_b[w / group] |= 1 (each nullable) for every window holding a NaN / Inf.  The
// flags must be zeroed before (stream-ordered).  The reference's NaN reaches every BN input value of its
// window (torch's conv / BN / ReLU / mean propagate it; CAM++'s context mean spreads it over all frames),
// while these kernels' ReLUs (v_max_f32) drop NaN, so the flag is taken at the source.
void nonfinite_windows(const float* x, int B, int64_t per_win, int group, int* win, int* grp_a, int* grp_b,
                       hipStream_t st);
// rows of `per_win` floats of every window w with win_a[w] | win_b[w] set -> NaN (the reference's logits of a
// window with a non-finite input are NaN; win_b nullable).
void poison_windows(float* x, int B, int64_t per_win, const int* win_a, const int* win_b, hipStream_t st);
// rows (b, spk, t) of a (B*NS*T, 2E) buffer: [ts[b,spk,:] | mix[b,t,:]] (+ pe[t]).
// mix rows t >= Tmix read as zeros (the pad of model.py:703-710 / :852-854).
// model.py:862-877 (ts_embeds repeat + cat) and :876 PositionalEncoding.
void build_speaker_input(const float* ts, const float* mix, int ldmix, int Tmix, int B, int NS,
                         int T, int E, const float* pe, float* out, hipStream_t st, const BnRelu& mix_bn = BnRelu());

// Chunk-streaming speaker input (ts_vad2_streaming/model.py:767-777): row (b, spk, t) =
// [ts[b, spk] | mix[b, t]] * scale + pe[pos(t)], pos(t) = start(t / C) + t % C with start(c) = 0
// (left < 0: the whole history is cached) or max(0, c - left) * C.  out (B * NS * T, 2E).
void build_stream_input(const float* ts, const float* mix, int B, int T, int NS, int E, float scale,
                        const float* pe, int C, int left, float* out, hipStream_t st);
// x[r, :] += pe[r % T, :]  (rows of length D at stride ld)
// (bn: the rows' BatchNorm1D + ReLU first, window = row / T)
void add_pe(float* x, int rows, int T, int D, int ld, const float* pe, hipStream_t st, const BnRelu& bn = BnRelu());

// Per-frame mean/std over channels then Linear(2 -> E): model.py:689-696.
// bn: speech_down_or_up's BatchNorm1D + ReLU applied to x first (window = row / rows_per_window).
void gsp_fc(const float* x, int rows, int C, int ldx, const float* w /*E x 2*/,
            const float* bias, int E, float* out, int ldo, hipStream_t st, const BnRelu& bn = BnRelu(),
            int rows_per_window = 1);

// (B*NS, T, E) speaker-major rows -> (B, T, NS*E) channel-concatenated rows.
void speakers_to_channels(const float* x, int B, int NS, int T, int E, void* out, bool out_bf16,
                          hipStream_t st);

// ---------------------------------------------------------------- conformer conv module
// Depthwise conv over time (kernel k, pad (k-1)/2, with bias), y: (S, T, C).
// glu_in: x is the pw1 output (S, T, 2C) with rows interleaved [16 values | 16 gates]
// (glu_interleave_row) and the GLU is applied on load; else x is already gated (S, T, C).
// Writes per (sequence, channel-block) partial sums for GroupNorm(1, C), or with
// fused_silu (BatchNorm already folded into w/bias) stores SiLU(y) and no partials.
void glu_dwconv(const void* x, int S, int T, int C, const float* w /*C x k*/,
                const float* bias, int k, void* y, float* partial /*S x nblk x 2*/, bool fused_silu,
                bool glu_in, bool io_bf16, hipStream_t st);
// GroupNorm(num_groups=1) over (T, C) of each sequence, affine, then SiLU (in place).
void groupnorm_silu(void* y, int S, int T, int C, const float* partial, const float* g,
                    const float* b, float eps, bool io_bf16, hipStream_t st);

// ---------------------------------------------------------------- lstm
// One bidirectional (or unidirectional) LSTM layer recurrence given the
// precomputed input projections gx (B, T, ndir*4H) (bias_ih + bias_hh folded in).
// whh: (ndir, 4H, H) fp32.  out: (B, T, ldo) at column dir*H.
// h0/c0 optional (ndir, B, H); hT/cT optional outputs (ndir, B, H).
// whh_bf16 (optional, same layout in bf16 bits): bf16-MFMA recurrence (bf16 mode); the
// cell state, gates and h stay fp32, h is rounded to bf16 only as the MFMA operand.
// whh_lo (optional, with whh_bf16 = bf16(W) as the hi part): bf16(W - hi), the bf16x3 mode's split
// recurrence (W_lo h_hi + W_hi h_lo + W_hi h_hi, h exchanged as hi + lo); where the persistent kernel cannot
// run, the exact-f32 step kernel (never the bf16 one).
// work: per-handle device scratch of lstm_work_floats(B, H, ndir) floats (the persistent bf16
// kernel keeps its h exchange and counters there).  host_err (optional, the DEVICE address of a pinned
// slot of the handle's PinnedFlags): a persistent launch whose poll timed out sets it to 1 from the
// kernel itself and nothing ever writes 0 there but the host's take(), so the report is sticky across
// any number of forwards enqueued before the handle raises kErrHip (sd_tsvad_status / sd_eda_status after
// the forward, or at the latest its next call).
int64_t lstm_work_floats(int B, int H, int ndir);
// Exchange floor of the persistent recurrence (sd_probe_lstm_handoff): us per step of its hand-off alone.
float lstm_handoff_probe(int steps, hipStream_t st);
// The same exchange on 8-byte {data, tag} granules (sd_probe_lstm_granule; lstm.hip): us per step.
// nwg 2: the two-workgroup 1-to-1 form (each lane polls only the other workgroup's half of its operand).
float lstm_granule_probe(int steps, hipStream_t st, int nwg = 4);
void lstm_recurrence(const float* gx, int B, int T, int H, int ndir, const float* whh,
                     const int* lengths, const float* h0, const float* c0, float* out, int ldo,
                     float* hT, float* cT, float* work, hipStream_t st, const void* whh_bf16 = nullptr,
                     int* host_err = nullptr, const void* whh_lo = nullptr);

// ---------------------------------------------------------------- frontend
// Kaldi fbank (torchaudio.compliance.kaldi.fbank semantics used by
// ts_vad_dataset.py:39-52): 25 ms / 10 ms frames, snip_edges, DC removal,
// pre-emphasis 0.97, hamming, 512-point power spectrum, HTK mel, log(max(.,eps)).
void fbank_kaldi(const float* wav, int64_t n_samples, float in_scale, int n_frames,
                 const float* mel_fb /*n_mels x 257*/, int n_mels, float* out,
                 hipStream_t st, int window = 0 /*0 hamming, 1 povey*/);

// Per-window CMN + zero pad: out[w, j, :] = feats[start_w + j, :] - mean_w for j < n_w,
// 0 for n_w <= j < T_out (ts_vad_dataset.py:55 + collater padding :676).
void window_cmn(const float* feats, int n_mels, const int* win_start, const int* win_n,
                int n_win, int T_out, float* out, hipStream_t st);

}  // namespace sd

namespace sd {
// Device-side weight packing (test ops): torch (N, Cin, taps) -> conv_gemm layout.
void pack_weight(const float* w, int N, int Cin, int taps, void* out, bool bf16, hipStream_t st);
}  // namespace sd

namespace sd {
// sigmoid=false: inputs are probabilities already (sd_overlap_mean).  numpy's pairwise
// summation is reproduced for up to kOverlapMaxWindows covering windows per frame.
constexpr int kOverlapMaxDepth = 6;
constexpr int kOverlapMaxWindows = (128 << kOverlapMaxDepth) / 2;
void overlap_average(const float* logits, int n_win, int NS, int Tw, const int* start, const int* len,
                     int dis, int chunk, int n_frames, float* out, hipStream_t st, bool sigmoid = true);

// ---------------------------------------------------------------- postprocess.hip
struct ThresholdSet {
  static constexpr int kMax = 16;
  int n = 0;
  int strict = 0;   // 1: speech iff x > thr (EEND make_rttm.py), 0: x >= thr (TS-VAD infer.py)
  float v[kMax] = {};
};
int segments_max_frames();
// scipy.signal.medfilt (zero padded, odd k <= 63) over each of `rows` tracks of T frames.
void medfilt(const float* x, int rows, int T, int k, float* y, hipStream_t st);
// Per (row, threshold): binarise, fill short silences, drop short speech, emit
// [begin, end) runs.  seg_*: (rows * thr.n, cap); n_seg: (rows * thr.n).
void run_segments(const float* med, int rows, int T, const ThresholdSet& thr, int lim_sil, int lim_sp, int cap,
                  int* seg_begin, int* seg_end, int* n_seg, hipStream_t st);
}  // namespace sd

namespace sd {
void f32_to_bf16(const float* x, int64_t n, void* y, hipStream_t st);
void bf16_to_f32(const void* x, int64_t n, float* y, hipStream_t st);

// ---------------------------------------------------------------- eend frontend + EDA glue (eend.hip)
// librosa-style centred STFT (float64) -> log10 mel power: out (n_frames, n_mels) float64.
void stft_logmel(const float* wav, int64_t n_samples, int n_frames, int n_fft, int hop, int win_len,
                 const float* mel_fb /*(n_mels, n_fft/2+1)*/, int n_mels, double* out, hipStream_t st);
// Streaming frontend of one FS-EEND chunk (sd_fseend_stream_push_audio): the logmel frames the splice of
// model frames [cursor[0], cursor[0] + rows) reads (frame0 = cursor[0] * sub - context, (rows - 1) * sub +
// 2 context + 1 frames into lm), then the spliced rows into out (rows, ld_out).  bound (device int[2]):
// [0] samples of the input (INT_MAX while open), [1] STFT frames of the input (INT_MAX while open).
// Per frame the arithmetic of stft_logmel + splice_subsample, bit for bit.
void stream_frontend(const float* wav, int64_t cap_samples, int rows, int n_fft, int hop, int win_len,
                     const float* mel_fb, int n_mels, int context, int sub, const int* cursor, const int* bound,
                     double* lm, float* out, int ld_out, hipStream_t st);
void col_mean(const double* x, int rows, int cols, double* mean, hipStream_t st);
// out (n_out, ld_out) f32: row r = splice of frame r*sub (±context, zero pad), minus mean (nullable).
void splice_subsample(const double* lm, int n_frames, int n_mels, const double* mean, int context, int sub,
                      int n_out, float* out, int ld_out, hipStream_t st);
// y[s, t] = x[s, perm[s, t]] for t < lengths[s], else x[s, t].  Rows of D floats.
void gather_rows(const float* x, int S, int T, int D, const int* perm, const int* lengths, float* y,
                 hipStream_t st);
void fill_rows(const float* row, int D, int rows, float* y, hipStream_t st);
// probs (S, n_att) = sigmoid(att · lw + lb); act (S, T, n_att-1) = sigmoid(emb · att[:-1]ᵀ).
void attractor_scores(const float* emb, int S, int T, int E, const float* att, int n_att, const float* lw,
                      const float* lb, float* probs, float* act, hipStream_t st);

// ---------------------------------------------------------------- fs-eend glue (fseend_ops.hip)
// y = x / |x| per row (D <= 512); slabs > 1: x is the sum of split-K slabs x + k * rows * D
void row_l2norm(const float* x, int rows, int D, float* y, hipStream_t st, int slabs = 1);
// out (T*C, D): out[t*C + c] = g[t] + p[c]
void slot_init(const float* g, int T, int C, int D, const float* p, float* out, hipStream_t st);
// scores (T, C) = emb[t]·att[t,c]/|att[t,c]|; write_norm: att normalised in place.
void slot_scores(const float* emb, float* att, int T, int C, int D, float* scores, bool write_norm,
                 hipStream_t st);
}  // namespace sd

namespace sd {
// ---------------------------------------------------------------- streaming (stream_ops.hip)
// Chunked causal attention against a K/V history (see stream_ops.hip).  Element offsets:
// query i of sequence s at q + i*q_tok + s*q_seq (+ head*64); key j at k/v + j*kv_tok + s*kv_seq;
// output like the query.  Query i sits at absolute position *pos + i and sees keys
// j <= *pos + i + delay; keys [0, *pos + nq) must be in the history.
struct DecodeAttnArgs {
  const void* q = nullptr;
  int64_t q_tok = 0, q_seq = 0;
  const void* k = nullptr;
  const void* v = nullptr;
  int64_t kv_tok = 0, kv_seq = 0;
  void* out = nullptr;
  int64_t o_tok = 0, o_seq = 0;
  int nseq = 1, nq = 1, nh = 1, hd = 64;
  float scale = 1.f;
  const int* pos = nullptr;   // device cursor
  int delay = 0;
  int max_keys = 0;           // history capacity: grid coverage
  int n_blocks = 0;           // workspace partials per (sequence, head) >= attn_decode_blocks(max_keys)
  float* ws = nullptr;        // nseq*nh*n_blocks*nq*(2+hd) floats
  bool io_bf16 = false;
  // optional: nseq*nh counters, zeroed once when allocated and shared only by launches that run one after
  // another -- the last block of each (sequence, head) then merges the partials (no combine launch)
  unsigned* cnt = nullptr;
  // optional, with cnt: the out-projection in the same launch (o2 = o W_outᵀ + b_out, rows laid out as out's, D =
  // nh * 64 <= 256): each (sequence, head)'s merging block publishes its head's partial write-through to ws2
  // (nseq*nh*nq*D floats) and the last head of a sequence (cnt2: nseq counters, zeroed once) sums them in head order
  const void* wo = nullptr;   // packed [D][D], io dtype
  const float* bo = nullptr;
  void* o2 = nullptr;
  float* ws2 = nullptr;
  unsigned* cnt2 = nullptr;
};
int attn_decode_blocks(int max_keys);
// FS-EEND streaming decoder, slot-attention sub-block of the fusion layer (fs_eend.py:468-471) for one chunk:
//   y = LN(x + t) (-> ln_out, the next residual);  qkv = y W_inᵀ + b_in;  o = softmax(q kᵀ scale) v across the
//   C slots of each frame, per head;  out = o W_outᵀ + b_out.
// ONE launch of nh workgroups (one per head): a head's q/k/v and attention stay in LDS, its out-projection
// partial (the head's 64 input features) is published write-through and the last workgroup to count itself
// sums the nh partials in head order (MI355X guide hand-off row 1; cnt monotonic, zeroed once).
// Supported: D == 256, D / nh == 64, c * C <= 16, C <= 8; returns false otherwise (caller runs the three-launch
// path).
struct SlotBlockArgs {
  const float* ln_x = nullptr;
  const void* ln_t = nullptr;
  bool t_bf16 = false;
  const float *ln_g = nullptr, *ln_b = nullptr;
  float eps = 1e-5f;
  float* ln_out = nullptr;
  const void* w_in = nullptr;   // packed [3D][D]
  const float* b_in = nullptr;
  const void* w_out = nullptr;  // packed [D][D]
  const float* b_out = nullptr;
  bool w_bf16 = false;
  void* out = nullptr;          // (c*C, D), bf16 when out_bf16
  bool out_bf16 = false;
  float* ws = nullptr;          // nh * c*C * D floats
  unsigned* cnt = nullptr;
  int c = 1, C = 1, D = 256, nh = 4;
  float scale = 0.125f;
};
bool stream_slot_block(const SlotBlockArgs& a, hipStream_t st);
// FS-EEND streaming feed-forward sub-block (nn.TransformerEncoderLayer linear1 -> relu -> linear2, fs_eend.py:
// 196-204 / 474-477) for one chunk of n rows, its input post-LN folded in:  y = LN(x + t) (-> ln_out);
// out = relu(y W1ᵀ + b1) W2ᵀ + b2.  ONE launch: each workgroup owns a slice of the hidden units, its down-projection
// partial is published write-through and the last workgroup to count itself sums the partials in workgroup order
// (cnt wraps to 0 per launch, zeroed once).  Supported: D == 256, F == 2048, 1 <= n <= 8, 16-B aligned operands;
// returns false otherwise (caller runs the two skinny GEMMs).  ws: 128 * 8 * D floats.
struct FfnPairArgs {
  const float* ln_x = nullptr;
  const void* ln_t = nullptr;
  bool t_bf16 = false;
  const float *ln_g = nullptr, *ln_b = nullptr;
  float eps = 1e-5f;
  float* ln_out = nullptr;
  const void* w1 = nullptr;   // packed [F][D]
  const float* b1 = nullptr;
  const void* w2 = nullptr;   // packed [D][F]
  const float* b2 = nullptr;
  bool w_bf16 = false;
  void* out = nullptr;        // (n, D), bf16 when out_bf16
  bool out_bf16 = false;
  float* ws = nullptr;
  unsigned* cnt = nullptr;
  int n = 1, D = 256, F = 2048;
};
bool stream_ffn_pair(const FfnPairArgs& a, hipStream_t st);
// returns true when it also ran the out-projection (wo set, the fused merge taken)
bool attn_decode(const DecodeAttnArgs& a, hipStream_t st);
// dst row (cursor*mult + r) = src row r, r < rows (16-B aligned rows of width_bytes).
void kv_append(const void* src, int64_t ld_src_bytes, int rows, int width_bytes, void* dst, int64_t ld_dst_bytes,
               const int* cursor, int mult, hipStream_t st);
// dst (rows, D) = hist rows [*cursor - pad, ...), zero outside [0, *n_valid).
void gather_window(const float* hist, int D, const int* cursor, const int* n_valid, int pad, int rows, float* dst,
                   hipStream_t st);
// *cursor += by; mirror (optional) = new value.
void cursor_advance(int* cursor, int by, int* mirror, hipStream_t st);
// Encoder chunk tail: v = LN(x + t)*g + b for rows < c (D % 256 == 0, D <= 1024); v -> hist row
// (*cursor + r); then *cursor += c and *mirror = *cursor.
void stream_enc_finish(const float* x, const void* t, bool t_bf16, const float* g, const float* b, float eps, int c,
                       int D, float* hist, int* cursor, int* mirror, hipStream_t st);
// Decoder chunk tail: a = LN(x + t)*g + b for the c*C (frame, slot) rows, scores[f, s] =
// emb[f]·a/|a| (fs_eend.py:88-90); then *cursor += c.
void stream_dec_finish(const float* x, const void* t, bool t_bf16, const float* g, const float* b, float eps, int c,
                       int C, int D, const float* emb, float* scores, int* cursor, hipStream_t st);
}  // namespace sd
