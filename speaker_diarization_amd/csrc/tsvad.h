// Native TS-VAD inference runner (owns folded weights + workspace).
#pragma once
#include <vector>
#include "campp.h"

namespace sd {

struct TsvadConfig {
  int variant = 0;            // 0: CAM++ + transformer (model.py:758-897); 1: CAM++_ots_vad (669-756)
  int max_num_speaker = 4;
  int rs_len = 4;
  int max_batch = 64;
  int max_fbank_frames = 398;
  bool bf16 = false;
  int num_transformer_layer = 2;
  int num_attention_head = 4;
  int embed_dim = 384;
  int ffn_dim = 1536;
  int speaker_embed_dim = 192;
  int conformer_layers = 6;
  int conformer_heads = 8;
  int conformer_ffn = 512;
  int conformer_kernel = 31;
  int lstm_hidden = 256;
};

class TsvadModel {
 public:
  explicit TsvadModel(const TsvadConfig& c) : cfg_(c) {}
  ParamStore& params() { return ps_; }
  void finalize();
  // ref_speech (B, T_fb, 80) fbank, target_speech (B, NS, 192), logits out (B, NS, T_lab).
  // forward_batch: windows per reference forward call, the scope of BatchNorm1D's NaN bypass (model.py:161-171),
  // i.e. the batch a NaN window disables speech_down_or_up's / backend_down's BatchNorm for; 0: the whole call.
  // force: the call is part of a larger reference batch that holds a non-finite input elsewhere: bit 0 skips
  // both BatchNorms for every window (a non-finite fbank), bit 1 backend_down's (a non-finite v0 embedding).
  void forward(const float* ref_speech, const float* target_speech, int B, int T_fb, int T_lab,
               float* logits, hipStream_t st, int forward_batch = 0, int force = 0);
  bool finalized() const { return finalized_; }
  size_t device_bytes() const { return arena_.total(); }
  // Diagnostics (graph-replay investigation): captures forward() once into a hipGraph on a capture stream
  // (the fork / join side stream included), then replays it `replays` times on st; `dot` (nullable) receives
  // hipGraphDebugDotPrint of the captured graph.
  void forward_graph(const float* ref_speech, const float* target_speech, int B, int T_fb, int T_lab, float* logits,
                     int replays, const char* dot, hipStream_t st);
  // Device buffers of the forward's stages for stage-by-stage comparisons: 0 mix (speech_down_or_up conv),
  // 1 mixg (gsp_fc), 2 X2 (conformer stack output), 3 H (BiLSTM gates), 4 Y (BiLSTM output).
  void debug_buffer(int which, void** ptr, int64_t* bytes) const;
  // waits for `st` and raises kErrHip if a persistent LSTM of the forwards enqueued on it timed out
  void status(hipStream_t st) {
    SD_HIP(hipStreamSynchronize(st));
    lstm_err_.raise_if_set();
    cam_.raise_if_set();
  }
  ~TsvadModel();

 private:
  ConvL conv_bn(const std::string& wname, const std::string& bn, const std::string& bias = "");
  LayerLoader loader() { return LayerLoader{ps_, arena_, cfg_.bf16}; }
  EncoderWork enc_work() const { return EncoderWork{Y_, QKV_, AO_, H_, partial_, cfg_.bf16}; }
  void alloc_workspace();
  float* ws(size_t n) { return static_cast<float*>(arena_.alloc(n * sizeof(float))); }

  TsvadConfig cfg_;
  ParamStore ps_;
  DeviceArena arena_;
  PinnedFlags lstm_err_;   // poll-timeout reports of the persistent LSTMs (lstm.hip), one slot each
  bool finalized_ = false;

  CamTrunk cam_;     // speech_encoder.* (CAM++ get_time_out=True)
  ConvL down_;        // speech_down_or_up conv: epilogue = + bias only (its BatchNorm1D is down_bn_)
  BnRelu down_bn_, backend_bn_;   // folded BatchNorms, applied (or bypassed) by the consumers
  int* nonfinite_ = nullptr;      // [win_fbank B | win_ts B | grp_speech B | grp_backend B]
  const float *gsp_w_ = nullptr, *gsp_b_ = nullptr;
  const float* pe_ = nullptr;
  int pe_len_ = 0;
  std::vector<TransformerL> single_, multi_;
  ConvL backend_down_;
  std::vector<ConformerL> conf_;
  PackedW lstm_ih_;
  const float *lstm_b_ = nullptr, *lstm_hh_ = nullptr;
  const void* lstm_hh_bf_ = nullptr;   // bf16 copy of W_hh (bf16 mode; the hi part in fp32 mode)
  const void* lstm_hh_lo_ = nullptr;   // bf16(W_hh - hi) (fp32 handles: the bf16x3 split recurrence)
  ConvL fc_;

  // CAM++ trunk of a large batch as two window slices, the second on side_ (fork / join events on the
  // caller's stream): the per-layer launches of one slice fill the CUs the other slice's last round of
  // workgroups leaves idle (cam_dense: 600 items on 256 CUs = 2.34 rounds of 3).
  hipStream_t side_ = nullptr;
  hipEvent_t ev_fork_ = nullptr, ev_join_ = nullptr;

  // Workspace.
  float *mix_ = nullptr, *mixg_ = nullptr;
  float *X_ = nullptr, *Y_ = nullptr, *QKV_ = nullptr, *AO_ = nullptr, *H_ = nullptr;
  float *X2_ = nullptr, *partial_ = nullptr, *lstm_work_ = nullptr;
};

}  // namespace sd
