// Chunk-streaming TS-VAD (egs/alimeeting/ts_vad2_streaming/model.py) on gfx950.
//
// The reference decodes a window chunk by chunk (forward_chunk_by_chunk_temp1, :594-655):
// CAM++ + down conv on each chunk alone, then per-speaker and multi-speaker wenet pre-LN
// transformers whose attention sees the KV caches of earlier chunks, backend_down over the
// chunk alone, fc.  Everything except the caches is chunk-local, and the caches only make
// chunk c attend to the keys of chunks max(0, c - left) .. c.  So the whole window runs as
// ONE forward: CAM++ batched over the chunks, block-causal attention masks (AttnArgs::chunk /
// left), the positional-encoding offsets the caches imply (offset - cache length, :774-776),
// backend_down batched over the chunks — the same numbers without a per-chunk host loop.
#pragma once
#include <vector>
#include "campp.h"

namespace sd {

struct TsvadStreamConfig {
  int max_num_speaker = 4;
  int max_labels = 200;        // label frames (25 Hz) per window
  int max_windows = 1;         // windows per forward
  bool bf16 = false;
  int num_transformer_layer = 2;
  int num_attention_head = 4;
  int embed_dim = 384;
  int ffn_dim = 1536;
  int speaker_embed_dim = 192;
};

struct WenetLayerL {           // transformer_chunk_streaming.TransformerEncoderLayer (pre-LN)
  PackedW qkv, out, w1, w2;    // linear_q|k|v packed as one (3E, E) projection
  const float *qkv_b = nullptr, *out_b = nullptr, *b1 = nullptr, *b2 = nullptr;
  const float *n1g = nullptr, *n1b = nullptr, *n2g = nullptr, *n2b = nullptr;
};

class TsvadStreamModel {
 public:
  explicit TsvadStreamModel(const TsvadStreamConfig& c) : cfg_(c) {}
  ParamStore& params() { return ps_; }
  void finalize();
  bool finalized() const { return finalized_; }
  size_t device_bytes() const { return arena_.total(); }
  // B independent windows: feats (B, 4 * T_lab, 80) fbank (padded to 4 x labels,
  // model.py:614-618); ts (B, NS, 192); chunk = decoding_chunk_size (label frames),
  // left = num_decoding_left_chunks; logits (B, NS, T_lab) pre-sigmoid.
  void forward(const float* feats, const float* ts, int B, int T_lab, int chunk, int left, float* logits,
               hipStream_t st);

 private:
  WenetLayerL load_layer(const std::string& prefix);
  void run_layers(const std::vector<WenetLayerL>& L, float* X, int S, int T, int chunk, int left, hipStream_t st);
  float* ws(size_t n) { return static_cast<float*>(arena_.alloc(n * sizeof(float))); }

  TsvadStreamConfig cfg_;
  ParamStore ps_;
  DeviceArena arena_;
  bool finalized_ = false;
  CamTrunk cam_;               // embed.speech_encoder.*
  ConvL down_;                 // embed.speech_down_or_up (Conv1d k5 s2 + BatchNorm1D + ReLU)
  std::vector<WenetLayerL> single_, multi_;
  ConvL backend_down_;         // Conv1d(NS*E -> E, k5, p2) + BatchNorm1D + ReLU
  ConvL fc_;
  const float* pe_ = nullptr;  // pos_encoder.pe (max_len, E)
  int pe_len_ = 0;
  float *mix_ = nullptr, *X_ = nullptr, *Y_ = nullptr, *QKV_ = nullptr, *AO_ = nullptr, *T1_ = nullptr,
        *H_ = nullptr, *X2_ = nullptr;
};

}  // namespace sd
