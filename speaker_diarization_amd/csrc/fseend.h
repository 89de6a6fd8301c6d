// Native FS-EEND inference runner (fs_eend/fs_eend.py OnlineTransformerDADiarization.test).
#pragma once
#include <vector>
#include "encoder.h"

namespace sd {

struct FsEendConfig {
  int in_size = 345;
  int n_units = 256;
  int n_heads = 4;
  int enc_n_layers = 4;
  int enc_ffn = 2048;       // MaskedTransformerEncoderModel default dim_feedforward
  int dec_n_layers = 2;     // applications of the ONE shared fusion layer
  int dec_ffn = 2048;
  int conv_delay = 9;       // Conv1d kernel 2*delay+1 (padding hard-coded 9, fs_eend.py:41)
  int mask_delay = 0;
  int has_mask = 1;
  int max_seqs = 1;
  int max_frames = 10000;   // chunk_size of the infer config
  int max_nspks = 6;        // max_speakers + 2
  bool bf16 = false;
};

struct FusionL {            // TransformerEncoderFusionLayer (fs_eend.py:282-333)
  PackedW in1, out1, in2, out2, l1, l2;
  const float *in1_b, *out1_b, *in2_b, *out2_b, *b1, *b2;
  const float *n11g, *n11b, *n21g, *n21b, *n22g, *n22b;
};

class FsEendStream;

class FsEendModel {
 public:
  explicit FsEendModel(const FsEendConfig& c) : cfg_(c) {}
  ParamStore& params() { return ps_; }
  void finalize();
  int in_ld() const { return in_ld_; }
  // feats (S, T, ld_in) f32 (pad_sequence(-1) rows beyond a sequence's length);
  // lengths_host (S) frames per sequence; C = max_nspks of test().
  // preds (S, T, C); emb_out (S, T, D) and att_out (S, T, C, D) optional (normalised, as test() returns).
  void forward(const float* feats, int ld_in, int S, int T, const int* lengths_host, int C, float* preds,
               float* emb_out, float* att_out, hipStream_t st);
  bool finalized() const { return finalized_; }
  size_t device_bytes() const { return arena_.total(); }

 private:
  friend class FsEendStream;
  float* ws(size_t n) { return static_cast<float*>(arena_.alloc(n * sizeof(float))); }
  void run_fusion(float* A, int S, int T, int C, hipStream_t st);

  FsEendConfig cfg_;
  ParamStore ps_;
  DeviceArena arena_;
  bool finalized_ = false;
  int in_ld_ = 352;

  ConvL in_;
  const float *norm_g_ = nullptr, *norm_b_ = nullptr;
  std::vector<TransformerL> enc_;
  ConvL cnn_;
  PackedW conv_emb_;            // convert.weight[:, :D]
  const float* slot_bias_ = nullptr;   // (max_nspks, D): pe[c]·W_peᵀ + convert.bias
  FusionL fus_;

  float *X_ = nullptr, *Y_ = nullptr, *EMB_ = nullptr, *G_ = nullptr;
  float *A_ = nullptr, *A2_ = nullptr, *QKV_ = nullptr, *AO_ = nullptr, *H_ = nullptr;
};

}  // namespace sd
