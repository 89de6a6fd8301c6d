// Native EEND-EDA inference runner (eend_eda/models.py TransformerEdaModel /
// EendEdaModel + encoder_decoder_attractor.py LstmEncoderDedecoderAttractor).
#pragma once
#include <vector>
#include "encoder.h"

namespace sd {

struct EdaConfig {
  int variant = 0;          // 0 TransformerEda, 1 EendEda(transformer), 2 EendEda(conformer),
                            // 3 plain EEND TransformerModel (eend/models.py:17-101)
  int n_speakers = 2;       // variant 3: decoder Linear(n_units, n_speakers)
  int in_size = 345;
  int n_units = 256;
  int n_heads = 4;
  int n_layers = 2;
  int dim_feedforward = 2048;
  int max_seqs = 8;         // workspace: sequences per forward
  int max_frames = 2000;    // workspace: frames per sequence (chunk_size)
  int max_n_speakers = 15;  // attractors decoded
  bool bf16 = false;
};

constexpr int kEdaInPad = 8;   // input rows are padded to a multiple of 8 floats (345 -> 352)

class EdaModel {
 public:
  explicit EdaModel(const EdaConfig& c) : cfg_(c) {}
  ParamStore& params() { return ps_; }
  void finalize();
  int in_ld() const { return in_ld_; }
  // feats (S, T, ld_in) fp32 with ld_in >= in_ld(), finite values in the pad columns;
  // lengths (S) device int32 (LSTM / shuffle lengths); key_len (S) device int32 or
  // nullptr (attention key mask); perm (S, T) device int32, rows < lengths[s] hold
  // randperm(lengths[s]).  probs (S, max_n_speakers); act (S, T, max_n_speakers-1).
  void forward(const float* feats, int ld_in, int S, int T, const int* lengths, const int* key_len,
               const int* perm, float* probs, float* act, hipStream_t st);
  bool finalized() const { return finalized_; }
  size_t device_bytes() const { return arena_.total(); }
  // waits for `st` and raises kErrHip if a persistent LSTM of the forwards enqueued on it timed out
  void status(hipStream_t st) { SD_HIP(hipStreamSynchronize(st)); lstm_err_.raise_if_set(); }

 private:
  float* ws(size_t n) { return static_cast<float*>(arena_.alloc(n * sizeof(float))); }

  EdaConfig cfg_;
  ParamStore ps_;
  DeviceArena arena_;
  PinnedFlags lstm_err_;   // poll-timeout reports of the persistent LSTMs (lstm.hip), one slot each
  bool finalized_ = false;
  int in_ld_ = 352;

  ConvL in_;
  const float *norm_g_ = nullptr, *norm_b_ = nullptr;
  std::vector<TransformerL> tfm_;
  std::vector<ConformerL> conf_;
  PackedW enc_ih_;
  const float *enc_b_ = nullptr, *enc_hh_ = nullptr;
  const float *dec_b_ = nullptr, *dec_hh_ = nullptr;
  const void *enc_hh_bf_ = nullptr, *dec_hh_bf_ = nullptr;   // bf16 copies (bf16 mode; the hi part in fp32 mode)
  const void *enc_hh_lo_ = nullptr, *dec_hh_lo_ = nullptr;   // bf16(W - hi) (fp32 handles: the bf16x3 recurrence)
  const float *lin_w_ = nullptr, *lin_b_ = nullptr;
  ConvL dec_;   // variant 3: decoder Linear -> sigmoid

  float *X_ = nullptr, *Y_ = nullptr, *QKV_ = nullptr, *AO_ = nullptr, *H_ = nullptr, *partial_ = nullptr;
  float *G_ = nullptr, *Gd_ = nullptr, *att_ = nullptr, *hT_ = nullptr, *cT_ = nullptr, *lstm_work_ = nullptr;
};

}  // namespace sd
