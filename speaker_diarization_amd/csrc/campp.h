// CAM++ (egs/alimeeting/ts_vad2/cam_pplus_wespeaker.py) on gfx950.
//
// CamTrunk is the FCM head + xvector up to transit3 (cam_pplus_wespeaker.py:271-372),
// shared by the TS-VAD speech encoder (get_time_out=True, model.py:385-395) and the
// target-speaker embedding extractor CamppModel (get_time_out=False: out_nonlinear ->
// StatsPool -> DenseLayer(batchnorm_), :374-399), which produces the (n_chunks, 192)
// embeddings generate_chunk_speaker_embedding_from_modelscope_for_diarization.py:271-304
// writes and ts_vad_dataset.py:494-537 reads back.
#pragma once
#include <string>
#include <vector>
#include "encoder.h"

namespace sd {

struct DenseL {
  ConvL bottleneck;       // nonlinear1 (prologue) -> linear1 (1x1) -> nonlinear2 (epilogue, relu)
  ConvL local;            // cam_layer.linear_local (k3, dilation)
  int dil = 1;
  const float *c1w = nullptr, *c1b = nullptr, *c2w = nullptr, *c2b = nullptr;
  int c1 = 0, c2 = 0;
};

// 1-D conv (channel-last rows of stride lda) as an implicit GEMM; out row stride ldo.
ConvGemmArgs cam_conv1d(Tens in, int B, int T, int lda, const ConvL& L, int stride, int pad, int dil, Tens out,
                        int ldo);
// Conv weight + optional folded BatchNorm (alpha/beta epilogue) + optional conv bias.
ConvL load_conv_bn(ParamStore& ps, DeviceArena& arena, bool bf16, const std::string& wname,
                   const std::string& bn, const std::string& bias = "");

class CamTrunk {
 public:
  static constexpr int kChannels = 512;   // transit3 output width
  // Reads `prefix`head.* and `prefix`xvector.{tdnn,block*,transit*,out_nonlinear}.*.
  void load(ParamStore& ps, DeviceArena& arena, const std::string& prefix, bool bf16);
  void alloc(DeviceArena& arena, int max_batch, int max_frames);
  static int out_frames(int Tf) { return (Tf - 1) / 2 + 1; }
  // fbank (B, Tf, 80) fp32 -> transit3 output (B, out_frames(Tf), 512), before out_nonlinear.
  // b0: the call covers windows [b0, b0 + B) of a batch (fbank = the batch's base; the result is the
  // batch's output map with this slice filled in), so disjoint slices may run on different streams.
  Tens forward(const float* fbank, int B, int Tf, hipStream_t st, int b0 = 0) const;
  // Folded out_nonlinear BatchNorm (the ReLU follows it).
  const float* out_s() const { return out_s_; }
  const float* out_h() const { return out_h_; }
  bool bf16() const { return bf16_; }
  // kErrHip if a cam_dense launch of an earlier forward lost a split item's exchange (its outputs are NaN;
  // cannot happen by construction, reported instead of hanging the GPU)
  void raise_if_set() const {
    err_.raise_if_set("cam_dense: the two parts of a split item lost their exchange (outputs poisoned with NaN)");
  }

 private:
  float* ws(DeviceArena& a, size_t n) { return static_cast<float*>(a.alloc(n * sizeof(float))); }
  bool bf16_ = false;
  ConvL fcm_conv1_;  // fp32 3x3 Cin=1 weights (32x9) + folded bn
  struct ResBlock { ConvL c1, c2, sc; bool has_sc; int stride; };
  std::vector<ResBlock> fcm_blocks_;
  ConvL fcm_conv2_;
  ConvL tdnn_;
  std::vector<std::vector<DenseL>> dense_;
  std::vector<ConvL> transit_;
  const float *out_s_ = nullptr, *out_h_ = nullptr;
  // Workspace.
  float *fcmA_ = nullptr, *fcmB_ = nullptr, *fcmC_ = nullptr, *x0_ = nullptr;
  float *d_[3] = {nullptr, nullptr, nullptr}, *x4_ = nullptr, *tmp_ = nullptr, *gate_ = nullptr;
  void* dense_rec_ = nullptr;          // cam_dense exchange records, one per window
  unsigned* dense_cnt_ = nullptr;      // cam_dense counters, one set per window (zeroed once)
  mutable PinnedFlags err_;            // cam_dense's sticky lost-exchange report (slot 0)
};

struct CamppConfig {
  int feat_dim = 80;
  int embedding_size = 192;
  int max_batch = 96;        // extract_embed batch_size default (generate_chunk_...py:45)
  int max_frames = 598;      // 6 s chunks: 1 + (96000 - 400) / 160
  bool bf16 = false;
};

class CamppModel {
 public:
  explicit CamppModel(const CamppConfig& c) : cfg_(c) {}
  ParamStore& params() { return ps_; }
  void finalize();
  bool finalized() const { return finalized_; }
  size_t device_bytes() const { return arena_.total(); }
  // fbank (B, Tf, 80) -> emb (B, embedding_size) (forward(x), :388-399) and/or
  // time_out (B, T', 512) channel-last = relu(out_nonlinear(x)) (forward(x, get_time_out=True)).
  void forward(const float* fbank, int B, int Tf, float* emb, float* time_out, hipStream_t st);

 private:
  CamppConfig cfg_;
  ParamStore ps_;
  DeviceArena arena_;
  bool finalized_ = false;
  CamTrunk trunk_;
  ConvL dense_;            // xvector.dense: Conv1d(1024 -> E, 1, bias=False) + BatchNorm1d(affine=False)
  float* stats_ = nullptr; // (max_batch, 1024) [mean | std]
};

}  // namespace sd
