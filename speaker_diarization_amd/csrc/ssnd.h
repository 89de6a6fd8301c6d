// SSND (egs/alimeeting/ssnd/ssnd_model.py) block inference on gfx950: the speaker-query
// cross-attention decoders of SSNDModel.infer (:752-776) behind sd_ssnd_* (include/sdiar.h).
//
//   extractor  ResNetExtractor('CAM++_wo_gsp') (:107-124, :164-170): the CAM++ trunk shared with
//              TS-VAD (CamTrunk), out_nonlinear BN-ReLU as the prologue of output_proj
//              (Linear 512 -> emb_dim, CAMPPlusWithGSP.forward, cam_pplus_wespeaker.py:513-525),
//              Conv1d k5 s2 + BN + ReLU (speech_down_or_up)
//   encoder    SSNDConformerEncoder (:172-195): input_proj + torchaudio Conformer (BatchNorm,
//              depthwise kernel 15) on the shared run_conformer
//   decoders   DetectionDecoder (:274-296) and RepresentationDecoder (:343-370): SWDecoderBlockV2
//              layers (:224-272) = Fq/Fk fusion (:198-222) folded into GEMM epilogues (1/sqrt(D)
//              in the weights, the residual in the epilogue), cross attention of the N speaker
//              queries over the T frames and self attention over the N queries (mha_small), FFN,
//              post-LNs; always exact fp32 (N <= 32 rows per block: latency, not bandwidth)
#pragma once
#include <vector>
#include "campp.h"
#include "encoder.h"

namespace sd {

struct SsndConfig {
  int max_batch = 8;          // blocks per call
  int max_fbank_frames = 800; // 8 s blocks (100 frames / s)
  int max_speakers = 4;       // N (det_query_emb rows)
  int feat_dim = 80;
  int emb_dim = 256;
  int q_det_aux_dim = 256;
  int q_rep_aux_dim = 256;
  int d_model = 256;
  int nhead = 8;
  int d_ff = 512;
  int num_layers = 4;
  int vad_out_len = 200;
  int pos_emb_dim = 256;
  int max_seq_len = 1000;
  int n_all_speakers = 1000;
  int conformer_kernel = 15;
  bool bf16 = false;          // extractor + encoder precision; the decoders are fp32
};

class SsndModel {
 public:
  explicit SsndModel(const SsndConfig& c) : cfg_(c) {}
  ParamStore& params() { return ps_; }
  void finalize();
  bool finalized() const { return finalized_; }
  size_t device_bytes() const { return arena_.total(); }
  // Label frames of a block of Tf fbank frames (CAM++ /2, speech_down_or_up /2).
  static int label_frames(int Tf) { return (CamTrunk::out_frames(Tf) - 1) / 2 + 1; }
  // SSNDModel.infer: feats (B, Tf, 80), speaker_embs (B, N, emb) -> vad (B, N, T), emb (B, N, emb).
  void infer(const float* feats, const float* spk, int B, int Tf, float* vad, float* emb, hipStream_t st);
  // infer after the encoder (the decoders alone): enc (B, T, d_model), x (B, T, emb_dim) fp32.
  void decode(const float* enc, const float* x, const float* spk, int B, int T, float* vad, float* emb,
              hipStream_t st);

 private:
  struct DecL {
    PackedW fq, fk, cq, ck, cv, co, sa_in, so, f1, f2;
    const float *fq_b, *fk_b, *cq_b, *ck_b, *cv_b, *co_b, *sa_in_b, *so_b, *f1_b, *f2_b;
    const float *n1g, *n1b, *n2g, *n2b, *n3g, *n3b;
  };
  std::vector<DecL> load_decoder(const std::string& pre, int d_aux);
  void run_decoder(const std::vector<DecL>& L, float* xdec, const float* qaux, int d_aux, const float* fea,
                   int B, int T, hipStream_t st);
  float* ws(size_t n) { return static_cast<float*>(arena_.alloc(n * sizeof(float))); }

  SsndConfig cfg_;
  ParamStore ps_;
  DeviceArena arena_;
  bool finalized_ = false;
  CamTrunk cam_;
  ConvL out_proj_, down_;
  ConvL enc_in_;
  std::vector<ConformerL> conf_;
  std::vector<DecL> det_, rep_;
  ConvL det_out_, rep_out_, rep_in_;
  const float *pos_ = nullptr, *det_q_ = nullptr, *rep_xdec_ = nullptr, *qaux_w_ = nullptr, *qaux_b_ = nullptr;
  // workspace
  float *x_ = nullptr, *xp_ = nullptr, *X_ = nullptr, *pos_t_ = nullptr, *xdec_ = nullptr, *qaux_ = nullptr;
  float *Qin_ = nullptr, *Kin_ = nullptr, *q_ = nullptr, *k_ = nullptr, *v_ = nullptr, *ctx_ = nullptr,
        *t1_ = nullptr, *xa_ = nullptr, *h_ = nullptr, *fea_ = nullptr;
  float *Y_ = nullptr, *QKV_ = nullptr, *AO_ = nullptr, *H_ = nullptr, *partial_ = nullptr;
};

}  // namespace sd
