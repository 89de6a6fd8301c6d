// Chunked (streaming) FS-EEND inference with per-layer K/V histories and hipGraph replay.
//
// Produces the same per-frame scores as OnlineTransformerDADiarization.test()
// (fs_eend.py:79-96) on the concatenation of the pushed frames, chunk by chunk:
//   encoder chunk  c new feature rows -> BN-folded Linear -> LN -> enc_n_layers causal
//                  transformer layers, each attending to its K|V history (stream_ops.hip)
//   decoder chunk  once 9 frames of look-ahead exist (Conv1d k 19 pad 9, fs_eend.py:41,85):
//                  conv window -> L2 norm -> slot init -> the shared fusion layer
//                  dec_n_layers times (time attention against each application's K|V
//                  history over the (t, slot) grid, slot attention, FFN) -> scores
// Requires has_mask = 1 and mask_delay = 0 (every shipped config; with a positive delay
// frame t would depend on future frames at every layer).  Each chunk's kernel sequence
// is captured once into a hipGraph (after a first direct run that performs the kernels'
// one-time setup) and replayed: positions live in a device cursor block.
#pragma once
#include "fseend.h"

namespace sd {

class FsEendStream {
 public:
  FsEendStream(FsEendModel& m, int chunk, int max_frames, int C, bool use_graph);
  ~FsEendStream();
  // feats: device (n, ld) f32, 1 <= n <= chunk.  A push of n < chunk frames ends the input.
  // Writes the scores of every frame that became final to preds (device, rows of C, capacity
  // cap rows) and returns their number.
  int push(const float* feats, int ld, int n, float* preds, int cap, hipStream_t st);
  // Audio input (fs_eend/dataset.py:217-223 + feature.py:130-184: centred STFT, logmel, splice ±context,
  // [::sub]) instead of feature rows: configure once on a fresh or reset stream (mel_fb: device
  // (n_mels, n_fft/2 + 1) f32, the librosa Slaney basis), then push_audio() any number of samples.  Each
  // chunk's frontend runs inside its captured encoder graph; the rows are the ones eend_features() computes
  // for the whole recording, bit for bit.
  void set_audio(const float* mel_fb, int n_mels, int frame_size, int frame_shift, int context, int sub);
  int push_audio(const float* samples, int64_t n, float* preds, int cap, hipStream_t st);
  // Ends the input (if not already) and emits the remaining frames.
  int flush(float* preds, int cap, hipStream_t st);
  void reset(hipStream_t st);
  int frames_in() const { return n_valid_; }
  int frames_out() const { return n_out_; }
  int chunk() const { return c_; }
  // chunks run so far (0 encoder, 1 decoder) and the nodes of the captured graph (0 if none yet)
  int64_t runs(int which) const { return runs_[which]; }
  int graph_nodes(int which) const;
  size_t device_bytes() const { return arena_.total(); }
  // diagnostics: the block-merge counters (attn_decode's C * n_heads, then the slot block's one) copied to the
  // host after `st` drains; returns how many there are (writes at most cap)
  int debug_counters(unsigned* host, int cap, hipStream_t st) const;

 private:
  void enc_chunk(hipStream_t st);
  void ffn(const PackedW& l1, const float* b1, const PackedW& l2, const float* b2, const float* ln_x, const void* ln_t,
           const float* ln_g, const float* ln_b, float* ln_out, int n, hipStream_t st);
  int after_enc(int n, float* preds, int cap, hipStream_t st);   // cursor bookkeeping + decoder chunks
  void dec_chunk(hipStream_t st);
  void run(int which, hipStream_t st);   // 0 encoder, 1 decoder: graph replay or direct launches
  int emit(float* preds, int cap, int rows, hipStream_t st);
  template <typename T>
  T* wsb(size_t elems) { return static_cast<T*>(arena_.alloc(elems * sizeof(T))); }

  FsEendModel& m_;
  const int c_, cap_, C_;
  const bool use_graph_;
  const bool bf_;
  const size_t es_;
  DeviceArena arena_;
  int* state_ = nullptr;               // [0] encoder frames, [1] valid frames, [2] decoder frames
  int n_enc_ = 0, n_valid_ = 0, n_dec_ = 0, n_out_ = 0;
  bool closed_ = false;
  int n_blocks_ = 0;
  // staging (chunk-sized)
  float *F_ = nullptr, *Y_ = nullptr, *X_ = nullptr, *W_ = nullptr, *Yc_ = nullptr, *E_ = nullptr;
  float *X2_ = nullptr, *A2_ = nullptr, *G_ = nullptr, *A_ = nullptr, *P_ = nullptr, *ws_ = nullptr;
  unsigned* dcnt_ = nullptr;           // attn_decode's per-(sequence, head) block counters (0..nblk-1, wrap)
  float* sws_ = nullptr;               // stream_slot_block's per-head out-projection partials
  unsigned* scnt_ = nullptr;           // its arrival counter (0..n_heads-1, wraps per launch)
  float* fws_ = nullptr;               // stream_ffn_pair's down-projection partials
  unsigned* fcnt_ = nullptr;           // its arrival counter (wraps per launch)
  float* ows_ = nullptr;               // attn_decode's out-projection head partials
  unsigned* ocnt_ = nullptr;           // their per-sequence arrival counters (0..n_heads-1, wrap)
  void *QKV_ = nullptr, *AO_ = nullptr, *T_ = nullptr, *H_ = nullptr;
  // histories
  std::vector<void*> kv_enc_, kv_dec_;
  float* hist_ = nullptr;
  // audio frontend (set_audio)
  bool audio_ = false;
  const float* fb_ = nullptr;
  int n_mels_ = 0, fsz_ = 0, hop_ = 0, nfft_ = 0, ctx_ = 0, sub_ = 0;
  float* aud_ = nullptr;               // every sample of the stream (the frontend reads its window by cursor)
  int64_t aud_cap_ = 0, n_samp_ = 0;
  double* lm_ = nullptr;               // the chunk's logmel frames
  int* bound_ = nullptr;               // [0] samples, [1] STFT frames of the input (INT_MAX while open)
  // graphs
  hipStream_t cap_st_ = nullptr;
  // graphs: 0 encoder chunk, 1 decoder chunk, 2 both back to back (the steady state of an audio stream: one
  // graph launch per push instead of two)
  hipGraph_t graph_[3] = {nullptr, nullptr, nullptr};
  hipGraphExec_t exec_[3] = {nullptr, nullptr, nullptr};
  bool ran_direct_[3] = {false, false, false};
  int64_t runs_[2] = {0, 0};
};

}  // namespace sd
