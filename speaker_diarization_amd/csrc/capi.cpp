// extern "C" boundary (include/sdiar.h).  Exceptions never cross it: every
// entry point maps sd::Error to a status code + thread-local message.
#include "../../include/sdiar.h"

#include <cmath>
#include <memory>
#include <string>

#include <algorithm>

#include "kernels.h"
#include "prof.h"
#include "eda.h"
#include "fseend.h"
#include "fseend_stream.h"
#include "tsvad.h"
#include "campp.h"
#include "tsvad_stream.h"
#include "ssnd.h"

namespace sd {
static thread_local std::string g_err;
void set_error(const std::string& m) { g_err = m; }
const char* last_error() { return g_err.c_str(); }
}  // namespace sd

struct sd_tsvad {
  bool x3 = false;   // precision 2: conv_gemm's exact path in bf16x3 (GemmX3Scope around compute)
  std::unique_ptr<sd::TsvadModel> model;
};

struct sd_eda {
  bool x3 = false;   // precision 2: conv_gemm's exact path in bf16x3 (GemmX3Scope around compute)
  std::unique_ptr<sd::EdaModel> model;
};

struct sd_campp {
  std::unique_ptr<sd::CamppModel> model;
};

struct sd_ssnd {
  std::unique_ptr<sd::SsndModel> model;
};

struct sd_tsvad_stream {
  std::unique_ptr<sd::TsvadStreamModel> model;
};

struct sd_fseend {
  bool x3 = false;   // precision 2: conv_gemm's exact path in bf16x3 (GemmX3Scope around compute)
  std::unique_ptr<sd::FsEendModel> model;
};

struct sd_fseend_stream {
  std::unique_ptr<sd::FsEendStream> s;
};

namespace {

template <typename F>
int guard(F&& f) {
  try {
    f();
    return SD_OK;
  } catch (const sd::Error& e) {
    sd::set_error(e.msg);
    return e.code;
  } catch (const std::exception& e) {
    sd::set_error(e.what());
    return SD_ERR_HIP;
  } catch (...) {
    sd::set_error("unknown error");
    return SD_ERR_HIP;
  }
}

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Scratch for test-only ops (packed weights); freed after the stream drains.
struct Scratch {
  void* p = nullptr;
  hipStream_t st;
  Scratch(size_t bytes, hipStream_t s) : st(s) { SD_HIP(hipMalloc(&p, bytes ? bytes : 4)); }
  ~Scratch() {
    (void)hipStreamSynchronize(st);
    (void)hipFree(p);
  }
};

}  // namespace

extern "C" {

const char* sd_last_error(void) { return sd::last_error(); }
int sd_version(void) { return 1; }

void sd_prof_enable(int on) { sd::prof_enable(on != 0); }
void sd_prof_reset(void) { sd::prof_reset(); }
int sd_prof_query(int i, char* name, int name_len, int64_t* launches, double* flops, double* bytes,
                  double* ms) {
  std::string n;
  long long l;
  if (!sd::prof_query(i, n, l, *flops, *bytes, *ms)) return 0;
  *launches = l;
  if (name && name_len > 0) {
    size_t k = std::min<size_t>(n.size(), (size_t)name_len - 1);
    n.copy(name, k);
    name[k] = '\0';
  }
  return 1;
}

double sd_prof_query_steps(int i) { return sd::prof_query_steps(i); }

int sd_probe_lstm_granule(int steps, float* us_per_step, void* stream) {
  return guard([&] {
    SD_CHECK(steps >= 1 && us_per_step, sd::kErrInvalid, "probe_lstm_granule: bad argument");
    *us_per_step = sd::lstm_granule_probe(steps, S(stream));
  });
}

int sd_probe_lstm_granule2(int steps, float* us_per_step, void* stream) {
  return guard([&] {
    SD_CHECK(steps >= 1 && us_per_step, sd::kErrInvalid, "probe_lstm_granule2: bad argument");
    *us_per_step = sd::lstm_granule_probe(steps, S(stream), 2);
  });
}

int sd_probe_lstm_handoff(int steps, float* us_per_step, void* stream) {
  return guard([&] {
    SD_CHECK(steps >= 1 && us_per_step, sd::kErrInvalid, "probe_lstm_handoff: bad argument");
    *us_per_step = sd::lstm_handoff_probe(steps, S(stream));
  });
}

int sd_tsvad_create(const sd_tsvad_config* c, sd_tsvad** out) {
  return guard([&] {
    SD_CHECK(c && out, sd::kErrInvalid, "null argument");
    SD_CHECK(c->variant == 0 || c->variant == 1, sd::kErrInvalid, "unknown TS-VAD variant");
    SD_CHECK(c->precision >= 0 && c->precision <= 2, sd::kErrInvalid, "precision must be 0, 1 or 2");
    SD_CHECK(c->max_batch > 0 && c->max_fbank_frames > 0, sd::kErrInvalid, "bad workspace sizes");
    SD_CHECK(c->max_num_speaker > 0 && c->num_transformer_layer >= 1 && c->transformer_ffn_embed_dim > 0 &&
                 c->speaker_embed_dim > 0, sd::kErrInvalid, "bad model dimensions");
    SD_CHECK(c->num_attention_head > 0 && c->transformer_embed_dim % c->num_attention_head == 0, sd::kErrInvalid,
             "transformer_embed_dim must be divisible by num_attention_head");
    sd::TsvadConfig t;
    t.variant = c->variant;
    t.max_num_speaker = c->max_num_speaker;
    t.rs_len = c->rs_len;
    t.max_batch = c->max_batch;
    t.max_fbank_frames = c->max_fbank_frames;
    t.bf16 = c->precision == 1;
    t.num_transformer_layer = c->num_transformer_layer;
    t.num_attention_head = c->num_attention_head;
    t.embed_dim = c->transformer_embed_dim;
    t.ffn_dim = c->transformer_ffn_embed_dim;
    t.speaker_embed_dim = c->speaker_embed_dim;
    auto* h = new sd_tsvad;
    h->x3 = c->precision == 2;
    h->model.reset(new sd::TsvadModel(t));
    *out = h;
  });
}

int sd_tsvad_set_param(sd_tsvad* h, const char* name, const float* data, const int64_t* shape,
                       int ndim) {
  return guard([&] {
    SD_CHECK(h && name && (data || ndim == 0), sd::kErrInvalid, "null argument");
    SD_CHECK(!h->model->finalized(), sd::kErrState, "set_param after finalize");
    h->model->params().set(name, data, shape, ndim);
  });
}

int sd_tsvad_finalize(sd_tsvad* h) {
  return guard([&] {
    SD_CHECK(h, sd::kErrInvalid, "null handle");
    h->model->finalize();
  });
}

int sd_tsvad_forward(sd_tsvad* h, const float* ref, const float* ts, int B, int Tf, int Tl,
                     float* logits, void* stream) {
  return guard([&] {
    const sd::GemmX3Scope x3(h && h->x3);
    SD_CHECK(h && ref && ts && logits, sd::kErrInvalid, "null argument");
    h->model->forward(ref, ts, B, Tf, Tl, logits, S(stream));
  });
}

int sd_tsvad_forward_graph(sd_tsvad* h, const float* ref, const float* ts, int B, int Tf, int Tl, float* logits,
                           int replays, const char* dot_path, void* stream) {
  return guard([&] {
    const sd::GemmX3Scope x3(h && h->x3);
    SD_CHECK(h && ref && ts && logits, sd::kErrInvalid, "null argument");
    h->model->forward_graph(ref, ts, B, Tf, Tl, logits, replays, dot_path, S(stream));
  });
}

int sd_tsvad_debug_buffer(const sd_tsvad* h, int which, void** ptr, int64_t* bytes) {
  return guard([&] {
    SD_CHECK(h && ptr && bytes, sd::kErrInvalid, "null argument");
    h->model->debug_buffer(which, ptr, bytes);
  });
}

int sd_tsvad_status(sd_tsvad* h, void* stream) {
  return guard([&] {
    SD_CHECK(h, sd::kErrInvalid, "null argument");
    h->model->status(S(stream));
  });
}

int sd_tsvad_forward_batched(sd_tsvad* h, const float* ref, const float* ts, int B, int Tf, int Tl,
                             int forward_batch, int force, float* logits, void* stream) {
  return guard([&] {
    const sd::GemmX3Scope x3(h && h->x3);
    SD_CHECK(h && ref && ts && logits, sd::kErrInvalid, "null argument");
    h->model->forward(ref, ts, B, Tf, Tl, logits, S(stream), forward_batch, force);
  });
}

int64_t sd_tsvad_device_bytes(const sd_tsvad* h) { return h ? (int64_t)h->model->device_bytes() : 0; }

int sd_tsvad_destroy(sd_tsvad* h) {
  return guard([&] { delete h; });
}

int sd_eda_create(const sd_eda_config* c, sd_eda** out) {
  return guard([&] {
    SD_CHECK(c && out, sd::kErrInvalid, "null argument");
    SD_CHECK(c->variant >= 0 && c->variant <= 3, sd::kErrInvalid, "Unknown model type.");
    SD_CHECK(c->variant != 3 || c->n_speakers > 0, sd::kErrInvalid, "n_speakers must be positive");
    SD_CHECK(c->precision >= 0 && c->precision <= 2, sd::kErrInvalid, "precision must be 0, 1 or 2");
    SD_CHECK(c->max_seqs > 0 && c->max_frames > 0 && c->max_n_speakers >= 2, sd::kErrInvalid,
             "bad workspace sizes");
    SD_CHECK(c->n_units > 0 && c->n_heads > 0 && c->n_units % c->n_heads == 0, sd::kErrInvalid,
             "n_units must be divisible by n_heads");
    sd::EdaConfig t;
    t.variant = c->variant;
    t.in_size = c->in_size;
    t.n_units = c->n_units;
    t.n_heads = c->n_heads;
    t.n_layers = c->n_layers;
    t.dim_feedforward = c->dim_feedforward;
    t.max_seqs = c->max_seqs;
    t.max_frames = c->max_frames;
    t.max_n_speakers = c->max_n_speakers;
    t.n_speakers = c->n_speakers;
    t.bf16 = c->precision == 1;
    auto* h = new sd_eda;
    h->x3 = c->precision == 2;
    h->model.reset(new sd::EdaModel(t));
    *out = h;
  });
}

int sd_eda_set_param(sd_eda* h, const char* name, const float* data, const int64_t* shape, int ndim) {
  return guard([&] {
    SD_CHECK(h && name && (data || ndim == 0), sd::kErrInvalid, "null argument");
    SD_CHECK(!h->model->finalized(), sd::kErrState, "set_param after finalize");
    h->model->params().set(name, data, shape, ndim);
  });
}

int sd_eda_finalize(sd_eda* h) {
  return guard([&] {
    SD_CHECK(h, sd::kErrInvalid, "null handle");
    h->model->finalize();
  });
}

int sd_eda_input_stride(const sd_eda* h) { return h && h->model->finalized() ? h->model->in_ld() : 0; }

int sd_eda_forward(sd_eda* h, const float* feats, int ld_feats, int S_, int T, const int* lengths,
                   const int* key_len, const int* perm, float* probs, float* act, void* stream) {
  return guard([&] {
    const sd::GemmX3Scope x3(h && h->x3);
    SD_CHECK(h && feats && act, sd::kErrInvalid, "null argument");
    h->model->forward(feats, ld_feats, S_, T, lengths, key_len, perm, probs, act, S(stream));
  });
}

int sd_eda_status(sd_eda* h, void* stream) {
  return guard([&] {
    SD_CHECK(h, sd::kErrInvalid, "null argument");
    h->model->status(S(stream));
  });
}

int64_t sd_eda_device_bytes(const sd_eda* h) { return h ? (int64_t)h->model->device_bytes() : 0; }

int sd_eda_destroy(sd_eda* h) {
  return guard([&] { delete h; });
}

int sd_fseend_create(const sd_fseend_config* c, sd_fseend** out) {
  return guard([&] {
    SD_CHECK(c && out, sd::kErrInvalid, "null argument");
    SD_CHECK(c->precision >= 0 && c->precision <= 2, sd::kErrInvalid, "precision must be 0, 1 or 2");
    SD_CHECK(c->max_seqs > 0 && c->max_frames > 0 && c->max_nspks > 0, sd::kErrInvalid, "bad workspace sizes");
    SD_CHECK(c->n_units > 0 && c->n_heads > 0 && c->n_units % c->n_heads == 0, sd::kErrInvalid,
             "n_units must be divisible by n_heads");
    SD_CHECK(c->dec_n_layers >= 1 && c->enc_n_layers >= 0 && c->mask_delay >= 0, sd::kErrInvalid,
             "bad layer counts");
    sd::FsEendConfig t;
    t.in_size = c->in_size;
    t.n_units = c->n_units;
    t.n_heads = c->n_heads;
    t.enc_n_layers = c->enc_n_layers;
    t.enc_ffn = c->enc_dim_feedforward;
    t.dec_n_layers = c->dec_n_layers;
    t.dec_ffn = c->dec_dim_feedforward;
    t.conv_delay = c->conv_delay;
    t.mask_delay = c->mask_delay;
    t.has_mask = c->has_mask;
    t.max_seqs = c->max_seqs;
    t.max_frames = c->max_frames;
    t.max_nspks = c->max_nspks;
    t.bf16 = c->precision == 1;
    auto* h = new sd_fseend;
    h->x3 = c->precision == 2;
    h->model.reset(new sd::FsEendModel(t));
    *out = h;
  });
}

int sd_fseend_set_param(sd_fseend* h, const char* name, const float* data, const int64_t* shape, int ndim) {
  return guard([&] {
    SD_CHECK(h && name && (data || ndim == 0), sd::kErrInvalid, "null argument");
    SD_CHECK(!h->model->finalized(), sd::kErrState, "set_param after finalize");
    h->model->params().set(name, data, shape, ndim);
  });
}

int sd_fseend_finalize(sd_fseend* h) {
  return guard([&] {
    SD_CHECK(h, sd::kErrInvalid, "null handle");
    h->model->finalize();
  });
}

int sd_fseend_input_stride(const sd_fseend* h) { return h && h->model->finalized() ? h->model->in_ld() : 0; }

int sd_fseend_test(sd_fseend* h, const float* feats, int ld_feats, int S_, int T, const int* ilens_host,
                   int max_nspks, float* preds, float* emb, float* attractors, void* stream) {
  return guard([&] {
    const sd::GemmX3Scope x3(h && h->x3);
    SD_CHECK(h && feats && preds, sd::kErrInvalid, "null argument");
    h->model->forward(feats, ld_feats, S_, T, ilens_host, max_nspks, preds, emb, attractors, S(stream));
  });
}

int64_t sd_fseend_device_bytes(const sd_fseend* h) { return h ? (int64_t)h->model->device_bytes() : 0; }

int sd_fseend_destroy(sd_fseend* h) {
  return guard([&] { delete h; });
}

int sd_fseend_stream_create(sd_fseend* h, int chunk, int max_frames, int max_nspks, int use_graph,
                            sd_fseend_stream** out) {
  return guard([&] {
    SD_CHECK(h && out, sd::kErrInvalid, "null argument");
    auto* s = new sd_fseend_stream;
    try {
      s->s.reset(new sd::FsEendStream(*h->model, chunk, max_frames, max_nspks, use_graph != 0));
    } catch (...) {
      delete s;
      throw;
    }
    *out = s;
  });
}

int sd_fseend_stream_push(sd_fseend_stream* s, const float* feats, int ld_feats, int n, float* preds, int cap,
                          int* n_out, void* stream) {
  return guard([&] {
    SD_CHECK(s && n_out, sd::kErrInvalid, "null argument");
    *n_out = s->s->push(feats, ld_feats, n, preds, cap, S(stream));
  });
}

int sd_fseend_stream_set_audio(sd_fseend_stream* s, const float* mel_fb, int n_mels, int frame_size, int frame_shift,
                               int context_size, int subsampling) {
  return guard([&] {
    SD_CHECK(s, sd::kErrInvalid, "null handle");
    s->s->set_audio(mel_fb, n_mels, frame_size, frame_shift, context_size, subsampling);
  });
}

int sd_fseend_stream_push_audio(sd_fseend_stream* s, const float* samples, int64_t n, float* preds, int cap,
                                int* n_out, void* stream) {
  return guard([&] {
    SD_CHECK(s && n_out, sd::kErrInvalid, "null argument");
    *n_out = s->s->push_audio(samples, n, preds, cap, S(stream));
  });
}

int sd_fseend_stream_flush(sd_fseend_stream* s, float* preds, int cap, int* n_out, void* stream) {
  return guard([&] {
    SD_CHECK(s && n_out, sd::kErrInvalid, "null argument");
    *n_out = s->s->flush(preds, cap, S(stream));
  });
}

int sd_fseend_stream_reset(sd_fseend_stream* s, void* stream) {
  return guard([&] {
    SD_CHECK(s, sd::kErrInvalid, "null handle");
    s->s->reset(S(stream));
  });
}

int sd_fseend_stream_stats(const sd_fseend_stream* s, int64_t* enc_runs, int64_t* dec_runs, int* enc_nodes,
                           int* dec_nodes) {
  return guard([&] {
    SD_CHECK(s && enc_runs && dec_runs && enc_nodes && dec_nodes, sd::kErrInvalid, "null argument");
    *enc_runs = s->s->runs(0);
    *dec_runs = s->s->runs(1);
    *enc_nodes = s->s->graph_nodes(0);
    *dec_nodes = s->s->graph_nodes(1);
  });
}

int sd_fseend_stream_debug_counters(const sd_fseend_stream* s, unsigned* host_out, int cap, int* n, void* stream) {
  return guard([&] {
    SD_CHECK(s && n && (host_out || cap == 0), sd::kErrInvalid, "null argument");
    *n = s->s->debug_counters(host_out, cap, S(stream));
  });
}

int64_t sd_fseend_stream_device_bytes(const sd_fseend_stream* s) {
  return s ? (int64_t)s->s->device_bytes() : 0;
}

int sd_fseend_stream_destroy(sd_fseend_stream* s) {
  return guard([&] { delete s; });
}

int sd_eend_features(const float* wav, int64_t n_samples, int frame_size, int frame_shift, int n_frames,
                     const float* mel_fb, int n_mels, int mean_norm, int context_size, int subsampling,
                     double* work, float* out, int ld_out, void* stream) {
  return guard([&] {
    SD_CHECK(wav && mel_fb && work && out, sd::kErrInvalid, "null argument");
    SD_CHECK(frame_size > 0 && frame_shift > 0 && subsampling > 0 && context_size >= 0, sd::kErrInvalid,
             "bad frame geometry");
    const int n_fft = 1 << (32 - __builtin_clz((unsigned)(frame_size - 1)));
    const int64_t nf_max = 1 + n_samples / frame_shift;
    SD_CHECK(n_frames >= 1 && n_frames <= nf_max, sd::kErrInvalid, "n_frames exceeds the STFT frames");
    hipStream_t st = S(stream);
    double* lm = work;
    double* mean = work + (int64_t)n_frames * n_mels;
    sd::stft_logmel(wav, n_samples, n_frames, n_fft, frame_shift, frame_size, mel_fb, n_mels, lm, st);
    if (mean_norm) sd::col_mean(lm, n_frames, n_mels, mean, st);
    const int n_out = (n_frames + subsampling - 1) / subsampling;
    sd::splice_subsample(lm, n_frames, n_mels, mean_norm ? mean : nullptr, context_size, subsampling, n_out,
                         out, ld_out, st);
  });
}

int sd_fbank_kaldi(const float* wav, int64_t n_samples, float in_scale, int n_frames,
                   const float* mel_fb, int n_mels, float* out, void* stream) {
  return guard([&] {
    SD_CHECK(n_frames >= 0 && (n_frames == 0 || n_samples >= 400 + (int64_t)(n_frames - 1) * 160),
             sd::kErrInvalid, "fbank: n_frames exceeds the samples");
    sd::fbank_kaldi(wav, n_samples, in_scale, n_frames, mel_fb, n_mels, out, S(stream));
  });
}

int sd_fbank_kaldi_ex(const float* wav, int64_t n_samples, float in_scale, int n_frames, const float* mel_fb,
                      int n_mels, int window_type, float* out, void* stream) {
  return guard([&] {
    SD_CHECK(n_frames >= 0 && (n_frames == 0 || n_samples >= 400 + (int64_t)(n_frames - 1) * 160),
             sd::kErrInvalid, "fbank: n_frames exceeds the samples");
    sd::fbank_kaldi(wav, n_samples, in_scale, n_frames, mel_fb, n_mels, out, S(stream), window_type);
  });
}

int sd_tsvad_stream_create(const sd_tsvad_stream_config* c, sd_tsvad_stream** out) {
  return guard([&] {
    SD_CHECK(c && out, sd::kErrInvalid, "null argument");
    SD_CHECK(c->precision == 0 || c->precision == 1, sd::kErrInvalid, "precision must be 0 or 1");
    SD_CHECK(c->max_labels > 0 && c->max_num_speaker > 0 && c->max_windows > 0, sd::kErrInvalid,
             "bad workspace sizes");
    SD_CHECK(c->num_attention_head > 0 && c->transformer_embed_dim % c->num_attention_head == 0, sd::kErrInvalid,
             "transformer_embed_dim must be divisible by num_attention_head");
    SD_CHECK(c->num_transformer_layer >= 1, sd::kErrInvalid, "num_transformer_layer must be >= 1");
    SD_CHECK(c->transformer_ffn_embed_dim > 0 && c->speaker_embed_dim > 0, sd::kErrInvalid,
             "transformer_ffn_embed_dim and speaker_embed_dim must be > 0");
    sd::TsvadStreamConfig t;
    t.max_num_speaker = c->max_num_speaker;
    t.max_labels = c->max_labels;
    t.max_windows = c->max_windows;
    t.bf16 = c->precision == 1;
    t.num_transformer_layer = c->num_transformer_layer;
    t.num_attention_head = c->num_attention_head;
    t.embed_dim = c->transformer_embed_dim;
    t.ffn_dim = c->transformer_ffn_embed_dim;
    t.speaker_embed_dim = c->speaker_embed_dim;
    auto* h = new sd_tsvad_stream;
    h->model.reset(new sd::TsvadStreamModel(t));
    *out = h;
  });
}

int sd_tsvad_stream_set_param(sd_tsvad_stream* h, const char* name, const float* data, const int64_t* shape,
                              int ndim) {
  return guard([&] {
    SD_CHECK(h && name && (data || ndim == 0), sd::kErrInvalid, "null argument");
    SD_CHECK(!h->model->finalized(), sd::kErrState, "set_param after finalize");
    h->model->params().set(name, data, shape, ndim);
  });
}

int sd_tsvad_stream_finalize(sd_tsvad_stream* h) {
  return guard([&] {
    SD_CHECK(h, sd::kErrInvalid, "null handle");
    h->model->finalize();
  });
}

int sd_tsvad_stream_forward(sd_tsvad_stream* h, const float* feats, const float* ts, int B, int T_label, int chunk,
                            int left_chunks, float* logits, void* stream) {
  return guard([&] {
    SD_CHECK(h && feats && ts && logits, sd::kErrInvalid, "null argument");
    SD_CHECK(chunk > 0, sd::kErrShape, "decoding_chunk_size must be > 0");
    h->model->forward(feats, ts, B, T_label, chunk, left_chunks, logits, S(stream));
  });
}

int64_t sd_tsvad_stream_device_bytes(const sd_tsvad_stream* h) {
  return h ? (int64_t)h->model->device_bytes() : 0;
}

int sd_tsvad_stream_destroy(sd_tsvad_stream* h) {
  return guard([&] { delete h; });
}

int sd_campp_create(const sd_campp_config* c, sd_campp** out) {
  return guard([&] {
    SD_CHECK(c && out, sd::kErrInvalid, "null argument");
    SD_CHECK(c->precision == 0 || c->precision == 1, sd::kErrInvalid, "precision must be 0 or 1");
    SD_CHECK(c->feat_dim == 80, sd::kErrInvalid, "CAM++ FCM head supports feat_dim 80 only");
    SD_CHECK(c->embedding_size > 0, sd::kErrInvalid, "embedding_size must be positive");
    SD_CHECK(c->max_batch > 0 && c->max_frames >= 8, sd::kErrInvalid, "bad workspace sizes");
    sd::CamppConfig t;
    t.feat_dim = c->feat_dim;
    t.embedding_size = c->embedding_size;
    t.max_batch = c->max_batch;
    t.max_frames = c->max_frames;
    t.bf16 = c->precision == 1;
    auto* h = new sd_campp;
    h->model.reset(new sd::CamppModel(t));
    *out = h;
  });
}

int sd_campp_set_param(sd_campp* h, const char* name, const float* data, const int64_t* shape, int ndim) {
  return guard([&] {
    SD_CHECK(h && name && (data || ndim == 0), sd::kErrInvalid, "null argument");
    SD_CHECK(!h->model->finalized(), sd::kErrState, "set_param after finalize");
    h->model->params().set(name, data, shape, ndim);
  });
}

int sd_campp_finalize(sd_campp* h) {
  return guard([&] {
    SD_CHECK(h, sd::kErrInvalid, "null handle");
    h->model->finalize();
  });
}

int sd_campp_forward(sd_campp* h, const float* feats, int B, int T, float* emb, float* time_out, void* stream) {
  return guard([&] {
    SD_CHECK(h && feats && (emb || time_out), sd::kErrInvalid, "null argument");
    h->model->forward(feats, B, T, emb, time_out, S(stream));
  });
}

int64_t sd_campp_device_bytes(const sd_campp* h) { return h ? (int64_t)h->model->device_bytes() : 0; }

int sd_campp_destroy(sd_campp* h) {
  return guard([&] { delete h; });
}

int sd_ssnd_create(const sd_ssnd_config* c, sd_ssnd** out) {
  return guard([&] {
    SD_CHECK(c && out, sd::kErrInvalid, "null argument");
    SD_CHECK(c->precision == 0 || c->precision == 1, sd::kErrInvalid, "precision must be 0 or 1");
    SD_CHECK(c->max_batch > 0 && c->max_fbank_frames >= 8 && c->max_speakers > 0, sd::kErrInvalid,
             "bad workspace sizes");
    SD_CHECK(c->num_layers >= 1 && c->nhead > 0 && c->d_model > 0 && c->d_ff > 0 && c->emb_dim > 0 &&
                 c->q_det_aux_dim > 0 && c->q_rep_aux_dim > 0 && c->pos_emb_dim > 0 && c->vad_out_len > 0 &&
                 c->max_seq_len >= c->vad_out_len && c->n_all_speakers > 0,
             sd::kErrInvalid, "bad model dimensions");
    SD_CHECK(c->conformer_kernel >= 1 && c->conformer_kernel % 2 == 1 && c->conformer_kernel <= 31, sd::kErrInvalid,
             "conformer_kernel must be odd and <= 31");
    SD_CHECK(c->q_det_aux_dim == c->emb_dim, sd::kErrInvalid,
             "q_det_aux_dim must equal emb_dim (the speaker embeddings are the detection queries)");
    sd::SsndConfig t;
    t.max_batch = c->max_batch; t.max_fbank_frames = c->max_fbank_frames; t.max_speakers = c->max_speakers;
    t.feat_dim = c->feat_dim; t.emb_dim = c->emb_dim; t.q_det_aux_dim = c->q_det_aux_dim;
    t.q_rep_aux_dim = c->q_rep_aux_dim; t.d_model = c->d_model; t.nhead = c->nhead; t.d_ff = c->d_ff;
    t.num_layers = c->num_layers; t.vad_out_len = c->vad_out_len; t.pos_emb_dim = c->pos_emb_dim;
    t.max_seq_len = c->max_seq_len; t.n_all_speakers = c->n_all_speakers; t.conformer_kernel = c->conformer_kernel;
    t.bf16 = c->precision == 1;
    auto* h = new sd_ssnd;
    h->model.reset(new sd::SsndModel(t));
    *out = h;
  });
}

int sd_ssnd_set_param(sd_ssnd* h, const char* name, const float* data, const int64_t* shape, int ndim) {
  return guard([&] {
    SD_CHECK(h && name && (data || ndim == 0), sd::kErrInvalid, "null argument");
    SD_CHECK(!h->model->finalized(), sd::kErrState, "set_param after finalize");
    h->model->params().set(name, data, shape, ndim);
  });
}

int sd_ssnd_finalize(sd_ssnd* h) {
  return guard([&] {
    SD_CHECK(h, sd::kErrInvalid, "null handle");
    h->model->finalize();
  });
}

int sd_ssnd_infer(sd_ssnd* h, const float* feats, const float* spk, int B, int T_fbank, float* vad, float* emb,
                  void* stream) {
  return guard([&] {
    SD_CHECK(h && feats && spk && vad && emb, sd::kErrInvalid, "null argument");
    h->model->infer(feats, spk, B, T_fbank, vad, emb, S(stream));
  });
}

int sd_ssnd_decode(sd_ssnd* h, const float* enc, const float* x, const float* spk, int B, int T, float* vad,
                   float* emb, void* stream) {
  return guard([&] {
    SD_CHECK(h && enc && x && spk && vad && emb, sd::kErrInvalid, "null argument");
    h->model->decode(enc, x, spk, B, T, vad, emb, S(stream));
  });
}

int64_t sd_ssnd_device_bytes(const sd_ssnd* h) { return h ? (int64_t)h->model->device_bytes() : 0; }

int sd_ssnd_destroy(sd_ssnd* h) {
  return guard([&] { delete h; });
}

int sd_window_cmn(const float* feats, int n_mels, const int* win_start, const int* win_n, int n_win,
                  int T_out, float* out, void* stream) {
  return guard([&] {
    if (n_win == 0) return;
    sd::window_cmn(feats, n_mels, win_start, win_n, n_win, T_out, out, S(stream));
  });
}

int sd_overlap_average(const float* logits, int n_win, int NS, int Tw, const int* start,
                       const int* len, int dis, int chunk, int n_frames, float* out, void* stream) {
  return guard([&] {
    SD_CHECK(dis > 0 && chunk > 0, sd::kErrInvalid, "overlap_average: bad window geometry");
    SD_CHECK((chunk + dis - 1) / dis <= sd::kOverlapMaxWindows, sd::kErrInvalid,
             "overlap_average: more covering windows per frame than the pairwise mean supports");
    sd::overlap_average(logits, n_win, NS, Tw, start, len, dis, chunk, n_frames, out, S(stream));
  });
}

int sd_overlap_mean(const float* probs, int n_win, int NS, int Tw, const int* start, const int* len, int dis,
                    int chunk, int n_frames, float* out, void* stream) {
  return guard([&] {
    SD_CHECK(dis > 0 && chunk > 0, sd::kErrInvalid, "overlap_mean: bad window geometry");
    SD_CHECK((chunk + dis - 1) / dis <= sd::kOverlapMaxWindows, sd::kErrInvalid,
             "overlap_mean: more covering windows per frame than the pairwise mean supports");
    sd::overlap_average(probs, n_win, NS, Tw, start, len, dis, chunk, n_frames, out, S(stream), false);
  });
}

int sd_postprocess_segments(const float* post, int rows, int T, int med_filter, const float* thresholds,
                            int n_thresholds, int min_silence_frames, int min_speech_frames, int cap,
                            int* seg_begin, int* seg_end, int* n_seg, int flags, void* stream) {
  return guard([&] {
    SD_CHECK(rows >= 0 && T >= 0, sd::kErrInvalid, "postprocess: negative shape");
    SD_CHECK(n_thresholds >= 1 && n_thresholds <= sd::ThresholdSet::kMax, sd::kErrInvalid,
             "postprocess: 1..16 thresholds");
    SD_CHECK(T <= sd::segments_max_frames(), sd::kErrInvalid, "postprocess: track too long");
    SD_CHECK(cap >= (T + 1) / 2, sd::kErrInvalid, "postprocess: cap < (T+1)/2");
    if (rows == 0 || T == 0) {
      if (rows > 0) SD_HIP(hipMemsetAsync(n_seg, 0, sizeof(int) * rows * n_thresholds, S(stream)));
      return;
    }
    hipStream_t st = S(stream);
    sd::ThresholdSet thr;
    thr.n = n_thresholds;
    thr.strict = flags & 1;
    for (int i = 0; i < n_thresholds; ++i) thr.v[i] = thresholds[i];
    Scratch med((size_t)rows * T * sizeof(float), st);
    sd::medfilt(post, rows, T, med_filter, static_cast<float*>(med.p), st);
    sd::run_segments(static_cast<const float*>(med.p), rows, T, thr, min_silence_frames, min_speech_frames, cap,
                     seg_begin, seg_end, n_seg, st);
  });
}

int sd_op_linear(const float* x, int M, int K, const float* w, const float* b, int N, int act,
                 float* out, int precision, void* stream) {
  return guard([&] {
    hipStream_t st = S(stream);
    const bool bf = precision >= 1;
    Scratch wt((size_t)N * K * (bf ? 2 : 4), st);
    sd::pack_weight(w, N, K, 1, wt.p, bf, st);
    Scratch xb(precision == 2 ? (size_t)M * K * 2 : 4, st);   // precision 2: bf16 activations
    if (precision == 2) sd::f32_to_bf16(x, (int64_t)M * K, xb.p, st);
    sd::ConvGemmArgs p = sd::linear_args(precision == 2 ? xb.p : (const void*)x, M, K, K, wt.p, N, out, N);
    p.a_bf16 = precision == 2;
    p.beta = b;
    p.act = act;
    sd::conv_gemm(p, bf, st);
  });
}

int sd_op_gemm_bf16(const void* x, int M, int K, int lda, int a_coff, const float* w, int N,
                    const float* pre_scale, const float* pre_shift, const float* alpha, const float* beta,
                    int act, void* out, int ldo, void* stream) {
  return guard([&] {
    hipStream_t st = S(stream);
    SD_CHECK(M > 0 && K > 0 && N > 0 && lda >= a_coff + K && ldo >= N, sd::kErrInvalid, "gemm_bf16: bad shape");
    SD_CHECK((pre_scale == nullptr) == (pre_shift == nullptr), sd::kErrInvalid, "gemm_bf16: pre_scale/pre_shift");
    Scratch wt((size_t)N * K * 2, st);
    sd::pack_weight(w, N, K, 1, wt.p, true, st);
    sd::ConvGemmArgs p = sd::linear_args(x, M, K, lda, wt.p, N, out, ldo);
    p.a_bf16 = true;
    p.a_coff = a_coff;
    p.out_bf16 = true;
    p.pre_scale = pre_scale;
    p.pre_shift = pre_shift;
    p.alpha = alpha;
    p.beta = beta;
    p.act = act;
    sd::conv_gemm(p, true, st);
  });
}

int sd_probe_graph_memset(int n, int replays, int fork, int* bad_per_replay, void* stream) {
  return guard([&] {
    SD_CHECK(n > 0 && replays > 0 && bad_per_replay, sd::kErrInvalid, "probe_graph_memset: bad argument");
    sd::graph_memset_probe(n, replays, fork != 0, bad_per_replay, S(stream));
  });
}

int sd_debug_cam_dense_probe(void* stamps) {
  return guard([&] { sd::cam_dense_set_probe(stamps); });
}

int sd_debug_rowprog_probe(void* stamps) {
  return guard([&] { sd::rowprog_set_probe(stamps); });
}

int sd_op_cam_dense(const void* x, int B, int T, int ld, int cin, int dil, const float* s1, const float* h1,
                    const float* wb, const float* a2, const float* b2, const float* wl, const float* bl,
                    const float* w1, const float* c1, const float* w2, const float* c2, void* out, int repeats,
                    void* stream) {
  return guard([&] {
    hipStream_t st = S(stream);
    SD_CHECK(B >= 1 && repeats >= 1 && ld >= cin + 32 &&
                 sd::cam_dense_supported(T, cin, ld, 128, 64, 32, 32, 3, dil, 100, true),
             sd::kErrInvalid, "cam_dense: unsupported shape");
    Scratch wbt((size_t)128 * cin * 2, st), wlt((size_t)32 * 3 * 128 * 2, st);
    sd::pack_weight(wb, 128, cin, 1, wbt.p, true, st);
    sd::pack_weight(wl, 32, 128, 3, wlt.p, true, st);   // Wt[o][tap * 128 + c]
    Scratch rec(sd::cam_dense_record_bytes(B), st), cnt(sd::cam_dense_counter_bytes(B), st);
    SD_HIP(hipMemsetAsync(cnt.p, 0, sd::cam_dense_counter_bytes(B), st));
    for (int r = 0; r < repeats; ++r)
      sd::cam_dense(x, B, T, ld, cin, dil, s1, h1, wbt.p, a2, b2, wlt.p, bl, w1, c1, w2, c2, out, rec.p,
                    static_cast<unsigned*>(cnt.p), st);
  });
}

int sd_op_mha_block(const void* y, const float* w, const float* bias, int nseq, int T, const int* key_len, void* out,
                    int variant, int flags, void* stream) {
  return guard([&] {
    hipStream_t st = S(stream);
    SD_CHECK(nseq >= 1 && sd::mha_block_supported(384, 8, T, true), sd::kErrInvalid, "mha_block: unsupported shape");
    SD_CHECK(flags >= 0 && flags <= 3, sd::kErrInvalid, "mha_block: flags");
    Scratch wt((size_t)3 * 384 * 384 * 2, st);
    sd::pack_weight(w, 3 * 384, 384, 1, wt.p, true, st);
    sd::MhaBlockArgs m;
    m.y = y; m.W = wt.p; m.bias = bias; m.out = out; m.ldo = 384;
    m.S = nseq; m.T = T; m.D = 384; m.nh = 8; m.scale = 1.f / std::sqrt(48.f); m.key_len = key_len;
    m.y_tiled = flags & 1;     // y in RowProgArgs::a_tiled's fragment layout (what the FFN programs hand over)
    m.out_tiled = (flags >> 1) & 1;   // the output in that layout (what the out-projection program reads)
    sd::mha_block(m, st, variant);
  });
}

int sd_op_conv1d(const float* x, int B, int T, int Cin, const float* w, const float* b, int Cout,
                 int k, int stride, int pad, int dil, int act, float* out, int precision,
                 void* stream) {
  return guard([&] {
    hipStream_t st = S(stream);
    const bool bf = precision >= 1;
    Scratch wt((size_t)Cout * Cin * k * (bf ? 2 : 4), st);
    sd::pack_weight(w, Cout, Cin, k, wt.p, bf, st);
    Scratch xb(precision == 2 ? (size_t)B * T * Cin * 2 : 4, st);
    if (precision == 2) sd::f32_to_bf16(x, (int64_t)B * T * Cin, xb.p, st);
    sd::ConvGemmArgs p;
    p.A = precision == 2 ? xb.p : (const void*)x; p.a_bf16 = precision == 2; p.B = B; p.H = 1; p.W = T; p.Cin = Cin; p.lda = Cin;
    p.kh = 1; p.kw = k; p.sw = stride; p.pw = pad; p.dw = dil;
    p.Ho = 1; p.Wo = (T + 2 * pad - dil * (k - 1) - 1) / stride + 1;
    SD_CHECK(p.Wo > 0, sd::kErrInvalid, "conv1d: empty output");
    p.Wt = wt.p; p.N = Cout; p.K = Cin * k;
    p.beta = b; p.act = act;
    p.out = out; p.o_sb = (int64_t)p.Wo * Cout; p.o_sw = Cout; p.o_sn = 1;
    sd::conv_gemm(p, bf, st);
  });
}

int sd_op_conv2d(const float* x, int B, int H, int W, int Cin, const float* w, int Cout, int kh,
                 int kw, int sh, int sw, int ph, int pw, float* out, int precision, void* stream) {
  return guard([&] {
    hipStream_t st = S(stream);
    const bool bf = precision >= 1;
    Scratch wt((size_t)Cout * Cin * kh * kw * (bf ? 2 : 4), st);
    sd::pack_weight(w, Cout, Cin, kh * kw, wt.p, bf, st);
    Scratch xb(precision == 2 ? (size_t)B * H * W * Cin * 2 : 4, st);
    if (precision == 2) sd::f32_to_bf16(x, (int64_t)B * H * W * Cin, xb.p, st);
    sd::ConvGemmArgs p;
    p.A = precision == 2 ? xb.p : (const void*)x; p.a_bf16 = precision == 2; p.B = B; p.H = H; p.W = W; p.Cin = Cin; p.lda = Cin;
    p.kh = kh; p.kw = kw; p.sh = sh; p.sw = sw; p.ph = ph; p.pw = pw;
    p.Ho = (H + 2 * ph - kh) / sh + 1;
    p.Wo = (W + 2 * pw - kw) / sw + 1;
    p.Wt = wt.p; p.N = Cout; p.K = Cin * kh * kw;
    p.out = out; p.o_sb = (int64_t)p.Ho * p.Wo * Cout; p.o_sh = (int64_t)p.Wo * Cout; p.o_sw = Cout;
    p.o_sn = 1;
    sd::conv_gemm(p, bf, st);
  });
}

namespace {
void op_attention(const float* qkv, int S_, int T, int D, int nh, int causal, int causal_delay, const int* key_len,
                  int chunk, int left, float* out, int precision, hipStream_t st, int* mask_dump = nullptr,
                  int grid_c = 0) {
  SD_CHECK(precision >= 0 && precision <= 2, sd::kErrInvalid, "precision must be 0, 1 or 2");
  sd::AttnArgs a;
  a.qkv = qkv; a.S = S_; a.T = T; a.D = D; a.nh = nh; a.ld_qkv = 3 * D;
  a.out = out; a.ldo = D; a.scale = 1.f / std::sqrt((float)(D / nh));
  a.causal = causal; a.causal_delay = causal_delay; a.key_len = key_len;
  a.chunk = chunk; a.left = left;
  a.mask_dump = mask_dump;
  if (grid_c > 0) {   // time attention over a (S/C, T, C) token grid: sequence (s, c) walks tokens with stride C
    a.seq_inner = grid_c; a.seq_outer = (int64_t)T * grid_c; a.seq_inner_stride = 1; a.tok_stride = grid_c;
  }
  if (precision == 2) {   // bf16 storage: qkv and out in bf16 (the encoders' layout)
    Scratch qb((size_t)S_ * T * 3 * D * 2, st), ob((size_t)S_ * T * D * 2, st);
    sd::f32_to_bf16(qkv, (int64_t)S_ * T * 3 * D, qb.p, st);
    a.qkv = qb.p; a.out = ob.p; a.io_bf16 = true;
    sd::attention(a, true, st);
    sd::bf16_to_f32(ob.p, (int64_t)S_ * T * D, out, st);
    return;
  }
  sd::attention(a, precision == 1, st);
}
}  // namespace

int sd_op_attention(const float* qkv, int S_, int T, int D, int nh, int causal, int causal_delay,
                    const int* key_len, float* out, int precision, void* stream) {
  return guard([&] { op_attention(qkv, S_, T, D, nh, causal, causal_delay, key_len, 0, -1, out, precision, S(stream)); });
}

int sd_op_attention_grid(const float* qkv, int S_, int T, int C, int D, int nh, int causal, int causal_delay,
                         float* out, int precision, void* stream) {
  return guard([&] {
    SD_CHECK(S_ >= 1 && C >= 1 && T >= 1, sd::kErrInvalid, "attention_grid: empty grid");
    op_attention(qkv, S_ * C, T, D, nh, causal, causal_delay, nullptr, 0, -1, out, precision, S(stream), nullptr, C);
  });
}

int sd_op_attention_chunk(const float* qkv, int S_, int T, int D, int nh, int chunk, int left, float* out,
                          int precision, void* stream) {
  return guard([&] {
    SD_CHECK(chunk > 0, sd::kErrInvalid, "decoding chunk must be > 0");
    op_attention(qkv, S_, T, D, nh, 0, 0, nullptr, chunk, left, out, precision, S(stream));
  });
}

int sd_probe_attention_mask(const float* qkv, int S_, int T, int D, int nh, int causal, int causal_delay,
                            const int* key_len, int chunk, int left, int* mask_dump, float* out,
                            int precision, void* stream) {
  return guard([&] {
    SD_CHECK(mask_dump != nullptr, sd::kErrInvalid, "mask_dump is required");
    op_attention(qkv, S_, T, D, nh, causal, causal_delay, key_len, chunk, left, out, precision, S(stream),
                 mask_dump);
  });
}

int sd_op_layernorm(const float* x, int rows, int D, const float* g, const float* b, float eps,
                    float* y, void* stream) {
  return guard([&] { sd::layernorm(x, rows, D, D, g, b, eps, y, D, false, S(stream)); });
}

int sd_op_add_layernorm(float* x, const void* t, int t_bf16, int rows, int D, const float* g, const float* b,
                        float eps, int write_x, void* y, int y_bf16, void* stream) {
  return guard([&] {
    sd::add_layernorm(x, t, t_bf16 != 0, rows, D, g, b, eps, write_x != 0, y, y_bf16 != 0, S(stream));
  });
}

int sd_op_lstm(const float* gx, int B, int T, int H, int ndir, const float* whh, const int* lengths,
               float* out, float* hT, float* cT, float* work, void* stream) {
  return guard([&] {
    sd::lstm_recurrence(gx, B, T, H, ndir, whh, lengths, nullptr, nullptr, out, ndir * H, hT, cT,
                        work, S(stream));
  });
}

}  // extern "C"
