/*
 * sdiar.h — C ABI of the MI355X (gfx950) diarization inference engine.
 *
 * Plain pointers, sizes and a hipStream_t passed as void*.  Device pointers are
 * caller-owned (torch tensors, hipMalloc); weights are copied from host arrays
 * into a handle-owned device arena.  Every call returns 0 (SD_OK) or a negative
 * status; sd_last_error() returns the message of the last failure on the
 * calling thread.  All compute calls are stream-ordered and do not allocate,
 * so they can be captured into a hipGraph.
 *
 * The reference has no FFI: its boundary is the PyTorch nn.Module surface.
 * Each entry point below names the reference callable it replaces; the Python
 * mirror (speaker_diarization_amd/) binds them with ctypes.
 */
#ifndef SDIAR_H_
#define SDIAR_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SD_OK 0
#define SD_ERR_INVALID (-1)  /* ValueError in the reference                       */
#define SD_ERR_SHAPE (-2)    /* AssertionError (label / feature length mismatch)  */
#define SD_ERR_PARAM (-3)    /* load_state_dict missing/unexpected key            */
#define SD_ERR_HIP (-4)      /* HIP runtime failure                               */
#define SD_ERR_STATE (-5)    /* handle used before finalize                       */

const char* sd_last_error(void);
int sd_version(void);

/* Opt-in kernel-family timing (HIP events on the launch stream) with
 * algorithmic FLOP/byte counts; used by bench.py for the live roofline.
 * sd_prof_query fills family i and returns 1, or returns 0 past the end. */
void sd_prof_enable(int on);
void sd_prof_reset(void);
int sd_prof_query(int i, char* name, int name_len, int64_t* launches, double* flops, double* bytes,
                  double* ms);
/* Sequential steps family i accumulated (latency-bound kernels: the LSTM recurrence counts its time steps). */
double sd_prof_query_steps(int i);
/* The persistent LSTM's exchange floor: one launch of the recurrence's 4-workgroup h hand-off protocol with
 * no gate arithmetic (same publish / poll / payload loads as lstm_group_bf16_kernel, batch 16) over `steps`
 * steps, timed with HIP events on `stream`; *us_per_step = its time / steps. */
int sd_probe_lstm_handoff(int steps, float* us_per_step, void* stream);
/* The same 4-workgroup exchange on data-tagged 8-byte granules (no counter, no barrier; MI355X guide
 * handoff-1to1): the hardware's hand-off price for the recurrence, us per step. */
int sd_probe_lstm_granule(int steps, float* us_per_step, void* stream);
/* Round 6: the granule exchange between TWO workgroups (each lane polls only the other one's half of its operand,
 * 1-to-1): the exchange floor of a recurrence that holds half of W_hh per CU. */
int sd_probe_lstm_granule2(int steps, float* us_per_step, void* stream);

/* ------------------------------------------------------------------ TS-VAD
 * Replaces TSVADModel (egs/alimeeting/ts_vad2/model.py:179-1142):
 *   construction  model.py:180-225 (TSVADConfig model.py:40-110)
 *   load_state_dict  (infer.py:184 loads checkpoint["model"])
 *   forward(ref_speech, target_speech, labels, num_updates)  model.py:899-921
 */
typedef struct sd_tsvad sd_tsvad;

typedef struct {
  int variant;                    /* 0: speech_encoder_type "CAM++", single/multi_backend "transformer"
                                     1: "CAM++_ots_vad", "conformer_ots_vad", "lstm_ots_vad", ots_vad_style "v1" */
  int max_num_speaker;            /* TSVADDataConfig.max_num_speaker (4)                     */
  int rs_len;                     /* seconds; PositionalEncoding max_len = rs_len * 25       */
  int max_batch;                  /* workspace sizing                                        */
  int max_fbank_frames;           /* workspace sizing: 1 + (rs_len*16000 - 400) / 160        */
  int precision;                  /* 0: fp32 (exact-f32 MFMA), 1: bf16 MFMA, fp32 accumulate, 2: bf16x3 (fp32 tensors; the GEMMs as bf16 hi+lo splits: hi·hi + hi·lo + lo·hi) */
  int num_transformer_layer;      /* TSVADConfig defaults: 2, 4, 384, 1536, 192              */
  int num_attention_head;
  int transformer_embed_dim;
  int transformer_ffn_embed_dim;
  int speaker_embed_dim;
} sd_tsvad_config;

int sd_tsvad_create(const sd_tsvad_config* cfg, sd_tsvad** out);
/* One state_dict entry by its reference key name (fp32 host data, torch shape). */
int sd_tsvad_set_param(sd_tsvad* h, const char* name, const float* host_data, const int64_t* shape,
                       int ndim);
/* Folds BatchNorms, packs/uploads weights, allocates the workspace.  Fails with
 * SD_ERR_PARAM listing missing or unexpected keys (strict load_state_dict). */
int sd_tsvad_finalize(sd_tsvad* h);
/* ref_speech: device (B, T_fbank, 80) fbank after per-window CMN + batch pad;
 * target_speech: device (B, max_num_speaker, speaker_embed_dim);
 * logits: device (B, max_num_speaker, T_label) — pre-sigmoid, like forward(). */
int sd_tsvad_forward(sd_tsvad* h, const float* ref_speech, const float* target_speech, int B,
                     int T_fbank, int T_label, float* logits, void* stream);
/* Waits for `stream` and returns SD_ERR_HIP if the ots_vad BiLSTM's persistent recurrence of a
 * forward enqueued on it lost workgroup co-residency (its logits are NaN).  The Python mirror
 * calls it after forward(), so the failing forward itself raises (RuntimeError); an
 * uncollected report is raised by the handle's next forward at the latest. */
int sd_tsvad_status(sd_tsvad* h, void* stream);
/* sd_tsvad_forward with the scope of BatchNorm1D's NaN bypass (ts_vad2/model.py:161-171) given per call (no
 * handle state): a window with a non-finite input makes the reference skip speech_down_or_up's (and, variant 0,
 * backend_down's) BatchNorm for every window of ITS batch.  forward_batch: windows per reference forward call
 * (the collater's batch, e.g. infer.py's 64) when this call covers several; 0: the call is one batch.
 * force: this call is a slice of a larger reference batch whose non-finite input lies in another slice —
 * bit 0: a non-finite fbank (both BatchNorms skipped for every window), bit 1: a non-finite variant-0
 * target-speaker embedding (backend_down's skipped).  sd_tsvad_forward = forward_batch 0, force 0. */
int sd_tsvad_forward_batched(sd_tsvad* h, const float* ref_speech, const float* target_speech, int B, int T_fbank,
                             int T_label, int forward_batch, int force, float* logits, void* stream);
int64_t sd_tsvad_device_bytes(const sd_tsvad* h);
/* Diagnostics only (not on the product path, which launches directly): capture sd_tsvad_forward once into a
 * hipGraph, optionally write its DOT dump to `dot_path`, replay it `replays` times on `stream` (each replay
 * rewrites logits) and wait; and the device buffers of the forward's stages (which: 0 mix, 1 mixg, 2 X2,
 * 3 H, 4 Y) for stage-by-stage comparisons. */
int sd_tsvad_forward_graph(sd_tsvad* h, const float* ref_speech, const float* target_speech, int B, int T_fbank,
                           int T_label, float* logits, int replays, const char* dot_path, void* stream);
int sd_tsvad_debug_buffer(const sd_tsvad* h, int which, void** ptr, int64_t* bytes);
int sd_tsvad_destroy(sd_tsvad* h);

/* ------------------------------------------------------------------ chunk-streaming TS-VAD
 * Replaces TSVADModel of egs/alimeeting/ts_vad2_streaming/model.py:95-1117 in its streaming
 * decode: forward_chunk_by_chunk(_temp1)(xs, target_speech, labels, decoding_chunk_size,
 * num_decoding_left_chunks) (model.py:368-461, 594-655; called through infer_debug :951-975 with
 * simulate_streaming, B = 1).  The KV caches are expressed as block-causal attention masks, so
 * one call decodes a whole window with the reference's per-chunk results.  State-dict keys are
 * the streaming model's (embed.speech_encoder.*, single_backend.{i}.self_attn.linear_q.*, ...). */
typedef struct sd_tsvad_stream sd_tsvad_stream;

typedef struct {
  int max_num_speaker;            /* 4 */
  int max_labels;                 /* workspace: label frames (25 Hz) per window */
  int precision;                  /* 0: fp32 (exact-f32 MFMA), 1: bf16 MFMA, fp32 accumulate */
  int num_transformer_layer;      /* TSVADConfig defaults (model.py:38-79): 2, 4, 384, 1536, 192 */
  int num_attention_head;
  int transformer_embed_dim;
  int transformer_ffn_embed_dim;
  int speaker_embed_dim;
  int max_windows;                /* workspace: windows per forward call (>= 1) */
} sd_tsvad_stream_config;

int sd_tsvad_stream_create(const sd_tsvad_stream_config* cfg, sd_tsvad_stream** out);
int sd_tsvad_stream_set_param(sd_tsvad_stream* h, const char* name, const float* host_data, const int64_t* shape,
                              int ndim);
int sd_tsvad_stream_finalize(sd_tsvad_stream* h);
/* B independent windows, each decoded as the reference's chunk loop decodes one (infer_debug,
 * batch 1, model.py:951-975).  feats: device (B, 4 * T_label, 80) fbank, already padded / trimmed
 * to 4 x labels (model.py:614-618); ts: device (B, max_num_speaker, speaker_embed_dim); chunk:
 * decoding_chunk_size (>= 1 label frame; a last partial chunk of any length, even 1 label = 4 fbank
 * frames, is decoded as the reference decodes it); left_chunks:
 * num_decoding_left_chunks (< 0: all history); logits: device (B, max_num_speaker, T_label),
 * pre-sigmoid. */
int sd_tsvad_stream_forward(sd_tsvad_stream* h, const float* feats, const float* ts, int B, int T_label, int chunk,
                            int left_chunks, float* logits, void* stream);
int64_t sd_tsvad_stream_device_bytes(const sd_tsvad_stream* h);
int sd_tsvad_stream_destroy(sd_tsvad_stream* h);

/* ------------------------------------------------------------------ CAM++ embeddings
 * Replaces CAMPPlus (egs/alimeeting/ts_vad2/cam_pplus_wespeaker.py:311-399) as the target-speaker
 * embedding extractor of generate_chunk_speaker_embedding_from_modelscope_for_diarization.py:
 *   construction  :256-260 (CAMPPLUS_COMMON: feat_dim 80, embedding_size 192)
 *   forward(x) / forward(x, get_time_out=True)  :264 / cam_pplus_wespeaker.py:388-399
 * State-dict keys are the standalone module's (head.*, xvector.*). */
typedef struct sd_campp sd_campp;

typedef struct {
  int feat_dim;        /* 80 */
  int embedding_size;  /* 192 (CAMPPLUS_COMMON) / 512 (CAMPPLUS_VOX)                     */
  int max_batch;       /* workspace: chunks per forward (extract_embed batch_size 96)      */
  int max_frames;      /* workspace: fbank frames per chunk (598 for 6 s)                  */
  int precision;       /* 0: fp32 (exact-f32 MFMA), 1: bf16 MFMA trunk (the pooled head stays fp32) */
} sd_campp_config;

int sd_campp_create(const sd_campp_config* cfg, sd_campp** out);
int sd_campp_set_param(sd_campp* h, const char* name, const float* host_data, const int64_t* shape, int ndim);
int sd_campp_finalize(sd_campp* h);
/* feats: device (B, T, 80) fbank; emb: device (B, embedding_size) or NULL; time_out: device
 * (B, (T-1)/2+1, 512) channel-last = xvector[:-2] output transposed, or NULL (one of the two). */
int sd_campp_forward(sd_campp* h, const float* feats, int B, int T, float* emb, float* time_out, void* stream);
int64_t sd_campp_device_bytes(const sd_campp* h);
int sd_campp_destroy(sd_campp* h);

/* ------------------------------------------------------------------ SSND
 * Replaces SSNDModel.infer (egs/alimeeting/ssnd/ssnd_model.py:752-776) with extractor
 * 'CAM++_wo_gsp' (:107-124), SSNDConformerEncoder (:172-195), DetectionDecoder (:274-296: the
 * speaker-query cross-attention decoder, SWDecoderBlockV2 :224-272) and RepresentationDecoder
 * (:343-370); construction :373-441 (training=False).  State-dict keys are SSNDModel's.  The
 * decoders always run exact fp32; precision selects the extractor / encoder arithmetic. */
typedef struct sd_ssnd sd_ssnd;

typedef struct {
  int max_batch;         /* workspace: blocks per call                                        */
  int max_fbank_frames;  /* workspace: fbank frames per block (800 = 8 s)                    */
  int max_speakers;      /* N: det_query_emb rows                                             */
  int feat_dim;          /* 80 */
  int emb_dim;           /* 256 */
  int q_det_aux_dim;     /* 256 */
  int q_rep_aux_dim;     /* 256 */
  int d_model;           /* 256 */
  int nhead;             /* 8 */
  int d_ff;              /* 512 */
  int num_layers;        /* 4 (encoder and both decoders) */
  int vad_out_len;       /* label frames per block (det_decoder.out_proj rows), 200 for 8 s */
  int pos_emb_dim;       /* 256 */
  int max_seq_len;       /* 1000 (pos_emb rows) */
  int n_all_speakers;    /* 1000 (E_all rows) */
  int conformer_kernel;  /* 15 (SSNDConformerEncoder cnn_kernel_size) */
  int precision;         /* 0: fp32, 1: bf16 MFMA extractor + encoder */
} sd_ssnd_config;

int sd_ssnd_create(const sd_ssnd_config* cfg, sd_ssnd** out);
int sd_ssnd_set_param(sd_ssnd* h, const char* name, const float* host_data, const int64_t* shape, int ndim);
int sd_ssnd_finalize(sd_ssnd* h);
/* SSNDModel.infer: feats device (B, T_fbank, 80) with (T_fbank - 1) / 2 + 1 CAM++ frames giving
 * vad_out_len label frames; speaker_embs device (B, max_speakers, emb_dim);
 * vad_pred device (B, max_speakers, vad_out_len) pre-sigmoid; emb_pred device (B, max_speakers, emb_dim). */
int sd_ssnd_infer(sd_ssnd* h, const float* feats, const float* speaker_embs, int B, int T_fbank, float* vad_pred,
                  float* emb_pred, void* stream);
/* The two decoders alone (infer after the encoder, :762-776): enc_out device (B, T, d_model),
 * x_fea device (B, T, emb_dim) (the extractor output), T == vad_out_len. */
int sd_ssnd_decode(sd_ssnd* h, const float* enc_out, const float* x_fea, const float* speaker_embs, int B, int T,
                   float* vad_pred, float* emb_pred, void* stream);
int64_t sd_ssnd_device_bytes(const sd_ssnd* h);
int sd_ssnd_destroy(sd_ssnd* h);

/* ------------------------------------------------------------------ EEND-EDA
 * Replaces TransformerEdaModel (speaker_diarization/eend_eda/models.py:161-347) and
 * EendEdaModel (models.py:466-652) with LstmEncoderDedecoderAttractor
 * (eend_eda/encoder_decoder_attractor.py:8-59):
 *   construction  infer_eda.py:50-71;  load_state_dict  infer_eda.py:88
 *   infer(src, infer_num_speakers, max_n_speakers, attractor_threshold)  models.py:297 / 601
 * The forward computes everything before speaker selection; the selection
 * (sort / first-n / threshold on the max_n_speakers probs) stays on the host.
 */
typedef struct sd_eda sd_eda;

typedef struct {
  int variant;          /* 0: TransformerEdaModel; 1: EendEdaModel(encoder_type "transformer");
                           2: EendEdaModel(encoder_type "conformer") (infer_eda.py model_type ConformerEda) */
  int in_size;          /* 345 = (2*context_size+1) * 23                                     */
  int n_units;          /* hidden_size (256)                                                  */
  int n_heads;          /* transformer_encoder_n_heads (4)                                    */
  int n_layers;         /* transformer_encoder_n_layers (2 / 4)                               */
  int dim_feedforward;  /* 2048 (never passed by infer_eda.py)                                */
  int max_seqs;         /* workspace: sequences (chunks) per forward                          */
  int max_frames;       /* workspace: frames per sequence (chunk_size, 2000)                  */
  int max_n_speakers;   /* attractors decoded (15)                                            */
  int precision;        /* 0: fp32 (exact-f32 MFMA), 1: bf16 MFMA, fp32 accumulate, 2: bf16x3 GEMMs */
  int n_speakers;       /* variant 3 only: decoder outputs                                    */
} sd_eda_config;
/* variant 3 is the plain EEND TransformerModel (speaker_diarization/eend/models.py:17-101,
 * called as model([chunk], activation=torch.sigmoid) from eend/eend_infer.py:69): the same
 * handle API; lengths/perm/probs may be NULL and act receives (S, T, n_speakers) sigmoid outputs. */

int sd_eda_create(const sd_eda_config* cfg, sd_eda** out);
int sd_eda_set_param(sd_eda* h, const char* name, const float* host_data, const int64_t* shape, int ndim);
int sd_eda_finalize(sd_eda* h);
/* Row stride (floats) the input features must have: in_size rounded up to 8 (352). */
int sd_eda_input_stride(const sd_eda* h);
/* feats: device (S, T, ld_feats) f32 (pad columns finite, e.g. zero or pad_sequence's -1);
 * lengths: device int32 (S) frames per sequence (ilens); key_len: device int32 (S) attention
 * key mask or NULL (the transformer variants attend to padded frames, models.py:216-226;
 * the conformer variant masks by ilens, :527-528); perm: device int32 (S, T), row s holds
 * torch.randperm(lengths[s]) drawn by the caller on the host CPU generator (models.py:229-233).
 * probs: device (S, max_n_speakers) attractor existence probabilities;
 * act: device (S, T, max_n_speakers - 1) = sigmoid(emb · attractors[:-1]ᵀ). */
int sd_eda_forward(sd_eda* h, const float* feats, int ld_feats, int S, int T, const int* lengths,
                   const int* key_len, const int* perm, float* probs, float* act, void* stream);
/* As sd_tsvad_status for the EDA encoder / decoder LSTMs (encoder_decoder_attractor.py:19-59). */
int sd_eda_status(sd_eda* h, void* stream);
int64_t sd_eda_device_bytes(const sd_eda* h);
int sd_eda_destroy(sd_eda* h);

/* ------------------------------------------------------------------ FS-EEND
 * Replaces OnlineTransformerDADiarization (speaker_diarization/fs_eend/fs_eend.py:20-96):
 *   construction  fs_eend/train.py:71-75 (config/spk_onl_tfm_enc_dec_nonautoreg_infer.yaml)
 *   test(src, ilens, max_nspks) -> (preds, emb, attractors)   fs_eend.py:79-96, called from
 *   fs_eend/model.py:198 with max_nspks = max_speakers + 2.
 * The causal encoder attends to all history: the path does not shard (replicas only). */
typedef struct sd_fseend sd_fseend;

typedef struct {
  int in_size;              /* (2 * context_recp + 1) * n_mels = 345                     */
  int n_units;              /* 256 */
  int n_heads;              /* 4   */
  int enc_n_layers;         /* 4   */
  int enc_dim_feedforward;  /* 2048 (MaskedTransformerEncoderModel default)             */
  int dec_n_layers;         /* 2: applications of the shared fusion layer               */
  int dec_dim_feedforward;  /* 2048 */
  int conv_delay;           /* 9 (Conv1d kernel 19, padding 9)                           */
  int mask_delay;           /* 0 */
  int has_mask;             /* 1: causal encoder                                          */
  int max_seqs;             /* workspace: sequences per call                              */
  int max_frames;           /* workspace: frames per sequence (chunk_size 10000)          */
  int max_nspks;            /* workspace: attractor slots (max_speakers + 2 = 6)         */
  int precision;            /* 0 fp32, 1 bf16 MFMA, 2 bf16x3 GEMMs (fp32 tensors) */
} sd_fseend_config;

int sd_fseend_create(const sd_fseend_config* cfg, sd_fseend** out);
int sd_fseend_set_param(sd_fseend* h, const char* name, const float* host_data, const int64_t* shape, int ndim);
int sd_fseend_finalize(sd_fseend* h);
int sd_fseend_input_stride(const sd_fseend* h);
/* feats: device (S, T, ld_feats) f32 = pad_sequence(src, -1) (pad columns finite);
 * ilens_host: host int32 (S); preds: device (S, T, max_nspks); emb: device (S, T, n_units) or NULL;
 * attractors: device (S, T, max_nspks, n_units) or NULL (both L2-normalised, as test() returns). */
int sd_fseend_test(sd_fseend* h, const float* feats, int ld_feats, int S, int T, const int* ilens_host,
                   int max_nspks, float* preds, float* emb, float* attractors, void* stream);
int64_t sd_fseend_device_bytes(const sd_fseend* h);
int sd_fseend_destroy(sd_fseend* h);

/* Streaming test(): the same scores as sd_fseend_test on the concatenated frames, produced
 * chunk by chunk from K/V histories (no reference counterpart: the reference recomputes the
 * causal forward over the whole recording, fs_eend.py:79-96 / fs_eend/model.py:198; the
 * causal masks of every shipped config, mask_delay 0, make the two identical).  A frame's
 * score is final 9 frames later (look-ahead Conv1d, fs_eend.py:41).  chunk: frames per push
 * (1..32; 1 frame = 100 ms at subsampling 10); use_graph: replay each chunk's kernels as a
 * captured hipGraph.  The stream keeps a pointer to its model handle: destroy it first. */
typedef struct sd_fseend_stream sd_fseend_stream;
int sd_fseend_stream_create(sd_fseend* h, int chunk, int max_frames, int max_nspks, int use_graph,
                            sd_fseend_stream** out);
/* feats: device (n, ld_feats) f32, 1 <= n <= chunk (n < chunk ends the input);
 * preds: device (cap, max_nspks) f32; *n_out = frames whose scores were written. */
int sd_fseend_stream_push(sd_fseend_stream* s, const float* feats, int ld_feats, int n, float* preds, int cap,
                          int* n_out, void* stream);
/* Audio input instead of feature rows (latency mode from raw audio): the FS-EEND frontend of
 * fs_eend/dataset.py:217-223 (transform 'logmel23' at the hardcoded 8 kHz: frame_size 200, frame_shift 80,
 * n_fft 256, 23 mels, no CMN) + feature.splice (context_size 7) + [::subsampling 10] (feature.py:130-184)
 * computed incrementally on the device: each chunk's STFT frames, logmel and spliced rows run inside its
 * captured encoder graph, reading the stream's audio history at the device cursor.  mel_fb: device
 * (n_mels, n_fft/2 + 1) f32 (librosa.filters.mel, Slaney), kept by pointer.  Call on a fresh or reset
 * stream; reset() returns the stream to feature rows.  push_audio: n samples (device f32, any n >= 0,
 * e.g. 640 = 80 ms); a model frame (100 ms) is encoded once its last spliced STFT frame has all its
 * samples, and scored 9 frames later (look-ahead); flush() then knows the length (feature.stft's frame
 * count, feature.py:176-184) and finishes.  The rows equal eend_features() of the whole recording bit
 * for bit, so the scores equal sd_fseend_test on them (as for feature pushes). */
int sd_fseend_stream_set_audio(sd_fseend_stream* s, const float* mel_fb, int n_mels, int frame_size, int frame_shift,
                               int context_size, int subsampling);
int sd_fseend_stream_push_audio(sd_fseend_stream* s, const float* samples, int64_t n, float* preds, int cap,
                                int* n_out, void* stream);
int sd_fseend_stream_flush(sd_fseend_stream* s, float* preds, int cap, int* n_out, void* stream);
/* reset: enqueues the cursor reset on `stream` and waits for it (and every chunk enqueued before it), so a
 * following set_audio() on any stream sees no chunk of the previous utterance still in flight. */
int sd_fseend_stream_reset(sd_fseend_stream* s, void* stream);
int64_t sd_fseend_stream_device_bytes(const sd_fseend_stream* s);
/* Counters for the latency model of bench.py's C5 line: encoder / decoder chunks run since creation and the
 * node count of each captured chunk graph (0 before the capture). */
int sd_fseend_stream_stats(const sd_fseend_stream* s, int64_t* enc_runs, int64_t* dec_runs, int* enc_nodes,
                           int* dec_nodes);
/* Diagnostics: the decode attention's per-(slot, head) block-merge counters, then the slot block's arrival
 * counter, copied to host_out (at most cap) after `stream` drains; *n = how many there are.  Each runs
 * 0..blocks-1 by a wrapping increment and is 0 between launches (test_gpu_fseend_stream.py). */
int sd_fseend_stream_debug_counters(const sd_fseend_stream* s, unsigned* host_out, int cap, int* n, void* stream);
int sd_fseend_stream_destroy(sd_fseend_stream* s);

/* feature.stft + feature.transform('logmel23_mn' | 'logmel23') + feature.splice + [::subsampling]
 * (speaker_diarization/feature.py:155-184, 56-73, 130-152; eend_eda/infer_eda.py:94-98).
 * wav: device f32 (n_samples) (soundfile values, computed in float64 like the reference);
 * n_frames: STFT frames = 1 + n_samples/frame_shift, minus one when divisible (feature.py:176-184);
 * mel_fb: device (n_mels, n_fft/2+1) Slaney mel (librosa.filters.mel, host-built);
 * mean_norm: 1 for logmel23_mn; work: device float64 (n_frames*n_mels + n_mels);
 * out: device (ceil(n_frames/subsampling), ld_out) f32, columns >= (2c+1)*n_mels zeroed. */
int sd_eend_features(const float* wav, int64_t n_samples, int frame_size, int frame_shift, int n_frames,
                     const float* mel_fb, int n_mels, int mean_norm, int context_size, int subsampling,
                     double* work, float* out, int ld_out, void* stream);

/* ------------------------------------------------------------------ frontend
 * FBank.__call__ (ts_vad2/ts_vad_dataset.py:29-56) over a whole recording at
 * dither 0: wav (n_samples) device fp32 in [-1,1), in_scale = 32768.
 * mel_fb: device (n_mels, 257) HTK banks (host-built, see frontend.py).
 * out: device (n_frames, n_mels), n_frames = 1 + (n_samples - 400) / 160. */
int sd_fbank_kaldi(const float* wav, int64_t n_samples, float in_scale, int n_frames,
                   const float* mel_fb, int n_mels, float* out, void* stream);
/* Same with the window chosen: window_type 0 hamming (TS-VAD FBank, ts_vad_dataset.py:45-52),
 * 1 povey (kaldi.fbank's default, used by the embedding extractor's FBank,
 * generate_chunk_speaker_embedding_from_modelscope_for_diarization.py:317-331, in_scale 1). */
int sd_fbank_kaldi_ex(const float* wav, int64_t n_samples, float in_scale, int n_frames, const float* mel_fb,
                      int n_mels, int window_type, float* out, void* stream);
/* Window slicing + per-window mean normalisation (mean_nor=True, :55) + the
 * collater's zero pad to the batch max (ts_vad_dataset.py:664-701).
 * win_start / win_n: device int32 (n_win). out: device (n_win, T_out, n_mels). */
int sd_window_cmn(const float* feats, int n_mels, const int* win_start, const int* win_n, int n_win,
                  int T_out, float* out, void* stream);

/* ------------------------------------------------------------------ posteriors
 * sigmoid (model.py:945-946) + mean over the overlapping windows covering each
 * label frame, in window order (ts_vad2/infer.py:90-94).  logits: device
 * (n_win, NS, Tw); start/len: device int32 (n_win) in label frames; windows start
 * every `dis` frames and span at most `chunk`.  out: device (NS, n_frames). */
int sd_overlap_average(const float* logits, int n_win, int NS, int Tw, const int* start,
                       const int* len, int dis, int chunk, int n_frames, float* out, void* stream);
/* The same mean over already-sigmoided probabilities (the res_dict lists of
 * TSVADModel.infer, model.py:945-966, averaged by infer.py:90-94): bit-identical to
 * np.mean of each frame's float32 list in window order (float32 sum from 0 in window
 * order, then one correctly rounded division by the count).  NaN where no window
 * covers a frame. */
int sd_overlap_mean(const float* probs, int n_win, int NS, int Tw, const int* start,
                    const int* len, int dis, int chunk, int n_frames, float* out, void* stream);

/* ------------------------------------------------------------------ postprocess
 * Replaces the host loop of ts_vad2/infer.py:72-130 (postprocess): per track
 * (one (meeting, speaker) posterior row of T frames) scipy.signal.medfilt(med_filter)
 * -> for each threshold: >= threshold (float32 compare), change_zeros_to_ones
 * (silence runs <= min_silence_frames become speech, :27-47), change_ones_to_zeros
 * (speech runs <= min_speech_frames become silence, :50-70) -> speech runs as
 * [begin, end) frame pairs.  min_*_frames = int(min_* // frame_len) as the recipe
 * computes it.  post: device (rows, T) f32.  thresholds: HOST array (1..16).
 * seg_begin/seg_end: device int32 (rows * n_thresholds, cap), cap >= (T+1)/2;
 * n_seg: device int32 (rows * n_thresholds), row-major (row, threshold).
 * RTTM formatting stays on the host (speaker_diarization_amd/ts_vad/postprocess.py).
 * flags bit 0: speech iff x > threshold (EEND bin/make_rttm.py:29, medfilt of the 0/1
 * decisions == threshold of the medfilt'd posteriors) instead of >=.
 * T <= 524288 frames. */
int sd_postprocess_segments(const float* post, int rows, int T, int med_filter, const float* thresholds,
                            int n_thresholds, int min_silence_frames, int min_speech_frames, int cap,
                            int* seg_begin, int* seg_end, int* n_seg, int flags, void* stream);

/* ------------------------------------------------------------------ ops (parity tests)
 * precision: 0 fp32, 1 bf16 MFMA (fp32 activations), 2 bf16 MFMA on bf16 activations
 * (the input is converted first; exercises the LDS-DMA GEMM path).
 * Weights are fp32 device arrays in torch layout. */
/* nn.Linear: out (M, N) = act(x (M, K) · w (N, K)ᵀ + b). act: 0 none 1 relu 2 sigmoid 3 silu */
int sd_op_linear(const float* x, int M, int K, const float* w, const float* b, int N, int act,
                 float* out, int precision, void* stream);
/* bf16 GEMM as the encoders run it: x bf16 bits (M rows, stride lda, columns
 * [a_coff, a_coff + K)); optional per-input-channel BN-ReLU prologue
 * x' = relu(x * pre_scale + pre_shift) (CAM++ nonlinear1, model.py dense layers);
 * out bf16 bits (M, ldo) = act(alpha * (x' · wᵀ) + beta). */
int sd_op_gemm_bf16(const void* x, int M, int K, int lda, int a_coff, const float* w, int N,
                    const float* pre_scale, const float* pre_shift, const float* alpha, const float* beta,
                    int act, void* out, int ldo, void* stream);
/* One CAM++ dense layer, bf16 (CAMDenseTDNNLayer + CAMLayer, egs/alimeeting/ts_vad2/cam_pplus_wespeaker.py:
 * 79-168) as the TS-VAD / embedding trunk runs it (cam_dense.hip): x bf16 bits (B, T, ld), input channels
 * [0, cin); out: bf16 bits at x's channels [cin, cin + 32) (out may alias x + cin).  s1/h1: nonlinear1
 * folded [cin]; wb: linear1 weight fp32 (128, cin); a2/b2: nonlinear2 folded [128]; wl: linear_local weight
 * fp32 (32, 128, 3); bl: its bias [32] or NULL; w1/c1: cam_layer.linear1 (64, 128)/(64); w2/c2:
 * cam_layer.linear2 (32, 64)/(32).  T <= 320, dil 1 or 2, cin % 32 == 0, cin <= 992.  repeats: run the
 * launch that many times on the same exchange records / counters (each must give the same bits). */
int sd_op_cam_dense(const void* x, int B, int T, int ld, int cin, int dil, const float* s1, const float* h1,
                    const float* wb, const float* a2, const float* b2, const float* wl, const float* bl,
                    const float* w1, const float* c1, const float* w2, const float* c2, void* out, int repeats,
                    void* stream);
/* Diagnostics: while `stamps` (device, >= 16 u64 per workgroup of a launch) is non-NULL, every cam_dense
 * launch records its workgroups' phase-boundary s_memrealtime stamps there (tools/cam_dense_probe.py). */
int sd_debug_cam_dense_probe(void* stamps);
/* Diagnostics: while `stamps` (device, >= 64 u64 per workgroup, zeroed) is non-NULL, every conformer pw2 + FFN
 * row-program launch (rowprog.hip, program 5) runs its stamping instantiation: lane 0 of every wave adds the
 * s_memtime cycles of its phases to stamps[(workgroup * 8 + wave) * 8 + k], k = 0 whole launch, 1 piece waits,
 * 2 refill issue, 3 epilogue, 4 tile loads (tools/rowprog_probe.py). */
int sd_debug_rowprog_probe(void* stamps);
/* Diagnostics: a captured graph [memsetAsync(X, 0) -> kernel: Y = X, then X = 7] (fork != 0: the kernel behind
 * an event fork / join of a second captured stream) replayed `replays` times; bad_per_replay (host, replays
 * ints) = Y values that were not 0 after each replay. */
int sd_probe_graph_memset(int n, int replays, int fork, int* bad_per_replay, void* stream);
/* The conformer self-attention block's in-projection + attention (mha_block.hip; torchaudio MHA with
 * batch_first, 8 heads of 48, D 384) on LayerNorm'd bf16 rows y (S, T, 384): w (1152, 384) / bias (1152) the
 * packed in_proj, key_len device int32 (S) or NULL, out bf16 (S, T, 384) = the heads' outputs before out_proj.
 * variant: the kernel layout (-1 or 0: the shipped <2 sequences, 8 waves, 3-slot ring, 48-wide Q / K rows>;
 * 1-7 the round-5 sweep's other layouts, mha_block.hip; tests).  flags (round 6): bit 0 = y given in the row
 * programs' MFMA-fragment layout (RowProgArgs::a_tiled), bit 1 = out written in it (S * T % 16 == 0). */
int sd_op_mha_block(const void* y, const float* w, const float* bias, int S, int T, const int* key_len, void* out,
                    int variant, int flags, void* stream);
/* nn.Conv1d on channel-last input x (B, T, Cin) with weight (Cout, Cin, k) -> out (B, To, Cout). */
int sd_op_conv1d(const float* x, int B, int T, int Cin, const float* w, const float* b, int Cout,
                 int k, int stride, int pad, int dil, int act, float* out, int precision, void* stream);
/* nn.Conv2d (Cin % 32 == 0) on NHWC x (B, H, W, Cin), weight (Cout, Cin, kh, kw) -> NHWC out. */
int sd_op_conv2d(const float* x, int B, int H, int W, int Cin, const float* w, int Cout, int kh,
                 int kw, int sh, int sw, int ph, int pw, float* out, int precision, void* stream);
/* Attention core on packed qkv (S*T, 3D) -> out (S*T, D). */
int sd_op_attention(const float* qkv, int S, int T, int D, int nh, int causal, int causal_delay,
                    const int* key_len, float* out, int precision, void* stream);
/* Chunk-streaming attention (ts_vad2_streaming forward_chunk_by_chunk's KV caches as one
 * block-causal mask): query i sees key j iff j / chunk <= i / chunk and, when left >= 0,
 * j / chunk >= i / chunk - left.  precision as sd_op_attention. */
/* Test op: time attention over a (S, T, C) token grid — qkv (S, T, C, 3D) rows, out (S, T, C, D) —
 * one sequence per (s, c) whose tokens are C rows apart, as the FS-EEND fusion decoder runs it
 * (fs_eend.py:459-478: MHA over time per speaker slot, causal mask).  precision as sd_op_attention. */
int sd_op_attention_grid(const float* qkv, int S, int T, int C, int D, int nh, int causal, int causal_delay,
                         float* out, int precision, void* stream);
int sd_op_attention_chunk(const float* qkv, int S, int T, int D, int nh, int chunk, int left, float* out,
                          int precision, void* stream);
/* Test probe: the attention above (causal / key_len / chunk terms as given) with every visited
 * (query, key) decision of sequence 0, head 0 written to mask_dump (T*T int32, caller-zeroed:
 * 0 = tile not visited, 1 = visible, 2 = masked).  Used by the mask tests only. */
int sd_probe_attention_mask(const float* qkv, int S, int T, int D, int nh, int causal, int causal_delay,
                            const int* key_len, int chunk, int left, int* mask_dump, float* out,
                            int precision, void* stream);
int sd_op_layernorm(const float* x, int rows, int D, const float* g, const float* b, float eps,
                    float* y, void* stream);
/* Residual add + LayerNorm of the encoder blocks: s = x + t (t fp32, or bf16 bits when
 * t_bf16); x <- s when write_x; y = LN(s) (bf16 bits when y_bf16). */
int sd_op_add_layernorm(float* x, const void* t, int t_bf16, int rows, int D, const float* g, const float* b,
                        float eps, int write_x, void* y, int y_bf16, void* stream);
/* LSTM recurrence on precomputed gx (B, T, ndir*4H) (biases included); whh (ndir, 4H, H). */
int sd_op_lstm(const float* gx, int B, int T, int H, int ndir, const float* whh, const int* lengths,
               float* out, float* hT, float* cT, float* work, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SDIAR_H_ */
