// EEND frontend + EDA glue kernels for gfx950.
//
// Frontend (speaker_diarization/feature.py, called from eend_eda/infer_eda.py:94-98
// and fs_eend/dataset.py):
//   stft_logmel  librosa.stft(n_fft, win_length, hop, 'hann', center=True,
//                pad_mode='constant') of the float64 wav (soundfile reads f64,
//                kaldi_data.py:82) -> |Y|^2 · mel^T (float64) -> log10(max(·, 1e-10)).
//                One wavefront per frame; the n_fft-point complex FFT runs in
//                float64 in LDS (the reference computes this stage in float64).
//   col_mean     per-recording mean of each mel channel ('logmel23_mn', feature.py:72).
//   splice       (x - mean) cast to f32, ±context zero-padded splice (feature.py:130-152)
//                and [::subsampling], written as 352-wide rows (in_size 345 + zero pad)
//                so the first Linear's K is a multiple of the MFMA k-step.
// EDA (eend_eda/models.py, encoder_decoder_attractor.py):
//   gather_rows       the frame shuffle emb[randperm(T)] (models.py:229-233)
//   fill_rows         decoder LSTM gates for the zero inputs = b_ih + b_hh (:50)
//   attractor_scores  sigmoid(linear(att)) (:53-58) and sigmoid(emb · att[:-1]ᵀ)
//                     (models.py:324-331)
#include <cmath>

#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {
namespace {

constexpr int kMaxMels = 64;

// One wave per frame, 8 frames per workgroup.  Everything a frame needs besides its samples is built
// once per workgroup in LDS: the twiddles, the Hann window (the same sincospi values the per-sample form
// computed) and each mel filter's nonzero bin range, so the projection runs over ~20 bins instead of
// BINS (the skipped terms are exact zeros: same sums, same order).  The butterfly stages of a frame
// belong to its wave alone, so they are ordered by a wave barrier, not a workgroup barrier.
// STREAM: the streaming frontend (sd_fseend_stream_push_audio) — local frame f is global frame
// f + frame0 with frame0 = cursor[0] * sub - context (the first frame a chunk's splice reads) and the
// sample bound min(n_samples, bound[0]) read from device memory, so one captured graph serves every
// chunk; the arithmetic per global frame is the whole-recording kernel's, bit for bit.
// STREAM also stages the mel filters in LDS (the projection's per-bin reads were dependent L2 round trips) and
// loads the frame's samples before the table prologue.  SPLICE (STREAM, FPB 16: a whole c = 1 chunk's 15
// logmel frames in one workgroup): the logmel frames stay in LDS and the same workgroup writes the chunk's
// spliced rows (splice_stream_kernel's arithmetic) -- no second launch.
template <int LOG2N, bool STREAM, int FPB = 8, bool SPLICE = false>
__global__ __launch_bounds__(FPB * 64) void stft_logmel_kernel(const float* __restrict__ wav, int64_t n_samples,
                                                               int n_frames, int hop, int win_len,
                                                               const float* __restrict__ mel_fb, int n_mels,
                                                               double* __restrict__ out, const int* __restrict__ cursor,
                                                               const int* __restrict__ bound, int sub, int context,
                                                               int rows = 0, float* __restrict__ sout = nullptr,
                                                               int ld_out = 0) {
  constexpr int N = 1 << LOG2N;
  constexpr int BINS = N / 2 + 1;
  static_assert(!SPLICE || STREAM, "the fused splice is the streaming frontend's");
  __shared__ double2 buf[FPB][N + N / 16];   // +1 element per 16: padded index pz(i) = i + i / 16
  __shared__ float melS[STREAM ? kMaxMels * BINS : 1];
  __shared__ double lmS[SPLICE ? FPB : 1][SPLICE ? kMaxMels : 1];
  // the bit-reversed scatter and the small-stride stages hit a few banks without the pad (PMC: 46 percent of
  // the LDS cycles were bank conflicts); the padded index spreads them, the arithmetic is unchanged
  auto pz = [](int i) { return i + (i >> 4); };
  __shared__ double2 tw[N / 2];
  __shared__ double win[N];
  __shared__ int mlo[kMaxMels], mhi[kMaxMels];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int f = blockIdx.x * FPB + w;
  const bool active = f < n_frames;
  // Frame f covers padded samples [f*hop, f*hop + N) of the wav zero-padded by N/2;
  // the periodic Hann window of win_len sits at offset (N - win_len)/2.
  const int lpad = (N - win_len) / 2;
  int64_t fg = f;
  const int64_t cap = n_samples;
  if constexpr (STREAM) {
    fg += (int64_t)cursor[0] * sub - context;
    n_samples = min(n_samples, (int64_t)bound[0]);
  }
  const int64_t base = fg * hop - N / 2 + lpad;
  // REG (whole-recording 512-point frames): the FFT as three register passes of three radix-2 stages with two LDS
  // transposes (the per-stage form moves every element through LDS nine times); same butterflies, same twiddles.
  // The lane then holds samples r6 + 64 u (r6 = bitrev6(lane)): its pass-A positions 8 lane + k are samples
  // bitrev3(k) * 64 + r6.
  constexpr bool REG = LOG2N == 9 && !STREAM;
  const int r6 = (int)(__brev((unsigned)lane) >> 26);
  // the frame's samples, in flight during the table prologue (clamped loads, masked after)
  float raw[N / 64];
#pragma unroll
  for (int u = 0; u < N / 64; ++u) {
    const int64_t gi = base + ((REG ? r6 : lane) + 64 * u) - lpad;
    raw[u] = cap > 0 ? wav[min(max(gi, (int64_t)0), cap - 1)] : 0.f;
  }
  for (int k = threadIdx.x; k < N / 2; k += blockDim.x) {
    double s, c;
    sincospi(-2.0 * (double)k / (double)N, &s, &c);
    tw[k] = make_double2(c, s);
  }
  for (int j = threadIdx.x; j < win_len; j += blockDim.x) {
    double s, c;
    sincospi(2.0 * (double)j / (double)win_len, &s, &c);
    win[j] = 0.5 - 0.5 * c;
  }
  for (int m = threadIdx.x; m < n_mels; m += blockDim.x) {
    mlo[m] = BINS;
    mhi[m] = 0;
  }
  __syncthreads();
  // each filter's nonzero bin range; the filter values' loads issued in batches of 8 (one round trip each)
  const int nfb = n_mels * BINS;
  for (int i0 = threadIdx.x; i0 < nfb; i0 += 8 * (int)blockDim.x) {
    float fv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) fv[u] = mel_fb[min(i0 + u * (int)blockDim.x, nfb - 1)];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * (int)blockDim.x;
      if (i < nfb) {
        if constexpr (STREAM) melS[i] = fv[u];
        if (fv[u] != 0.f) {
          const int m = i / BINS, k = i - m * BINS;
          atomicMin(&mlo[m], k);
          atomicMax(&mhi[m], k + 1);
        }
      }
    }
  }
  __syncthreads();   // window table, filter ranges
  if constexpr (REG) {
    auto bfly = [](double2& a, double2& b, double2 t0) {
      const double2 t = make_double2(b.x * t0.x - b.y * t0.y, b.x * t0.y + b.y * t0.x);
      const double2 a0 = a;
      a = make_double2(a0.x + t.x, a0.y + t.y);
      b = make_double2(a0.x - t.x, a0.y - t.y);
    };
    double2 X[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {   // pass A positions 8 lane + k
      const int u = (int)(__brev((unsigned)k) >> 29);
      const int n = r6 + 64 * u;
      double v = 0.0;
      const int j = n - lpad;
      if (active && j >= 0 && j < win_len) {
        const int64_t gi = base + j;
        if (gi >= 0 && gi < n_samples) v = (double)raw[u] * win[j];
      }
      X[k] = make_double2(v, 0.0);
    }
#pragma unroll
    for (int half = 1; half < 8; half <<= 1)
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (!(k & half)) bfly(X[k], X[k + half], tw[(k & (half - 1)) * (N / 2 / half)]);
#pragma unroll
    for (int k = 0; k < 8; ++k) buf[w][pz(8 * lane + k)] = X[k];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int pb = 64 * (lane >> 3) + (lane & 7);   // pass B: positions 64 b + r + 8 m (lane = 8 b + r)
#pragma unroll
    for (int m = 0; m < 8; ++m) X[m] = buf[w][pz(pb + 8 * m)];
#pragma unroll
    for (int h = 1; h < 8; h <<= 1)   // half = 8 h
#pragma unroll
      for (int m = 0; m < 8; ++m)
        if (!(m & h)) bfly(X[m], X[m + h], tw[((lane & 7) + 8 * m) % (8 * h) * (N / 16 / h)]);
#pragma unroll
    for (int m = 0; m < 8; ++m) buf[w][pz(pb + 8 * m)] = X[m];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int m = 0; m < 8; ++m) X[m] = buf[w][pz(lane + 64 * m)];   // pass C: positions lane + 64 m
#pragma unroll
    for (int h = 1; h < 8; h <<= 1)   // half = 64 h
#pragma unroll
      for (int m = 0; m < 8; ++m)
        if (!(m & h)) bfly(X[m], X[m + h], tw[(lane + 64 * m) % (64 * h) * (N / 128 / h)]);
#pragma unroll
    for (int m = 0; m < 8; ++m) buf[w][pz(lane + 64 * m)] = X[m];
  } else {
#pragma unroll
  for (int u = 0; u < N / 64; ++u) {
    const int n = lane + 64 * u;
    double v = 0.0;
    const int j = n - lpad;
    if (active && j >= 0 && j < win_len) {
      const int64_t gi = base + j;
      if (gi >= 0 && gi < n_samples) v = (double)raw[u] * win[j];
    }
    const int r = (int)(__brev((unsigned)n) >> (32 - LOG2N));
    buf[w][pz(r)] = make_double2(v, 0.0);
  }
  for (int half = 1; half < N; half <<= 1) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int tstride = N / (2 * half);
    for (int bfly = lane; bfly < N / 2; bfly += 64) {
      const int grp = bfly / half, pos = bfly % half;
      const int i0 = grp * 2 * half + pos, i1 = i0 + half;
      const double2 t0 = tw[pos * tstride];
      const double2 a = buf[w][pz(i0)], b = buf[w][pz(i1)];
      const double2 t = make_double2(b.x * t0.x - b.y * t0.y, b.x * t0.y + b.y * t0.x);
      buf[w][pz(i0)] = make_double2(a.x + t.x, a.y + t.y);
      buf[w][pz(i1)] = make_double2(a.x - t.x, a.y - t.y);
    }
  }
  }   // REG
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (active) {
    for (int m = lane; m < n_mels; m += 64) {
      const float* fr = STREAM ? melS + m * BINS : mel_fb + (int64_t)m * BINS;
      double acc = 0.0;
      for (int k = mlo[m]; k < mhi[m]; ++k) {
        const double2 c = buf[w][pz(k)];
        acc = fma((double)fr[k], c.x * c.x + c.y * c.y, acc);
      }
      const double y = log10(fmax(acc, 1e-10));
      if constexpr (SPLICE) lmS[w][m] = y;
      else out[(int64_t)f * n_mels + m] = y;
    }
  }
  if constexpr (SPLICE) {
    // splice_stream_kernel over this workgroup's frames (local frame r * sub + c of row r)
    __syncthreads();
    const int nf = bound[1], i0 = cursor[0];
    const int width = (2 * context + 1) * n_mels;
    for (int r = 0; r < rows; ++r) {
      const int i = i0 + r;
      const bool row_live = (int64_t)i * sub < (int64_t)nf;
      for (int e = threadIdx.x; e < ld_out; e += blockDim.x) {
        float v = 0.f;
        if (row_live && e < width) {
          const int c = e / n_mels, m = e % n_mels;
          const int64_t fgl = (int64_t)i * sub + c - context;
          if (fgl >= 0 && fgl < nf) v = (float)lmS[r * sub + c][m];
        }
        sout[(int64_t)r * ld_out + e] = v;
      }
    }
  }
}

// One block per mel channel: fixed-order strided partial sums + tree -> deterministic.
__global__ __launch_bounds__(256) void col_mean_kernel(const double* __restrict__ x, int rows, int cols,
                                                       double* __restrict__ mean) {
  __shared__ double red[256];
  const int c = blockIdx.x;
  double s = 0.0;
  for (int r = threadIdx.x; r < rows; r += 256) s += x[(int64_t)r * cols + c];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) mean[c] = red[0] / (double)rows;
}

__global__ __launch_bounds__(256) void splice_kernel(const double* __restrict__ lm, int n_frames, int n_mels,
                                                     const double* __restrict__ mean, int context, int sub,
                                                     int n_out, float* __restrict__ out, int ld_out) {
  const int r = blockIdx.x;
  if (r >= n_out) return;
  const int width = (2 * context + 1) * n_mels;
  for (int i = threadIdx.x; i < ld_out; i += blockDim.x) {
    float v = 0.f;
    if (i < width) {
      const int c = i / n_mels, m = i % n_mels;
      const int f = r * sub + c - context;
      if (f >= 0 && f < n_frames) {
        const double y = lm[(int64_t)f * n_mels + m] - (mean ? mean[m] : 0.0);
        v = (float)y;
      }
    }
    out[(int64_t)r * ld_out + i] = v;
  }
}

// Streaming splice: row r is model frame i = cursor[0] + r, built from the chunk's logmel frames
// (local frame = global frame - (cursor[0] * sub - context)); frames outside [0, bound[1]) are the splice's
// zero padding and rows of model frames >= ceil(bound[1] / sub) (past the end of the input) are zero.
__global__ __launch_bounds__(128) void splice_stream_kernel(const double* __restrict__ lm, int n_mels, int context,
                                                            int sub, const int* __restrict__ cursor,
                                                            const int* __restrict__ bound, float* __restrict__ out,
                                                            int ld_out) {
  const int r = blockIdx.x;
  const int i = cursor[0] + r;
  const int nf = bound[1];
  const bool row_live = (int64_t)i * sub < (int64_t)nf;
  const int width = (2 * context + 1) * n_mels;
  for (int e = threadIdx.x; e < ld_out; e += blockDim.x) {
    float v = 0.f;
    if (row_live && e < width) {
      const int c = e / n_mels, m = e % n_mels;
      const int64_t fgl = (int64_t)i * sub + c - context;
      if (fgl >= 0 && fgl < nf) v = (float)lm[(int64_t)(r * sub + c) * n_mels + m];
    }
    out[(int64_t)r * ld_out + e] = v;
  }
}

__global__ __launch_bounds__(256) void gather_rows_kernel(const float* __restrict__ x, int T, int D,
                                                          const int* __restrict__ perm,
                                                          const int* __restrict__ lengths,
                                                          float* __restrict__ y) {
  const int s = blockIdx.y, t = blockIdx.x;
  const int len = lengths ? lengths[s] : T;
  const int src = t < len ? perm[(int64_t)s * T + t] : t;
  const float* xr = x + ((int64_t)s * T + src) * D;
  float* yr = y + ((int64_t)s * T + t) * D;
  for (int i = threadIdx.x; i < D; i += blockDim.x) yr[i] = xr[i];
}

__global__ __launch_bounds__(256) void fill_rows_kernel(const float* __restrict__ row, int D, int rows,
                                                        float* __restrict__ y) {
  const int64_t n = (int64_t)rows * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = row[i % D];
}

constexpr int kScoreRows = 32;

// One block per (sequence, 32 frames): attractors of the sequence in LDS.
__global__ __launch_bounds__(256) void attractor_scores_kernel(
    const float* __restrict__ emb, int T, int E, const float* __restrict__ att, int n_att,
    const float* __restrict__ lw, const float* __restrict__ lb, float* __restrict__ probs,
    float* __restrict__ act) {
  extern __shared__ float sm[];
  const int ES = E + 1;
  float* as = sm;                       // [n_att][ES]
  float* es = as + n_att * ES;          // [kScoreRows][ES]
  const int s = blockIdx.y;
  const int t0 = blockIdx.x * kScoreRows;
  const float* a = att + (int64_t)s * n_att * E;
  for (int i = threadIdx.x; i < n_att * E; i += blockDim.x) as[(i / E) * ES + i % E] = a[i];
  const int nr = min(kScoreRows, T - t0);
  for (int i = threadIdx.x; i < nr * E; i += blockDim.x)
    es[(i / E) * ES + i % E] = emb[((int64_t)s * T + t0 + i / E) * E + i % E];
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x < n_att) {
    const int j = threadIdx.x;
    float acc = 0.f;
    for (int k = 0; k < E; ++k) acc = fmaf(as[j * ES + k], lw[k], acc);
    acc += lb[0];
    probs[(int64_t)s * n_att + j] = 1.f / (1.f + expf(-acc));
  }
  const int ns = n_att - 1;
  for (int i = threadIdx.x; i < nr * ns; i += blockDim.x) {
    const int r = i / ns, j = i % ns;
    float acc = 0.f;
    for (int k = 0; k < E; ++k) acc = fmaf(es[r * ES + k], as[j * ES + k], acc);
    act[((int64_t)s * T + t0 + r) * ns + j] = 1.f / (1.f + expf(-acc));
  }
}

}  // namespace

void stft_logmel(const float* wav, int64_t n_samples, int n_frames, int n_fft, int hop, int win_len,
                 const float* mel_fb, int n_mels, double* out, hipStream_t st) {
  SD_CHECK(n_fft == 256 || n_fft == 512, kErrInvalid, "stft: n_fft must be 256 or 512");
  SD_CHECK(win_len > 0 && win_len <= n_fft && hop > 0, kErrInvalid, "stft: bad frame_size/frame_shift");
  SD_CHECK(n_mels > 0 && n_mels <= kMaxMels, kErrInvalid, "stft: n_mels out of range");
  if (n_frames <= 0) return;
  ProfScope prof("stft_logmel", 5.0 * n_fft * std::log2((double)n_fft) * n_frames,
                 4.0 * (double)n_frames * hop + 8.0 * n_frames * n_mels, st);
  const dim3 grid(cdiv(n_frames, 8));
  if (n_fft == 512)
    hipLaunchKernelGGL((stft_logmel_kernel<9, false>), grid, dim3(512), 0, st, wav, n_samples, n_frames, hop, win_len,
                       mel_fb, n_mels, out, nullptr, nullptr, 0, 0);
  else
    hipLaunchKernelGGL((stft_logmel_kernel<8, false>), grid, dim3(512), 0, st, wav, n_samples, n_frames, hop, win_len,
                       mel_fb, n_mels, out, nullptr, nullptr, 0, 0);
  SD_LAUNCH_CHECK();
}

void stream_frontend(const float* wav, int64_t cap_samples, int rows, int n_fft, int hop, int win_len,
                     const float* mel_fb, int n_mels, int context, int sub, const int* cursor, const int* bound,
                     double* lm, float* out, int ld_out, hipStream_t st) {
  SD_CHECK(n_fft == 256 || n_fft == 512, kErrInvalid, "stream frontend: n_fft must be 256 or 512");
  SD_CHECK(win_len > 0 && win_len <= n_fft && hop > 0, kErrInvalid, "stream frontend: bad frame_size/frame_shift");
  SD_CHECK(n_mels > 0 && n_mels <= kMaxMels, kErrInvalid, "stream frontend: n_mels out of range");
  SD_CHECK(ld_out >= (2 * context + 1) * n_mels, kErrInvalid, "stream frontend: ld_out < spliced width");
  const int n_frames = (rows - 1) * sub + 2 * context + 1;   // logmel frames the chunk's splice reads
  ProfScope prof("stream_frontend", 5.0 * n_fft * std::log2((double)n_fft) * n_frames,
                 4.0 * (double)n_frames * hop + 4.0 * rows * ld_out, st);
  if (n_fft == 256 && n_frames <= 16) {   // the chunk in one workgroup, splice included
    hipLaunchKernelGGL((stft_logmel_kernel<8, true, 16, true>), dim3(1), dim3(1024), 0, st, wav, cap_samples, n_frames,
                       hop, win_len, mel_fb, n_mels, lm, cursor, bound, sub, context, rows, out, ld_out);
    SD_LAUNCH_CHECK();
    return;
  }
  const dim3 grid(cdiv(n_frames, 8));
  if (n_fft == 512)
    hipLaunchKernelGGL((stft_logmel_kernel<9, true>), grid, dim3(512), 0, st, wav, cap_samples, n_frames, hop,
                       win_len, mel_fb, n_mels, lm, cursor, bound, sub, context);
  else
    hipLaunchKernelGGL((stft_logmel_kernel<8, true>), grid, dim3(512), 0, st, wav, cap_samples, n_frames, hop,
                       win_len, mel_fb, n_mels, lm, cursor, bound, sub, context);
  hipLaunchKernelGGL(splice_stream_kernel, dim3(rows), dim3(128), 0, st, lm, n_mels, context, sub, cursor, bound, out,
                     ld_out);
  SD_LAUNCH_CHECK();
}

void col_mean(const double* x, int rows, int cols, double* mean, hipStream_t st) {
  SD_CHECK(rows > 0, kErrInvalid, "col_mean: empty input");
  hipLaunchKernelGGL(col_mean_kernel, dim3(cols), dim3(256), 0, st, x, rows, cols, mean);
  SD_LAUNCH_CHECK();
}

void splice_subsample(const double* lm, int n_frames, int n_mels, const double* mean, int context,
                      int sub, int n_out, float* out, int ld_out, hipStream_t st) {
  SD_CHECK(ld_out >= (2 * context + 1) * n_mels, kErrInvalid, "splice: ld_out < spliced width");
  if (n_out <= 0) return;
  ProfScope prof("splice", 0.0, 4.0 * (double)n_out * ld_out + 8.0 * n_frames * n_mels, st);
  hipLaunchKernelGGL(splice_kernel, dim3(n_out), dim3(128), 0, st, lm, n_frames, n_mels, mean, context, sub,
                     n_out, out, ld_out);
  SD_LAUNCH_CHECK();
}

void gather_rows(const float* x, int S, int T, int D, const int* perm, const int* lengths, float* y,
                 hipStream_t st) {
  hipLaunchKernelGGL(gather_rows_kernel, dim3(T, S), dim3(64), 0, st, x, T, D, perm, lengths, y);
  SD_LAUNCH_CHECK();
}

void fill_rows(const float* row, int D, int rows, float* y, hipStream_t st) {
  const int64_t n = (int64_t)rows * D;
  if (n <= 0) return;
  const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(fill_rows_kernel, dim3(blocks), dim3(256), 0, st, row, D, rows, y);
  SD_LAUNCH_CHECK();
}

void attractor_scores(const float* emb, int S, int T, int E, const float* att, int n_att, const float* lw,
                      const float* lb, float* probs, float* act, hipStream_t st) {
  const size_t smem = sizeof(float) * (size_t)(n_att + kScoreRows) * (E + 1);
  SD_CHECK(smem <= 160 * 1024, kErrInvalid, "attractor_scores: too many attractors for LDS");
  static bool attr = false;
  if (!attr) {
    SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(attractor_scores_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  ProfScope prof("attractor_scores", 2.0 * S * T * E * (n_att - 1), 4.0 * S * T * (E + n_att), st);
  hipLaunchKernelGGL(attractor_scores_kernel, dim3(cdiv(T, kScoreRows), S), dim3(256), smem, st, emb, T, E,
                     att, n_att, lw, lb, probs, act);
  SD_LAUNCH_CHECK();
}

}  // namespace sd
