// Kaldi-compatible log-mel filterbank on gfx950 (one wavefront per frame).
//
// Semantics follow torchaudio.compliance.kaldi.fbank as called from
// ts_vad2/ts_vad_dataset.py:39-52 (FBank.__call__): waveform * 2^15, frames of
// 400 samples every 160 (snip_edges=True), per-frame DC removal, pre-emphasis
// 0.97 (first sample against itself), symmetric Hamming (or povey) window, zero pad to 512,
// |rFFT|^2, HTK-mel triangular banks (host-built, 80 x 257), log(max(e, FLT_EPS)).
// dither is 0 here: the reference's default dither=1.0 adds fresh noise per
// call, so parity is defined at dither 0.
//
// The whole meeting is framed once; windows (ts_vad_dataset.py:242-271) start
// every 25 label frames = 400 fbank frames/s * k, so each window's frames are a
// contiguous slice of the meeting's frames and window_cmn() only subtracts the
// per-window mean.  That removes the 6x frame recomputation of overlapping
// 6 s / 1 s-shift windows.
#include <algorithm>
#include <cstdlib>
#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {
namespace {

constexpr int kFrameLen = 400;
constexpr int kShift = 160;
constexpr int kNfft = 512;
constexpr int kBins = kNfft / 2 + 1;
constexpr int kFramesPerBlock = 8;
constexpr int kMaxFbMels = 128;
constexpr int kMelCap = 2 * kBins + 2 * kMaxFbMels;   // triangular banks: each bin in at most two filters

__device__ __forceinline__ void wave_sync() {   // order one wave's LDS accesses (no workgroup barrier)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One wave per frame, 8 frames per workgroup.  Built once per workgroup in LDS: the twiddles, the
// window (the same cospif / powf values the per-sample form computed) and each mel filter's nonzero bin
// range and values, so the projection runs over a filter's ~10 bins instead of all 257 (the skipped terms
// are exact zeros: same sums, same order).  A frame's FFT stages belong to its wave alone: wave barriers only.
__global__ __launch_bounds__(512) void fbank_kernel(const float* __restrict__ wav, int64_t n_samples,
                                                    float in_scale, int n_frames,
                                                    const float* __restrict__ mel_fb, int n_mels,
                                                    const float2* __restrict__ twiddle, int window,
                                                    float* __restrict__ out) {
  __shared__ float2 buf[kFramesPerBlock][kNfft + kNfft / 32];   // padded index pz(i) = i + i / 32
  // the bit-reversed scatter and the small-stride stages hit a few banks without the pad (PMC: 46 percent of
  // the LDS cycles were bank conflicts); the padded index spreads them, the arithmetic is unchanged
  auto pz = [](int i) { return i + (i >> 5); };
  __shared__ float pw[kFramesPerBlock][kBins + 3];
  __shared__ float2 tw[kNfft / 2];
  __shared__ float win[kFrameLen];
  __shared__ int mlo[kMaxFbMels], mhi[kMaxFbMels], moff[kMaxFbMels + 1];
  __shared__ float melv[kMelCap];   // every filter's nonzero run, packed (moff[m] = its start)
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;

  for (int k = threadIdx.x; k < kNfft / 2; k += blockDim.x) tw[k] = twiddle[k];
  for (int n = threadIdx.x; n < kFrameLen; n += blockDim.x) {
    const float cw = cospif(2.f * (float)n / (float)(kFrameLen - 1));
    // hamming (ts_vad_dataset.py:50) or povey = hann^0.85 (kaldi default, used by the
    // embedding extractor, generate_chunk_speaker_embedding_...py:326-327).
    win[n] = window == 0 ? 0.54f - 0.46f * cw : powf(0.5f - 0.5f * cw, 0.85f);
  }
  for (int m = threadIdx.x; m < n_mels; m += blockDim.x) {
    mlo[m] = kBins;
    mhi[m] = 0;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n_mels * kBins; i += blockDim.x) {
    const int m = i / kBins, k = i - m * kBins;
    if (mel_fb[i] != 0.f) {
      atomicMin(&mlo[m], k);
      atomicMax(&mhi[m], k + 1);
    }
  }
  __syncthreads();   // mel ranges
  if (threadIdx.x == 0) {
    int o = 0;
    for (int m = 0; m < n_mels; ++m) {
      moff[m] = o;
      o += max(mhi[m] - mlo[m], 0);
    }
    moff[n_mels] = o;
  }
  __syncthreads();
  // the filters' runs in LDS (the projection read them from global memory, one dependent load per bin: most of
  // the kernel's time); a mel matrix with more nonzero runs than kMelCap keeps the global reads
  const bool lds_mel = moff[n_mels] <= kMelCap;
  if (lds_mel)
    for (int i = threadIdx.x; i < n_mels * kBins; i += blockDim.x) {
      const int m = i / kBins, k = i - m * kBins;
      if (k >= mlo[m] && k < mhi[m]) melv[moff[m] + k - mlo[m]] = mel_fb[i];
    }
  __syncthreads();   // window table, twiddles, mel runs

  // The workgroup walks frame groups blockIdx.x, + gridDim.x, ...: the tables above (a 20 k-entry scan of the
  // mel matrix) are built once per workgroup instead of once per 8 frames.
  const int n_groups = (n_frames + kFramesPerBlock - 1) / kFramesPerBlock;
  // a frame group's samples are requested one group ahead (in flight during the previous group's FFT)
  float xr[7];
  auto load_x = [&](int fg) {
    const int f = fg * kFramesPerBlock + w;
    const bool active = f < n_frames;
    const float* x = wav + (int64_t)(active ? f : 0) * kShift;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      int n = lane + i * 64;
      int64_t gi = (int64_t)(active ? f : 0) * kShift + n;
      xr[i] = (fg < n_groups && n < kFrameLen && gi < n_samples) ? x[n] : 0.f;
    }
  };
  load_x(blockIdx.x);
  for (int fg = blockIdx.x; fg < n_groups; fg += gridDim.x) {
    const int f = fg * kFramesPerBlock + w;
    const bool active = f < n_frames;
    // Load, DC removal.
    float v[7];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      int n = lane + i * 64;
      int64_t gi = (int64_t)(active ? f : 0) * kShift + n;
      v[i] = (n < kFrameLen && gi < n_samples) ? xr[i] * in_scale : 0.f;
      s += v[i];
    }
    load_x(fg + gridDim.x);
    s = warp_sum(s);
    const float mean = s / (float)kFrameLen;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      int n = lane + i * 64;
      if (n < kFrameLen) buf[w][pz(n)].x = v[i] - mean;   // scratch (real part)
    }
    wave_sync();   // this frame's scratch
    {
      // Radix-2 DIT in three register passes of three stages each, the wave's LDS only for the two
      // transposes between them (round 5; the nine-stage LDS form it replaced moved every element through LDS
      // nine times).
      // Same butterflies, same twiddles, same order per element.
      // pass A: bit-reversed positions 8 lane + k (sample bitrev3(k) * 64 + bitrev6(lane)), stages 1, 2, 4
      float2 X[8];
      const int r6 = (int)(__brev((unsigned)lane) >> 26);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int n = (int)(__brev((unsigned)k) >> 29) * 64 + r6;
        float val = 0.f;
        if (n < kFrameLen) {
          float cur = buf[w][pz(n)].x;
          float prev = n > 0 ? buf[w][pz(n - 1)].x : cur;
          val = (cur - 0.97f * prev) * win[n];
        }
        X[k] = make_float2(val, 0.f);
      }
      auto bfly = [](float2& a, float2& b, float2 t0) {
        const float2 t = make_float2(b.x * t0.x - b.y * t0.y, b.x * t0.y + b.y * t0.x);
        const float2 a0 = a;
        a = make_float2(a0.x + t.x, a0.y + t.y);
        b = make_float2(a0.x - t.x, a0.y - t.y);
      };
#pragma unroll
      for (int half = 1; half < 8; half <<= 1)
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (!(k & half)) bfly(X[k], X[k + half], tw[(k & (half - 1)) * (kNfft / 2 / half)]);
      wave_sync();   // every lane's pre-emphasis reads of the scratch are done
#pragma unroll
      for (int k = 0; k < 8; ++k) buf[w][pz(8 * lane + k)] = X[k];
      wave_sync();
      // pass B: positions 64 b + r + 8 m (lane = 8 b + r), stages 8, 16, 32
      const int pb = 64 * (lane >> 3) + (lane & 7);
#pragma unroll
      for (int m = 0; m < 8; ++m) X[m] = buf[w][pz(pb + 8 * m)];
#pragma unroll
      for (int h = 1; h < 8; h <<= 1)   // half = 8 h
#pragma unroll
        for (int m = 0; m < 8; ++m)
          if (!(m & h)) bfly(X[m], X[m + h], tw[((lane & 7) + 8 * m) % (8 * h) * (kNfft / 16 / h)]);
#pragma unroll
      for (int m = 0; m < 8; ++m) buf[w][pz(pb + 8 * m)] = X[m];
      wave_sync();
      // pass C: positions lane + 64 m, stages 64, 128, 256
#pragma unroll
      for (int m = 0; m < 8; ++m) X[m] = buf[w][pz(lane + 64 * m)];
#pragma unroll
      for (int h = 1; h < 8; h <<= 1)   // half = 64 h
#pragma unroll
        for (int m = 0; m < 8; ++m)
          if (!(m & h)) bfly(X[m], X[m + h], tw[(lane + 64 * m) % (64 * h) * (kNfft / 128 / h)]);
#pragma unroll
      for (int m = 0; m < 5; ++m)
        if (lane + 64 * m < kBins) pw[w][lane + 64 * m] = X[m].x * X[m].x + X[m].y * X[m].y;
    }
    wave_sync();
    if (active) {
      const float eps = 1.1920928955078125e-07f;
      for (int m = lane; m < n_mels; m += 64) {
        float acc = 0.f;
        if (lds_mel) {
          const int lo = mlo[m], base = moff[m];
          for (int k = lo; k < mhi[m]; ++k) acc = fmaf(melv[base + (k - lo)], pw[w][k], acc);
        } else {
          const float* fr = mel_fb + (int64_t)m * kBins;
          for (int k = mlo[m]; k < mhi[m]; ++k) acc = fmaf(fr[k], pw[w][k], acc);
        }
        out[(int64_t)f * n_mels + m] = logf(fmaxf(acc, eps));
      }
    }
    wave_sync();   // the next frame group rewrites buf[w] / pw[w]
  }
}

float2* g_twiddle = nullptr;

}  // namespace

void fbank_kaldi(const float* wav, int64_t n_samples, float in_scale, int n_frames,
                 const float* mel_fb, int n_mels, float* out, hipStream_t st, int window) {
  SD_CHECK(window == 0 || window == 1, kErrInvalid, "fbank window_type must be hamming (0) or povey (1)");
  if (!g_twiddle) {
    float2 h[kNfft / 2];
    for (int k = 0; k < kNfft / 2; ++k) {
      double ang = -2.0 * 3.14159265358979323846 * k / kNfft;
      h[k] = make_float2((float)cos(ang), (float)sin(ang));
    }
    SD_HIP(hipMalloc(&g_twiddle, sizeof(h)));
    SD_HIP(hipMemcpy(g_twiddle, h, sizeof(h), hipMemcpyHostToDevice));
  }
  if (n_frames <= 0) return;
  ProfScope prof("fbank_kaldi", 0.0, 4.0 * ((double)n_frames * kShift + (double)n_frames * n_mels), st);
  SD_CHECK(n_mels > 0 && n_mels <= kMaxFbMels, kErrInvalid, "fbank: n_mels out of range");
  // as many workgroups as are resident at once (each builds its tables once and walks frame groups)
  static int slots = 0;
  if (!slots) {
    int dev = 0, cus = 0, per_cu = 0;
    SD_HIP(hipGetDevice(&dev));
    SD_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    SD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fbank_kernel, 512, 0));
    slots = std::max(1, cus * std::max(1, per_cu));
  }
  const int groups = cdiv(n_frames, kFramesPerBlock);
  const dim3 grid(std::min(groups, slots));
  hipLaunchKernelGGL(fbank_kernel, grid, dim3(512), 0, st, wav, n_samples, in_scale, n_frames, mel_fb, n_mels,
                     g_twiddle, window, out);
  SD_LAUNCH_CHECK();
}

}  // namespace sd
