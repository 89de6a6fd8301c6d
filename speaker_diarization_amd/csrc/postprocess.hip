// Posteriors -> speech segments on the GPU (ts_vad2/infer.py:27-130).
//
// The recipe post-processes each (meeting, speaker) posterior track on the host:
// scipy.signal.medfilt(k) (zero-padded), then for each of 10 thresholds
// change_zeros_to_ones (silence runs <= min_silence//frame_len frames become
// speech, infer.py:27-47) and change_ones_to_zeros (speech runs <= min_speech
// frames become silence, 50-70), then one RTTM line per remaining speech run.
// Here:
//   medfilt_kernel      one thread per frame: the k-window median by rank
//                       selection from an LDS tile (the median is one of the
//                       inputs, so the result is exact);
//   run_segments_kernel one workgroup per (track, threshold): the binarised track
//                       lives as a bitmask in LDS, each run-length filter is a
//                       block-wide max/min scan of run boundaries, and the
//                       surviving runs are compacted with a sum scan into
//                       [begin, end) frame pairs.
// The host only formats the RTTM lines (start/duration quirks of infer.py).
// Comparison `x >= threshold` is done in float32, as numpy does for a float32
// element against a Python float (NEP 50).
#include "common.h"
#include "kernels.h"

namespace sd {

namespace {

constexpr int kMedMaxK = 63;
constexpr int kMedBlock = 256;
constexpr int kSegThreads = 256;

__global__ void __launch_bounds__(kMedBlock) medfilt_kernel(const float* __restrict__ x, int T, int k,
                                                            float* __restrict__ y) {
  __shared__ float tile[kMedBlock + kMedMaxK];
  const int row = blockIdx.y;
  const int t0 = blockIdx.x * kMedBlock;
  const int h = k / 2;
  const float* xr = x + (int64_t)row * T;
  for (int i = threadIdx.x; i < kMedBlock + k - 1; i += kMedBlock) {
    const int t = t0 - h + i;
    tile[i] = (t >= 0 && t < T) ? xr[t] : 0.f;
  }
  __syncthreads();
  const int t = t0 + threadIdx.x;
  if (t >= T) return;
  const float* w = tile + threadIdx.x;
  // Element j is the median iff #(< w[j]) + #(== w[j] before j) == h.
  float med = 0.f;
  for (int j = 0; j < k; ++j) {
    const float v = w[j];
    int rank = 0;
    for (int l = 0; l < k; ++l) {
      const float u = w[l];
      rank += (u < v) | ((u == v) & (l < j));
    }
    if (rank == h) med = v;
  }
  y[(int64_t)row * T + t] = med;
}

template <typename Op>
__device__ __forceinline__ int block_scan_excl(int v, Op op, int identity, int* sm, int& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(inc, o, 64);
    if (lane >= o) inc = op(inc, y);
  }
  if (lane == 63) sm[wid] = inc;
  __syncthreads();
  int pre = identity;
  for (int w = 0; w < wid; ++w) pre = op(pre, sm[w]);
  int tot = identity;
  for (int w = 0; w < kSegThreads / 64; ++w) tot = op(tot, sm[w]);
  int ex = __shfl_up(inc, 1, 64);
  if (lane == 0) ex = identity;
  __syncthreads();
  total = tot;
  return op(pre, ex);
}

__device__ __forceinline__ int bit_at(const uint32_t* m, int i) { return (m[i >> 5] >> (i & 31)) & 1; }

// One run-length filter pass over `in` (T frames) into `out`.
//   mode 0 (change_zeros_to_ones): 0-runs of length <= lim become 1;
//   mode 1 (change_ones_to_zeros): 1-runs of length <= lim become 0.
// Thread t owns words [t*wpt, (t+1)*wpt) i.e. frames [c0, c1).
__device__ void run_filter(const uint32_t* in, uint32_t* out, int T, int lim, int mode, int wpt, int* sm) {
  const int W = (T + 31) >> 5;
  const int w0 = min(W, (int)threadIdx.x * wpt), w1 = min(W, w0 + wpt);
  const int c0 = w0 * 32, c1 = min(T, w1 * 32);
  // Run starts s (s == 0 or bit(s) != bit(s-1)) and run ends e (e == T or
  // bit(e) != bit(e-1)); a thread owns starts in [c0, c1) and ends in (c0, c1].
  int last_start = -1, first_end = 0x7fffffff;
  for (int i = c0; i < c1; ++i)
    if (i == 0 || bit_at(in, i) != bit_at(in, i - 1)) last_start = i;
  for (int e = c1; e > c0; --e)
    if (e == T || bit_at(in, e) != bit_at(in, e - 1)) first_end = e;
  int tot;
  const int start_in = block_scan_excl(last_start, [](int a, int b) { return max(a, b); }, -1, sm, tot);
  // Reverse exclusive min-scan: thread t needs min over threads > t.
  __shared__ int rev[kSegThreads];
  rev[kSegThreads - 1 - threadIdx.x] = first_end;
  __syncthreads();
  const int r = rev[threadIdx.x];
  __syncthreads();
  const int end_r = block_scan_excl(r, [](int a, int b) { return min(a, b); }, 0x7fffffff, sm, tot);
  rev[kSegThreads - 1 - threadIdx.x] = end_r;
  __syncthreads();
  const int end_in = rev[threadIdx.x];
  __syncthreads();
  if (c0 >= c1) return;
  int i = c0;
  int s = (c0 == 0 || bit_at(in, c0) != bit_at(in, c0 - 1)) ? c0 : start_in;
  uint32_t word = 0;
  int wi = w0;
  while (i < c1) {
    const int v = bit_at(in, i);
    int j = i + 1;
    while (j < c1 && bit_at(in, j) == v) ++j;
    const int e = (j < c1 || j == T || bit_at(in, j) != v) ? j : end_in;
    const int len = e - s;
    const int o = mode == 0 ? (v | (len <= lim)) : (v & (len > lim));
    for (int f = i; f < j; ++f) {
      if ((f >> 5) != wi) {
        out[wi] = word;
        word = 0;
        wi = f >> 5;
      }
      word |= (uint32_t)o << (f & 31);
    }
    i = j;
    s = j;
  }
  out[wi] = word;
  for (int w = wi + 1; w < w1; ++w) out[w] = 0;
}

__global__ void __launch_bounds__(kSegThreads)
run_segments_kernel(const float* __restrict__ med, int T, ThresholdSet thr, int lim_sil, int lim_sp, int cap,
                    int* __restrict__ seg_begin, int* __restrict__ seg_end, int* __restrict__ n_seg) {
  extern __shared__ uint32_t bits[];
  __shared__ int sm[kSegThreads / 64];
  const int W = (T + 31) >> 5;
  uint32_t* A = bits;
  uint32_t* B = bits + W;
  const int row = blockIdx.x / thr.n, ti = blockIdx.x % thr.n;
  const float th = thr.v[ti];
  const float* m = med + (int64_t)row * T;
  // Binarise: one coalesced 64-frame load + ballot per wave iteration.
  const int lane = threadIdx.x & 63;
  for (int f0 = (threadIdx.x >> 6) * 64; f0 < T; f0 += kSegThreads) {
    const bool p = f0 + lane < T && (thr.strict ? m[f0 + lane] > th : m[f0 + lane] >= th);
    const uint64_t b = __ballot(p);
    if (lane == 0) {
      A[f0 >> 5] = (uint32_t)b;
      if ((f0 >> 5) + 1 < W) A[(f0 >> 5) + 1] = (uint32_t)(b >> 32);
    }
  }
  __syncthreads();
  const int wpt = (W + kSegThreads - 1) / kSegThreads;
  run_filter(A, B, T, lim_sil, 0, wpt, sm);
  __syncthreads();
  run_filter(B, A, T, lim_sp, 1, wpt, sm);
  __syncthreads();
  // Compact the surviving 1-runs.
  const int w0 = min(W, (int)threadIdx.x * wpt), w1 = min(W, w0 + wpt);
  const int c0 = w0 * 32, c1 = min(T, w1 * 32);
  int nb = 0, ne = 0;
  for (int i = c0; i < c1; ++i) nb += bit_at(A, i) && (i == 0 || !bit_at(A, i - 1));
  for (int e = c0 + 1; e <= c1; ++e) ne += bit_at(A, e - 1) && (e == T || !bit_at(A, e));
  int total_b, total_e;
  auto add = [](int a, int b) { return a + b; };
  int ob = block_scan_excl(nb, add, 0, sm, total_b);
  int oe = block_scan_excl(ne, add, 0, sm, total_e);
  const int64_t base = (int64_t)blockIdx.x * cap;
  for (int i = c0; i < c1; ++i)
    if (bit_at(A, i) && (i == 0 || !bit_at(A, i - 1))) {
      if (ob < cap) seg_begin[base + ob] = i;
      ++ob;
    }
  for (int e = c0 + 1; e <= c1; ++e)
    if (bit_at(A, e - 1) && (e == T || !bit_at(A, e))) {
      if (oe < cap) seg_end[base + oe] = e;
      ++oe;
    }
  if (threadIdx.x == 0) n_seg[blockIdx.x] = total_b;
}

}  // namespace

int segments_max_frames() { return 32 * 16384; }   // two 64 KB bitmasks in LDS (5.8 h at 25 Hz)

void medfilt(const float* x, int rows, int T, int k, float* y, hipStream_t st) {
  SD_CHECK(k >= 1 && k <= kMedMaxK && (k & 1), kErrInvalid, "medfilt: kernel size must be odd and <= 63");
  if (rows == 0 || T == 0) return;
  hipLaunchKernelGGL(medfilt_kernel, dim3(cdiv(T, kMedBlock), rows), dim3(kMedBlock), 0, st, x, T, k, y);
  SD_LAUNCH_CHECK();
}

void run_segments(const float* med, int rows, int T, const ThresholdSet& thr, int lim_sil, int lim_sp, int cap,
                  int* seg_begin, int* seg_end, int* n_seg, hipStream_t st) {
  SD_CHECK(thr.n >= 1 && thr.n <= ThresholdSet::kMax, kErrInvalid, "run_segments: 1..16 thresholds");
  SD_CHECK(T <= segments_max_frames(), kErrInvalid, "run_segments: track longer than the LDS bitmask");
  SD_CHECK(cap >= (T + 1) / 2, kErrInvalid, "run_segments: cap < (T+1)/2");
  if (rows == 0 || T == 0) return;
  const int W = (T + 31) / 32;
  const size_t lds = 2 * (size_t)W * sizeof(uint32_t);
  static bool attr = false;
  if (!attr) {
    SD_HIP(hipFuncSetAttribute((const void*)run_segments_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               160 * 1024 - 4096));
    attr = true;
  }
  hipLaunchKernelGGL(run_segments_kernel, dim3(rows * thr.n), dim3(kSegThreads), lds, st, med, T, thr, lim_sil,
                     lim_sp, cap, seg_begin, seg_end, n_seg);
  SD_LAUNCH_CHECK();
}

}  // namespace sd
