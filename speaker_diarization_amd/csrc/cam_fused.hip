// CAM++ dense layer tail, fused: CAMLayer context gate + linear_local conv + gating
// (egs/alimeeting/ts_vad2/cam_pplus_wespeaker.py:106-123, CAMDenseTDNNLayer 158-167).
//
//   y[t, n]   = sum_{tap, c} W[n][tap][c] * x[t + (tap - 1) * dil, c]  (+ bias[n])
//   ctx[s, c] = mean_t x[t, c] + mean_{t in segment s} x[t, c]           (seg_len 100)
//   gate[s,:] = sigmoid(W2 relu(W1 ctx[s] + b1) + b2)
//   out[t, n] = y[t, n] * gate[t / 100, n]
//
// x is the bottleneck output (128 channels, bf16) of one item.  The unfused path ran a
// context kernel (reading x) and then the N = 32 implicit-GEMM conv (reading x again, a
// skinny GEMM the tiled kernels serve poorly); here one workgroup per (item, segment)
// streams the item's rows once for the whole-sequence sum, keeps its own segment's rows
// (+ dil halo rows each side) in LDS while doing so, evaluates the gate, and runs the
// conv for its <= 100 output rows on MFMA from LDS (transposed: 4 consecutive output
// channels per lane -> 8-B stores into the dense block's channel slice).
#include <algorithm>

#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {
namespace {

constexpr int kC = 128, kC1 = 64, kC2 = 32;   // bn_channels, reduction 2, growth rate
constexpr int kSeg = 100;
constexpr int kMaxDil = 2;
constexpr int kRows = kSeg + 2 * kMaxDil;     // staged rows per segment
constexpr int kL = kC / 4;                    // lanes per row (4 channels = 8 B each)
constexpr int kP = 256 / kL;                  // rows in flight per pass

// Staged rows are 256 B (the full bank row): the conv's fragment reads take 16 rows at one
// channel offset, so 16-B chunk q of row r is stored at q ^ (r & 15) (conflict-free reads).
__device__ __forceinline__ int xs_off(int r, int c) { return r * kC + ((((c >> 3) ^ (r & 15)) << 3) | (c & 7)); }

// FUSED: the workgroup computes its segment's gate (whole-sequence + segment means, MLP);
// otherwise the gate comes from cam_context()'s buffer and only the window rows are read.
template <bool FUSED>
__global__ __launch_bounds__(256) void cam_local_fused_kernel(
    const uint16_t* __restrict__ x, int T, int dil, const uint16_t* __restrict__ wt /*[32][3*128] bf16*/,
    const float* __restrict__ bias, const float* __restrict__ w1, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ b2, const float* __restrict__ gate_in,
    uint16_t* __restrict__ out, int ldo, int nseg, int ntask) {
  __shared__ __attribute__((aligned(16))) uint16_t xs[kRows * kC];   // rows s0 - dil .. s0 + 100 + dil
  __shared__ float4 red_t[kP][kL];
  __shared__ float4 red_s[kP][kL];
  __shared__ float ctx[kC];
  __shared__ float h1[kC1];
  __shared__ float gate[kC2];
  const int tid = threadIdx.x;
  const int part = tid / kL, l = tid % kL;
  // The conv's weight fragments (rows n = nt*16 + l15, k = kk*32 + lk*8; L2-resident) are
  // requested first so their latency hides behind the row pass, and kept for every task of this
  // persistent workgroup (they are as many bytes as a task's rows: one load per task doubled the
  // L2 -> CU traffic).
  const int lane = tid & 63, wv = tid >> 6;
  const int l15 = lane & 15, lk = lane >> 4;
  bf16x8 wf[2][12];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int kk = 0; kk < 12; ++kk)
      wf[nt][kk] = *reinterpret_cast<const bf16x8*>(wt + (nt * 16 + l15) * (3 * kC) + kk * 32 + lk * 8);
  for (int task = blockIdx.x; task < ntask; task += gridDim.x) {
  if (task != (int)blockIdx.x) __syncthreads();   // the previous task's LDS reads are done
  const int lid = xcd_remap(task, ntask);        // the nseg tasks of an item share an XCD
  const int b = lid / nseg, s = lid - b * nseg;
  const int t0 = s * kSeg, t1 = min(T, t0 + kSeg);
  const int r_lo = t0 - dil, r_hi = t1 + dil;          // staged window [r_lo, r_hi)
  const uint16_t* xb = x + (int64_t)b * T * kC;

  if constexpr (!FUSED) {
    // Only the window rows: every 16-B chunk of them requested at once (one HBM round trip per task,
    // the row pass below keeps four in flight per lane), halo rows outside [0, T) zero-filled.
    constexpr int CH = kC / 8;                        // 16-B chunks per row
    constexpr int NL = (kRows * CH + 255) / 256;      // chunks per thread
    const int nr = r_hi - r_lo;
    uint4 v[NL];
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = tid + 256 * i, r = c / CH, q = c - r * CH;
      const int t = r_lo + r;
      v[i] = make_uint4(0u, 0u, 0u, 0u);
      if (r < nr && t >= 0 && t < T) v[i] = *reinterpret_cast<const uint4*>(xb + (int64_t)t * kC + q * 8);
    }
    if (tid < kC2) gate[tid] = gate_in[((int64_t)b * nseg + s) * kC2 + tid];
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = tid + 256 * i, r = c / CH, q = c - r * CH;
      if (r < nr) *reinterpret_cast<uint4*>(xs + xs_off(r, q * 8)) = v[i];
    }
    __syncthreads();
  } else {
  // ---- pass over all rows: whole-sequence sum, segment sum, stage the window rows
  float4 at = make_float4(0.f, 0.f, 0.f, 0.f), as = at;
  auto take = [&](int t, const uint2& u) {
    const float4 v = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                                 __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
    at.x += v.x; at.y += v.y; at.z += v.z; at.w += v.w;
    if (t >= t0 && t < t1) { as.x += v.x; as.y += v.y; as.z += v.z; as.w += v.w; }
    if (t >= r_lo && t < r_hi) *reinterpret_cast<uint2*>(xs + xs_off(t - r_lo, 4 * l)) = u;
  };
  auto row = [&](int t) { return *reinterpret_cast<const uint2*>(xb + (int64_t)t * kC + 4 * l); };
  const int p_lo = FUSED ? 0 : max(r_lo, 0), p_hi = FUSED ? T : min(r_hi, T);
  int t = p_lo + part;
  for (; t + 3 * kP < p_hi; t += 4 * kP) {     // four rows in flight per lane
    const uint2 u0 = row(t), u1 = row(t + kP), u2 = row(t + 2 * kP), u3 = row(t + 3 * kP);
    take(t, u0); take(t + kP, u1); take(t + 2 * kP, u2); take(t + 3 * kP, u3);
  }
  for (; t < p_hi; t += kP) take(t, row(t));
  // zero halo rows outside [0, T) (the conv's zero padding)
  for (int r = part; r < r_hi - r_lo; r += kP) {
    const int t = r_lo + r;
    if (t < 0 || t >= T) *reinterpret_cast<uint2*>(xs + xs_off(r, 4 * l)) = make_uint2(0u, 0u);
  }
  {
  red_t[part][l] = at;
  red_s[part][l] = as;
  __syncthreads();
  if (tid < kC) {
    const int ll = tid / 4, k = tid % 4;
    float tt = 0.f, ss = 0.f;
#pragma unroll
    for (int q = 0; q < kP; ++q) {
      tt += reinterpret_cast<const float*>(&red_t[q][ll])[k];
      ss += reinterpret_cast<const float*>(&red_s[q][ll])[k];
    }
    ctx[tid] = tt / (float)T + ss / (float)(t1 - t0);
  }
  __syncthreads();
  {   // h1 = relu(W1 ctx + b1): 4 threads per output
    const int j = tid / 4, q = tid % 4;
    const float* wr = w1 + j * kC + q * 32;
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) a = fmaf(wr[k], ctx[q * 32 + k], a);
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    if (q == 0) h1[j] = fmaxf(a + b1[j], 0.f);
  }
  __syncthreads();
  {   // gate = sigmoid(W2 h1 + b2): 8 threads per output
    const int j = tid / 8, q = tid % 8;
    const float* wr = w2 + j * kC1 + q * 8;
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) a = fmaf(wr[k], h1[q * 8 + k], a);
    a += __shfl_xor(a, 1, 64);
    a += __shfl_xor(a, 2, 64);
    a += __shfl_xor(a, 4, 64);
    if (q == 0) gate[j] = 1.f / (1.f + expf(-(a + b2[j])));
  }
  __syncthreads();
  }
  }   // FUSED

  // ---- conv rows t0..t1-1 on MFMA: C'[n][t] = sum_k W[n][k] X[t][k], k = tap*128 + c
  const int nrows = t1 - t0;
  const int n_rt = (nrows + 15) / 16;
  float g4[2][4], bb4[2][4];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = nt * 16 + lk * 4 + r;
      g4[nt][r] = gate[n];
      bb4[nt][r] = bias ? bias[n] : 0.f;
    }
  uint16_t* ob = out + (int64_t)b * T * ldo;
  for (int rt = wv; rt < n_rt; rt += 4) {
    const int tr = rt * 16 + l15;                  // this lane's output row (segment-local)
    floatx4 acc[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int kk = 0; kk < 12; ++kk) {
      const int tap = kk >> 2, c = (kk & 3) * 32 + lk * 8;
      const int r = tr + dil + (tap - 1) * dil;    // staged row (window starts at t0 - dil)
      bf16x8 xf;
      if (tr < nrows) xf = *reinterpret_cast<const bf16x8*>(xs + xs_off(r, c));
      else xf = bf16x8{};
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[nt][kk], xf, acc[nt], 0, 0, 0);
    }
    if (tr < nrows) {
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = (acc[nt][r] + bb4[nt][r]) * g4[nt][r];
        *reinterpret_cast<uint2*>(ob + (int64_t)(t0 + tr) * ldo + nt * 16 + lk * 4) =
            make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
      }
    }
  }
  }   // task
}

// Persistent grid: tasks (item, segment) are dealt to at most kCamWgPerCu workgroups per CU.
constexpr int kCamWgPerCu = 4;
dim3 cam_grid(int B, int nseg) {
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    SD_HIP(hipGetDevice(&dev));
    SD_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  return dim3((unsigned)std::min(B * nseg, kCamWgPerCu * n_cu));
}

}  // namespace

bool cam_local_fused_supported(int C, int C1, int C2, int N, int taps, int dil, int seg_len, int ldo,
                               bool bf16) {
  return bf16 && C == kC && C1 == kC1 && C2 == kC2 && N == kC2 && taps == 3 && dil >= 1 && dil <= kMaxDil &&
         seg_len == kSeg && ldo % 4 == 0;
}

void cam_local_fused(const void* x, int B, int T, int dil, const void* wt, const float* bias, const float* w1,
                     const float* b1, const float* w2, const float* b2, void* out, int ldo, hipStream_t st) {
  SD_CHECK(T >= 1 && B >= 1, kErrInvalid, "cam_local_fused: empty input");
  SD_CHECK((reinterpret_cast<uintptr_t>(out) & 7) == 0, kErrInvalid, "cam_local_fused: output must be 8-B aligned");
  const int nseg = cdiv(T, kSeg);
  ProfScope prof("cam_local_fused", 2.0 * B * T * kC2 * 3 * kC + 2.0 * B * nseg * (kC * kC1 + kC1 * kC2),
                 2.0 * B * T * (kC + kC2), st);
  hipLaunchKernelGGL(cam_local_fused_kernel<true>, cam_grid(B, nseg), dim3(256), 0, st, static_cast<const uint16_t*>(x),
                     T, dil, static_cast<const uint16_t*>(wt), bias, w1, b1, w2, b2, nullptr,
                     static_cast<uint16_t*>(out), ldo, nseg, B * nseg);
  SD_LAUNCH_CHECK();
}

void cam_local_conv(const void* x, int B, int T, int dil, const void* wt, const float* bias, const float* gate,
                    void* out, int ldo, hipStream_t st) {
  SD_CHECK(T >= 1 && B >= 1, kErrInvalid, "cam_local_conv: empty input");
  SD_CHECK((reinterpret_cast<uintptr_t>(out) & 7) == 0, kErrInvalid, "cam_local_conv: output must be 8-B aligned");
  const int nseg = cdiv(T, kSeg);
  ProfScope prof("cam_local_conv", 2.0 * B * T * kC2 * 3 * kC, 2.0 * B * T * (kC + kC2), st);
  hipLaunchKernelGGL(cam_local_fused_kernel<false>, cam_grid(B, nseg), dim3(256), 0, st,
                     static_cast<const uint16_t*>(x), T, dil, static_cast<const uint16_t*>(wt), bias, nullptr, nullptr,
                     nullptr, nullptr, gate, static_cast<uint16_t*>(out), ldo, nseg, B * nseg);
  SD_LAUNCH_CHECK();
}

}  // namespace sd
