// LSTM recurrence (torch.nn.LSTM gate order i, f, g, o) for gfx950.
//
// The input projection W_ih·x_t + b_ih + b_hh for every step is one big
// conv_gemm launched beforehand; this file only runs the sequential part.
// One launch per time step covers both directions: workgroup (u-block, dir,
// b-block) owns 8 hidden units = 32 gate rows of W_hh, stages them and
// h_{t-1} in LDS and computes the 64x32 gate tile with exact-f32 MFMA, then
// updates c/h for its units.  Sequence lengths follow pack_padded_sequence
// semantics (encoder_decoder_attractor.py:45-49): the reverse direction starts
// at len-1 and states freeze after a sequence ends.
// Serves ts_vad2/model.py:360-366,752 (BiLSTM) and eend_eda EDA LSTMs.
#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {
namespace {

constexpr int kUB = 8;       // hidden units per workgroup
constexpr int kRows = 4 * kUB;
constexpr int kBB = 64;      // batch rows per workgroup

__global__ __launch_bounds__(256) void lstm_step_kernel(
    const float* __restrict__ gx, int B, int T, int H, int ndir, const float* __restrict__ whh,
    const int* __restrict__ lengths, const float* __restrict__ h_in, float* __restrict__ h_out,
    float* __restrict__ c_state, float* __restrict__ out, int ldo, int step) {
  extern __shared__ float sm[];
  const int HS = H + 4;                  // padded stride (== 4 mod 32 for H % 32 == 0)
  float* hs = sm;                        // [kBB][HS]
  float* ws = hs + kBB * HS;             // [kRows][HS]
  float* zs = ws + kRows * HS;           // [kBB][kRows + 1]
  const int u0 = blockIdx.x * kUB;
  const int d = blockIdx.y;
  const int b0 = blockIdx.z * kBB;
  const int nb = min(kBB, B - b0);
  const int tid = threadIdx.x;
  const float* hprev = h_in + ((int64_t)d * B + b0) * H;
  const float* wd = whh + (int64_t)d * 4 * H * H;

  for (int i = tid; i < kBB * (H / 4); i += 256) {
    int b = i / (H / 4), k4 = (i % (H / 4)) * 4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (b < nb) v = *reinterpret_cast<const float4*>(hprev + (int64_t)b * H + k4);
    float* dst = hs + b * HS + k4;
    dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
  }
  for (int i = tid; i < kRows * (H / 4); i += 256) {
    int r = i / (H / 4), k4 = (i % (H / 4)) * 4;
    int gate = r / kUB, u = r % kUB;
    float4 v = *reinterpret_cast<const float4*>(wd + ((int64_t)gate * H + u0 + u) * H + k4);
    float* dst = ws + r * HS + k4;
    dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
  }
  __syncthreads();

  // 4 waves x (16 batch rows) x (32 gate rows = 2 subtiles).
  const int lane = tid & 63, wid = tid >> 6;
  const int l15 = lane & 15, g = lane >> 4;
  floatx4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  for (int kk = 0; kk < H / 4; ++kk) {
    float a = hs[(wid * 16 + l15) * HS + kk * 4 + g];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      float bw = ws[(nt * 16 + l15) * HS + kk * 4 + g];
      acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bw, acc[nt], 0, 0, 0);
    }
  }
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) zs[(wid * 16 + g * 4 + r) * (kRows + 1) + nt * 16 + l15] = acc[nt][r];
  __syncthreads();

  for (int i = tid; i < nb * kUB; i += 256) {
    const int b = i / kUB, u = i % kUB;
    const int gb = b0 + b;
    const int len = lengths ? lengths[gb] : T;
    const int64_t hidx = ((int64_t)d * B + gb) * H + u0 + u;
    if (step >= len) {
      h_out[hidx] = h_in[hidx];
      continue;
    }
    const int t = d == 0 ? step : len - 1 - step;
    const float* gr = gx + ((int64_t)gb * T + t) * (ndir * 4 * H) + d * 4 * H + u0 + u;
    const float* zr = zs + b * (kRows + 1) + u;
    float zi = zr[0 * kUB] + gr[0 * H];
    float zf = zr[1 * kUB] + gr[1 * H];
    float zg = zr[2 * kUB] + gr[2 * H];
    float zo = zr[3 * kUB] + gr[3 * H];
    float ig = 1.f / (1.f + expf(-zi));
    float fg = 1.f / (1.f + expf(-zf));
    float gg = tanhf(zg);
    float og = 1.f / (1.f + expf(-zo));
    float c = fg * c_state[hidx] + ig * gg;
    float hv = og * tanhf(c);
    c_state[hidx] = c;
    h_out[hidx] = hv;
    if (out) out[((int64_t)gb * T + t) * ldo + d * H + u0 + u] = hv;
  }
}

// bf16 variant: 32 hidden units (128 gate rows) x 64 batch rows per workgroup, so the
// h tile is re-read by 4x fewer workgroups and both operands move as bf16: W slice
// 128 x H and h 64 x H staged with 16-B loads, v_mfma_f32_16x16x32_bf16, each wave
// owns 16 batch rows x 128 gate rows (8 accumulators).
constexpr int kUB2 = 32;
constexpr int kRows2 = 4 * kUB2;

__global__ __launch_bounds__(256) void lstm_step_bf16_kernel(
    const float* __restrict__ gx, int B, int T, int H, int ndir, const uint16_t* __restrict__ whh,
    const int* __restrict__ lengths, const float* __restrict__ h_in, float* __restrict__ h_out,
    float* __restrict__ c_state, float* __restrict__ out, int ldo, int step) {
  extern __shared__ __attribute__((aligned(16))) uint16_t sm2[];
  const int HS = H + 8;                         // bf16 row stride (16-B aligned, conflict-spread)
  uint16_t* hs = sm2;                           // [kBB][HS]
  uint16_t* ws = hs + kBB * HS;                 // [kRows2][HS]
  float* zs = reinterpret_cast<float*>(ws + kRows2 * HS);   // [kBB][kRows2 + 1]
  const int u0 = blockIdx.x * kUB2;
  const int d = blockIdx.y;
  const int b0 = blockIdx.z * kBB;
  const int nb = min(kBB, B - b0);
  const int tid = threadIdx.x;
  const float* hprev = h_in + ((int64_t)d * B + b0) * H;
  const uint16_t* wd = whh + (int64_t)d * 4 * H * H;
  const int H8 = H / 8;
  for (int i = tid; i < kBB * H8; i += 256) {
    const int b = i / H8, k8 = (i % H8) * 8;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (b < nb) {
      const float4 x0 = *reinterpret_cast<const float4*>(hprev + (int64_t)b * H + k8);
      const float4 x1 = *reinterpret_cast<const float4*>(hprev + (int64_t)b * H + k8 + 4);
      v.x = (uint32_t)f2bf_bits(x0.x) | ((uint32_t)f2bf_bits(x0.y) << 16);
      v.y = (uint32_t)f2bf_bits(x0.z) | ((uint32_t)f2bf_bits(x0.w) << 16);
      v.z = (uint32_t)f2bf_bits(x1.x) | ((uint32_t)f2bf_bits(x1.y) << 16);
      v.w = (uint32_t)f2bf_bits(x1.z) | ((uint32_t)f2bf_bits(x1.w) << 16);
    }
    *reinterpret_cast<uint4*>(hs + b * HS + k8) = v;
  }
  for (int i = tid; i < kRows2 * H8; i += 256) {
    const int r = i / H8, k8 = (i % H8) * 8;
    const int gate = r / kUB2, u = r % kUB2;
    *reinterpret_cast<uint4*>(ws + r * HS + k8) =
        *reinterpret_cast<const uint4*>(wd + ((int64_t)gate * H + u0 + u) * H + k8);
  }
  __syncthreads();
  const int lane = tid & 63, wid = tid >> 6;
  const int l15 = lane & 15, g = lane >> 4;
  floatx4 acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < H; k0 += 32) {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(hs + (wid * 16 + l15) * HS + k0 + g * 8);
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      const bf16x8 bw = *reinterpret_cast<const bf16x8*>(ws + (nt * 16 + l15) * HS + k0 + g * 8);
      acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw, acc[nt], 0, 0, 0);
    }
  }
#pragma unroll
  for (int nt = 0; nt < 8; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) zs[(wid * 16 + g * 4 + r) * (kRows2 + 1) + nt * 16 + l15] = acc[nt][r];
  __syncthreads();
  for (int i = tid; i < nb * kUB2; i += 256) {
    const int b = i / kUB2, u = i % kUB2;
    const int gb = b0 + b;
    const int len = lengths ? lengths[gb] : T;
    const int64_t hidx = ((int64_t)d * B + gb) * H + u0 + u;
    if (step >= len) {
      h_out[hidx] = h_in[hidx];
      continue;
    }
    const int t = d == 0 ? step : len - 1 - step;
    const float* gr = gx + ((int64_t)gb * T + t) * (ndir * 4 * H) + d * 4 * H + u0 + u;
    const float* zr = zs + b * (kRows2 + 1) + u;
    const float zi = zr[0 * kUB2] + gr[0 * H];
    const float zf = zr[1 * kUB2] + gr[1 * H];
    const float zg = zr[2 * kUB2] + gr[2 * H];
    const float zo = zr[3 * kUB2] + gr[3 * H];
    const float ig = 1.f / (1.f + expf(-zi));
    const float fg = 1.f / (1.f + expf(-zf));
    const float gg = tanhf(zg);
    const float og = 1.f / (1.f + expf(-zo));
    const float c = fg * c_state[hidx] + ig * gg;
    const float hv = og * tanhf(c);
    c_state[hidx] = c;
    h_out[hidx] = hv;
    if (out) out[((int64_t)gb * T + t) * ldo + d * H + u0 + u] = hv;
  }
}

}  // namespace

void lstm_recurrence(const float* gx, int B, int T, int H, int ndir, const float* whh,
                     const int* lengths, const float* h0, const float* c0, float* out, int ldo,
                     float* hT, float* cT, float* work, hipStream_t st, const void* whh_bf16) {
  SD_CHECK(H % 32 == 0, kErrInvalid, "lstm: H must be a multiple of 32");
  const int64_t n = (int64_t)ndir * B * H;
  float* hA = work;
  float* hB = work + n;
  float* c = work + 2 * n;
  if (h0) SD_HIP(hipMemcpyAsync(hA, h0, n * 4, hipMemcpyDeviceToDevice, st));
  else SD_HIP(hipMemsetAsync(hA, 0, n * 4, st));
  if (c0) SD_HIP(hipMemcpyAsync(c, c0, n * 4, hipMemcpyDeviceToDevice, st));
  else SD_HIP(hipMemsetAsync(c, 0, n * 4, st));
  const size_t smem = sizeof(float) * ((kBB + kRows) * (H + 4) + kBB * (kRows + 1));
  static bool attr_set = false;
  if (!attr_set) {
    SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(lstm_step_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  ProfScope prof("lstm_recurrence", 2.0 * ndir * B * T * 4.0 * H * H,
                 4.0 * ((double)B * T * ndir * 4 * H + (double)T * ndir * 4 * H * H), st);
  if (whh_bf16 && H % kUB2 == 0) {
    const size_t smem2 = sizeof(uint16_t) * (size_t)(kBB + kRows2) * (H + 8) + sizeof(float) * kBB * (kRows2 + 1);
    SD_CHECK(smem2 <= 160 * 1024, kErrInvalid, "lstm: hidden size too large for the bf16 step kernel");
    static bool attr2 = false;
    if (!attr2) {
      SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(lstm_step_bf16_kernel),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      attr2 = true;
    }
    dim3 grid2(H / kUB2, ndir, cdiv(B, kBB));
    for (int s = 0; s < T; ++s) {
      const float* hin = (s & 1) ? hB : hA;
      float* hout = (s & 1) ? hA : hB;
      hipLaunchKernelGGL(lstm_step_bf16_kernel, grid2, dim3(256), smem2, st, gx, B, T, H, ndir,
                         reinterpret_cast<const uint16_t*>(whh_bf16), lengths, hin, hout, c, out, ldo, s);
    }
    SD_LAUNCH_CHECK();
    const float* hfin = (T & 1) ? hB : hA;
    if (hT) SD_HIP(hipMemcpyAsync(hT, hfin, n * 4, hipMemcpyDeviceToDevice, st));
    if (cT) SD_HIP(hipMemcpyAsync(cT, c, n * 4, hipMemcpyDeviceToDevice, st));
    return;
  }
  dim3 grid(H / kUB, ndir, cdiv(B, kBB));
  for (int s = 0; s < T; ++s) {
    const float* hin = (s & 1) ? hB : hA;
    float* hout = (s & 1) ? hA : hB;
    hipLaunchKernelGGL(lstm_step_kernel, grid, dim3(256), smem, st, gx, B, T, H, ndir, whh, lengths,
                       hin, hout, c, out, ldo, s);
  }
  SD_LAUNCH_CHECK();
  const float* hfin = (T & 1) ? hB : hA;
  if (hT) SD_HIP(hipMemcpyAsync(hT, hfin, n * 4, hipMemcpyDeviceToDevice, st));
  if (cT) SD_HIP(hipMemcpyAsync(cT, c, n * 4, hipMemcpyDeviceToDevice, st));
}

}  // namespace sd
