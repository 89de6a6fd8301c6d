// SSND speaker-query decoder kernels (egs/alimeeting/ssnd/ssnd_model.py:198-370) for gfx950.
//
//   mha_small            nn.MultiheadAttention core (softmax(q kᵀ / sqrt(hd)) v per head) for the
//                        decoders' cross attention (N speaker queries over T frames, :261) and
//                        self attention (N over N, :265): q, k, v are separate row sets (the
//                        cross attention's K and V come from different tensors), fp32.
//   tile_rows            learnable query / position tables expanded over the batch (:764-767)
//   mean_sigmoid_affine  RepresentationDecoder's pooled auxiliary query:
//                        Linear(1 -> d)(mean_t sigmoid(vad_pred)) (:361-363, :773)
//
// The decoder's work is tiny (N <= 32 queries per block), so these kernels are latency-shaped:
// one wave per (block, head, query), keys spread over the 64 lanes, the query held in SGPRs
// (readlane), online softmax across key chunks, the probability of each key broadcast by
// readlane into the lane-per-feature output accumulation.
#include <algorithm>

#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {
namespace {

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int HDL>   // feature slots per lane: hd <= 64 * HDL
__global__ __launch_bounds__(256) void mha_small_kernel(MhaSmallArgs a) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int bh = blockIdx.x;
  const int b = bh / a.nh, h = bh % a.nh;
  const int i = blockIdx.y * 4 + w;
  if (i >= a.Nq) return;   // waves are independent: no block barrier below
  const int hd = a.hd;
  const float* qr = a.q + (int64_t)b * a.q_bs + (int64_t)i * a.ldq + h * hd;
  float qv[HDL];
#pragma unroll
  for (int u = 0; u < HDL; ++u) qv[u] = (lane + 64 * u < hd) ? qr[lane + 64 * u] * a.scale : 0.f;
  const float* kb = a.k + (int64_t)b * a.k_bs + h * hd;
  const float* vb = a.v + (int64_t)b * a.v_bs + h * hd;
  const int Tk = a.key_len ? min(a.key_len[b], a.Tk) : a.Tk;
  float o[HDL];
#pragma unroll
  for (int u = 0; u < HDL; ++u) o[u] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;
  for (int k0 = 0; k0 < Tk; k0 += 64) {
    const int key = k0 + lane;
    const bool valid = key < Tk;
    const float* kr = kb + (int64_t)(valid ? key : k0) * a.ldk;
    float s = 0.f;
    for (int d0 = 0; d0 < hd; d0 += 4) {
      const float4 kk = *reinterpret_cast<const float4*>(kr + d0);
      // the query feature d is wave-uniform: readlane from the lane that holds it
      const int u = d0 >> 6, l0 = d0 & 63;
      const float q0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qv[u]), l0));
      const float q1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qv[u]), l0 + 1));
      const float q2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qv[u]), l0 + 2));
      const float q3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qv[u]), l0 + 3));
      s = fmaf(q0, kk.x, s);
      s = fmaf(q1, kk.y, s);
      s = fmaf(q2, kk.z, s);
      s = fmaf(q3, kk.w, s);
    }
    s = valid ? s : -INFINITY;
    const float m_new = fmaxf(m_run, wave_max(s));
    const float corr = (m_run == -INFINITY) ? 0.f : __expf(m_run - m_new);
    const float p = valid ? __expf(s - m_new) : 0.f;
    l_run = l_run * corr + wave_sum(p);
    m_run = m_new;
#pragma unroll
    for (int u = 0; u < HDL; ++u) o[u] *= corr;
    const int nk = min(64, Tk - k0);
    for (int jj = 0; jj < nk; ++jj) {
      const float pj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), jj));
      const float* vr = vb + (int64_t)(k0 + jj) * a.ldv;
#pragma unroll
      for (int u = 0; u < HDL; ++u)
        if (lane + 64 * u < hd) o[u] = fmaf(pj, vr[lane + 64 * u], o[u]);
    }
  }
  const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
  float* orow = a.o + (int64_t)b * a.o_bs + (int64_t)i * a.ldo + h * hd;
#pragma unroll
  for (int u = 0; u < HDL; ++u)
    if (lane + 64 * u < hd) orow[lane + 64 * u] = o[u] * inv;
}

__global__ void tile_rows_kernel(const float* __restrict__ src, int src_rows, int D, float* __restrict__ dst,
                                 int64_t n) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / D;
    const int d = (int)(e % D);
    dst[e] = src[(r % src_rows) * D + d];
  }
}

__global__ __launch_bounds__(256) void mean_sigmoid_affine_kernel(const float* __restrict__ x, int rows, int T,
                                                                  int ldx, const float* __restrict__ w,
                                                                  const float* __restrict__ bias, int N,
                                                                  float* __restrict__ out, int ldo) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  float s = 0.f;
  for (int t = lane; t < T; t += 64) s += 1.f / (1.f + expf(-x[(int64_t)r * ldx + t]));
  const float m = wave_sum(s) / (float)T;
  for (int j = lane; j < N; j += 64) out[(int64_t)r * ldo + j] = fmaf(m, w[j], bias[j]);
}

}  // namespace

void mha_small(const MhaSmallArgs& a, hipStream_t st) {
  SD_CHECK(a.hd > 0 && a.hd % 4 == 0 && a.hd <= 128, kErrInvalid, "mha_small: head dim must be 4..128, % 4");
  SD_CHECK(a.ldk % 4 == 0 && a.k_bs % 4 == 0, kErrInvalid, "mha_small: key rows must be 16-B aligned");
  if (a.B <= 0 || a.Nq <= 0 || a.Tk <= 0) return;
  ProfScope prof("mha_small", 4.0 * a.B * a.nh * (double)a.Nq * a.Tk * a.hd,
                 4.0 * a.B * ((double)a.Nq * 2 + 2.0 * a.Tk) * a.nh * a.hd, st);
  const dim3 grid(a.B * a.nh, cdiv(a.Nq, 4));
  if (a.hd <= 64)
    hipLaunchKernelGGL(mha_small_kernel<1>, grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(mha_small_kernel<2>, grid, dim3(256), 0, st, a);
  SD_LAUNCH_CHECK();
}

void tile_rows(const float* src, int src_rows, int D, float* dst, int dst_rows, hipStream_t st) {
  const int64_t n = (int64_t)dst_rows * D;
  if (n == 0) return;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(tile_rows_kernel, dim3(blocks), dim3(256), 0, st, src, src_rows, D, dst, n);
  SD_LAUNCH_CHECK();
}

void mean_sigmoid_affine(const float* x, int rows, int T, int ldx, const float* w, const float* b, int N, float* out,
                         int ldo, hipStream_t st) {
  if (rows <= 0) return;
  hipLaunchKernelGGL(mean_sigmoid_affine_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, st, x, rows, T, ldx, w, b, N, out,
                     ldo);
  SD_LAUNCH_CHECK();
}

}  // namespace sd
