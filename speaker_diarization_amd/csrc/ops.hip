// Small fused kernels around the GEMMs: FCM stem, CAMLayer context gate,
// LayerNorm, GroupNorm+SiLU, GLU+depthwise conv, GSP, layout glue.
// HBM-bound; written for coalesced 64-lane access, no MFMA.
#include <algorithm>

#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {

ConvGemmArgs linear_args(const void* A, int M, int K, int lda, const void* Wt, int N,
                         void* out, int ldo) {
  ConvGemmArgs p;
  p.A = A; p.B = 1; p.H = 1; p.W = M; p.Cin = K; p.lda = lda; p.a_coff = 0;
  p.Ho = 1; p.Wo = M;
  p.Wt = Wt; p.N = N; p.K = K;
  p.out = out; p.o_sb = 0; p.o_sh = 0; p.o_sw = ldo; p.o_sn = 1;
  return p;
}

// ------------------------------------------------------------------ FCM stem
template <bool OBF>
__global__ __launch_bounds__(256) void fcm_conv1_kernel(const float* __restrict__ fb, int B, int T,
                                                        int F, const float* __restrict__ w,
                                                        const float* __restrict__ alpha,
                                                        const float* __restrict__ beta,
                                                        void* __restrict__ out) {
  __shared__ float ws[32 * 9];
  __shared__ float al[32], be[32];
  for (int i = threadIdx.x; i < 32 * 9; i += blockDim.x) ws[i] = w[i];
  if (threadIdx.x < 32) { al[threadIdx.x] = alpha[threadIdx.x]; be[threadIdx.x] = beta[threadIdx.x]; }
  __syncthreads();
  int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = (int64_t)B * F * T;
  if (idx >= total) return;
  int t = idx % T;
  int64_t r = idx / T;
  int f = r % F;
  int b = r / F;
  float x[9];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      int ff = f + i - 1, tt = t + j - 1;
      x[i * 3 + j] = (ff >= 0 && ff < F && tt >= 0 && tt < T) ? fb[((int64_t)b * T + tt) * F + ff] : 0.f;
    }
#pragma unroll
  for (int c8 = 0; c8 < 4; ++c8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      int c = c8 * 8 + u;
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 9; ++k) acc = fmaf(ws[c * 9 + k], x[k], acc);
      v[u] = fmaxf(acc * al[c] + be[c], 0.f);
    }
    if constexpr (OBF) {
      uint4 pk;
      pk.x = (uint32_t)f2bf_bits(v[0]) | ((uint32_t)f2bf_bits(v[1]) << 16);
      pk.y = (uint32_t)f2bf_bits(v[2]) | ((uint32_t)f2bf_bits(v[3]) << 16);
      pk.z = (uint32_t)f2bf_bits(v[4]) | ((uint32_t)f2bf_bits(v[5]) << 16);
      pk.w = (uint32_t)f2bf_bits(v[6]) | ((uint32_t)f2bf_bits(v[7]) << 16);
      reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(out) + idx * 32)[c8] = pk;
    } else {
      float4* o = reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + idx * 32);
      o[2 * c8] = make_float4(v[0], v[1], v[2], v[3]);
      o[2 * c8 + 1] = make_float4(v[4], v[5], v[6], v[7]);
    }
  }
}

void fcm_conv1(const float* fbank, int B, int T, int F, const float* w, const float* alpha,
               const float* beta, void* out, bool out_bf16, hipStream_t st) {
  int64_t total = (int64_t)B * F * T;
  ProfScope prof("fcm_conv1", 2.0 * total * 32 * 9, 4.0 * total * 33, st);
  if (out_bf16)
    hipLaunchKernelGGL(fcm_conv1_kernel<true>, dim3((unsigned)cdiv((int)total, 256)), dim3(256), 0, st,
                       fbank, B, T, F, w, alpha, beta, out);
  else
    hipLaunchKernelGGL(fcm_conv1_kernel<false>, dim3((unsigned)cdiv((int)total, 256)), dim3(256), 0, st,
                       fbank, B, T, F, w, alpha, beta, out);
  SD_LAUNCH_CHECK();
}

// ------------------------------------------------------------------ CAM context
constexpr int kMaxSeg = 32;

// One workgroup per batch item: segment sums over time (4 independent
// accumulators per thread for load ILP), then the 2-layer context MLP with both
// weight matrices staged in LDS at a padded (+1) row stride.
template <bool XBF>
__global__ __launch_bounds__(256) void cam_context_kernel(
    const void* __restrict__ xv, int T, int C, int ldx, int seg_len,
    const float* __restrict__ w1, const float* __restrict__ b1, int C1,
    const float* __restrict__ w2, const float* __restrict__ b2, int C2, float* __restrict__ gate) {
  extern __shared__ float sm[];
  const int b = blockIdx.x;
  const int nseg = (T + seg_len - 1) / seg_len;
  const int parts = blockDim.x / C;
  float* psum = sm;                         // [parts][nseg][C]
  float* ctx = psum + parts * nseg * C;     // [nseg][C]
  float* h1 = ctx + nseg * C;               // [nseg][C1]
  float* W1 = h1 + nseg * C1;               // [C1][C+1]
  float* W2 = W1 + C1 * (C + 1);            // [C2][C1+1]
  const int tid = threadIdx.x;
  for (int i = tid; i < C1 * C; i += blockDim.x) W1[(i / C) * (C + 1) + i % C] = w1[i];
  for (int i = tid; i < C2 * C1; i += blockDim.x) W2[(i / C1) * (C1 + 1) + i % C1] = w2[i];
  const int c = tid % C;
  const int part = tid / C;
  if (part < parts) {
    for (int s = 0; s < nseg; ++s) {
      float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
      const int t1 = min(T, (s + 1) * seg_len);
      int t = s * seg_len + part;
      auto ld = [&](int tt) -> float {
        const int64_t o = ((int64_t)b * T + tt) * ldx + c;
        if constexpr (XBF) return bf_bits2f(reinterpret_cast<const uint16_t*>(xv)[o]);
        else return reinterpret_cast<const float*>(xv)[o];
      };
      for (; t + 3 * parts < t1; t += 4 * parts) {
        a0 += ld(t); a1 += ld(t + parts); a2 += ld(t + 2 * parts); a3 += ld(t + 3 * parts);
      }
      for (; t < t1; t += parts) a0 += ld(t);
      psum[(part * nseg + s) * C + c] = (a0 + a1) + (a2 + a3);
    }
  }
  __syncthreads();
  if (tid < C) {
    float tot = 0.f;
    for (int s = 0; s < nseg; ++s) {
      float ss = 0.f;
      for (int q = 0; q < parts; ++q) ss += psum[(q * nseg + s) * C + tid];
      ctx[s * C + tid] = ss;
      tot += ss;
    }
    const float mean = tot / (float)T;
    for (int s = 0; s < nseg; ++s) {
      const int cnt = min(T, (s + 1) * seg_len) - s * seg_len;
      ctx[s * C + tid] = mean + ctx[s * C + tid] / (float)cnt;
    }
  }
  __syncthreads();
  for (int i = tid; i < nseg * C1; i += blockDim.x) {
    const int s = i / C1, j = i % C1;
    const float* wr = W1 + j * (C + 1);
    const float* cr = ctx + s * C;
    float a0 = b1[j], a1 = 0.f;
    for (int k = 0; k < C; k += 2) {
      a0 = fmaf(wr[k], cr[k], a0);
      a1 = fmaf(wr[k + 1], cr[k + 1], a1);
    }
    h1[i] = fmaxf(a0 + a1, 0.f);
  }
  __syncthreads();
  for (int i = tid; i < nseg * C2; i += blockDim.x) {
    const int s = i / C2, o = i % C2;
    const float* wr = W2 + o * (C1 + 1);
    const float* hr = h1 + s * C1;
    float a0 = b2[o], a1 = 0.f;
    for (int k = 0; k < C1; k += 2) {
      a0 = fmaf(wr[k], hr[k], a0);
      a1 = fmaf(wr[k + 1], hr[k + 1], a1);
    }
    gate[((int64_t)b * nseg + s) * C2 + o] = 1.f / (1.f + expf(-(a0 + a1)));
  }
}


// Segment-parallel variant: one workgroup per (segment, batch item), so a batch of B
// items launches B * nseg workgroups instead of B (the per-item kernel above left most
// CUs idle at the embedding extractor's B = 96 and ran latency-bound).  Each workgroup
// streams all T rows once with 8/16-B loads (4 channels per lane, 256/(C/4) rows in
// flight), accumulating the whole-sequence sum and its own segment's sum in the same
// pass, then evaluates its segment's context MLP straight from the (L2-resident)
// weights with shuffle-reduced dot products.
template <bool XBF, int C, int C1, int C2>
__global__ __launch_bounds__(256) void cam_context_seg_kernel(
    const void* __restrict__ xv, int T, int ldx, int seg_len, int nseg_arg,
    const float* __restrict__ w1, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ b2, float* __restrict__ gate) {
  constexpr int L = C / 4;          // lanes per row
  constexpr int P = 256 / L;        // rows in flight
  constexpr int G1 = 256 / C1;      // threads per first-layer output
  constexpr int G2 = 256 / C2;
  static_assert(C % 4 == 0 && 256 % L == 0 && 256 % C1 == 0 && 256 % C2 == 0, "cam_context_seg shape");
  static_assert(C % G1 == 0 && C1 % G2 == 0 && G1 <= 64 && G2 <= 64, "cam_context_seg split");
  __shared__ float4 red_t[P][L];
  __shared__ float4 red_s[P][L];
  __shared__ float ctx[C];
  __shared__ float h1[C1];
  // 1-D grid, remapped so the nseg workgroups of one item are consecutive logical ids on one
  // XCD: the item's rows are fetched into that XCD's L2 once instead of once per segment.
  const int nseg = nseg_arg;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int b = lid / nseg, s = lid - b * nseg;
  const int tid = threadIdx.x;
  const int part = tid / L, l = tid % L;
  const int t0 = s * seg_len, t1 = min(T, t0 + seg_len);
  float4 at = make_float4(0.f, 0.f, 0.f, 0.f), as = at;
  auto load = [&](int t) -> float4 {
    const int64_t o = ((int64_t)b * T + t) * ldx + 4 * l;
    if constexpr (XBF) {
      const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(xv) + o);
      return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                         __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
    } else {
      return *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(xv) + o);
    }
  };
  auto acc = [&](int t, const float4& v) {
    at.x += v.x; at.y += v.y; at.z += v.z; at.w += v.w;
    if (t >= t0 && t < t1) { as.x += v.x; as.y += v.y; as.z += v.z; as.w += v.w; }
  };
  int t = part;
  for (; t + 3 * P < T; t += 4 * P) {    // four rows in flight per lane
    const float4 v0 = load(t), v1 = load(t + P), v2 = load(t + 2 * P), v3 = load(t + 3 * P);
    acc(t, v0); acc(t + P, v1); acc(t + 2 * P, v2); acc(t + 3 * P, v3);
  }
  for (; t < T; t += P) acc(t, load(t));
  red_t[part][l] = at;
  red_s[part][l] = as;
  __syncthreads();
  if (tid < C) {
    const int ll = tid / 4, k = tid % 4;
    float tt = 0.f, ss = 0.f;
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const float* a = reinterpret_cast<const float*>(&red_t[q][ll]);
      const float* z = reinterpret_cast<const float*>(&red_s[q][ll]);
      tt += a[k];
      ss += z[k];
    }
    ctx[tid] = tt / (float)T + ss / (float)(t1 - t0);
  }
  __syncthreads();
  {
    const int j = tid / G1, q = tid % G1;
    constexpr int KC = C / G1;
    const float* wr = w1 + (int64_t)j * C + q * KC;
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < KC; ++k) a = fmaf(wr[k], ctx[q * KC + k], a);
#pragma unroll
    for (int o = G1 / 2; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
    if (q == 0) h1[j] = fmaxf(a + b1[j], 0.f);
  }
  __syncthreads();
  {
    const int j = tid / G2, q = tid % G2;
    constexpr int KC = C1 / G2;
    const float* wr = w2 + (int64_t)j * C1 + q * KC;
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < KC; ++k) a = fmaf(wr[k], h1[q * KC + k], a);
#pragma unroll
    for (int o = G2 / 2; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
    if (q == 0) gate[((int64_t)b * nseg + s) * C2 + j] = 1.f / (1.f + expf(-(a + b2[j])));
  }
}

void cam_context(const void* x, bool x_bf16, int B, int T, int C, int ldx, int seg_len, const float* w1,
                 const float* b1, int C1, const float* w2, const float* b2, int C2, float* gate,
                 hipStream_t st) {
  SD_CHECK(C <= 256 && 256 % C == 0 && C % 2 == 0 && C1 % 2 == 0, kErrInvalid,
           "cam_context: C must divide 256");
  const int nseg = cdiv(T, seg_len);
  SD_CHECK(nseg <= kMaxSeg, kErrInvalid, "cam_context: too many segments");
  const size_t smem = sizeof(float) * ((256 / C) * nseg * C + nseg * C + nseg * C1 + C1 * (C + 1) +
                                       C2 * (C1 + 1));
  ProfScope prof("cam_context", 2.0 * B * nseg * (C * C1 + C1 * C2), (x_bf16 ? 2.0 : 4.0) * B * T * C, st);
  const uintptr_t align = x_bf16 ? 8 : 16;
  if (C == 128 && C1 == 64 && C2 == 32 && ldx % 4 == 0 && reinterpret_cast<uintptr_t>(x) % align == 0) {
    // CAM++ dense layers (bn_channels 128, reduction 2, growth 32)
    if (x_bf16)
      hipLaunchKernelGGL((cam_context_seg_kernel<true, 128, 64, 32>), dim3(nseg * B), dim3(256), 0, st, x, T, ldx,
                         seg_len, nseg, w1, b1, w2, b2, gate);
    else
      hipLaunchKernelGGL((cam_context_seg_kernel<false, 128, 64, 32>), dim3(nseg * B), dim3(256), 0, st, x, T, ldx,
                         seg_len, nseg, w1, b1, w2, b2, gate);
    SD_LAUNCH_CHECK();
    return;
  }
  if (x_bf16)
    hipLaunchKernelGGL(cam_context_kernel<true>, dim3(B), dim3(256), smem, st, x, T, C, ldx, seg_len, w1,
                       b1, C1, w2, b2, C2, gate);
  else
    hipLaunchKernelGGL(cam_context_kernel<false>, dim3(B), dim3(256), smem, st, x, T, C, ldx, seg_len, w1,
                       b1, C1, w2, b2, C2, gate);
  SD_LAUNCH_CHECK();
}

// ------------------------------------------------------------------ LayerNorm
template <int PER, bool YBF, int TM>
__global__ __launch_bounds__(256) void layernorm_kernel(const float* __restrict__ x, int rows, int D,
                                                        int ldx, const void* __restrict__ t,
                                                        float* __restrict__ xo, const float* __restrict__ g,
                                                        const float* __restrict__ bb, float eps,
                                                        act_t<YBF>* __restrict__ y, int ldy) {
  // TM: 0 plain LN of x; 1 / 2: LN of x + t with t fp32 / bf16 (the residual add of the
  // encoder blocks, fused here so the producing GEMM stores its output only); xo: the sum
  // is also written back (pre-LN residual stream).
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + (int64_t)row * ldx;
  float v[PER];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    int c = lane + i * 64;
    float a = c < D ? xr[c] : 0.f;
    if constexpr (TM == 1) a += c < D ? reinterpret_cast<const float*>(t)[(int64_t)row * D + c] : 0.f;
    if constexpr (TM == 2) a += c < D ? bf_bits2f(reinterpret_cast<const uint16_t*>(t)[(int64_t)row * D + c]) : 0.f;
    v[i] = a;
    s += a;
  }
  s = warp_sum(s);
  const float mean = s / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    int c = lane + i * 64;
    float d = c < D ? v[i] - mean : 0.f;
    q += d * d;
  }
  q = warp_sum(q);
  const float rstd = rsqrtf(q / (float)D + eps);
  if (xo) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      int c = lane + i * 64;
      if (c < D) xo[(int64_t)row * ldx + c] = v[i];
    }
  }
  act_t<YBF>* yr = y + (int64_t)row * ldy;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    int c = lane + i * 64;
    if (c < D) st_act(yr, c, (v[i] - mean) * rstd * g[c] + bb[c]);
  }
}

// Vector LayerNorm for D % 128 == 0 (D = 128 * NV <= 1024): half a wave per row, each
// lane owns NV float4 column groups (16-B loads/stores, 8-B bf16 t/y), so a row is
// moved in full 512-B wave instructions with no idle lanes (the one-wave-per-row
// kernel above leaves 1/4 of its lanes idle at D = 384 and issues 4-B accesses).
// Same math: sum -> mean, centred sum of squares -> rstd; the reductions stay inside
// each 32-lane half (xor masks < 32).
__device__ __forceinline__ float half_sum(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int NV, bool YBF, int TM>
__global__ __launch_bounds__(256) void layernorm_vec_kernel(const float* __restrict__ x, int rows, int D, int ldx,
                                                            const void* __restrict__ t, float* __restrict__ xo,
                                                            const float* __restrict__ g,
                                                            const float* __restrict__ bb, float eps,
                                                            act_t<YBF>* __restrict__ y, int ldy,
                                                            uint16_t* __restrict__ y2, int t_slabs) {
  const int hl = threadIdx.x & 31;
  const int row = blockIdx.x * 8 + (threadIdx.x >> 5);
  if (row >= rows) return;   // whole 32-lane halves leave together
  const float* xr = x + (int64_t)row * ldx;
  float4 v[NV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (hl + i * 32) * 4;
    float4 a = *reinterpret_cast<const float4*>(xr + c);
    if constexpr (TM == 1) {
      for (int sl = 0; sl < t_slabs; ++sl) {   // split-K partial slabs, summed in slab order
        const float4 b = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(t) +
                                                           ((int64_t)sl * rows + row) * D + c);
        a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
      }
    }
    if constexpr (TM == 2) {
      const uint2 b = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(t) + (int64_t)row * D + c);
      a.x += __uint_as_float(b.x << 16); a.y += __uint_as_float(b.x & 0xffff0000u);
      a.z += __uint_as_float(b.y << 16); a.w += __uint_as_float(b.y & 0xffff0000u);
    }
    v[i] = a;
    s += (a.x + a.y) + (a.z + a.w);
  }
  const float mean = half_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const float dx = v[i].x - mean, dy = v[i].y - mean, dz = v[i].z - mean, dw = v[i].w - mean;
    q += (dx * dx + dy * dy) + (dz * dz + dw * dw);
  }
  const float rstd = rsqrtf(half_sum(q) / (float)D + eps);
  if (xo) {
#pragma unroll
    for (int i = 0; i < NV; ++i)
      *reinterpret_cast<float4*>(xo + (int64_t)row * ldx + (hl + i * 32) * 4) = v[i];
  }
  act_t<YBF>* yr = y + (int64_t)row * ldy;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (hl + i * 32) * 4;
    const float4 gg = *reinterpret_cast<const float4*>(g + c);
    const float4 b4 = *reinterpret_cast<const float4*>(bb + c);
    const float o0 = (v[i].x - mean) * rstd * gg.x + b4.x, o1 = (v[i].y - mean) * rstd * gg.y + b4.y;
    const float o2 = (v[i].z - mean) * rstd * gg.z + b4.z, o3 = (v[i].w - mean) * rstd * gg.w + b4.w;
    if constexpr (YBF)
      *reinterpret_cast<uint2*>(yr + c) = make_uint2(pack_bf16x2(o0, o1), pack_bf16x2(o2, o3));
    else
      *reinterpret_cast<float4*>(yr + c) = make_float4(o0, o1, o2, o3);
    if (y2)   // bf16 shadow of an fp32 y (the next GEMM's A operand; the bf16 GEMMs round A the same way)
      *reinterpret_cast<uint2*>(y2 + (int64_t)row * ldy + c) = make_uint2(pack_bf16x2(o0, o1), pack_bf16x2(o2, o3));
  }
}

template <int NV, int TM>
static void lnv_launch2(const float* x, int rows, int D, int ldx, const void* t, float* xo, const float* g,
                        const float* b, float eps, void* y, int ldy, bool ybf, uint16_t* y2, int t_slabs,
                        hipStream_t st) {
  dim3 grid(cdiv(rows, 8));
  if (ybf)
    hipLaunchKernelGGL((layernorm_vec_kernel<NV, true, TM>), grid, dim3(256), 0, st, x, rows, D, ldx, t, xo, g, b,
                       eps, reinterpret_cast<uint16_t*>(y), ldy, y2, t_slabs);
  else
    hipLaunchKernelGGL((layernorm_vec_kernel<NV, false, TM>), grid, dim3(256), 0, st, x, rows, D, ldx, t, xo, g, b,
                       eps, reinterpret_cast<float*>(y), ldy, y2, t_slabs);
}

template <int NV>
static void lnv_launch(const float* x, int rows, int D, int ldx, const void* t, int tm, float* xo,
                       const float* g, const float* b, float eps, void* y, int ldy, bool ybf, uint16_t* y2,
                       int t_slabs, hipStream_t st) {
  if (tm == 0) lnv_launch2<NV, 0>(x, rows, D, ldx, t, xo, g, b, eps, y, ldy, ybf, y2, t_slabs, st);
  else if (tm == 1) lnv_launch2<NV, 1>(x, rows, D, ldx, t, xo, g, b, eps, y, ldy, ybf, y2, t_slabs, st);
  else lnv_launch2<NV, 2>(x, rows, D, ldx, t, xo, g, b, eps, y, ldy, ybf, y2, t_slabs, st);
}

static bool aligned16(const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

template <int PER, int TM>
static void ln_launch2(const float* x, int rows, int D, int ldx, const void* t, float* xo, const float* g,
                       const float* b, float eps, void* y, int ldy, bool ybf, hipStream_t st) {
  dim3 grid(cdiv(rows, 4));
  if (ybf)
    hipLaunchKernelGGL((layernorm_kernel<PER, true, TM>), grid, dim3(256), 0, st, x, rows, D, ldx, t, xo, g, b,
                       eps, reinterpret_cast<uint16_t*>(y), ldy);
  else
    hipLaunchKernelGGL((layernorm_kernel<PER, false, TM>), grid, dim3(256), 0, st, x, rows, D, ldx, t, xo, g, b,
                       eps, reinterpret_cast<float*>(y), ldy);
}

template <int PER>
static void ln_launch(const float* x, int rows, int D, int ldx, const void* t, int tm, float* xo,
                      const float* g, const float* b, float eps, void* y, int ldy, bool ybf, hipStream_t st) {
  if (tm == 0) ln_launch2<PER, 0>(x, rows, D, ldx, t, xo, g, b, eps, y, ldy, ybf, st);
  else if (tm == 1) ln_launch2<PER, 1>(x, rows, D, ldx, t, xo, g, b, eps, y, ldy, ybf, st);
  else ln_launch2<PER, 2>(x, rows, D, ldx, t, xo, g, b, eps, y, ldy, ybf, st);
}

static void ln_dispatch(const float* x, int rows, int D, int ldx, const void* t, int tm, float* xo,
                        const float* g, const float* b, float eps, void* y, int ldy, bool y_bf16, hipStream_t st,
                        uint16_t* y2 = nullptr, int t_slabs = 1) {
  SD_CHECK(!y2 || !y_bf16, kErrInvalid, "layernorm: the bf16 shadow output needs an fp32 y");
  SD_CHECK(t_slabs == 1 || tm == 1, kErrInvalid, "layernorm: t slabs need an fp32 t");
  const bool vec = D % 128 == 0 && D <= 1024 && ldx % 4 == 0 && ldy % 4 == 0 && aligned16(x) && aligned16(xo) &&
                   aligned16(g) && aligned16(b) && (reinterpret_cast<uintptr_t>(y) & (y_bf16 ? 7 : 15)) == 0 &&
                   (reinterpret_cast<uintptr_t>(t) & (tm == 2 ? 7 : 15)) == 0 &&
                   (reinterpret_cast<uintptr_t>(y2) & 7) == 0;
  if (vec) {
    switch (D / 128) {
      case 1: lnv_launch<1>(x, rows, D, ldx, t, tm, xo, g, b, eps, y, ldy, y_bf16, y2, t_slabs, st); break;
      case 2: lnv_launch<2>(x, rows, D, ldx, t, tm, xo, g, b, eps, y, ldy, y_bf16, y2, t_slabs, st); break;
      case 3: lnv_launch<3>(x, rows, D, ldx, t, tm, xo, g, b, eps, y, ldy, y_bf16, y2, t_slabs, st); break;
      case 4: lnv_launch<4>(x, rows, D, ldx, t, tm, xo, g, b, eps, y, ldy, y_bf16, y2, t_slabs, st); break;
      case 5: lnv_launch<5>(x, rows, D, ldx, t, tm, xo, g, b, eps, y, ldy, y_bf16, y2, t_slabs, st); break;
      case 6: lnv_launch<6>(x, rows, D, ldx, t, tm, xo, g, b, eps, y, ldy, y_bf16, y2, t_slabs, st); break;
      case 7: lnv_launch<7>(x, rows, D, ldx, t, tm, xo, g, b, eps, y, ldy, y_bf16, y2, t_slabs, st); break;
      default: lnv_launch<8>(x, rows, D, ldx, t, tm, xo, g, b, eps, y, ldy, y_bf16, y2, t_slabs, st); break;
    }
  } else if (t_slabs > 1) {
    SD_CHECK(false, kErrInvalid, "layernorm: t slabs need D % 128 == 0 and 16-B aligned rows");
  } else if (y2) {
    ln_dispatch(x, rows, D, ldx, t, tm, xo, g, b, eps, y, ldy, false, st);
    SD_CHECK(ldy == D, kErrInvalid, "layernorm: bf16 shadow needs ldy == D");
    f32_to_bf16(reinterpret_cast<const float*>(y), (int64_t)rows * D, y2, st);
    return;
  } else if (D <= 256) ln_launch<4>(x, rows, D, ldx, t, tm, xo, g, b, eps, y, ldy, y_bf16, st);
  else if (D <= 512) ln_launch<8>(x, rows, D, ldx, t, tm, xo, g, b, eps, y, ldy, y_bf16, st);
  else if (D <= 1024) ln_launch<16>(x, rows, D, ldx, t, tm, xo, g, b, eps, y, ldy, y_bf16, st);
  else SD_CHECK(false, kErrInvalid, "layernorm: D > 1024 unsupported");
  SD_LAUNCH_CHECK();
}

void layernorm(const float* x, int rows, int D, int ldx, const float* g, const float* b,
               float eps, void* y, int ldy, bool y_bf16, hipStream_t st, uint16_t* y2) {
  ProfScope prof("layernorm", 0.0, (4.0 + (y_bf16 ? 2.0 : 4.0) + (y2 ? 2.0 : 0.0)) * rows * D, st);
  ln_dispatch(x, rows, D, ldx, nullptr, 0, nullptr, g, b, eps, y, ldy, y_bf16, st, y2);
}

void add_layernorm(float* x, const void* t, bool t_bf16, int rows, int D, const float* g, const float* b,
                   float eps, bool write_x, void* y, bool y_bf16, hipStream_t st, uint16_t* y2, int t_slabs) {
  ProfScope prof("add_layernorm", 0.0,
                 (4.0 + (t_bf16 ? 2.0 : 4.0 * t_slabs) + (write_x ? 4.0 : 0.0) + (y_bf16 ? 2.0 : 4.0) +
                  (y2 ? 2.0 : 0.0)) * rows * D, st);
  ln_dispatch(x, rows, D, D, t, t_bf16 ? 2 : 1, write_x ? x : nullptr, g, b, eps, y, D, y_bf16, st, y2, t_slabs);
}

// ------------------------------------------------------------------ zero fill
// Stream-ordered zeroing as a kernel, used instead of hipMemsetAsync inside every forward: a memset
// captured into a hipGraph (a caller may capture our forwards) is a memset node, and on ROCm 7.2 such
// nodes were observed not to take effect before the next kernel node from the second launch of the
// instantiated graph on (graph-replay root cause) -- a kernel node is ordered like any other.
__global__ __launch_bounds__(256) void fill_u32_kernel(uint32_t* __restrict__ p, int64_t n, uint32_t v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = v;
}

void fill_u32(void* p, size_t bytes, uint32_t value, hipStream_t st) {
  SD_CHECK(bytes % 4 == 0 && (reinterpret_cast<uintptr_t>(p) & 3) == 0, kErrInvalid, "fill: 4-byte words only");
  const int64_t n = (int64_t)(bytes / 4);
  if (n == 0) return;
  const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(fill_u32_kernel, dim3(blocks), dim3(256), 0, st, static_cast<uint32_t*>(p), n, value);
  SD_LAUNCH_CHECK();
}

void zero_fill(void* p, size_t bytes, hipStream_t st) { fill_u32(p, bytes, 0u, st); }

// ------------------------------------------------------------------ TS-VAD glue
__device__ __forceinline__ float bn_relu(const BnRelu& p, int window, int c, float x) {
  if (!p.a) return x;
  const bool bypass = p.grp && p.grp[(window + p.win0) / p.group];
  return fmaxf(bypass ? x : fmaf(p.a[c], x, p.b[c]), 0.f);
}

__global__ __launch_bounds__(256) void nonfinite_windows_kernel(const float* __restrict__ x, int64_t per_win, int group,
                                                                int* win, int* grp_a, int* grp_b) {
  const int w = blockIdx.x;
  const float4* xr = reinterpret_cast<const float4*>(x + (int64_t)w * per_win);
  const int64_t n4 = per_win / 4;
  bool bad = false;
  for (int64_t i = (int64_t)blockIdx.y * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.y * blockDim.x) {
    const float4 v = xr[i];
    bad |= ((__float_as_uint(v.x) | 0x807fffffu) == 0xffffffffu) | ((__float_as_uint(v.y) | 0x807fffffu) == 0xffffffffu) |
           ((__float_as_uint(v.z) | 0x807fffffu) == 0xffffffffu) | ((__float_as_uint(v.w) | 0x807fffffu) == 0xffffffffu);
  }
  if (blockIdx.y == 0)
    for (int64_t i = n4 * 4 + threadIdx.x; i < per_win; i += blockDim.x)
      bad |= (__float_as_uint(x[(int64_t)w * per_win + i]) | 0x807fffffu) == 0xffffffffu;
  if (__any(bad) && (threadIdx.x & 63) == 0) {   // one atomic per wave that saw one
    atomicOr(win + w, 1);
    if (grp_a) atomicOr(grp_a + w / group, 1);
    if (grp_b) atomicOr(grp_b + w / group, 1);
  }
}

void nonfinite_windows(const float* x, int B, int64_t per_win, int group, int* win, int* grp_a, int* grp_b,
                       hipStream_t st) {
  SD_CHECK(B >= 1 && per_win >= 1 && group >= 1 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 && per_win % 4 == 0,
           kErrInvalid, "nonfinite_windows: bad shape");
  const int chunks = (int)std::min<int64_t>(64, cdiv((int)std::min<int64_t>(per_win / 4, 1 << 30), 256 * 8));
  hipLaunchKernelGGL(nonfinite_windows_kernel, dim3(B, std::max(chunks, 1)), dim3(256), 0, st, x, per_win, group, win,
                     grp_a, grp_b);
  SD_LAUNCH_CHECK();
}

__global__ void poison_windows_kernel(float* x, int64_t per_win, const int* __restrict__ win_a,
                                      const int* __restrict__ win_b) {
  const int w = blockIdx.x;
  if (!win_a[w] && !(win_b && win_b[w])) return;
  for (int64_t i = threadIdx.x; i < per_win; i += blockDim.x) x[(int64_t)w * per_win + i] = __int_as_float(0x7fc00000);
}

void poison_windows(float* x, int B, int64_t per_win, const int* win_a, const int* win_b, hipStream_t st) {
  hipLaunchKernelGGL(poison_windows_kernel, dim3(B), dim3(256), 0, st, x, per_win, win_a, win_b);
  SD_LAUNCH_CHECK();
}

__global__ void build_speaker_input_kernel(const float* __restrict__ ts, const float* __restrict__ mix,
                                           int ldmix, int Tmix, int B, int NS, int T, int E,
                                           const float* __restrict__ pe, float* __restrict__ out, BnRelu bn) {
  const int row = blockIdx.x;  // (b, spk, t)
  const int t = row % T;
  const int bs = row / T;
  const int b = bs / NS;
  float* o = out + (int64_t)row * 2 * E;
  const float* ts_r = ts + (int64_t)bs * E;
  const bool mv = t < Tmix;
  const float* mx = mix + ((int64_t)b * Tmix + (mv ? t : 0)) * ldmix;
  const float* pr = pe ? pe + (int64_t)t * 2 * E : nullptr;
  for (int c = threadIdx.x; c < 2 * E; c += blockDim.x) {
    float v = c < E ? ts_r[c] : (mv ? bn_relu(bn, b, c - E, mx[c - E]) : 0.f);
    if (pr) v += pr[c];
    o[c] = v;
  }
}

void build_speaker_input(const float* ts, const float* mix, int ldmix, int Tmix, int B, int NS,
                         int T, int E, const float* pe, float* out, hipStream_t st, const BnRelu& mix_bn) {
  hipLaunchKernelGGL(build_speaker_input_kernel, dim3(B * NS * T), dim3(128), 0, st, ts, mix,
                     ldmix, Tmix, B, NS, T, E, pe, out, mix_bn);
  SD_LAUNCH_CHECK();
}

__global__ void build_stream_input_kernel(const float* __restrict__ ts, const float* __restrict__ mix, int T,
                                          int NS, int E, float scale, const float* __restrict__ pe, int C,
                                          int left, float* __restrict__ out) {
  const int row = blockIdx.x;   // (window, spk, t)
  const int t = row % T, spk = row / T, w = spk / NS;
  const int ch = t / C;
  const int pos = (left < 0 ? 0 : max(0, ch - left) * C) + t % C;
  float* o = out + (int64_t)row * 2 * E;
  const float* pr = pe + (int64_t)pos * 2 * E;
  for (int c = threadIdx.x; c < 2 * E; c += blockDim.x) {
    const float v = c < E ? ts[(int64_t)spk * E + c] : mix[((int64_t)w * T + t) * E + c - E];
    o[c] = v * scale + pr[c];
  }
}

void build_stream_input(const float* ts, const float* mix, int B, int T, int NS, int E, float scale,
                        const float* pe, int C, int left, float* out, hipStream_t st) {
  hipLaunchKernelGGL(build_stream_input_kernel, dim3(B * NS * T), dim3(128), 0, st, ts, mix, T, NS, E, scale, pe, C,
                     left, out);
  SD_LAUNCH_CHECK();
}

__global__ void add_pe_kernel(float* __restrict__ x, int rows, int T, int D, int ld,
                              const float* __restrict__ pe, BnRelu bn) {
  const int row = blockIdx.x;
  const int t = row % T;
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    float* p = x + (int64_t)row * ld + c;
    *p = bn_relu(bn, row / T, c, *p) + pe[(int64_t)t * D + c];
  }
}

void add_pe(float* x, int rows, int T, int D, int ld, const float* pe, hipStream_t st, const BnRelu& bn) {
  hipLaunchKernelGGL(add_pe_kernel, dim3(rows), dim3(128), 0, st, x, rows, T, D, ld, pe, bn);
  SD_LAUNCH_CHECK();
}

__global__ __launch_bounds__(256) void gsp_fc_kernel(const float* __restrict__ x, int rows, int C,
                                                     int ldx, const float* __restrict__ w,
                                                     const float* __restrict__ bias, int E,
                                                     float* __restrict__ out, int ldo, BnRelu bn, int rpw) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + (int64_t)row * ldx;
  constexpr int kMaxPer = 4;                      // C <= 256
  float v[kMaxPer];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < kMaxPer; ++k) {
    const int c = lane + 64 * k;
    v[k] = c < C ? bn_relu(bn, row / rpw, c, xr[c]) : 0.f;
    s += v[k];
  }
  s = warp_sum(s);
  const float mean = s / (float)C;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < kMaxPer; ++k)
    if (lane + 64 * k < C) { const float d = v[k] - mean; q += d * d; }
  q = warp_sum(q);
  const float sd = sqrtf(q / (float)(C - 1));   // torch.std default: unbiased
  float* o = out + (int64_t)row * ldo;
  for (int e = lane; e < E; e += 64) o[e] = fmaf(w[e * 2], mean, fmaf(w[e * 2 + 1], sd, bias[e]));
}

void gsp_fc(const float* x, int rows, int C, int ldx, const float* w, const float* bias, int E,
            float* out, int ldo, hipStream_t st, const BnRelu& bn, int rows_per_window) {
  SD_CHECK(C >= 2 && C <= 256 && rows_per_window >= 1, kErrInvalid, "gsp_fc: C must be in [2, 256]");
  hipLaunchKernelGGL(gsp_fc_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, st, x, rows, C, ldx, w, bias,
                     E, out, ldo, bn, rows_per_window);
  SD_LAUNCH_CHECK();
}

template <bool OBF>
__global__ void speakers_to_channels_kernel(const float* __restrict__ x, int B, int NS, int T, int E,
                                            act_t<OBF>* __restrict__ out) {
  const int row = blockIdx.x;  // (b, t)
  const int t = row % T;
  const int b = row / T;
  act_t<OBF>* o = out + (int64_t)row * NS * E;
  for (int c = threadIdx.x; c < NS * E; c += blockDim.x) {
    int spk = c / E, e = c % E;
    st_act(o, c, x[(((int64_t)b * NS + spk) * T + t) * E + e]);
  }
}

void speakers_to_channels(const float* x, int B, int NS, int T, int E, void* out, bool out_bf16,
                          hipStream_t st) {
  if (out_bf16)
    hipLaunchKernelGGL(speakers_to_channels_kernel<true>, dim3(B * T), dim3(256), 0, st, x, B, NS, T, E,
                       reinterpret_cast<uint16_t*>(out));
  else
    hipLaunchKernelGGL(speakers_to_channels_kernel<false>, dim3(B * T), dim3(256), 0, st, x, B, NS, T, E,
                       reinterpret_cast<float*>(out));
  SD_LAUNCH_CHECK();
}

// ------------------------------------------------------------------ conformer conv module
constexpr int kDwCB = 64;    // channels per block
constexpr int kDwTT = 64;    // time tile

// One block per (sequence, 64 channels); lane = channel, so every LDS column read is
// conflict-free and every output row store is one coalesced 64-channel segment.
// Time is processed in tiles of kDwTT outputs: the GLU'd inputs of the tile (+ k-1
// halo rows) are staged in LDS with 16-B vector loads, then each wave produces runs
// of kDwR consecutive outputs from a register window (kDwR + k - 1 LDS reads for
// kDwR * k FMAs).  The channel's k taps live in registers.
constexpr int kDwR = 8;
constexpr int kDwMaxK = 31;

template <bool BF>
__global__ __launch_bounds__(256) void glu_dwconv_kernel(const act_t<BF>* __restrict__ x, int T, int C,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ bias, int k,
                                                         act_t<BF>* __restrict__ y,
                                                         float* __restrict__ partial, int fused_silu,
                                                         int glu_in) {
  // bf16 mode stages bf16 (the activations already are), so a whole 150-frame conformer
  // sequence (+ halo) fits one stage in 24 KiB: every global load of the block is in flight
  // at once instead of one latency per 64-frame tile.
  constexpr int TT = BF ? 160 : kDwTT;
  __shared__ act_t<BF> g[(TT + kDwMaxK - 1) * kDwCB];
  __shared__ float red[2][256];
  // bf16 mode: each wave's run of kDwR output rows is transposed through LDS so the stores
  // leave as 16-B lanes (8 rows x 128 B per wave-instruction) instead of 2-B lanes.
  __shared__ uint16_t otile[BF ? 4 : 1][kDwR * kDwCB];
  const int pad = (k - 1) / 2;
  const int s = blockIdx.y;
  const int c0 = blockIdx.x * kDwCB;
  const int nblk = gridDim.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = c0 + lane;
  float wr[kDwMaxK];
#pragma unroll
  for (int j = 0; j < kDwMaxK; ++j) wr[j] = (j < k && c < C) ? w[(int64_t)c * k + j] : 0.f;
  const float bv = (bias && c < C) ? bias[c] : 0.f;
  const act_t<BF>* xs = x + (int64_t)s * T * (glu_in ? 2 : 1) * C;
  act_t<BF>* ys = y + (int64_t)s * T * C;
  float lsum = 0.f, lsq = 0.f;
  constexpr int VEC = BF ? 8 : 4;             // elements per 16-B load
  constexpr int CPR = kDwCB / VEC;            // vector chunks per row
  for (int t0 = 0; t0 < T; t0 += TT) {
    const int span = min(TT, T - t0) + k - 1;
    __syncthreads();
    for (int i = threadIdx.x; i < span * CPR; i += blockDim.x) {
      const int tt = i / CPR, ch = (i % CPR) * VEC;
      const int t = t0 - pad + tt;
      uint4 out = {0u, 0u, 0u, 0u};            // VEC elements of act_t<BF>
      if (t >= 0 && t < T && c0 + ch < C && !glu_in) {
        out = *reinterpret_cast<const uint4*>(xs + (int64_t)t * C + c0 + ch);   // already gated (pw1 GLU epilogue)
      } else if (t >= 0 && t < T && c0 + ch < C) {
        // pw1 rows interleaved in 32-column groups [16 values | 16 gates] (glu_interleave_row)
        const int cc = c0 + ch;
        const act_t<BF>* ra = xs + (int64_t)t * 2 * C + (cc / 16) * 32 + cc % 16;
        if constexpr (BF) {
          const uint4 a4 = *reinterpret_cast<const uint4*>(ra);
          const uint4 g4 = *reinterpret_cast<const uint4*>(ra + 16);
          const uint32_t aw[4] = {a4.x, a4.y, a4.z, a4.w}, gw[4] = {g4.x, g4.y, g4.z, g4.w};
          uint32_t o[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const float a0 = __uint_as_float(aw[u] << 16), a1 = __uint_as_float(aw[u] & 0xffff0000u);
            const float g0 = __uint_as_float(gw[u] << 16), g1 = __uint_as_float(gw[u] & 0xffff0000u);
            o[u] = pack_bf16x2(a0 * sigmoid_rcp(g0), a1 * sigmoid_rcp(g1));
          }
          out = make_uint4(o[0], o[1], o[2], o[3]);
        } else {
          const float4 a4 = *reinterpret_cast<const float4*>(ra);
          const float4 g4 = *reinterpret_cast<const float4*>(ra + 16);
          out = make_uint4(__float_as_uint(a4.x / (1.f + __expf(-g4.x))), __float_as_uint(a4.y / (1.f + __expf(-g4.y))),
                           __float_as_uint(a4.z / (1.f + __expf(-g4.z))), __float_as_uint(a4.w / (1.f + __expf(-g4.w))));
        }
      }
      *reinterpret_cast<uint4*>(g + tt * kDwCB + ch) = out;
    }
    __syncthreads();
    const int nout = min(TT, T - t0);
    for (int r0 = wv * kDwR; r0 < nout; r0 += 4 * kDwR) {
      float win[kDwR + kDwMaxK - 1];
#pragma unroll
      for (int i = 0; i < kDwR + kDwMaxK - 1; ++i)
        win[i] = (i < kDwR + k - 1) ? ld_act(g, (r0 + i) * kDwCB + lane) : 0.f;
#pragma unroll
      for (int r = 0; r < kDwR; ++r) {
        float acc = bv;
#pragma unroll
        for (int j = 0; j < kDwMaxK; ++j) acc = fmaf(wr[j], win[r + j], acc);
        if (fused_silu) acc = acc * sigmoid_rcp(acc);
        const int t = t0 + r0 + r;
        if constexpr (BF) {
          otile[wv][r * kDwCB + lane] = f2bf_bits(acc);
        } else if (r0 + r < nout && c < C) {
          st_act(ys, (int64_t)t * C + c, acc);
        }
        if (r0 + r < nout && c < C) {
          lsum += acc;
          lsq += acc * acc;
        }
      }
      if constexpr (BF) {
        // lane l: row l / 8 of the run, channels 8 * (l % 8) .. +7 (same-wave LDS round trip)
        const int rr = lane >> 3, cc = (lane & 7) * 8;
        const uint4 v = *reinterpret_cast<const uint4*>(&otile[wv][rr * kDwCB + cc]);
        if (r0 + rr < nout && c0 + cc < C) *reinterpret_cast<uint4*>(ys + (int64_t)(t0 + r0 + rr) * C + c0 + cc) = v;
      }
    }
  }
  if (fused_silu) return;   // uniform across the block
  red[0][threadIdx.x] = lsum;
  red[1][threadIdx.x] = lsq;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      red[0][threadIdx.x] += red[0][threadIdx.x + o];
      red[1][threadIdx.x] += red[1][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    partial[((int64_t)s * nblk + blockIdx.x) * 2 + 0] = red[0][0];
    partial[((int64_t)s * nblk + blockIdx.x) * 2 + 1] = red[1][0];
  }
}


// bf16 depthwise conv with the tap count K and the run length R fixed at compile time (the conformer
// kernels 15 and 31): a lane owns a channel PAIR and produces R consecutive output rows, so every tap is
// one packed FMA (v_pk_fma_f32) over the pair, the window element arrives as one 4-B LDS read (the pair's
// bf16x2) + two bit ops, and nothing in the unrolled body branches (the runtime-k kernel above predicates
// every window element).  A wave is two half-waves of 32 pairs = the block's 64 channels; the 8 half-waves
// of the block take runs 0..7 of an 8R-row tile, rows of 128 B so the halves (R odd) read opposite bank
// halves.  The tile's staged rows are all requested before the first LDS store (one HBM latency per
// tile).  Per output element and tap the FMA order is the runtime kernel's (bias, then taps in order),
// so the conv values are bit-identical to it; only the GroupNorm partial sums' summation order differs.
typedef float float2v __attribute__((ext_vector_type(2)));

// R output rows of a half-wave run from the staged rows g[(r0 + i) * 32 + cp] (i < R + K - 1): per tap one packed
// FMA over the lane's channel pair, bias first, taps in order; optional SiLU; bf16 stores of the valid rows and
// their GroupNorm partial sums (lsum, lsq).
template <int K, int R>
__device__ __forceinline__ void dw_run(const uint32_t* g, int r0, int cp, int nout, const float2v (&wr)[K], float2v bv,
                                       bool fused_silu, uint16_t* yrow, int C, float& lsum, float& lsq) {
  float2v acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = bv;
  constexpr int kN = R + K - 1, kPf = 4;   // window elements; LDS reads issued kPf elements ahead
  uint32_t uw[kN];
#pragma unroll
  for (int i = 0; i < kPf; ++i) uw[i] = g[(r0 + i) * 32 + cp];
#pragma unroll
  for (int i = 0; i < kN; ++i) {
    if (i + kPf < kN) uw[i + kPf] = g[(r0 + i + kPf) * 32 + cp];
    const uint32_t u = uw[i];
    const float2v xv = float2v{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int j = i - r;
      if (j >= 0 && j < K) acc[r] = __builtin_elementwise_fma(wr[j], xv, acc[r]);
    }
    // keep the FMAs of one window element together: left alone the scheduler emits each
    // accumulator's 31-FMA dependent chain back to back (a dependency stall per FMA)
#pragma unroll
    for (int r = 0; r < R; ++r) asm volatile("" : "+v"(acc[r]));
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float2v v = acc[r];
    if (fused_silu) v = float2v{v.x * sigmoid_rcp(v.x), v.y * sigmoid_rcp(v.y)};
    if (r < nout) {
      *reinterpret_cast<uint32_t*>(yrow + (int64_t)r * C) = pack_bf16x2(v.x, v.y);
      lsum += v.x + v.y;
      lsq = fmaf(v.x, v.x, lsq);
      lsq = fmaf(v.y, v.y, lsq);
    }
  }
}

// Workgroup barrier for LDS hand-offs only: __syncthreads()' release fence also waits for vmcnt(0), which would
// drain the persistent kernel's next-sequence prefetch at every barrier.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// The block's (sum, sum of squares) over its 256 threads, in the order of a halving tree (t += t + o for
// o = 128 .. 1): the two cross-wave levels through LDS, the six in-wave ones as shfl_down (same operands, same
// association, 2 barriers instead of 8).  Thread 0 stores them at out[0], out[1].
__device__ __forceinline__ void dw_gn_partial(float (&red)[2][256], int tid, float lsum, float lsq, float* out) {
  lds_barrier();   // red may still be read by the previous call's wave 0
  red[0][tid] = lsum;
  red[1][tid] = lsq;
  lds_barrier();
  if (tid < 128) {
    red[0][tid] += red[0][tid + 128];
    red[1][tid] += red[1][tid + 128];
  }
  lds_barrier();
  if (tid < 64) {
    float a = red[0][tid] + red[0][tid + 64], b = red[1][tid] + red[1][tid + 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      a += __shfl_down(a, o, 64);
      b += __shfl_down(b, o, 64);
    }
    if (tid == 0) {
      out[0] = a;
      out[1] = b;
    }
  }
}

// bf16 depthwise conv with the tap count K and the run length R fixed at compile time (the conformer
// kernels 15 and 31): a lane owns a channel PAIR and produces R consecutive output rows, so every tap is
// one packed FMA (v_pk_fma_f32) over the pair, the window element arrives as one 4-B LDS read (the pair's
// bf16x2) + two bit ops, and nothing in the unrolled body branches (the runtime-k kernel above predicates
// every window element).  A wave is two half-waves of 32 pairs = the block's 64 channels; the 8 half-waves
// of the block take runs 0..7 of an 8R-row tile, rows of 128 B so the halves (R odd) read opposite bank
// halves.  The tile's staged rows are all requested before the first LDS store (one HBM latency per
// tile).  Per output element and tap the FMA order is the runtime kernel's (bias, then taps in order),
// so the conv values are bit-identical to it; only the GroupNorm partial sums' summation order differs.
template <int K, int R>
__global__ __launch_bounds__(256) void dwconv_pk_kernel(const uint16_t* __restrict__ x, int T, int C,
                                                        const float* __restrict__ w, const float* __restrict__ bias,
                                                        uint16_t* __restrict__ y, float* __restrict__ partial,
                                                        int fused_silu, int glu_in) {
  constexpr int kRows = 8 * R + K - 1;                  // staged rows per tile
  constexpr int kItems = kRows * 8;                     // 16-B chunks (8 channels) per tile
  constexpr int kIters = (kItems + 255) / 256;
  constexpr int pad = (K - 1) / 2;
  __shared__ uint32_t g[kRows * 32];                    // [row][32 channel pairs] bf16x2
  __shared__ float red[2][256];
  const int s = blockIdx.y, c0 = blockIdx.x * kDwCB, nblk = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int cp = lane & 31, slot = wv * 2 + (lane >> 5);
  const int c = c0 + 2 * cp;                            // C % 64 == 0 (host check): both channels exist
  float2v wr[K];
#pragma unroll
  for (int j = 0; j < K; ++j) wr[j] = float2v{w[(int64_t)c * K + j], w[(int64_t)(c + 1) * K + j]};
  const float2v bv = bias ? float2v{bias[c], bias[c + 1]} : float2v{0.f, 0.f};
  const uint16_t* xs = x + (int64_t)s * T * (glu_in ? 2 : 1) * C;
  uint16_t* ys = y + (int64_t)s * T * C;
  float lsum = 0.f, lsq = 0.f;
  for (int t0 = 0; t0 < T; t0 += 8 * R) {
    uint4 va[kIters], vg[kIters];
#pragma unroll
    for (int u = 0; u < kIters; ++u) {
      const int i = tid + u * 256, tt = i >> 3, ch = (i & 7) * 8, t = t0 - pad + tt;
      va[u] = vg[u] = make_uint4(0u, 0u, 0u, 0u);
      if (i < kItems && t >= 0 && t < T) {
        if (!glu_in) {
          va[u] = *reinterpret_cast<const uint4*>(xs + (int64_t)t * C + c0 + ch);
        } else {
          const int cc = c0 + ch;   // pw1 rows interleaved in 32-column groups [16 values | 16 gates]
          const uint16_t* ra = xs + (int64_t)t * 2 * C + (cc / 16) * 32 + cc % 16;
          va[u] = *reinterpret_cast<const uint4*>(ra);
          vg[u] = *reinterpret_cast<const uint4*>(ra + 16);
        }
      }
    }
    __syncthreads();   // the previous tile's reads of g are done
#pragma unroll
    for (int u = 0; u < kIters; ++u) {
      const int i = tid + u * 256;
      if (i >= kItems) break;
      uint4 o = va[u];
      if (glu_in) {
        const uint32_t aw[4] = {va[u].x, va[u].y, va[u].z, va[u].w}, gw[4] = {vg[u].x, vg[u].y, vg[u].z, vg[u].w};
        uint32_t r[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float a0 = __uint_as_float(aw[q] << 16), a1 = __uint_as_float(aw[q] & 0xffff0000u);
          const float g0 = __uint_as_float(gw[q] << 16), g1 = __uint_as_float(gw[q] & 0xffff0000u);
          r[q] = pack_bf16x2(a0 * sigmoid_rcp(g0), a1 * sigmoid_rcp(g1));
        }
        o = make_uint4(r[0], r[1], r[2], r[3]);
      }
      *reinterpret_cast<uint4*>(g + (i >> 3) * 32 + (i & 7) * 4) = o;
    }
    __syncthreads();
    const int r0 = slot * R, nout = min(8 * R, T - t0) - r0;   // valid rows of this run
    if (nout > 0) dw_run<K, R>(g, r0, cp, nout, wr, bv, fused_silu, ys + (int64_t)(t0 + r0) * C + c, C, lsum, lsq);
  }
  if (fused_silu) return;   // uniform across the block
  dw_gn_partial(red, tid, lsum, lsq, partial + ((int64_t)s * nblk + blockIdx.x) * 2);
}

// The same conv for sequences of one tile (T <= 8R, no GLU input), PERSISTENT: workgroup b keeps channel block
// b % (C / 64) (its taps stay in registers) and walks sequences b / (C / 64), + gridDim.x / (C / 64), ...; the
// next sequence's rows are requested as soon as the current ones are in LDS, so their HBM latency runs under
// the current sequence's taps, stores and GroupNorm sums (the one-tile-per-workgroup kernel above exposes one
// HBM latency per 64 channels x T rows).  Values and partial sums bit-identical to dwconv_pk_kernel.
template <int K, int R>
__global__ __launch_bounds__(256) void dwconv_pp_kernel(const uint16_t* __restrict__ x, int S, int T, int C,
                                                        const float* __restrict__ w, const float* __restrict__ bias,
                                                        uint16_t* __restrict__ y, float* __restrict__ partial,
                                                        int fused_silu) {
  constexpr int kRows = 8 * R + K - 1;
  constexpr int kItems = kRows * 8;
  constexpr int kIters = (kItems + 255) / 256;
  constexpr int pad = (K - 1) / 2;
  __shared__ uint32_t g[kRows * 32];
  __shared__ float red[2][256];
  const int ncb = C / kDwCB, cb = blockIdx.x % ncb, c0 = cb * kDwCB, sstep = gridDim.x / ncb;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int cp = lane & 31, slot = wv * 2 + (lane >> 5);
  const int c = c0 + 2 * cp;
  float2v wr[K];
#pragma unroll
  for (int j = 0; j < K; ++j) wr[j] = float2v{w[(int64_t)c * K + j], w[(int64_t)(c + 1) * K + j]};
  const float2v bv = bias ? float2v{bias[c], bias[c + 1]} : float2v{0.f, 0.f};
  uint4 va[kIters];
  auto fetch = [&](int s) {
    const uint16_t* xs = x + (int64_t)s * T * C + c0;
#pragma unroll
    for (int u = 0; u < kIters; ++u) {
      const int i = tid + u * 256, tt = i >> 3, ch = (i & 7) * 8, t = tt - pad;
      // rows outside [0, T) and chunks past the tile read row 0 (any finite data) and are zeroed below
      const bool in = i < kItems && t >= 0 && t < T;
      va[u] = *reinterpret_cast<const uint4*>(xs + (int64_t)(in ? t : 0) * C + ch);
      if (!in) va[u] = make_uint4(0u, 0u, 0u, 0u);
    }
  };
  int s = blockIdx.x / ncb;
  if (s < S) fetch(s);
  for (; s < S; s += sstep) {
    lds_barrier();   // the previous sequence's reads of g are done
#pragma unroll
    for (int u = 0; u < kIters; ++u) {
      const int i = tid + u * 256;
      if (i < kItems) *reinterpret_cast<uint4*>(g + (i >> 3) * 32 + (i & 7) * 4) = va[u];
    }
    lds_barrier();
    if (s + sstep < S) fetch(s + sstep);   // in flight during this sequence's conv
    float lsum = 0.f, lsq = 0.f;
    const int r0 = slot * R, nout = T - r0;
    if (nout > 0)
      dw_run<K, R>(g, r0, cp, nout, wr, bv, fused_silu, y + ((int64_t)s * T + r0) * C + c, C, lsum, lsq);
    if (!fused_silu) dw_gn_partial(red, tid, lsum, lsq, partial + ((int64_t)s * ncb + cb) * 2);
  }
}

// run length for the packed kernel: the R in {9, 13, 19} that stages the fewest rows over the sequence
static int dwconv_pk_runlen(int T, int K) {
  int best = 0;
  long cost = 0;
  for (int R : {9, 13, 19}) {
    const long c = (long)cdiv(T, 8 * R) * (8 * R + K - 1);
    if (!best || c < cost) best = R, cost = c;
  }
  return best;
}

template <int K>
static void launch_dwconv_pk(int R, dim3 grid, hipStream_t st, const uint16_t* x, int T, int C, const float* w,
                             const float* bias, uint16_t* y, float* partial, int fused_silu, int glu_in) {
  if (R == 9)
    hipLaunchKernelGGL((dwconv_pk_kernel<K, 9>), grid, dim3(256), 0, st, x, T, C, w, bias, y, partial, fused_silu, glu_in);
  else if (R == 13)
    hipLaunchKernelGGL((dwconv_pk_kernel<K, 13>), grid, dim3(256), 0, st, x, T, C, w, bias, y, partial, fused_silu, glu_in);
  else
    hipLaunchKernelGGL((dwconv_pk_kernel<K, 19>), grid, dim3(256), 0, st, x, T, C, w, bias, y, partial, fused_silu, glu_in);
}

// persistent grid: as many workgroups as fit on the device at once, a multiple of the channel blocks
template <int K, int R>
static void launch_dwconv_pp_r(int S, int T, int C, hipStream_t st, const uint16_t* x, const float* w, const float* bias,
                               uint16_t* y, float* partial, int fused_silu) {
  static int resident = 0;
  if (!resident) {
    int dev = 0, cus = 0, per = 0;
    SD_HIP(hipGetDevice(&dev));
    SD_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    SD_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, dwconv_pp_kernel<K, R>, 256, 0));
    resident = std::max(1, cus * std::max(1, per));
  }
  const int ncb = C / kDwCB;
  const int per_cb = std::max(1, std::min(S, resident / ncb));
  hipLaunchKernelGGL((dwconv_pp_kernel<K, R>), dim3(per_cb * ncb), dim3(256), 0, st, x, S, T, C, w, bias, y, partial,
                     fused_silu);
}

template <int K>
static void launch_dwconv_pp(int R, int S, int T, int C, hipStream_t st, const uint16_t* x, const float* w,
                             const float* bias, uint16_t* y, float* partial, int fused_silu) {
  if (R == 9) launch_dwconv_pp_r<K, 9>(S, T, C, st, x, w, bias, y, partial, fused_silu);
  else if (R == 13) launch_dwconv_pp_r<K, 13>(S, T, C, st, x, w, bias, y, partial, fused_silu);
  else launch_dwconv_pp_r<K, 19>(S, T, C, st, x, w, bias, y, partial, fused_silu);
}

void glu_dwconv(const void* x, int S, int T, int C, const float* w, const float* bias, int k,
                void* y, float* partial, bool fused_silu, bool glu_in, bool io_bf16, hipStream_t st) {
  SD_CHECK(fused_silu || partial, kErrInvalid, "glu_dwconv: GroupNorm partials buffer required");
  SD_CHECK(k >= 1 && k <= kDwMaxK && k % 2 == 1, kErrInvalid, "glu_dwconv: kernel size must be odd and <= 31");
  SD_CHECK(C % 16 == 0, kErrInvalid, "glu_dwconv: channels must be a multiple of 16");
  dim3 grid(cdiv(C, kDwCB), S);
  const double eb = io_bf16 ? 2.0 : 4.0;
  ProfScope prof(glu_in ? "glu_dwconv" : "dwconv", 2.0 * S * T * C * k, eb * S * T * (glu_in ? 3.0 : 2.0) * C, st);
  if (io_bf16 && (k == 15 || k == 31) && C % kDwCB == 0 && !glu_in && T <= 8 * 19) {
    auto xp = reinterpret_cast<const uint16_t*>(x);
    auto yp = reinterpret_cast<uint16_t*>(y);
    const int R = T <= 8 * 9 ? 9 : T <= 8 * 13 ? 13 : 19;
    if (k == 31) launch_dwconv_pp<31>(R, S, T, C, st, xp, w, bias, yp, partial, (int)fused_silu);
    else launch_dwconv_pp<15>(R, S, T, C, st, xp, w, bias, yp, partial, (int)fused_silu);
  } else if (io_bf16 && (k == 15 || k == 31) && C % kDwCB == 0) {
    const int R = dwconv_pk_runlen(T, k);
    auto xp = reinterpret_cast<const uint16_t*>(x);
    auto yp = reinterpret_cast<uint16_t*>(y);
    if (k == 31) launch_dwconv_pk<31>(R, grid, st, xp, T, C, w, bias, yp, partial, (int)fused_silu, (int)glu_in);
    else launch_dwconv_pk<15>(R, grid, st, xp, T, C, w, bias, yp, partial, (int)fused_silu, (int)glu_in);
  } else if (io_bf16)
    hipLaunchKernelGGL(glu_dwconv_kernel<true>, grid, dim3(256), 0, st, reinterpret_cast<const uint16_t*>(x), T,
                       C, w, bias, k, reinterpret_cast<uint16_t*>(y), partial, (int)fused_silu, (int)glu_in);
  else
    hipLaunchKernelGGL(glu_dwconv_kernel<false>, grid, dim3(256), 0, st, reinterpret_cast<const float*>(x), T, C,
                       w, bias, k, reinterpret_cast<float*>(y), partial, (int)fused_silu, (int)glu_in);
  SD_LAUNCH_CHECK();
}

// GroupNorm(1 group) statistics from the dwconv partials, then y = silu(GN(y)) in place.
// Each thread owns 8 consecutive channels of a row (one 16-B bf16 / 2 x 16-B fp32 access);
// a sequence's T x C elements are split over kGnBlocks workgroups.
constexpr int kGnBlocks = 4;

template <bool BF>
__global__ __launch_bounds__(256) void groupnorm_silu_kernel(act_t<BF>* __restrict__ y, int T, int C,
                                                             const float* __restrict__ partial, int nblk,
                                                             const float* __restrict__ g,
                                                             const float* __restrict__ b, float eps) {
  const int s = blockIdx.y;
  double sum = 0.0, sq = 0.0;
  for (int i = 0; i < nblk; ++i) {
    sum += partial[((int64_t)s * nblk + i) * 2];
    sq += partial[((int64_t)s * nblk + i) * 2 + 1];
  }
  const double n = (double)T * C;
  const double mean = sum / n;
  double var = sq / n - mean * mean;
  if (var < 0) var = 0;
  const float fm = (float)mean;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  act_t<BF>* ys = y + (int64_t)s * T * C;
  const int cv = C / 8;                         // 8-channel vectors per row
  const int nvec = T * cv;
  const int per = (nvec + gridDim.x - 1) / gridDim.x;
  const int v0 = blockIdx.x * per, v1 = min(nvec, v0 + per);
  for (int v = v0 + threadIdx.x; v < v1; v += blockDim.x) {
    const int c = (v % cv) * 8;
    act_t<BF>* p = ys + (int64_t)v * 8;
    float x[8];
    if constexpr (BF) {
      const uint4 u = *reinterpret_cast<const uint4*>(p);
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        x[2 * i] = __uint_as_float(w[i] << 16);
        x[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
      }
    } else {
      const float4 a = *reinterpret_cast<const float4*>(p), bq = *reinterpret_cast<const float4*>(p + 4);
      x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w; x[4] = bq.x; x[5] = bq.y; x[6] = bq.z; x[7] = bq.w;
    }
    const float4 g0 = *reinterpret_cast<const float4*>(g + c), g1 = *reinterpret_cast<const float4*>(g + c + 4);
    const float4 b0 = *reinterpret_cast<const float4*>(b + c), b1 = *reinterpret_cast<const float4*>(b + c + 4);
    const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float t = (x[i] - fm) * rstd * gg[i] + bb[i];
      x[i] = t * sigmoid_rcp(t);
    }
    if constexpr (BF) {
      const uint4 u = {pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3]), pack_bf16x2(x[4], x[5]),
                       pack_bf16x2(x[6], x[7])};
      *reinterpret_cast<uint4*>(p) = u;
    } else {
      *reinterpret_cast<float4*>(p) = make_float4(x[0], x[1], x[2], x[3]);
      *reinterpret_cast<float4*>(p + 4) = make_float4(x[4], x[5], x[6], x[7]);
    }
  }
}

void groupnorm_silu(void* y, int S, int T, int C, const float* partial, const float* g,
                    const float* b, float eps, bool io_bf16, hipStream_t st) {
  SD_CHECK(C % 8 == 0, kErrInvalid, "groupnorm_silu: channels must be a multiple of 8");
  int nblk = cdiv(C, kDwCB);
  dim3 grid(kGnBlocks, S);
  ProfScope prof("groupnorm_silu", 0.0, (io_bf16 ? 4.0 : 8.0) * S * T * C, st);
  if (io_bf16)
    hipLaunchKernelGGL(groupnorm_silu_kernel<true>, grid, dim3(256), 0, st, reinterpret_cast<uint16_t*>(y), T,
                       C, partial, nblk, g, b, eps);
  else
    hipLaunchKernelGGL(groupnorm_silu_kernel<false>, grid, dim3(256), 0, st, reinterpret_cast<float*>(y), T,
                       C, partial, nblk, g, b, eps);
  SD_LAUNCH_CHECK();
}

// ------------------------------------------------------------------ window CMN
__global__ __launch_bounds__(256) void window_cmn_kernel(const float* __restrict__ feats, int n_mels,
                                                         const int* __restrict__ win_start,
                                                         const int* __restrict__ win_n, int T_out,
                                                         float* __restrict__ out) {
  __shared__ double part[4][128];
  __shared__ float mean[128];
  const int w = blockIdx.x;
  const int start = win_start[w];
  const int n = win_n[w];
  const int c = threadIdx.x & 127;
  const int q = threadIdx.x >> 7;   // 0..1
  if (c < n_mels) {
    // rows j = q, q + 2, ... in order (the sum's association is unchanged); their loads issued 8 at a time
    // (the plain loop waited on each load: ~300 dependent round trips per window)
    double acc = 0.0;
    const float* fc = feats + (int64_t)start * n_mels + c;
    int j = q;
    for (; j + 14 < n; j += 16) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = fc[(int64_t)(j + 2 * u) * n_mels];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; j < n; j += 2) acc += fc[(int64_t)j * n_mels];
    part[q][c] = acc;
  }
  __syncthreads();
  if (threadIdx.x < n_mels) mean[threadIdx.x] = (float)((part[0][threadIdx.x] + part[1][threadIdx.x]) / (double)n);
  __syncthreads();
  float* o = out + (int64_t)w * T_out * n_mels;
  if ((n_mels & 3) == 0) {
    // float4 units (n_mels % 4 == 0: the window rows and the output stay 16-B aligned)
    const int m4 = n_mels >> 2;
    const int64_t total4 = (int64_t)T_out * m4;
    const float4* f4 = reinterpret_cast<const float4*>(feats + (int64_t)start * n_mels);
    float4* o4 = reinterpret_cast<float4*>(o);
    for (int64_t i = threadIdx.x; i < total4; i += blockDim.x) {
      const int j = (int)(i / m4), c4 = (int)(i - (int64_t)j * m4) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (j < n) {
        const float4 x = f4[i];
        v = make_float4(x.x - mean[c4], x.y - mean[c4 + 1], x.z - mean[c4 + 2], x.w - mean[c4 + 3]);
      }
      o4[i] = v;
    }
    return;
  }
  const int64_t total = (int64_t)T_out * n_mels;
  for (int64_t i = threadIdx.x; i < total; i += blockDim.x) {
    int j = i / n_mels, cc = i % n_mels;
    o[i] = j < n ? feats[((int64_t)start + j) * n_mels + cc] - mean[cc] : 0.f;
  }
}

void window_cmn(const float* feats, int n_mels, const int* win_start, const int* win_n, int n_win,
                int T_out, float* out, hipStream_t st) {
  SD_CHECK(n_mels <= 128, kErrInvalid, "window_cmn: n_mels > 128");
  hipLaunchKernelGGL(window_cmn_kernel, dim3(n_win), dim3(256), 0, st, feats, n_mels, win_start,
                     win_n, T_out, out);
  SD_LAUNCH_CHECK();
}

}  // namespace sd

namespace sd {

// Torch conv/linear weight (N, Cin, taps) -> Wt[N][tap*Cin + c] (fp32 or bf16 bits).
__global__ void pack_weight_kernel(const float* __restrict__ w, int N, int Cin, int taps,
                                   void* __restrict__ out, int bf16) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = (int64_t)N * Cin * taps;
  if (i >= total) return;
  int tp = i % taps;
  int64_t r = i / taps;
  int c = r % Cin;
  int n = r / Cin;
  int64_t o = ((int64_t)n * taps + tp) * Cin + c;
  if (bf16) reinterpret_cast<uint16_t*>(out)[o] = f2bf_bits(w[i]);
  else reinterpret_cast<float*>(out)[o] = w[i];
}

void pack_weight(const float* w, int N, int Cin, int taps, void* out, bool bf16, hipStream_t st) {
  int64_t total = (int64_t)N * Cin * taps;
  hipLaunchKernelGGL(pack_weight_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, w,
                     N, Cin, taps, out, bf16 ? 1 : 0);
  SD_LAUNCH_CHECK();
}

}  // namespace sd

namespace sd {

// Overlap-average of window posteriors (ts_vad2/infer.py:90-94 np.mean over the
// windows covering a frame, in window order) with the sigmoid of model.py:945-946
// fused.  logits: (n_win, NS, Tw); window w covers label frames
// [start_w, start_w + len_w).  out: (NS, n_frames); frames no window covers -> NaN.
//
// np.mean over a float32 list is numpy's float32 add.reduce followed by one correctly rounded
// float32 division.  The reduction is numpy's pairwise summation (umath loops, pairwise_sum):
// n < 8 values are summed from 0 in order; 8 <= n <= 128 go into 8 accumulators r[j] = v[j],
// r[j] += v[i + j] for each full group of 8, combined as ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)),
// then the n % 8 tail is added in order; n > 128 splits at n2 = n/2 rounded down to a multiple
// of 8 and adds the two halves' sums.  Reproduced exactly (adds only, __fadd_rn: no FMA can
// form), so the result is bit-identical to numpy for the same probabilities.
struct OverlapList {     // the covering windows of one (frame, speaker), in window order
  const float* logits;
  const int* start;
  const int* len;
  int64_t stride;        // NS * Tw
  int64_t base;          // spk * Tw + t
  int t, w_lo, w_hi;
  int first;             // first covering window
  bool contiguous;       // covering windows form [first, first + n)
};

template <bool kSigmoid>
__device__ __forceinline__ float ol_value(const OverlapList& L, int w) {
  const float x = L.logits[(int64_t)w * L.stride + L.base - L.start[w]];
  return kSigmoid ? 1.f / (1.f + expf(-x)) : x;
}

template <bool kSigmoid>
__device__ __forceinline__ float ol_at(const OverlapList& L, int k) {   // k-th covering value
  if (L.contiguous) return ol_value<kSigmoid>(L, L.first + k);
  for (int w = L.first; w <= L.w_hi; ++w) {
    const int off = L.t - L.start[w];
    if (off < 0 || off >= L.len[w]) continue;
    if (k-- == 0) return ol_value<kSigmoid>(L, w);
  }
  return 0.f;
}

template <bool kSigmoid>
__device__ float ol_block_sum(const OverlapList& L, int k0, int n) {     // n <= 128
  if (n < 8) {
    float s = 0.f;
    for (int k = 0; k < n; ++k) s = __fadd_rn(s, ol_at<kSigmoid>(L, k0 + k));
    return s;
  }
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = ol_at<kSigmoid>(L, k0 + j);
  int k = 8;
  for (; k < n - (n % 8); k += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = __fadd_rn(r[j], ol_at<kSigmoid>(L, k0 + k + j));
  }
  float s = __fadd_rn(__fadd_rn(__fadd_rn(r[0], r[1]), __fadd_rn(r[2], r[3])),
                      __fadd_rn(__fadd_rn(r[4], r[5]), __fadd_rn(r[6], r[7])));
  for (; k < n; ++k) s = __fadd_rn(s, ol_at<kSigmoid>(L, k0 + k));
  return s;
}

// numpy's recursion for n > 128, unrolled by depth (kDepth levels cover n <= 128 << kDepth;
// the host rejects geometries with more windows per frame than that).
template <bool kSigmoid, int kDepth>
__device__ __attribute__((noinline)) float ol_pairwise(const OverlapList& L, int k0, int n) {
  if constexpr (kDepth == 0) {
    return ol_block_sum<kSigmoid>(L, k0, n);
  } else {
    if (n <= 128) return ol_block_sum<kSigmoid>(L, k0, n);
    int n2 = n / 2;
    n2 -= n2 % 8;
    return __fadd_rn(ol_pairwise<kSigmoid, kDepth - 1>(L, k0, n2),
                     ol_pairwise<kSigmoid, kDepth - 1>(L, k0 + n2, n - n2));
  }
}

template <bool kSigmoid>
__global__ void overlap_average_kernel(const float* __restrict__ logits, int n_win, int NS, int Tw,
                                       const int* __restrict__ start, const int* __restrict__ len,
                                       int dis, int chunk, int n_frames, float* __restrict__ out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)NS * n_frames) return;
  const int t = i % n_frames;
  const int spk = i / n_frames;
  int w_lo = (t - chunk + 1 + dis - 1);
  w_lo = w_lo > 0 ? w_lo / dis : 0;
  const int w_hi = min(n_win - 1, t / dis);
  int cnt = 0, first = -1, last = -1;
  for (int w = w_lo; w <= w_hi; ++w) {
    const int off = t - start[w];
    if (off < 0 || off >= len[w]) continue;
    if (first < 0) first = w;
    last = w;
    ++cnt;
  }
  if (cnt == 0) {
    out[i] = __int_as_float(0x7fc00000);
    return;
  }
  OverlapList L{logits, start, len, (int64_t)NS * Tw, (int64_t)spk * Tw + t, t, w_lo, w_hi, first,
                last - first + 1 == cnt};
  const float s = cnt <= 128 ? ol_block_sum<kSigmoid>(L, 0, cnt)
                             : ol_pairwise<kSigmoid, kOverlapMaxDepth>(L, 0, cnt);
  out[i] = __fdiv_rn(s, (float)cnt);
}

void overlap_average(const float* logits, int n_win, int NS, int Tw, const int* start, const int* len,
                     int dis, int chunk, int n_frames, float* out, hipStream_t st, bool sigmoid) {
  int64_t total = (int64_t)NS * n_frames;
  if (total == 0) return;
  auto k = sigmoid ? overlap_average_kernel<true> : overlap_average_kernel<false>;
  hipLaunchKernelGGL(k, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     logits, n_win, NS, Tw, start, len, dis, chunk, n_frames, out);
  SD_LAUNCH_CHECK();
}

}  // namespace sd

namespace sd {

__global__ void f32_to_bf16_kernel(const float* __restrict__ x, int64_t n, uint16_t* __restrict__ y) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = f2bf_bits(x[i]);
}

void f32_to_bf16(const float* x, int64_t n, void* y, hipStream_t st) {
  if (n == 0) return;
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, n,
                     reinterpret_cast<uint16_t*>(y));
  SD_LAUNCH_CHECK();
}

__global__ void bf16_to_f32_kernel(const uint16_t* __restrict__ x, int64_t n, float* __restrict__ y) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = bf_bits2f(x[i]);
}

void bf16_to_f32(const void* x, int64_t n, float* y, hipStream_t st) {
  if (n == 0) return;
  hipLaunchKernelGGL(bf16_to_f32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     reinterpret_cast<const uint16_t*>(x), n, y);
  SD_LAUNCH_CHECK();
}

}  // namespace sd
