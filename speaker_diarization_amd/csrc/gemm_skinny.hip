// Skinny GEMM (M <= 16 output rows) for the streaming FS-EEND chunks on gfx950.
//
// A chunk of c frames turns every linear layer into an (c or c*C rows) x K x N product:
// the weights (N*K) dominate the bytes, an MFMA tile of 64-128 rows would be >90 % padding,
// and the tile kernels give each workgroup a 128-column panel -> 2-16 workgroups for
// N = 256..2048.  Here the A rows (M*K, a few KB) are staged once per workgroup in LDS as
// fp32, and each wave streams NC weight rows (16-B loads, coalesced along K) against them,
// so the grid has N/NC waves and the kernel runs at the weight-streaming rate.  The
// look-ahead Conv1d (k 19, stride 1, no padding in the streaming window) is the same
// product: output row m's im2col row is the contiguous span A[m*Cin, m*Cin + 19*Cin).
//
// Epilogue = conv_gemm's: v = acc*alpha[n] + beta[n] (+res[m*res_ld + n]), activation,
// out[b*o_sb + ho*o_sh + wo*o_sw + n*o_sn] (fp32 or bf16).  fp32 arithmetic throughout.
#include <algorithm>

#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {
namespace {

constexpr int kSkinnyLdsFloats = 16384;   // 64 KiB of staged A

template <int NC, bool WBF>
__device__ __forceinline__ void skinny_load(const ConvGemmArgs& p, int n0, int kv0, int nv, uint4 (&w)[NC][4]) {
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const int64_t row = (int64_t)min(n0 + j, p.N - 1) * p.K;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int kv = kv0 + b * 64;
      if (kv < nv) {
        if constexpr (WBF) w[j][b] = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(p.Wt) + row + kv * 8);
        else w[j][b] = *reinterpret_cast<const uint4*>(static_cast<const float*>(p.Wt) + row + kv * 4);
      } else {
        w[j][b] = make_uint4(0u, 0u, 0u, 0u);
      }
    }
  }
}

// Staging of n float4 units over the 256 threads, loads issued in batches of 8 per thread before any is stored
// (one memory round trip per batch; a plain strided loop waits on each load or is unrolled with a remainder
// loop that does).  ld(i) -> float4 for unit i, st(i, v); both called with i clamped to n - 1.
template <class Ld, class St>
__device__ __forceinline__ void stage4(int n, int tid, Ld ld, St st) {
  for (int i0 = tid; i0 < n; i0 += 8 * 256) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = ld(min(i0 + u * 256, n - 1));
    // units past n store unit n - 1's value again (unconditional stores: a store under a branch lets the
    // compiler sink its load behind the branch, one round trip per unit again)
#pragma unroll
    for (int u = 0; u < 8; ++u) st(min(i0 + u * 256, n - 1), v[u]);
  }
}

template <int MMAX, int NC, bool WBF>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(ConvGemmArgs p, int M, int a_rs) {
  extern __shared__ float As[];
  constexpr int VE = WBF ? 8 : 4;   // weight elements per 16-B load
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int K = p.K, nv = K / VE;
  const int n0 = (blockIdx.x * 4 + wid) * NC;
  const bool active = n0 < p.N;
  // Issue the first weight batch and the epilogue operands before staging A, so their
  // latency overlaps the staging round trip.
  uint4 cur[NC][4];
  if (active) skinny_load<NC, WBF>(p, n0, lane, nv, cur);
  const int me = lane / NC, mj = lane % NC, mn = min(n0 + mj, p.N - 1);
  const bool owner = active && me < M && n0 + mj < p.N;
  float ea = 1.f, eb = 0.f, er = 0.f;
  if (owner) {
    if (p.alpha) ea = p.alpha[mn];
    if (p.beta) eb = p.beta[mn];
    if (p.res)
      er = p.res_bf16 ? bf_bits2f(static_cast<const uint16_t*>(p.res)[(int64_t)me * p.res_ld + mn])
                      : static_cast<const float*>(p.res)[(int64_t)me * p.res_ld + mn];
  }
  const int span = (M - 1) * a_rs + K;
  if (p.ln_g) {
    // LayerNorm prologue (post-LN residual of the previous sub-block), one wave per row
    for (int m = wid; m < M; m += 4) {
      const float* xr = p.ln_x + (int64_t)m * K;
      float4 v[4];
      float sum = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = i * 256 + lane * 4;
        if (c < K) {
          float4 a = *reinterpret_cast<const float4*>(xr + c);
          if (p.ln_t) {
            if (p.ln_t_bf16) {
              const uint2 u = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(p.ln_t) + (int64_t)m * K + c);
              a.x += __uint_as_float(u.x << 16); a.y += __uint_as_float(u.x & 0xffff0000u);
              a.z += __uint_as_float(u.y << 16); a.w += __uint_as_float(u.y & 0xffff0000u);
            } else {
              const float4 u = *reinterpret_cast<const float4*>(static_cast<const float*>(p.ln_t) + (int64_t)m * K + c);
              a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
            }
          }
          v[i] = a;
          sum += (a.x + a.y) + (a.z + a.w);
        }
      }
      const float mean = warp_sum(sum) / (float)K;
      float q = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i * 256 + lane * 4 < K) {
          const float dx = v[i].x - mean, dy = v[i].y - mean, dz = v[i].z - mean, dw = v[i].w - mean;
          q += (dx * dx + dy * dy) + (dz * dz + dw * dw);
        }
      }
      const float rstd = rsqrtf(warp_sum(q) / (float)K + p.ln_eps);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = i * 256 + lane * 4;
        if (c < K) {
          const float4 gg = *reinterpret_cast<const float4*>(p.ln_g + c);
          const float4 bb = *reinterpret_cast<const float4*>(p.ln_b + c);
          float4 y;
          y.x = (v[i].x - mean) * rstd * gg.x + bb.x;
          y.y = (v[i].y - mean) * rstd * gg.y + bb.y;
          y.z = (v[i].z - mean) * rstd * gg.z + bb.z;
          y.w = (v[i].w - mean) * rstd * gg.w + bb.w;
          *reinterpret_cast<float4*>(As + m * K + c) = y;
          if (blockIdx.x == 0) *reinterpret_cast<float4*>(p.ln_out + (int64_t)m * K + c) = y;
        }
      }
    }
  } else if (p.pro_mode == 1) {
    // row_l2norm (fseend_ops.hip) per row: lane + 64 j elements, fmaf sum of squares in j order, warp sum
    for (int m = wid; m < M; m += 4) {
      const float* xr = p.ln_x + (int64_t)m * K;
      float v[8];
      float sq = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = lane + 64 * j;
        v[j] = i < K ? xr[i] : 0.f;
        sq = fmaf(v[j], v[j], sq);
      }
      const float nrm = sqrtf(warp_sum(sq));
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = lane + 64 * j;
        if (i < K) {
          const float y = v[j] / nrm;
          As[m * K + i] = y;
          if (blockIdx.x == 0) p.ln_out[(int64_t)m * K + i] = y;
        }
      }
    }
  } else if (p.pro_mode == 2) {
    // slot_init: row r = t * C + c is ln_x[t] + pro_p[c] (float4 units, K % 8 == 0)
    const int kv4 = K / 4;
    stage4(M * kv4, tid, [&](int i) {
      const int r = i / kv4, d = (i - r * kv4) * 4;
      const float4 x = *reinterpret_cast<const float4*>(p.ln_x + (int64_t)(r / p.pro_C) * K + d);
      const float4 b = *reinterpret_cast<const float4*>(p.pro_p + (int64_t)(r % p.pro_C) * K + d);
      return make_float4(x.x + b.x, x.y + b.y, x.z + b.z, x.w + b.w);
    }, [&](int i, float4 y) {
      *reinterpret_cast<float4*>(As + 4 * i) = y;
      if (blockIdx.x == 0) *reinterpret_cast<float4*>(p.ln_out + 4 * (int64_t)i) = y;
    });
  } else if (p.pro_mode == 3) {
    // gather_window: staged row r is history row *cursor - pad + r, zero outside [0, *n_valid)
    // (float4 units: lda % 4 == 0; rows outside read a clamped row and are replaced by zeros)
    const int base = *p.pro_cursor - p.pro_pad, nv = *p.pro_nvalid, ld4 = p.lda / 4;
    stage4(span / 4, tid, [&](int i) {
      const int r = i / ld4, d = (i - r * ld4) * 4;
      const int src = base + r;
      const float4 v = *reinterpret_cast<const float4*>(p.ln_x + (int64_t)min(max(src, 0), max(nv - 1, 0)) * p.lda + d);
      return (src >= 0 && src < nv) ? v : make_float4(0.f, 0.f, 0.f, 0.f);
    }, [&](int i, float4 y) { *reinterpret_cast<float4*>(As + 4 * i) = y; });
  } else if (p.a_bf16) {
    // 4 bf16 (8 B) per unit: a_coff % 4 == 0, span % 4 == 0
    const uint2* a = reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(p.A) + p.a_coff);
    stage4(span / 4, tid, [&](int i) {
      const uint2 u = a[i];
      return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                         __uint_as_float(u.y & 0xffff0000u));
    }, [&](int i, float4 y) { *reinterpret_cast<float4*>(As + 4 * i) = y; });
  } else {
    const float4* a = reinterpret_cast<const float4*>(static_cast<const float*>(p.A) + p.a_coff);
    stage4(span / 4, tid, [&](int i) { return a[i]; },
           [&](int i, float4 y) { *reinterpret_cast<float4*>(As + 4 * i) = y; });
  }
  __syncthreads();
  if (!active) return;
  float acc[MMAX][NC];
#pragma unroll
  for (int m = 0; m < MMAX; ++m)
#pragma unroll
    for (int j = 0; j < NC; ++j) acc[m][j] = 0.f;
  for (int kv0 = lane; kv0 < nv; kv0 += 256) {
    uint4 nxt[NC][4];
    const bool more = kv0 + 256 < nv;
    if (more) skinny_load<NC, WBF>(p, n0, kv0 + 256, nv, nxt);   // next batch in flight during the FMAs
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int kv = kv0 + b * 64;
      if (kv < nv) {
        float w[NC][VE];
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          const uint32_t q[4] = {cur[j][b].x, cur[j][b].y, cur[j][b].z, cur[j][b].w};
          if constexpr (WBF) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              w[j][2 * e] = __uint_as_float(q[e] << 16);
              w[j][2 * e + 1] = __uint_as_float(q[e] & 0xffff0000u);
            }
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) w[j][e] = __uint_as_float(q[e]);
          }
        }
#pragma unroll
        for (int m = 0; m < MMAX; ++m) {
          if (m < M) {
            const float* ar = As + m * a_rs + kv * VE;
            float av[VE];
#pragma unroll
            for (int e = 0; e < VE; e += 4) {
              const float4 t = *reinterpret_cast<const float4*>(ar + e);
              av[e] = t.x; av[e + 1] = t.y; av[e + 2] = t.z; av[e + 3] = t.w;
            }
#pragma unroll
            for (int j = 0; j < NC; ++j)
#pragma unroll
              for (int e = 0; e < VE; ++e) acc[m][j] = fmaf(av[e], w[j][e], acc[m][j]);
          }
        }
      }
    }
    if (more) {
#pragma unroll
      for (int j = 0; j < NC; ++j)
#pragma unroll
        for (int b = 0; b < 4; ++b) cur[j][b] = nxt[j][b];
    }
  }
  // reduce over the wave; lane (m*NC + j) owns element (m, n0 + j)
  float mine = 0.f;
#pragma unroll
  for (int m = 0; m < MMAX; ++m) {
    if (m < M) {
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        const float s = warp_sum(acc[m][j]);
        if (lane == m * NC + j) mine = s;
      }
    }
  }
  if (!owner) return;
  float v = apply_act(mine * ea + eb + er, p.act);
  const int hw = p.Ho * p.Wo;
  const int b = me / hw, r = me % hw, ho = r / p.Wo, wo = r % p.Wo;
  const int64_t o = (int64_t)b * p.o_sb + (int64_t)ho * p.o_sh + (int64_t)wo * p.o_sw + (int64_t)mn * p.o_sn;
  if (p.out_bf16) static_cast<uint16_t*>(p.out)[o] = f2bf_bits(v);
  else static_cast<float*>(p.out)[o] = v;
  if (p.kv_out && mn >= p.kv_col0) {
    const int64_t ko = ((int64_t)(*p.kv_cursor) * p.kv_mult + me) * p.kv_ld + (mn - p.kv_col0);
    if (p.out_bf16) static_cast<uint16_t*>(p.kv_out)[ko] = f2bf_bits(v);
    else static_cast<float*>(p.kv_out)[ko] = v;
  }
}

// A(m, k) = A[a_coff + m*a_rs + k]: a plain linear (row stride lda), or a stride-1
// unpadded 1-D conv whose taps are consecutive rows (Cin == lda).
int skinny_row_stride(const ConvGemmArgs& p) {
  if (p.ln_g || p.pro_mode == 1 || p.pro_mode == 2) return p.K;   // prologue rows of K built in LDS
  if (a_rows_linear(p)) return p.lda;
  if (p.B == 1 && p.H == 1 && p.Ho == 1 && p.kh == 1 && p.sw == 1 && p.dw == 1 && p.pw == 0 && p.ph == 0 &&
      p.Cin == p.lda && p.W >= p.Wo + p.kw - 1)
    return p.lda;
  return -1;
}

template <int MMAX, int NC>
void launch_skinny(const ConvGemmArgs& p, int M, int rs, bool wbf, hipStream_t st) {
  const int span = (M - 1) * rs + p.K;
  const size_t lds = (size_t)span * sizeof(float);
  const dim3 grid(cdiv(p.N, 4 * NC));
  static bool attr_set[2] = {false, false};   // once per instantiation, before any graph capture
  if (!attr_set[wbf]) {
    SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_skinny_kernel<MMAX, NC, true>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, kSkinnyLdsFloats * 4));
    SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_skinny_kernel<MMAX, NC, false>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, kSkinnyLdsFloats * 4));
    attr_set[wbf] = true;
  }
  if (wbf) {
    hipLaunchKernelGGL((gemm_skinny_kernel<MMAX, NC, true>), grid, dim3(256), lds, st, p, M, rs);
  } else {
    hipLaunchKernelGGL((gemm_skinny_kernel<MMAX, NC, false>), grid, dim3(256), lds, st, p, M, rs);
  }
  SD_LAUNCH_CHECK();
}

}  // namespace

bool gemm_skinny_supported(const ConvGemmArgs& p) {
  const int M = p.B * p.Ho * p.Wo;
  if (M < 1 || M > 16 || p.pre_scale || p.gate || p.glu) return false;
  if (p.K % 8 != 0) return false;
  const int rs = skinny_row_stride(p);
  if (rs < 0) return false;
  if (((int64_t)(M - 1) * rs + p.K) > kSkinnyLdsFloats) return false;
  if (p.ln_g && (p.K % 256 != 0 || p.K > 1024 || !p.ln_x || !p.ln_b || !p.ln_out || p.ln_out == p.ln_x))
    return false;
  if (p.pro_mode != 0) {
    if (p.ln_g || !p.ln_x || p.a_bf16) return false;
    if (p.pro_mode == 1 && (p.K > 512 || !p.ln_out || p.ln_out == p.ln_x || !a_rows_linear(p) || p.lda != p.K))
      return false;
    if (p.pro_mode == 2 && (!p.pro_p || p.pro_C < 1 || !p.ln_out || p.ln_out == p.ln_x || !a_rows_linear(p) ||
                            p.lda != p.K))
      return false;
    if (p.pro_mode == 3 && (!p.pro_cursor || !p.pro_nvalid)) return false;
    if (p.pro_mode > 3) return false;
  }
  // the vectorised staging: 16-B (fp32) / 8-B (bf16) A units, 16-B prologue rows
  auto al = [](const void* q, int b) { return reinterpret_cast<uintptr_t>(q) % b == 0; };
  if (p.pro_mode == 0 && !p.ln_g && !al(p.A, p.a_bf16 ? 8 : 16)) return false;
  if ((p.pro_mode == 2 || p.pro_mode == 3) && !al(p.ln_x, 16)) return false;
  if (p.pro_mode == 2 && !al(p.pro_p, 16)) return false;
  return p.a_coff % 4 == 0 && rs % 4 == 0;
}

void conv_gemm_skinny(const ConvGemmArgs& p, bool wbf, hipStream_t st) {
  const int M = p.B * p.Ho * p.Wo;
  const int rs = skinny_row_stride(p);
  ProfScope prof(wbf ? "gemm_skinny_bf16" : "gemm_skinny_f32", 2.0 * M * p.N * (double)p.K,
                 (wbf ? 2.0 : 4.0) * p.N * p.K + 4.0 * M * (p.K + p.N), st);
  // 4 weight rows per wave once there are >= 512 waves' worth of columns, else 1.
  const bool nc4 = p.N >= 2048;
  if (M == 1) {
    if (nc4) launch_skinny<1, 4>(p, M, rs, wbf, st); else launch_skinny<1, 1>(p, M, rs, wbf, st);
  } else if (M <= 8) {
    if (nc4) launch_skinny<8, 4>(p, M, rs, wbf, st); else launch_skinny<8, 1>(p, M, rs, wbf, st);
  } else {
    if (nc4) launch_skinny<16, 4>(p, M, rs, wbf, st); else launch_skinny<16, 1>(p, M, rs, wbf, st);
  }
}

}  // namespace sd
