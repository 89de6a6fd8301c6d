// Fused multi-head self-attention core (softmax(q·kᵀ·scale + mask)·v) for gfx950.
//
// Flash-style: per workgroup 64 queries (4 waves x 16), key/value tiles of 32
// keys staged in LDS, online softmax in registers.  The score tile is computed
// SWAPPED (Sᵀ = K·Qᵀ), so each lane holds the scores of ONE query for 8 keys:
// the row max/sum need only two cross-lane steps, and P feeds the P·V MFMA as
// its A operand straight from registers (the MFMA k-slot order is permuted to
// match, and V is read with the same permutation).
//
// Serves nn.TransformerEncoderLayer / nn.MultiheadAttention in
//   ts_vad2/model.py:238-246,335-343 (TS-VAD per-speaker / multi-speaker encoders)
//   torchaudio Conformer self_attn (ts_vad2/model.py:259-267)
//   eend_eda/models.py:193-194, fs_eend/fs_eend.py:163-171 (causal mask).
#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {
namespace {

constexpr int kQB = 64;   // queries per block
constexpr int kKT = 32;   // keys per tile

constexpr int f32_stride(int hd) { return hd + (((4 - hd) % 32) + 32) % 32; }

template <bool BF16, int HD, bool IOBF>
__global__ __launch_bounds__(256) void attn_kernel(AttnArgs a) {
  using io_t = act_t<IOBF>;
  constexpr int HDP = BF16 ? ((HD + 31) / 32) * 32 : HD;   // padded head dim for bf16 k-chunks
  constexpr int KS_BF = HDP + 8;                           // bf16 K row stride
  constexpr int VT_BF = kKT + 8;                           // bf16 Vᵀ row stride
  constexpr int FS = f32_stride(HD);                       // fp32 K/V row stride
  constexpr int DT = HD / 16;                              // output d-subtiles
  static_assert(HD % 16 == 0, "head dim must be a multiple of 16");

  __shared__ __attribute__((aligned(16))) uint16_t Kb[BF16 ? kKT * KS_BF : 1];
  __shared__ __attribute__((aligned(16))) uint16_t Vtb[BF16 ? HDP * VT_BF : 1];
  __shared__ __attribute__((aligned(16))) float Kf[BF16 ? 1 : kKT * FS];
  __shared__ __attribute__((aligned(16))) float Vf[BF16 ? 1 : kKT * FS];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int g = lane >> 4;
  const int l15 = lane & 15;
  const int sh = blockIdx.y;
  const int s = sh / a.nh;
  const int h = sh % a.nh;
  const int T = a.T;
  const int q0 = blockIdx.x * kQB + wid * 16;
  const int myq = q0 + l15;
  const int D = a.D;
  const int64_t row0 = (int64_t)(s / a.seq_inner) * (a.seq_outer ? a.seq_outer : (int64_t)T) +
                       (int64_t)(s % a.seq_inner) * a.seq_inner_stride;
  const int64_t tstr = (int64_t)a.tok_stride * a.ld_qkv;   // elements between consecutive tokens
  const io_t* base = reinterpret_cast<const io_t*>(a.qkv) + row0 * a.ld_qkv;
  const int klen = a.key_len ? min(a.key_len[s], T) : T;

  // Q operand (B operand of Sᵀ = K·Qᵀ), pre-scaled.
  constexpr int QN = BF16 ? HDP / 32 : HD / 4;
  typename std::conditional<BF16, bf16x8, float>::type qf[QN];
  {
    const io_t* qr = base + (int64_t)min(myq, T - 1) * tstr + h * HD;
    const bool qv = myq < T;
    if constexpr (BF16) {
#pragma unroll
      for (int kc = 0; kc < QN; ++kc) {
        bf16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          int d = kc * 32 + g * 8 + j;
          float x = (qv && d < HD) ? ld_act(qr, d) * a.scale : 0.f;
          uint16_t bits = f2bf_bits(x);
          v[j] = __builtin_bit_cast(__bf16, bits);
        }
        qf[kc] = v;
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < QN; ++kk) qf[kk] = qv ? ld_act(qr, kk * 4 + g) * a.scale : 0.f;
    }
  }

  floatx4 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) o[i] = floatx4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  int k_end = klen;
  if (a.causal) k_end = min(k_end, blockIdx.x * kQB + kQB + a.causal_delay);
  for (int k0 = 0; k0 < k_end; k0 += kKT) {
    __syncthreads();
    // Stage K and V for keys [k0, k0+32).
    constexpr int F4 = HD / 4;
    for (int i = tid; i < kKT * F4; i += 256) {
      int kr = i / F4, d4 = (i % F4) * 4;
      int key = k0 + kr;
      float4 kv = make_float4(0.f, 0.f, 0.f, 0.f), vv = kv;
      if (key < T) {
        const io_t* r = base + (int64_t)key * tstr + h * HD + d4;
        if constexpr (IOBF) {
          uint2 k2 = *reinterpret_cast<const uint2*>(r + D);
          uint2 v2 = *reinterpret_cast<const uint2*>(r + 2 * D);
          kv = make_float4(__uint_as_float(k2.x << 16), __uint_as_float(k2.x & 0xffff0000u),
                           __uint_as_float(k2.y << 16), __uint_as_float(k2.y & 0xffff0000u));
          vv = make_float4(__uint_as_float(v2.x << 16), __uint_as_float(v2.x & 0xffff0000u),
                           __uint_as_float(v2.y << 16), __uint_as_float(v2.y & 0xffff0000u));
        } else {
          kv = *reinterpret_cast<const float4*>(r + D);
          vv = *reinterpret_cast<const float4*>(r + 2 * D);
        }
      }
      if constexpr (BF16) {
        uint2 pk;
        pk.x = (uint32_t)f2bf_bits(kv.x) | ((uint32_t)f2bf_bits(kv.y) << 16);
        pk.y = (uint32_t)f2bf_bits(kv.z) | ((uint32_t)f2bf_bits(kv.w) << 16);
        *reinterpret_cast<uint2*>(&Kb[kr * KS_BF + d4]) = pk;
        Vtb[(d4 + 0) * VT_BF + kr] = f2bf_bits(vv.x);
        Vtb[(d4 + 1) * VT_BF + kr] = f2bf_bits(vv.y);
        Vtb[(d4 + 2) * VT_BF + kr] = f2bf_bits(vv.z);
        Vtb[(d4 + 3) * VT_BF + kr] = f2bf_bits(vv.w);
      } else {
        float* kd = &Kf[kr * FS + d4];
        kd[0] = kv.x; kd[1] = kv.y; kd[2] = kv.z; kd[3] = kv.w;
        float* vd = &Vf[kr * FS + d4];
        vd[0] = vv.x; vd[1] = vv.y; vd[2] = vv.z; vd[3] = vv.w;
      }
    }
    if constexpr (BF16) {
      if (HDP > HD) {
        for (int i = tid; i < kKT * (HDP - HD); i += 256) {
          int kr = i / (HDP - HD), d = HD + i % (HDP - HD);
          Kb[kr * KS_BF + d] = 0;
        }
      }
    }
    __syncthreads();

    // Sᵀ tile: 2 subtiles of 16 keys; lane holds keys st*16 + 4g + r of query l15.
    floatx4 sc[2];
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
      if constexpr (BF16) {
#pragma unroll
        for (int kc = 0; kc < QN; ++kc) {
          bf16x8 kf = *reinterpret_cast<const bf16x8*>(&Kb[(st * 16 + l15) * KS_BF + kc * 32 + g * 8]);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[kc], acc, 0, 0, 0);
        }
      } else {
#pragma unroll
        for (int kk = 0; kk < QN; ++kk) {
          float kf = Kf[(st * 16 + l15) * FS + kk * 4 + g];
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(kf, qf[kk], acc, 0, 0, 0);
        }
      }
      sc[st] = acc;
    }
    // Mask + online softmax (per query = per l15; reduce over r and over g).
    float tmax = -INFINITY;
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int key = k0 + st * 16 + g * 4 + r;
        bool ok = key < klen && (!a.causal || key <= myq + a.causal_delay);
        float v = ok ? sc[st][r] : -INFINITY;
        sc[st][r] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_new = fmaxf(m_run, tmax);
    const float alpha = (m_new == -INFINITY) ? 1.f : __expf(m_run - m_new);
    float psum = 0.f;
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float p = (m_new == -INFINITY) ? 0.f : __expf(sc[st][r] - m_new);
        sc[st][r] = p;
        psum += p;
      }
    psum += __shfl_xor(psum, 16, 64);
    psum += __shfl_xor(psum, 32, 64);
    l_run = l_run * alpha + psum;
    m_run = m_new;
    // Rescale O rows (row q' = 4g + r) with that query's alpha.
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float ar = __shfl(alpha, g * 4 + r, 64);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt][r] *= ar;
    }
    // O += P·V.
    if constexpr (BF16) {
      bf16x8 pa;
#pragma unroll
      for (int j = 0; j < 8; ++j) pa[j] = __builtin_bit_cast(__bf16, f2bf_bits(sc[j >> 2][j & 3]));
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const uint16_t* vr = &Vtb[(dt * 16 + l15) * VT_BF];
        uint2 lo = *reinterpret_cast<const uint2*>(vr + g * 4);
        uint2 hi = *reinterpret_cast<const uint2*>(vr + 16 + g * 4);
        bf16x8 vb;
        uint32_t w[4] = {lo.x, lo.y, hi.x, hi.y};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          vb[2 * j] = __builtin_bit_cast(__bf16, (uint16_t)(w[j] & 0xffff));
          vb[2 * j + 1] = __builtin_bit_cast(__bf16, (uint16_t)(w[j] >> 16));
        }
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vb, o[dt], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = st * 16 + g * 4 + r;
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            float vb = Vf[key * FS + dt * 16 + l15];
            o[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(sc[st][r], vb, o[dt], 0, 0, 0);
          }
        }
    }
  }

  // Normalise and store rows q' = q0 + 4g + r.
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int qi = g * 4 + r;
    const float lr = __shfl(l_run, qi, 64);
    const int q = q0 + qi;
    if (q >= T) continue;
    const float inv = lr > 0.f ? 1.f / lr : 0.f;
    io_t* orow = reinterpret_cast<io_t*>(a.out) + (row0 + (int64_t)q * a.tok_stride) * a.ldo + h * HD;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) st_act(orow, dt * 16 + l15, o[dt][r] * inv);
  }
}

// Short sequences (T <= 256, bf16 compute and storage): one workgroup per (sequence,
// head) stages the WHOLE K and Vᵀ of that head in LDS once with 16-B loads and its 4
// waves walk the 16-query tiles — no K/V re-reads per query block, no 64-query
// padding waste (conformer T = 150; FS-EEND slot attention T = 6).  Same S-transposed
// MFMA formulation and online softmax as attn_kernel above.
template <int HD>
__global__ __launch_bounds__(256) void attn_short_kernel(AttnArgs a, int TP) {
  constexpr int HDP = ((HD + 31) / 32) * 32;
  constexpr int KS = HDP + 8;         // K row stride (bf16)
  constexpr int QN = HDP / 32;
  constexpr int DT = HD / 16;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Kb = smem;                 // [TP][KS]
  uint16_t* Vt = smem + TP * KS;       // [HDP][TP + 8]
  const int VS = TP + 8;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, l15 = lane & 15;
  const int s = blockIdx.x / a.nh, h = blockIdx.x % a.nh;
  const int T = a.T, D = a.D;
  const int64_t row0 = (int64_t)(s / a.seq_inner) * (a.seq_outer ? a.seq_outer : (int64_t)T) +
                       (int64_t)(s % a.seq_inner) * a.seq_inner_stride;
  const int64_t tstr = (int64_t)a.tok_stride * a.ld_qkv;
  const uint16_t* base = reinterpret_cast<const uint16_t*>(a.qkv) + row0 * a.ld_qkv + h * HD;
  const int klen = a.key_len ? min(a.key_len[s], T) : T;

  // ---- stage K (rows) and Vᵀ for all keys; zero padding beyond T and HD
  constexpr int CH = HDP / 8;          // 16-B chunks per padded row
  for (int i = tid; i < TP * CH; i += 256) {
    const int key = i / CH, c8 = (i % CH) * 8;
    uint4 kv = make_uint4(0u, 0u, 0u, 0u), vv = kv;
    if (key < T && c8 < HD) {
      const uint16_t* r = base + (int64_t)key * tstr + c8;
      kv = *reinterpret_cast<const uint4*>(r + D);
      vv = *reinterpret_cast<const uint4*>(r + 2 * D);
    }
    *reinterpret_cast<uint4*>(Kb + key * KS + c8) = kv;
    const uint32_t vw[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      Vt[(c8 + 2 * u) * VS + key] = (uint16_t)(vw[u] & 0xffffu);
      Vt[(c8 + 2 * u + 1) * VS + key] = (uint16_t)(vw[u] >> 16);
    }
  }
  __syncthreads();

  const int n_qt = (T + 15) / 16;
  for (int qt = wid; qt < n_qt; qt += 4) {
    const int q0 = qt * 16;
    const int myq = q0 + l15;
    bf16x8 qf[QN];
    {
      const uint16_t* qr = base + (int64_t)min(myq, T - 1) * tstr;
#pragma unroll
      for (int kc = 0; kc < QN; ++kc) {
        const int d0 = kc * 32 + g * 8;
        bf16x8 v;
        if (myq < T && d0 < HD) {
          const uint4 q4 = *reinterpret_cast<const uint4*>(qr + d0);
          const uint32_t qw[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            v[2 * u] = __builtin_bit_cast(__bf16, f2bf_bits(__uint_as_float(qw[u] << 16) * a.scale));
            v[2 * u + 1] = __builtin_bit_cast(__bf16, f2bf_bits(__uint_as_float(qw[u] & 0xffff0000u) * a.scale));
          }
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = __builtin_bit_cast(__bf16, (uint16_t)0);
        }
        qf[kc] = v;
      }
    }
    floatx4 o[DT];
#pragma unroll
    for (int i = 0; i < DT; ++i) o[i] = floatx4{0.f, 0.f, 0.f, 0.f};
    float m_run = -INFINITY, l_run = 0.f;
    int k_end = klen;
    if (a.causal) k_end = min(k_end, q0 + 16 + a.causal_delay);
    for (int k0 = 0; k0 < k_end; k0 += 32) {
      floatx4 sc[2];
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < QN; ++kc) {
          const bf16x8 kf = *reinterpret_cast<const bf16x8*>(&Kb[(k0 + st * 16 + l15) * KS + kc * 32 + g * 8]);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[kc], acc, 0, 0, 0);
        }
        sc[st] = acc;
      }
      float tmax = -INFINITY;
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = k0 + st * 16 + g * 4 + r;
          const bool ok = key < klen && (!a.causal || key <= myq + a.causal_delay);
          const float v = ok ? sc[st][r] : -INFINITY;
          sc[st][r] = v;
          tmax = fmaxf(tmax, v);
        }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float m_new = fmaxf(m_run, tmax);
      const float alpha = (m_new == -INFINITY) ? 1.f : __expf(m_run - m_new);
      float psum = 0.f;
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = (m_new == -INFINITY) ? 0.f : __expf(sc[st][r] - m_new);
          sc[st][r] = pv;
          psum += pv;
        }
      psum += __shfl_xor(psum, 16, 64);
      psum += __shfl_xor(psum, 32, 64);
      l_run = l_run * alpha + psum;
      m_run = m_new;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float ar = __shfl(alpha, g * 4 + r, 64);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) o[dt][r] *= ar;
      }
      bf16x8 pa;
#pragma unroll
      for (int j = 0; j < 8; ++j) pa[j] = __builtin_bit_cast(__bf16, f2bf_bits(sc[j >> 2][j & 3]));
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const uint16_t* vr = &Vt[(dt * 16 + l15) * VS + k0];
        const uint2 lo = *reinterpret_cast<const uint2*>(vr + g * 4);
        const uint2 hi = *reinterpret_cast<const uint2*>(vr + 16 + g * 4);
        bf16x8 vb;
        const uint32_t w[4] = {lo.x, lo.y, hi.x, hi.y};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          vb[2 * j] = __builtin_bit_cast(__bf16, (uint16_t)(w[j] & 0xffff));
          vb[2 * j + 1] = __builtin_bit_cast(__bf16, (uint16_t)(w[j] >> 16));
        }
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vb, o[dt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int qi = g * 4 + r;
      const float lr = __shfl(l_run, qi, 64);
      const int q = q0 + qi;
      if (q >= T) continue;
      const float inv = lr > 0.f ? 1.f / lr : 0.f;
      uint16_t* orow = reinterpret_cast<uint16_t*>(a.out) + (row0 + (int64_t)q * a.tok_stride) * a.ldo + h * HD;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) orow[dt * 16 + l15] = f2bf_bits(o[dt][r] * inv);
    }
  }
}

template <int HD>
bool launch_short(const AttnArgs& a, bool bf16, hipStream_t st) {
  constexpr int HDP = ((HD + 31) / 32) * 32;
  if (!bf16 || !a.io_bf16 || a.T > 256 || (a.ld_qkv % 8) || (a.D % 8) || (HD % 8)) return false;
  const int TP = (a.T + 31) / 32 * 32;
  const size_t smem = sizeof(uint16_t) * ((size_t)TP * (HDP + 8) + (size_t)HDP * (TP + 8));
  static bool attr = false;
  if (!attr) {
    SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(attn_short_kernel<HD>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL(attn_short_kernel<HD>, dim3(a.S * a.nh), dim3(256), smem, st, a, TP);
  return true;
}

template <int HD>
void launch_hd(const AttnArgs& a, bool bf16, hipStream_t st) {
  if (launch_short<HD>(a, bf16, st)) return;
  dim3 grid(cdiv(a.T, kQB), a.S * a.nh);
  if (bf16 && a.io_bf16)
    hipLaunchKernelGGL((attn_kernel<true, HD, true>), grid, dim3(256), 0, st, a);
  else if (bf16)
    hipLaunchKernelGGL((attn_kernel<true, HD, false>), grid, dim3(256), 0, st, a);
  else if (a.io_bf16)
    hipLaunchKernelGGL((attn_kernel<false, HD, true>), grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((attn_kernel<false, HD, false>), grid, dim3(256), 0, st, a);
}

}  // namespace

void attention(const AttnArgs& a, bool bf16, hipStream_t st) {
  SD_CHECK(a.nh > 0 && a.D % a.nh == 0, kErrInvalid, "attention: D % nh != 0");
  SD_CHECK(a.ld_qkv % 4 == 0 && a.D % 4 == 0, kErrInvalid, "attention: ld_qkv % 4 != 0");
  const int hd = a.D / a.nh;
  const double flops = 4.0 * a.S * a.nh * (double)a.T * a.T * hd * (a.causal ? 0.5 : 1.0);
  const double bytes = (a.io_bf16 ? 2.0 : 4.0) * a.S * a.T * (3.0 * a.D + a.D);
  ProfScope prof(bf16 ? "attention_bf16" : "attention_f32", flops, bytes, st);
  switch (hd) {
    case 48: launch_hd<48>(a, bf16, st); break;
    case 64: launch_hd<64>(a, bf16, st); break;
    case 96: launch_hd<96>(a, bf16, st); break;
    case 128: launch_hd<128>(a, bf16, st); break;
    default: SD_CHECK(false, kErrInvalid, "attention: unsupported head dim");
  }
  SD_LAUNCH_CHECK();
}

}  // namespace sd
