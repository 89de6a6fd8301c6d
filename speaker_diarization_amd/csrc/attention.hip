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

template <int HD>
void launch_hd(const AttnArgs& a, bool bf16, hipStream_t st) {
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
