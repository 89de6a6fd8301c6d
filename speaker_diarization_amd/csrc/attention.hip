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
#include <mutex>
#include <unordered_map>

#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {
namespace {

constexpr int kQB = 64;   // queries per block

// Chunk-streaming visibility (AttnArgs::chunk / left) as the key window [lo, hi) of query q:
// keys of chunks max(0, c - left) .. c, c = q / chunk.  One division per query.
struct KeyWindow { int lo, hi; };
__device__ __forceinline__ KeyWindow chunk_window(const AttnArgs& a, int q) {
  if (!a.chunk) return {0, 0x7fffffff};
  const int qc = q / a.chunk;
  return {a.left < 0 ? 0 : max(0, qc - a.left) * a.chunk, (qc + 1) * a.chunk};
}
// Key visibility of query myq (key_len, causal and chunk-window terms).  a.mask_dump (tests,
// sd_probe_attention_mask) records the decision of every visited (query, key) pair of sequence 0, head 0.
__device__ __forceinline__ bool key_visible(const AttnArgs& a, const KeyWindow& kw, int klen, int key, int myq) {
  return key < klen && (!a.causal || key <= myq + a.causal_delay) && key >= kw.lo && key < kw.hi;
}
__device__ __forceinline__ void dump_mask(const AttnArgs& a, int s, int h, int T, int key, int myq, bool ok) {
  if (a.mask_dump && s == 0 && h == 0 && myq < T && key < T) a.mask_dump[(int64_t)myq * T + key] = ok ? 1 : 2;
}
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

  const KeyWindow kw = chunk_window(a, myq);
  int k_end = klen;
  if (a.causal) k_end = min(k_end, blockIdx.x * kQB + kQB + a.causal_delay);
  const bool clip = a.chunk != 0;
  if (clip) k_end = min(k_end, ((blockIdx.x * kQB + kQB - 1) / a.chunk + 1) * a.chunk);
  // left >= 0: tiles wholly before the block's first query window hold no visible key
  const int k_begin = (clip && a.left >= 0) ? chunk_window(a, blockIdx.x * kQB).lo / kKT * kKT : 0;
  for (int k0 = k_begin; k0 < k_end; k0 += kKT) {
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
        bool ok = key_visible(a, kw, klen, key, myq);
        dump_mask(a, s, h, T, key, myq, ok);
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
// group of heads).  For each head it stages the head's whole K (zero-padded to a
// multiple of 32 in d) and V — both row-major, straight 16-B copies — in LDS, and
// its 4 waves walk the 16-query tiles.  Both products run "transposed" so every
// softmax statistic and output row is lane-local:
//   S^T = K Q^T   (mfma(K frag, Q frag)): lane (g, l15) holds keys 4g+r of query l15;
//   O^T = V^T P^T (mfma(V frag, P frag)): lane holds d = 16dt + 4g + r of query l15,
//                 so the output leaves as 8-B bf16 stores;
// the V^T operand comes from the row-major V image through ds_read_b64_tr_b16 (gfx950
// transpose read), so staging needs no scattered 2-B LDS writes.  One workgroup per
// sequence (all heads) when there are enough sequences: each QKV row is then fetched
// by one CU instead of by nh workgroups spread over the XCDs.  LDS row strides
// (K: HDP+16, V: HD or HD+16 elements) are bank-conflict free for the ds_read_b128
// fragment reads and the transpose reads.
template <int HD, bool XREMAP>
__global__ __launch_bounds__(256) void attn_short_kernel(AttnArgs a, int TP, int hpw) {
  constexpr int HDP = ((HD + 31) / 32) * 32;
  constexpr int KS = HDP + 16;
  constexpr int VS = HD == 48 ? HD : HD + 16;
  constexpr int QN = HDP / 32;
  constexpr int DT = HD / 16;
  typedef short v4s __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Kb = smem;                 // [TP][KS]
  uint16_t* Vb = smem + TP * KS;       // [TP][VS]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, l15 = lane & 15;
  const int n_hg = (a.nh + hpw - 1) / hpw;
  const int lid = XREMAP ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int s = lid / n_hg, h_beg = (lid % n_hg) * hpw;
  const int h_end = min(h_beg + hpw, a.nh);
  const int T = a.T, D = a.D;
  const int64_t row0 = (int64_t)(s / a.seq_inner) * (a.seq_outer ? a.seq_outer : (int64_t)T) +
                       (int64_t)(s % a.seq_inner) * a.seq_inner_stride;
  const int64_t tstr = (int64_t)a.tok_stride * a.ld_qkv;
  const int klen = a.key_len ? min(a.key_len[s], T) : T;
  const int n_qt = (T + 15) / 16;
  // Transpose-read lane address inside a 4-row x 16-column block: row q = (l15 >> 2),
  // columns 4 * (l15 & 3) .. +3; block origin (keys k0 + 4g [+16], columns 16 dt).
  const int tr_off = ((4 * g + (l15 >> 2)) * VS + 4 * (l15 & 3)) * 2;

  for (int h = h_beg; h < h_end; ++h) {
    const uint16_t* base = reinterpret_cast<const uint16_t*>(a.qkv) + row0 * a.ld_qkv + h * HD;
    if (h > h_beg) __syncthreads();   // previous head's LDS reads done
    // Raw Q chunks of this wave's first query tile: in flight during the K/V staging.
    auto load_q = [&](int qt, uint4* raw) {
      const int myq = qt * 16 + l15;
      const uint16_t* qr = base + (int64_t)min(myq, T - 1) * tstr;
#pragma unroll
      for (int kc = 0; kc < QN; ++kc) {
        const int d0 = kc * 32 + g * 8;
        raw[kc] = (qt < n_qt && myq < T && d0 < HD) ? *reinterpret_cast<const uint4*>(qr + d0)
                                                     : make_uint4(0u, 0u, 0u, 0u);
      }
    };
    uint4 qraw[QN];
    load_q(wid, qraw);
    // K/V staging: up to 8 16-B loads per thread issued back to back, then stored.
    constexpr int CK = HDP / 8, CV = HD / 8;
    const int nk = TP * CK, nv = TP * CV;
    for (int r0 = 0; r0 < nk + nv; r0 += 8 * 256) {
      uint4 st[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = r0 + u * 256 + tid;
        st[u] = make_uint4(0u, 0u, 0u, 0u);
        if (i < nk) {
          const int key = i / CK, c8 = (i % CK) * 8;
          if (key < T && c8 < HD) st[u] = *reinterpret_cast<const uint4*>(base + (int64_t)key * tstr + D + c8);
        } else if (i < nk + nv) {
          const int key = (i - nk) / CV, c8 = ((i - nk) % CV) * 8;
          if (key < T) st[u] = *reinterpret_cast<const uint4*>(base + (int64_t)key * tstr + 2 * D + c8);
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = r0 + u * 256 + tid;
        if (i < nk) {
          const int key = i / CK, c8 = (i % CK) * 8;
          *reinterpret_cast<uint4*>(Kb + key * KS + c8) = st[u];
        } else if (i < nk + nv) {
          const int key = (i - nk) / CV, c8 = ((i - nk) % CV) * 8;
          *reinterpret_cast<uint4*>(Vb + key * VS + c8) = st[u];
        }
      }
    }
    __syncthreads();

    for (int qt = wid; qt < n_qt; qt += 4) {
      const int q0 = qt * 16;
      const int myq = q0 + l15;
      bf16x8 qf[QN];
#pragma unroll
      for (int kc = 0; kc < QN; ++kc) {
        const uint32_t qw[4] = {qraw[kc].x, qraw[kc].y, qraw[kc].z, qraw[kc].w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          qf[kc][2 * u] = (__bf16)(__uint_as_float(qw[u] << 16) * a.scale);
          qf[kc][2 * u + 1] = (__bf16)(__uint_as_float(qw[u] & 0xffff0000u) * a.scale);
        }
      }
      load_q(qt + 4, qraw);   // next tile's Q in flight during this tile
      floatx4 o[DT];
#pragma unroll
      for (int i = 0; i < DT; ++i) o[i] = floatx4{0.f, 0.f, 0.f, 0.f};
      float m_run = -INFINITY, l_run = 0.f;   // statistics of query myq
      const KeyWindow kw = chunk_window(a, myq);
      int k_end = klen;
      if (a.causal) k_end = min(k_end, q0 + 16 + a.causal_delay);
      const bool clip = a.chunk != 0;
      if (clip) k_end = min(k_end, ((q0 + 15) / a.chunk + 1) * a.chunk);
      const int k_begin = (clip && a.left >= 0) ? chunk_window(a, q0).lo / 32 * 32 : 0;
      for (int k0 = k_begin; k0 < k_end; k0 += 32) {
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
            const bool ok = key_visible(a, kw, klen, key, myq);
            dump_mask(a, s, h, T, key, myq, ok);
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
        // P^T operand: k-index 8g + j <-> key k0 + 4g + j (j < 4), k0 + 16 + 4g + j - 4.
        bf16x8 pb;
#pragma unroll
        for (int j = 0; j < 8; ++j) pb[j] = (__bf16)sc[j >> 2][j & 3];
        typedef __attribute__((address_space(3))) v4s* lds_v4s_t;
        const uint32_t vbase = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) void*)Vb) +
                               (uint32_t)(k0 * VS * 2) + (uint32_t)tr_off;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t)(uintptr_t)(vbase + dt * 32));
          const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t)(uintptr_t)(vbase + 16 * VS * 2 + dt * 32));
          const bf16x8 va = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
          for (int r = 0; r < 4; ++r) o[dt][r] *= alpha;
          o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pb, o[dt], 0, 0, 0);
        }
      }
      if (myq < T) {
        const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
        uint16_t* orow = reinterpret_cast<uint16_t*>(a.out) + (row0 + (int64_t)myq * a.tok_stride) * a.ldo + h * HD;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
          *reinterpret_cast<uint2*>(orow + dt * 16 + 4 * g) =
              make_uint2(pack_bf16x2(o[dt][0] * inv, o[dt][1] * inv), pack_bf16x2(o[dt][2] * inv, o[dt][3] * inv));
      }
    }
  }
}

// Long-sequence bf16 flash attention (FS-EEND: causal T = 6000 encoder and the decoder's strided time
// attention; fs_eend.py:163-171).  bf16 in / out, so K and V tiles are staged in LDS with 16-B copies (no
// fp32 round trip, no scattered 2-B transposes): K row-major for the Sᵀ = K·Qᵀ A operand, V row-major read
// back as the Vᵀ A operand of Oᵀ = Vᵀ·Pᵀ with ds_read_b64_tr_b16 (the attn_short scheme).
//
// A workgroup is 8 waves over 64 queries: waves w and w + 4 own the same 16 queries and split the keys by
// 64-key tile parity (each 128-key pair of tiles is staged once; the even tile feeds waves 0-3, the odd one
// waves 4-7), which doubles the waves in flight over the 1.5 per SIMD a T = 6000, 4-head causal launch
// gives with one wave per 16 queries.  The two halves' (max, sum, O) are merged through LDS at the end.
// Per tile: row max by 15 fmax + permlane16/32_swap (VALU, no LDS round trip), p = exp2(s·log2e - m·log2e)
// as one FMA + v_exp, the row sum kept per lane and reduced once at the end.  Pairs are double-buffered in
// LDS and fetched two pairs ahead into registers (one barrier per pair).  Tiles wholly visible skip the
// mask; causal query blocks run heaviest first.
constexpr int kLKT = 64;   // keys per tile (per wave); a pair of tiles per staging step
__device__ __forceinline__ float vmax(float x, float y) {   // v_max_f32 without the canonicalising pre-ops
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}
__device__ __forceinline__ float vmax3(float x, float y, float z) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(z));
  return r;
}
__device__ __forceinline__ float xor16_max(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return vmax(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return vmax(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// Small grids (fewer (sequence, head) pairs than XCDs: the FS-EEND encoder's 4 heads of one recording): each pair's
// query blocks go to 8 / nsh XCDs (block b runs on XCD b % 8), alternating between them in heaviest-first order so
// the XCDs of a pair get the same mix of long and short blocks, and a pair's K/V prefix is fetched into 8 / nsh
// L2s instead of all eight (round 5: FETCH_SIZE 55 MB per C5 encoder launch for 12.3 MB of Q, K, V and O).
// Identity when the split is not exact.
__device__ __forceinline__ int xcd_group_remap(int lin, int nqb, int nsh) {
  if (nsh >= 8 || 8 % nsh != 0) return lin;
  const int per = 8 / nsh;
  if (nqb % per != 0) return lin;
  const int x = lin & 7, k = lin >> 3;
  return (x / per) * nqb + k * per + x % per;
}

template <int HD, int HOIST>   // 0: reads next to their MFMAs; 1: K + first V half hoisted; 2: all hoisted
__global__ __launch_bounds__(512) void attn_long_kernel(AttnArgs a) {
  // row strides (bf16) HD + 16: the only padding up to 32 with conflict-free ds_read_b128 K fragments
  // (16-lane groups) AND ds_read_b64_tr_b16 V reads (32-lane groups) for HD = 32, 64, 128 (pad 8 / 0 cost
  // 2x / 4x: SQ_LDS_BANK_CONFLICT was 4.5 extra cycles per LDS instruction)
  constexpr int KS = HD + 16;
  constexpr int VS = HD + 16;
  constexpr int KC = HD / 32;                // 32-wide d chunks of Q / K
  constexpr int DT = HD / 16;                // 16-wide d tiles of O
  constexpr int CPR = HD / 8;                // 16-B chunks per row
  constexpr int PK = 2 * kLKT;               // keys per staged pair
  constexpr int CHK = PK * CPR / 512;        // 16-B chunks per thread per matrix and pair
  constexpr float kL2E = 1.4426950408889634f;
  static_assert(HD % 32 == 0 && CHK >= 1, "head dim");
  __shared__ __attribute__((aligned(16))) uint16_t Ks[2][PK * KS];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[2][PK * VS];
  typedef short v4s __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) v4s* lds_v4s_t;

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = wid >> 2, qw = wid & 3;   // key-tile parity, query group (wave-uniform: SGPR branches)
  const int g = lane >> 4, l15 = lane & 15;
  // XCD-aware order: the query blocks of one (sequence, head) are consecutive logical ids on one XCD, so
  // its K/V prefix (1.5 MB at T 6000, d 64) is fetched into that XCD's L2 once instead of into all eight
  // (FETCH_SIZE: 150 MB per decoder launch for 37 MB of K/V)
  const int nqb = (int)gridDim.x;
  // (large grids only: a small grid's heads would land whole on few XCDs, heavy query blocks together)
  const int lin = (int)(blockIdx.y * nqb + (int)blockIdx.x);
  const int lid = HOIST == 2 ? (a.xcd_small ? xcd_group_remap(lin, nqb, (int)gridDim.y) : lin)
                             : xcd_remap(lin, nqb * (int)gridDim.y);
  const int sh = lid / nqb, s = sh / a.nh, h = sh % a.nh;
  const int T = a.T, D = a.D;
  const int qbi = lid - sh * nqb;
  const int qb = a.causal ? nqb - 1 - qbi : qbi;   // heaviest first
  const int qblk0 = qb * kQB;
  const int myq = qblk0 + qw * 16 + l15;
  const int64_t row0 = (int64_t)(s / a.seq_inner) * (a.seq_outer ? a.seq_outer : (int64_t)T) +
                       (int64_t)(s % a.seq_inner) * a.seq_inner_stride;
  const int64_t tstr = (int64_t)a.tok_stride * a.ld_qkv;
  const uint16_t* base = reinterpret_cast<const uint16_t*>(a.qkv) + row0 * a.ld_qkv + h * HD;
  const int klen = a.key_len ? min(a.key_len[s], T) : T;

  bf16x8 qf[KC];
  {
    const float qs = a.scale * kL2E;
    const uint16_t* qr = base + (int64_t)min(myq, T - 1) * tstr;
    const bool qv = myq < T;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const uint4 u = *reinterpret_cast<const uint4*>(qr + kc * 32 + g * 8);
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
      uint32_t pk[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)   // bf16(q * scale * log2 e): scores arrive in log2 units
        pk[j] = qv ? pack_bf16x2(__uint_as_float(w[j] << 16) * qs, __uint_as_float(w[j] & 0xffff0000u) * qs) : 0u;
      qf[kc] = __builtin_bit_cast(bf16x8, make_uint4(pk[0], pk[1], pk[2], pk[3]));
    }
  }

  int k_end = klen;
  if (a.causal) k_end = min(k_end, qblk0 + kQB + a.causal_delay);
  const int ntile = k_end > 0 ? (k_end + kLKT - 1) / kLKT : 0;
  const int npair = (ntile + 1) / 2;
  const int nit = npair;
  auto P = [&](int i) { return i; };
  // staging map: chunk c = tid + 512 i -> pair row c / CPR, 16-B chunk c % CPR.  Two register sets: pair
  // p + 1 is staged from one at the end of pair p while pair p + 2 is in flight in the other.
  struct KV { u32x4_t k[CHK], v[CHK]; };   // native vectors: HIP's uint4 wrapper kept the sets in scratch
  KV ra, rb;
  auto fetch = [&](int p, KV& r) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < CHK; ++i) {
      const int c = tid + 512 * i, kr = c / CPR, ch = c % CPR;
      const int key = p * PK + kr;
      const uint16_t* src = base + (int64_t)min(key, T - 1) * tstr + ch * 8;
      // rows past T re-read row T - 1 (finite data; those keys are masked, p = 0): no branch around the load
      r.k[i] = *reinterpret_cast<const u32x4_t*>(src + D);
      r.v[i] = *reinterpret_cast<const u32x4_t*>(src + 2 * D);
    }
  };
  auto stage = [&](int buf, const KV& r) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < CHK; ++i) {
      const int c = tid + 512 * i, kr = c / CPR, ch = c % CPR;
      *reinterpret_cast<u32x4_t*>(&Ks[buf][kr * KS + ch * 8]) = r.k[i];
      *reinterpret_cast<u32x4_t*>(&Vs[buf][kr * VS + ch * 8]) = r.v[i];
    }
  };

  // Softmax against a per-query REFERENCE m (log2 units) that is raised only when a tile's max exceeds it
  // by more than kTau (or the query sees its first key): the MFMA accumulators start at -m, so on the
  // common path p = exp2(acc) with no subtraction and O is not rescaled.  The row sum l comes from the
  // MFMA too (a ones A operand against Pᵀ: every accumulator row is the column sum), so it needs no
  // VALU adds and no cross-lane reduction.  p <= 2^kTau keeps f32 sums and bf16 P exact enough.
  constexpr float kTau = 8.f;
  floatx4 o[DT], ls = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < DT; ++i) o[i] = floatx4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY;   // reference (log2 units); -inf: no visible key yet
  const int tr_off = ((4 * g + (l15 >> 2)) * VS + 4 * (l15 & 3)) * 2;   // attn_short's Vᵀ lane offset (bytes)
  const int krow0 = half * kLKT;                                        // this half's tile inside a pair
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.f;

  auto tile = [&](int t, int buf) __attribute__((always_inline)) {
    const int k0 = t * kLKT;
    const uint16_t* kb = &Ks[buf][krow0 * KS];
    const float mb = m_run == -INFINITY ? 0.f : m_run;   // accumulator origin
    // Every LDS fragment of the tile is requested up front, in source order ahead of the softmax's rare
    // branch (a block boundary the scheduler does not hoist loads across): the Vᵀ reads' latency then hides
    // behind the S MFMAs and the softmax instead of stalling the P·V MFMAs (the waves of a workgroup run
    // phase-locked between barriers, so other waves do not cover it).
    // HOIST (small grids, latency-bound: ILP over occupancy) — large grids keep the reads next to their
    // MFMAs, which leaves 114 instead of 142 VGPRs (4 waves per SIMD instead of 3) at HD 64.
    bf16x8 kf[4][KC];
    bf16x8 vf[HOIST == 2 ? 2 : 1][HOIST ? DT : 1];
    const uint32_t vb0 = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) void*)&Vs[buf][0]) +
                         (uint32_t)(krow0 * VS * 2) + (uint32_t)tr_off;
    auto vfrag = [&](int kh, int dt) __attribute__((always_inline)) {
      const uint32_t vbase = vb0 + (uint32_t)(32 * kh * VS * 2);
      const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t)(uintptr_t)(vbase + dt * 32));
      const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t)(uintptr_t)(vbase + 16 * VS * 2 + dt * 32));
      return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    if constexpr (HOIST) {
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int kc = 0; kc < KC; ++kc)
          kf[st][kc] = *reinterpret_cast<const bf16x8*>(&kb[(st * 16 + l15) * KS + kc * 32 + g * 8]);
#pragma unroll
      for (int kh = 0; kh < (HOIST == 2 ? 2 : 1); ++kh)
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) vf[kh][dt] = vfrag(kh, dt);
    }
    // Sᵀ - m: 4 subtiles of 16 keys; lane holds keys k0 + 16 st + 4g + r of query myq
    floatx4 sc[4];
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      floatx4 acc = {-mb, -mb, -mb, -mb};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        if constexpr (!HOIST) kf[st][kc] = *reinterpret_cast<const bf16x8*>(&kb[(st * 16 + l15) * KS + kc * 32 + g * 8]);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[st][kc], qf[kc], acc, 0, 0, 0);
      }
      sc[st] = acc;
    }
    // mask only where a key of the tile can be invisible to some query of the block (a uniform branch:
    // the per-element `full || visible` select form gave wrong scores on masked tiles; not root-caused)
    const bool full = k0 + kLKT <= klen && (!a.causal || k0 + kLKT - 1 <= qblk0 + a.causal_delay);
    if (!full) {
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = k0 + st * 16 + g * 4 + r;
          const bool ok = key < klen && (!a.causal || key <= myq + a.causal_delay);
          sc[st][r] = ok ? sc[st][r] : -INFINITY;
        }
    }
    float tmax = vmax3(sc[0][0], sc[0][1], sc[0][2]);
    tmax = vmax3(tmax, sc[0][3], sc[1][0]);
    tmax = vmax3(tmax, sc[1][1], sc[1][2]);
    tmax = vmax3(tmax, sc[1][3], sc[2][0]);
    tmax = vmax3(tmax, sc[2][1], sc[2][2]);
    tmax = vmax3(tmax, sc[2][3], sc[3][0]);
    tmax = vmax3(tmax, sc[3][1], sc[3][2]);
    tmax = vmax(tmax, sc[3][3]);
    tmax = xor32_max(xor16_max(tmax));   // relative to mb; -inf: every key of the tile masked
    const bool dead = m_run == -INFINITY;
    const bool raise = dead ? tmax != -INFINITY : tmax > kTau;
    if (__ballot(raise)) {   // rare, wave-uniform: move the reference to this tile's max where raised
      const float m_new = raise ? mb + tmax : m_run;
      const float shift = raise ? tmax : 0.f;
      const float alpha = raise && !dead ? __builtin_amdgcn_exp2f(m_run - m_new) : 1.f;
#pragma unroll
      for (int st = 0; st < 4; ++st)
#pragma unroll
        for (int r = 0; r < 4; ++r) sc[st][r] -= shift;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[dt][r] *= alpha;   // Oᵀ: lane's column is its own query
#pragma unroll
      for (int r = 0; r < 4; ++r) ls[r] *= alpha;
      m_run = m_new;
    }
#pragma unroll
    for (int st = 0; st < 4; ++st)
#pragma unroll
      for (int r = 0; r < 4; ++r) sc[st][r] = __builtin_amdgcn_exp2f(sc[st][r]);   // exp2(-inf) = 0
    // Oᵀ += Vᵀ·Pᵀ, l += 1ᵀ·Pᵀ over the tile's two 32-key halves
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      bf16x8 pb;   // Pᵀ operand: k-index 8g + j <-> key 32 kh + 4g + j (j < 4), 32 kh + 16 + 4g + j - 4
#pragma unroll
      for (int j = 0; j < 8; ++j) pb[j] = (__bf16)sc[2 * kh + (j >> 2)][j & 3];
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        bf16x8 va;
        if (HOIST == 2 || (HOIST == 1 && kh == 0)) va = vf[HOIST == 2 ? kh : 0][dt];
        else va = vfrag(kh, dt);
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pb, o[dt], 0, 0, 0);
      }
      ls = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pb, ls, 0, 0, 0);
    }
  };
  // buf as a compile-time constant: the two unrolled copies differ, so they are not merged into one body
  // selecting between the register sets (which put the sets in scratch)
  auto pair = [&](int p, KV& r, auto bufc) __attribute__((always_inline)) {
    constexpr int buf = decltype(bufc)::value;
    const int t = 2 * P(p) + half;
    tile(t, buf);   // t >= ntile (odd half, last pair): every key masked, no-op; no branch (see below)
    // unconditional (a pair past the end lands in the idle buffer, clamped rows): a skipped path makes
    // the compiler's vmcnt tracking assume the younger set is the one staged next, draining both sets
    stage(buf ^ 1, r);
    fetch(P(p + 3), r);
    __syncthreads();
  };
  if (nit > 0) {
    fetch(P(0), ra);
    stage(0, ra);
    fetch(P(1), ra);
    fetch(P(2), rb);
  }
  __syncthreads();
  int p = 0;
  for (; p + 1 < nit; p += 2) {
    pair(p, ra, std::integral_constant<int, 0>{});
    pair(p + 1, rb, std::integral_constant<int, 1>{});
  }
  if (p < nit) pair(p, ra, std::integral_constant<int, 0>{});

  // merge the odd-tile half into the even-tile half (LDS reuse: every wave passed the last barrier)
  constexpr int MW = 2 + 4 * DT;   // floats per lane: m, l, O
  static_assert(4 * 64 * MW * 4 <= (int)sizeof(Ks), "merge scratch");
  float* mg = reinterpret_cast<float*>(&Ks[0][0]) + (qw * 64 + lane);
  if (half) {
    mg[0] = m_run;
    mg[256] = ls[0];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) mg[256 * (2 + 4 * dt + r)] = o[dt][r];
  }
  __syncthreads();
  if (half) return;
  float l_run;
  {
    const float m1 = mg[0], l1 = mg[256];
    const float m = vmax(m_run, m1);
    const float f0 = m_run == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m_run - m);
    const float f1 = m1 == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m1 - m);
    l_run = ls[0] * f0 + l1 * f1;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[dt][r] = o[dt][r] * f0 + mg[256 * (2 + 4 * dt + r)] * f1;
    m_run = m;
  }
  if (myq < T) {
    const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
    uint16_t* orow = reinterpret_cast<uint16_t*>(a.out) + (row0 + (int64_t)myq * a.tok_stride) * a.ldo + h * HD;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
      *reinterpret_cast<uint2*>(orow + dt * 16 + 4 * g) =
          make_uint2(pack_bf16x2(o[dt][0] * inv, o[dt][1] * inv), pack_bf16x2(o[dt][2] * inv, o[dt][3] * inv));
  }
}

// Tiny-sequence attention (T <= 16: FS-EEND's per-frame attention across its C speaker slots,
// fs_eend.py:456-478 self_attn2 over the slot axis; S = frames x batch sequences).  The work is a few
// kFLOP per sequence, so the kernel is a bf16 stream (read q, k, v once, write o once): one thread per
// (sequence, head, query) computes its T scores, softmax and output row in f32 registers; the T threads of
// a (sequence, head) sit in adjacent lanes, so their k / v rows are one cache-line fetch per wave.
template <int HD>
__global__ __launch_bounds__(256) void attn_tiny_kernel(AttnArgs a) {
  constexpr int C8 = HD / 8;   // 16-B chunks per head row
  const int T = a.T, D = a.D;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (int64_t)a.S * a.nh * T) return;
  const int i = (int)(gid % T);
  const int64_t sh = gid / T;
  const int h = (int)(sh % a.nh), s = (int)(sh / a.nh);
  const int64_t row0 = (int64_t)(s / a.seq_inner) * (a.seq_outer ? a.seq_outer : (int64_t)T) +
                       (int64_t)(s % a.seq_inner) * a.seq_inner_stride;
  const int64_t tstr = (int64_t)a.tok_stride * a.ld_qkv;
  const uint16_t* base = reinterpret_cast<const uint16_t*>(a.qkv) + row0 * a.ld_qkv + h * HD;
  const int klen = a.key_len ? min(a.key_len[s], T) : T;
  float q[HD];
  {
    const uint16_t* qr = base + (int64_t)i * tstr;
#pragma unroll
    for (int c = 0; c < C8; ++c) {
      const uint4 u = *reinterpret_cast<const uint4*>(qr + 8 * c);
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {   // the MFMA kernels' rounding: bf16(q * scale)
        const uint32_t pk = pack_bf16x2(__uint_as_float(w[j] << 16) * a.scale, __uint_as_float(w[j] & 0xffff0000u) * a.scale);
        q[8 * c + 2 * j] = __uint_as_float(pk << 16);
        q[8 * c + 2 * j + 1] = __uint_as_float(pk & 0xffff0000u);
      }
    }
  }
  float sc[16];
  float m = -INFINITY;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    sc[j] = -INFINITY;
    if (j < T && j < klen && (!a.causal || j <= i + a.causal_delay)) {
      const uint16_t* kr = base + (int64_t)j * tstr + D;
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < C8; ++c) {
        const uint4 u = *reinterpret_cast<const uint4*>(kr + 8 * c);
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc = fmaf(q[8 * c + 2 * e], __uint_as_float(w[e] << 16), acc);
          acc = fmaf(q[8 * c + 2 * e + 1], __uint_as_float(w[e] & 0xffff0000u), acc);
        }
      }
      sc[j] = acc;
      m = fmaxf(m, acc);
    }
  }
  float o[HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) o[d] = 0.f;
  float l = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    if (sc[j] != -INFINITY) {
      const float p = __expf(sc[j] - m);
      l += p;
      const uint16_t* vr = base + (int64_t)j * tstr + 2 * D;
#pragma unroll
      for (int c = 0; c < C8; ++c) {
        const uint4 u = *reinterpret_cast<const uint4*>(vr + 8 * c);
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o[8 * c + 2 * e] = fmaf(p, __uint_as_float(w[e] << 16), o[8 * c + 2 * e]);
          o[8 * c + 2 * e + 1] = fmaf(p, __uint_as_float(w[e] & 0xffff0000u), o[8 * c + 2 * e + 1]);
        }
      }
    }
  }
  const float inv = l > 0.f ? 1.f / l : 0.f;
  uint16_t* orow = reinterpret_cast<uint16_t*>(a.out) + (row0 + (int64_t)i * a.tok_stride) * a.ldo + h * HD;
#pragma unroll
  for (int c = 0; c < C8; ++c)
    *reinterpret_cast<uint4*>(orow + 8 * c) =
        make_uint4(pack_bf16x2(o[8 * c] * inv, o[8 * c + 1] * inv), pack_bf16x2(o[8 * c + 2] * inv, o[8 * c + 3] * inv),
                   pack_bf16x2(o[8 * c + 4] * inv, o[8 * c + 5] * inv), pack_bf16x2(o[8 * c + 6] * inv, o[8 * c + 7] * inv));
}

template <int HD>
bool launch_tiny(const AttnArgs& a, bool bf16, hipStream_t st) {
  if (!bf16 || !a.io_bf16 || a.chunk || a.mask_dump || a.T > 16 || HD % 8 || HD > 128 ||
      (a.ld_qkv % 8) || (a.D % 8) || (a.ldo % 8) || (a.tok_stride * a.ld_qkv) % 8)
    return false;
  const int64_t n = (int64_t)a.S * a.nh * a.T;
  hipLaunchKernelGGL(attn_tiny_kernel<HD>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a);
  return true;
}

template <int HD>
bool launch_long(const AttnArgs& a, bool bf16, hipStream_t st) {
  static const bool off = getenv("SDIAR_NO_ATTN_LONG") != nullptr;   // A/B switch: the generic kernel
  if (off || !bf16 || !a.io_bf16 || a.chunk || a.mask_dump || HD % 32 || a.T <= 256 ||
      (a.ld_qkv % 8) || (a.D % 8) || (a.ldo % 4) || (a.tok_stride * a.ld_qkv) % 8)
    return false;
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    SD_HIP(hipGetDevice(&dev));
    SD_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  dim3 grid(cdiv(a.T, kQB), a.S * a.nh);
  // fewer than 2 workgroups per CU: latency-bound, hoist the fragment reads (measured: T 6000 with 4
  // heads 67 -> 57 us; with 24 sequence-heads the occupancy loss made it 215 -> 244 us)
  if ((int64_t)grid.x * grid.y < 2LL * n_cu) {
    // (a split of each query block's key pairs over two workgroups measured 60 -> 54 us here, but the split
    // depends on the grid, so sharded runs — EDA chunk shards, bit-identical for any world size — would
    // differ by world size; not kept)
    AttnArgs b = a;
    b.xcd_small = 1;
    hipLaunchKernelGGL((attn_long_kernel<HD, 2>), grid, dim3(512), 0, st, b);
  } else {
    // large grids: K and the first V half hoisted (126 VGPRs, still 4 waves per SIMD): 187 -> 178 us on the
    // FS-EEND decoder shape against the unhoisted variant (116 VGPRs)
    hipLaunchKernelGGL((attn_long_kernel<HD, 1>), grid, dim3(512), 0, st, a);
  }
  return true;
}

template <int HD>
bool launch_short(const AttnArgs& a, bool bf16, hipStream_t st) {
  constexpr int HDP = ((HD + 31) / 32) * 32;
  constexpr int KS = HDP + 16;
  constexpr int VS = HD == 48 ? HD : HD + 16;
  if (!bf16 || !a.io_bf16 || a.T > 256 || (a.ld_qkv % 8) || (a.D % 8) || (a.ldo % 4) || (HD % 16)) return false;
  const int TP = (a.T + 31) / 32 * 32;
  const size_t smem = sizeof(uint16_t) * (size_t)TP * (KS + VS);
  // One head per workgroup (measured best at S = 2400, T = 150: more, smaller workgroups
  // overlap their staging); XCD-aware order keeps the heads of a sequence on one L2.
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    SD_HIP(hipGetDevice(&dev));
    SD_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const int hpw = 1;
  static bool attr = false;
  if (!attr) {
    SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(attn_short_kernel<HD, true>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const dim3 grid(a.S * ((a.nh + hpw - 1) / hpw));
  hipLaunchKernelGGL((attn_short_kernel<HD, true>), grid, dim3(256), smem, st, a, TP, hpw);
  return true;
}

template <int HD>
void launch_hd(const AttnArgs& a, bool bf16, hipStream_t st) {
  if (launch_tiny<HD>(a, bf16, st)) return;
  if (launch_short<HD>(a, bf16, st)) return;
  if constexpr (HD % 32 == 0) {
    if (launch_long<HD>(a, bf16, st)) return;
  }
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

void attention(const AttnArgs& a_in, bool bf16, hipStream_t st) {
  const AttnArgs& a = a_in;
  SD_CHECK(a.nh > 0 && a.D % a.nh == 0, kErrInvalid, "attention: D % nh != 0");
  SD_CHECK(a.ld_qkv % 4 == 0 && a.D % 4 == 0, kErrInvalid, "attention: ld_qkv % 4 != 0");
  const int hd = a.D / a.nh;
  const double flops = 4.0 * a.S * a.nh * (double)a.T * a.T * hd * (a.causal ? 0.5 : 1.0);
  const double bytes = (a.io_bf16 ? 2.0 : 4.0) * a.S * a.T * (3.0 * a.D + a.D);
  ProfScope prof(bf16 ? "attention_bf16" : "attention_f32", flops, bytes, st);
  switch (hd) {
    case 32: launch_hd<32>(a, bf16, st); break;
    case 48: launch_hd<48>(a, bf16, st); break;
    case 64: launch_hd<64>(a, bf16, st); break;
    case 96: launch_hd<96>(a, bf16, st); break;
    case 128: launch_hd<128>(a, bf16, st); break;
    default: SD_CHECK(false, kErrInvalid, "attention: unsupported head dim");
  }
  SD_LAUNCH_CHECK();
}

}  // namespace sd
