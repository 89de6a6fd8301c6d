// Conformer self-attention block fused for gfx950 (C2: torchaudio ConformerLayer, ts_vad2/model.py:259-267,
// restated in oracle/tsvad_ref.py conformer()): the residual add of the ffn1 output, self_attn_layer_norm,
// the packed in-projection (Q, K, V) and the multi-head attention core in ONE launch.  Replaces
// add_layernorm + the QKV GEMM (gemm_areg) + attn_short, whose (S*T, 3D) bf16 QKV intermediate made a
// full HBM round trip (2.3 KiB per token each way at D = 384).
//
// A workgroup owns TWO sequences = 20 16-token MFMA row tiles (tile t: sequence t / 10, tokens 16 (t % 10)
// .. +15) over 8 waves: wave w takes tiles w, w + 8 and, for w < 4, w + 16, so each SIMD (waves w, w + 4)
// carries 5 tiles — the earlier 10-wave layout (2 tiles per wave) put 3 waves on two SIMDs and 2 on the
// others, and the 2-wave SIMDs spent 21 % of the block parked at the per-piece barrier (s_memtime stamps).
// D = 384, 8 heads of 48:
//   prologue  the LayerNorm'd bf16 rows (the preceding row program / add_layernorm writes them) become
//             the wave's MFMA B-operand fragments (up to 3 x 16 tokens x 384, 144 VGPRs), read once from HBM;
//   pieces    16 in-projection rows (one head's 16 features of q, k or v), 12 KiB, stream through a
//             3-slot LDS-DMA ring (buffer_load ... lds, 16-B chunk c of row r at c ^ (r & 7)), two pieces
//             in flight behind counted vmcnt waits; each weight fragment read from LDS feeds both row
//             tiles (the LDS read rate, not MFMA, bounded the one-tile-per-wave version); transposed MFMA
//             (weights as A operand) leaves 4 consecutive features per lane for one token: + bias, q
//             scaled by 1/sqrt(hd), 8-B LDS stores into the sequence's Q / K (row stride 64, features
//             48..63 zero) and V (row stride 48) images;
//   attention after a head's last V piece: Sᵀ = K·Qᵀ, online softmax, Oᵀ = Vᵀ·Pᵀ with Vᵀ from
//             ds_read_b64_tr_b16 (the attn_short scheme), 8-B bf16 stores of the head's 48 features.
// The in-projection weights (864 KiB bf16) come from L2 once per workgroup, i.e. once per two sequences;
// HBM sees the normalised rows and the attention output only.
#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {
namespace {

constexpr int kD = 384, kHD = 48, kNH = 8;
constexpr int kKT32 = kD / 32;                 // 32-wide k-steps of the projection
constexpr int kKC = kD / 64;                   // 64-wide k-blocks of a weight piece
constexpr int kTP = 160;                       // padded tokens per sequence
constexpr int kTilesPerSeq = kTP / 16;         // 10 row tiles of 16 tokens
constexpr int kPR = 16;                        // weight rows per piece (one MFMA column tile)
constexpr int kSlot = kKC * kPR * 64;          // bf16 elements per ring slot (12 KiB)
constexpr int kDmaPerPiece = kKC * (kPR / 8);  // 1-KiB DMA instructions per piece (12)
constexpr int kVS = 48;                        // V row stride
constexpr int kPieces = kNH * 3 * (kHD / kPR); // 72
typedef __attribute__((address_space(3))) void* lds_ptr_t;

// Layouts of the same arithmetic (bit-identical outputs, tests/test_gpu_mha_block.py), <SEQ, W, NSLOT, QS>:
//   <2, 8, 3, 64>  two sequences per 8-wave workgroup, 3-slot ring, Q / K rows padded to 64 (151 KiB: one
//                  workgroup per CU) - rounds 2-4;
//   <2, 8, 3, 48>  round 5, shipped: the same with Q / K rows of 48 (133 KiB).  With 48-wide rows the second
//                  32-deep QK^T k-step reads features 48..63 from the next row (finite values), multiplied by the
//                  query fragment's features 48..63, which are zeroed in registers; the 96-B row stride also
//                  spreads the K-fragment reads over more LDS banks than the 128-B one (0.4-0.7 ms per C2 step);
//   <1, 4, 2, 48>  one sequence per 4-wave workgroup, 2-slot ring (73.5 KiB: two workgroups per CU, so one's
//                  HBM prologue, piece waits and softmax overlap the other's MFMAs) - 0.1-0.2 ms behind.
template <int SEQ, int W, int NSLOT, int QS>
struct MhaL {
  static constexpr int kTiles = SEQ * kTilesPerSeq;
  static constexpr int kMaxTiles = (kTiles + W - 1) / W;
  static constexpr int kThreads = W * 64;
  static constexpr int kSeqLds = 2 * kTP * QS + kTP * kVS;   // bf16 elements of one sequence's Q, K, V images
  static constexpr size_t kSmem = sizeof(uint16_t) * ((size_t)NSLOT * kSlot + (size_t)SEQ * kSeqLds) +
                                  sizeof(float) * 3 * kD;
  static_assert(kMaxTiles == 2 || kMaxTiles == 3, "2 or 3 row tiles per wave (af registers)");
};

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// PROBE (timing diagnostics, sd_op_mha_block variants 8-10, wrong outputs): bit 0 skips the attention phase, bit 1 the
// projection MFMAs
template <int SEQ, int W, int NSLOT, int QS, int PROBE = 0>
__global__ __launch_bounds__(W * 64) void mha_block_kernel(MhaBlockArgs a) {
  using L = MhaL<SEQ, W, NSLOT, QS>;
  constexpr int kTiles = L::kTiles, kMaxTiles = L::kMaxTiles, kThreads = L::kThreads, kSeqLds = L::kSeqLds;
  extern __shared__ __attribute__((aligned(1024))) uint16_t sm[];
  uint16_t* Ws = sm;                                          // [NSLOT][kKC][16][64]
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, lk = lane >> 4;
  float* s_bias = reinterpret_cast<float*>(Ws + NSLOT * kSlot + SEQ * kSeqLds);   // [3 * kD]
  const int T = a.T;
  const int ntile = w < kTiles - (kMaxTiles - 1) * W ? kMaxTiles : kMaxTiles - 1;   // wave-uniform
  // tile j of this wave: sequence slot sqj[j], token row rowj[j] (this lane's token)
  int sqj[kMaxTiles], rowj[kMaxTiles];
#pragma unroll
  for (int j = 0; j < kMaxTiles; ++j) {
    const int t = w + W * j;
    sqj[j] = min(t, kTiles - 1) / kTilesPerSeq;
    rowj[j] = (min(t, kTiles - 1) % kTilesPerSeq) * 16 + l15;
  }
  auto qimg = [&](int sq) { return Ws + NSLOT * kSlot + sq * kSeqLds; };   // [kTP][QS] Q, then K, then V

  const int lrow = lane >> 3, lch = lane & 7;
  // Piece i: head h = i / 9, component c = (i / 3) % 3, feature tile ft = i % 3 -> in_proj rows
  // c*D + 48h + 16ft .. +15, all K, as 12 1-KiB DMA instructions (k-block kc, 8-row group) over the waves.
  auto issue_piece = [&](int i) {
    const int h = i / 9, c = (i / 3) % 3, ft = i % 3;
    uint16_t* slot = Ws + (i % NSLOT) * kSlot;
    for (int j = w; j < kDmaPerPiece; j += W) {
      const int kc = j >> 1, rg = j & 1;
      const int r = rg * 8 + lrow;
      const uint32_t off =
          (uint32_t)((((int64_t)(c * kD + h * kHD + ft * kPR + r)) * kD + kc * 64 + ((lch ^ (r & 7)) * 8)) * 2);
      // asm DMA (common.h dma_lds16): with the builtin, the compiler put s_waitcnt vmcnt(0) in front of
      // every fragment read of the piece loop (it cannot tell the slots apart), draining the ring
      dma_lds16(reinterpret_cast<const char*>(a.W) + off, (lds_ptr_t)(slot + ((size_t)kc * kPR + rg * 8) * 64));
    }
  };
  const int my_dma = (kDmaPerPiece - w + W - 1) / W;          // instructions this wave issues per piece
#pragma unroll
  for (int i = 0; i < NSLOT - 1; ++i) issue_piece(i);
  for (int i = tid; i < 3 * kD; i += kThreads) s_bias[i] = a.bias[i];
  if constexpr (QS > kHD) {
    for (int i = tid; i < SEQ * kTP * 2; i += kThreads) {   // zero Q/K features 48..63 (never written later)
      const int q = i / (kTP * 2), r = (i >> 1) % kTP, c = kHD + (i & 1) * 8;
      uint16_t* qs = Ws + NSLOT * kSlot + q * kSeqLds;
      *reinterpret_cast<uint4*>(qs + r * QS + c) = make_uint4(0u, 0u, 0u, 0u);
      *reinterpret_cast<uint4*>(qs + kTP * QS + r * QS + c) = make_uint4(0u, 0u, 0u, 0u);
    }
  }

  // ---- prologue: af[rt][kk] = y[32kk + 8lk .. +7] of the LayerNorm'd bf16 rows (B-operand fragments)
  bf16x8 af[kMaxTiles][kKT32];
#pragma unroll
  for (int rt = 0; rt < kMaxTiles; ++rt) {
    const int row = rowj[rt];
    const int s = blockIdx.x * SEQ + sqj[rt];
    const bool live = rt < ntile && s < a.S && row < T;
    const int64_t r = (int64_t)s * T + row;
    // row-major: features 32 kk + 8 lk of row r; tiled (RowProgArgs::a_tiled layout): fragment kk of r's 16-row
    // group, lane (r % 16) + 16 lk
    const uint16_t* yr = a.y_tiled ? reinterpret_cast<const uint16_t*>(a.y) + (r >> 4) * (16 * kD) + ((r & 15) + 16 * lk) * 8
                                   : reinterpret_cast<const uint16_t*>(a.y) + r * kD + 8 * lk;
    const int ks = a.y_tiled ? 512 : 32;
#pragma unroll
    for (int kk = 0; kk < kKT32; ++kk)
      af[rt][kk] = __builtin_bit_cast(bf16x8, live ? *reinterpret_cast<const uint4*>(yr + ks * kk)
                                                   : make_uint4(0u, 0u, 0u, 0u));
  }

  int klenj[SEQ];
#pragma unroll
  for (int q = 0; q < SEQ; ++q) {
    const int s = blockIdx.x * SEQ + q;
    klenj[q] = s < a.S ? (a.key_len ? min(a.key_len[s], T) : T) : 0;
  }
  const int tr_off = ((4 * lk + (l15 >> 2)) * kVS + 4 * (l15 & 3)) * 2;
  typedef short v4s __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) v4s* lds_v4s_t;
  bool drain = true;   // VMEM ops younger than the last DMA issue are pending: wait for everything

  for (int i = 0; i < kPieces; ++i) {
    // Piece i landed: the only younger DMAs are the NSLOT - 2 pieces issued after it (this wave's my_dma
    // instructions each), unless stores were issued after them (attention outputs) -> full drain.
    if constexpr (NSLOT == 4) {
      // two younger pieces in flight, except at the end of the ring (one, then none)
      if (drain || i + 1 >= kPieces) wait_vm<0>();
      else if (i + 2 >= kPieces) {
        if (my_dma == 3) wait_vm<3>(); else if (my_dma == 2) wait_vm<2>(); else wait_vm<1>();
      } else {
        if (my_dma == 3) wait_vm<6>(); else if (my_dma == 2) wait_vm<4>(); else wait_vm<2>();
      }
    } else if constexpr (NSLOT == 3) {
      if (drain || i + 1 >= kPieces) wait_vm<0>();
      else if (my_dma == 3) wait_vm<3>();
      else if (my_dma == 2) wait_vm<2>();
      else wait_vm<1>();
    } else {
      static_assert(NSLOT == 2, "ring depth");
      wait_vm<0>();
    }
    drain = false;
    __syncthreads();   // every wave's part of piece i is in LDS; the slot of piece i-1 is free
    if (i + NSLOT - 1 < kPieces) issue_piece(i + NSLOT - 1);
    const int h = i / 9, c = (i / 3) % 3, ft = i % 3;
    const uint16_t* slot = Ws + (i % NSLOT) * kSlot;
    floatx4 acc[kMaxTiles];
#pragma unroll
    for (int rt = 0; rt < kMaxTiles; ++rt) acc[rt] = floatx4{0.f, 0.f, 0.f, 0.f};
    auto wfrag = [&](int kk) {
      const int kc = kk >> 1, cc = (kk & 1) * 4 + lk;
      return *reinterpret_cast<const bf16x8*>(slot + (kc * kPR + l15) * 64 + ((cc ^ (l15 & 7)) * 8));
    };
    // The fragment of k-step kk + 1 is read while kk's two MFMAs run; the empty asm keeps the
    // compiler from hoisting every step's reads to the top.
    constexpr int kWPD = 3;   // weight fragment reads in flight ahead of their MFMAs
    bf16x8 wq[kWPD];
#pragma unroll
    for (int q = 0; q < kWPD; ++q) wq[q] = wfrag(q);
#pragma unroll
    for (int kk = 0; kk < kKT32; ++kk) {
      const bf16x8 wcur = wq[kk % kWPD];
      if (kk + kWPD < kKT32) wq[kk % kWPD] = wfrag(kk + kWPD);
      if constexpr (PROBE & 2) {
        asm volatile("" :: "v"(wcur));
        continue;
      }
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wcur, af[0][kk], acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wcur, af[1][kk], acc[1], 0, 0, 0);
      // the 4-wave layout does not skip the third tile's MFMA for its two-tile waves (af[2] = 0 there): with the
      // uniform branch around it the compiler shuttled the accumulators through AGPR copies every k-step and the
      // results came out wrong (0.1-2.4 off on every tile at T >= 100, tests/test_gpu_mha_block.py; not
      // root-caused further: the branch-free stream is also the faster one)
      if constexpr (kMaxTiles > 2) {
        if (W == 4 || ntile > 2) acc[2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wcur, af[2][kk], acc[2], 0, 0, 0);
      }
      asm volatile("" ::: "memory");
    }
    // lane holds features 16ft + 4lk + r of token rowj[rt]
    const int ld = c == 2 ? kVS : QS;
    const int coff = c * kTP * QS;                  // Q, K or V image within the sequence's block
    const float scl = c == 0 ? a.scale : 1.f;
    const int n0 = ft * 16 + 4 * lk;
    const float4 bv = *reinterpret_cast<const float4*>(s_bias + c * kD + h * kHD + n0);
#pragma unroll
    for (int rt = 0; rt < kMaxTiles; ++rt)
      if (rt < ntile)
        *reinterpret_cast<uint2*>(qimg(sqj[rt]) + coff + rowj[rt] * ld + n0) =
            make_uint2(pack_bf16x2((acc[rt][0] + bv.x) * scl, (acc[rt][1] + bv.y) * scl),
                       pack_bf16x2((acc[rt][2] + bv.z) * scl, (acc[rt][3] + bv.w) * scl));
    if (c != 2 || ft != 2 || (PROBE & 1)) continue;
    __syncthreads();   // head h's Q, K, V images complete (every sequence of the workgroup)

    // ---- attention of head h for this wave's 16-query tiles
#pragma unroll 1
    for (int rt = 0; rt < ntile; ++rt) {
      const int row = rowj[rt];
      const int s = blockIdx.x * SEQ + sqj[rt];
      if (s >= a.S) continue;
      const uint16_t* Qs = qimg(sqj[rt]);
      const uint16_t* Ks = Qs + kTP * QS;
      const uint16_t* Vs = Ks + kTP * QS;
      const int klen = klenj[sqj[rt]];
      bf16x8 qf[2];
#pragma unroll
      for (int kc = 0; kc < 2; ++kc) qf[kc] = *reinterpret_cast<const bf16x8*>(Qs + row * QS + kc * 32 + lk * 8);
      if constexpr (QS == kHD) {   // features 48..63 of the second k-step: the next row's (see MhaL), zeroed
        if (lk >= 2) qf[1] = __builtin_bit_cast(bf16x8, make_uint4(0u, 0u, 0u, 0u));
      }
      floatx4 o[3] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      float m_run = -INFINITY, l_run = 0.f;
      for (int k0 = 0; k0 < klen; k0 += 32) {
        floatx4 sc[2];
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          floatx4 sacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kc = 0; kc < 2; ++kc) {
            const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + (k0 + st * 16 + l15) * QS + kc * 32 + lk * 8);
            sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[kc], sacc, 0, 0, 0);
          }
          sc[st] = sacc;
        }
        float tmax = -INFINITY;
#pragma unroll
        for (int st = 0; st < 2; ++st)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = k0 + st * 16 + lk * 4 + r;
            const float v = key < klen ? sc[st][r] : -INFINITY;
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
        bf16x8 pb;   // Pᵀ operand: k-index 8g + j <-> key k0 + 4g + j (j < 4), k0 + 16 + 4g + j - 4
#pragma unroll
        for (int j = 0; j < 8; ++j) pb[j] = (__bf16)sc[j >> 2][j & 3];
        const uint32_t vbase = (uint32_t)reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) void*)Vs) +
                               (uint32_t)(k0 * kVS * 2) + (uint32_t)tr_off;
#pragma unroll
        for (int dt = 0; dt < 3; ++dt) {
          const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t)(uintptr_t)(vbase + dt * 32));
          const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_t)(uintptr_t)(vbase + 16 * kVS * 2 + dt * 32));
          const bf16x8 va = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
          for (int r = 0; r < 4; ++r) o[dt][r] *= alpha;
          o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pb, o[dt], 0, 0, 0);
        }
      }
      if (row < T) {
        const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
        const int64_t r = (int64_t)s * T + row;
        uint16_t* ob = reinterpret_cast<uint16_t*>(a.out);
#pragma unroll
        for (int dt = 0; dt < 3; ++dt) {
          const int f = h * kHD + dt * 16 + 4 * lk;   // this lane's 4 features f .. f + 3 of row r
          // tiled (RowProgArgs::a_tiled): fragment f / 32 of the row's 16-row group, lane (r % 16) + 16 ((f % 32) / 8)
          const int64_t off = a.out_tiled ? (((r >> 4) * kKT32 + (f >> 5)) * 64 + (r & 15) + 16 * ((f & 31) >> 3)) * 8 + (f & 7)
                                          : r * a.ldo + f;
          *reinterpret_cast<uint2*>(ob + off) =
              make_uint2(pack_bf16x2(o[dt][0] * inv, o[dt][1] * inv), pack_bf16x2(o[dt][2] * inv, o[dt][3] * inv));
        }
        drain = true;
      }
    }
  }
}

template <int SEQ, int W, int NSLOT, int QS, int PROBE = 0>
void launch_mha(const MhaBlockArgs& a, hipStream_t st) {
  using L = MhaL<SEQ, W, NSLOT, QS>;
  static bool attr = false;
  if (!attr) {
    SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(mha_block_kernel<SEQ, W, NSLOT, QS, PROBE>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)L::kSmem));
    attr = true;
  }
  hipLaunchKernelGGL((mha_block_kernel<SEQ, W, NSLOT, QS, PROBE>), dim3((a.S + SEQ - 1) / SEQ), dim3(L::kThreads),
                     L::kSmem, st, a);
}

}  // namespace

bool mha_block_supported(int D, int nh, int T, bool bf16) {
  static const bool off = getenv("SDIAR_NO_MHA_BLOCK") != nullptr;   // A/B switch: the unfused path
  return !off && bf16 && D == kD && nh == kNH && T >= 1 && T <= kTP;
}

void mha_block(const MhaBlockArgs& a, hipStream_t st, int variant) {
  SD_CHECK(mha_block_supported(kD, a.nh, a.T, true) && a.D == kD, kErrInvalid, "mha_block: unsupported shape");
  SD_CHECK(a.ldo % 4 == 0, kErrInvalid, "mha_block: output row stride must be a multiple of 4");
  SD_CHECK(!(a.out_tiled || a.y_tiled) || ((int64_t)a.S * a.T % 16 == 0 && a.ldo == kD), kErrInvalid,
           "mha_block: the tiled layouts need S * T % 16 == 0 and ldo == D");
  if (a.S <= 0) return;
  SD_CHECK(a.y != nullptr, kErrInvalid, "mha_block: y (LayerNorm'd bf16 rows) is required");
  const double rows = (double)a.S * a.T;
  const double flops = 2.0 * rows * 3 * kD * kD + 4.0 * a.S * (double)a.T * a.T * kD;
  const double bytes = rows * kD * (2.0 + 2.0) + 2.0 * 3 * kD * kD;
  ProfScope prof("mha_block", flops, bytes, st);
  // variant (sd_op_mha_block, tests / probes only; the product passes -1 = 0): 1 <2,8,3,64> (rounds 2-4),
  // 2 <1,4,2,64>, 3 <1,4,2,48>, 4 <1,4,3,48>, 5 <1,8,3,64>, 6 <1,8,2,48>, 7 <2,8,4,48>
  // Round 5 sweep on C2 (ms per step, one box, 2-3 rounds): <2,8,3,48> 26.39-26.79 (shipped), <1,4,2,48> 26.53-26.97,
  // <2,8,4,48> 26.55-26.61, <2,8,3,64> 27.15-27.18, <1,8,2,48> 28.35-28.42, <1,8,3,64> 28.83-28.90,
  // <1,4,2,64> / <1,4,3,48> 29.26-29.36 (over 80 KiB: one 4-wave workgroup per CU)
  const int var = variant >= 0 ? variant : 0;
  switch (var) {
    case 1: launch_mha<2, 8, 3, 64>(a, st); break;
    case 2: launch_mha<1, 4, 2, 64>(a, st); break;
    case 3: launch_mha<1, 4, 2, 48>(a, st); break;
    case 4: launch_mha<1, 4, 3, 48>(a, st); break;
    case 5: launch_mha<1, 8, 3, 64>(a, st); break;
    case 6: launch_mha<1, 8, 2, 48>(a, st); break;
    case 7: launch_mha<2, 8, 4, 48>(a, st); break;
    case 8: launch_mha<2, 8, 3, 48, 1>(a, st); break;    // probes: no attention
    case 9: launch_mha<2, 8, 3, 48, 2>(a, st); break;    //         no projection MFMAs
    case 10: launch_mha<2, 8, 3, 48, 3>(a, st); break;   //         neither (prologue, weight stream, barriers)
    default: launch_mha<2, 8, 3, 48>(a, st); break;
  }
  SD_LAUNCH_CHECK();
}

}  // namespace sd
