// Conformer row programs for gfx950 (C2: torchaudio ConformerLayer, ts_vad2/model.py:259-267, restated in
// oracle/tsvad_ref.py conformer()).  Everything in a conformer layer that is per token — the residual adds,
// every LayerNorm, the out-projection, pointwise_conv2 and both half-step FFN modules — runs as a short
// "program" over a 128-token tile whose fp32 residual rows never leave the registers between steps:
//
//   acc  = X                                           (fp32 residual, the MFMA accumulators themselves)
//   acc += A · W0ᵀ + b0                                 optional pre-GEMM, A bf16 from HBM (out_proj / pw2)
//   per FFN i:  acc += ½(W2 · silu(W1 · LN_i(acc) + b1) + b2)    then optionally acc = LN_post(acc)
//   Xo   = acc ;  y = LN_y(acc) (bf16)                  optional
//
// so a layer is  [ffn1 + attn-LN] -> mha_block -> [out_proj + conv-LN] -> pw1/GLU -> dwconv ->
// [pw2 + ffn2 + final LN + next layer's ffn1 + attn-LN].  HBM sees X, the bf16 A rows and y once each;
// the 512-wide FFN hidden layer, the sub-block outputs and every LN input stay on chip.
//
// Layout (transposed MFMA, v_mfma_f32_16x16x32_bf16 with weights as the A operand): a workgroup is 8 waves
// (two per SIMD, <= 256 VGPRs each), a wave owns 16 tokens as one 16-token column tile (TT = 1; the
// template keeps TT for the 2-tile layout, which measured slower at one wave per SIMD).  acc[ft][tt] holds
// features 16 ft + 4 g + r (g = lane / 16) of token 16 tt + lane % 16, i.e. a token's 384 features over the
// 4 lanes that share lane % 16 (LN statistics = 2 shuffles).  The B operand of the next GEMM is built from
// that layout without any data movement: k-step kk of a lane holds features 32 kk + 4 g + {0..3} (tile 2kk)
// and 32 kk + 16 + 4 g + {0..3} (tile 2kk + 1), and the weights are packed with the same k permutation
// (rowprog_pack_*).  The FFN hidden layer is produced 32 features at a time (2 up-projection tiles), SiLU'd
// in registers and consumed at once as one k-step of the down projection.
//
// Weights stream from L2 as 24-KiB pieces of 24 pre-packed 1-KiB MFMA fragments (lane-linear, so every
// ds_read_b128 is conflict-free) through a 5-slot LDS ring (global_load_lds, 4 pieces in flight, counted
// vmcnt waits).  The workgroups are persistent over tiles; the ring runs across tile boundaries, so the next
// tile's first weights are in flight during the current tile's epilogue.  One workgroup barrier per piece hands
// the slots over.  (Round 6 replaced it by per-slot FULL / FREE words in LDS -- a wave published FULL(g + 1) once
// its own share of g + 1 had landed and FREE(g - 1) as it started piece g, waited for all 8 FULL(g) before reading
// and all 8 FREE(g - 1) before refilling, so the waves could drift by about a piece: the pw2 + FFN program went
// 5.69 -> 6.38 ms per C2 step; the phase stamps, profiles/r06/rowprog_ring/, put the loss in the slot-free polls
// (36.8k -> 66.5k cycles per tile) while the piece waits did not shrink (46.6k -> 51.6k): the polls take LDS
// issue slots from the fragment reads that already bound the streaming phase, and a one-piece drift absorbs
// none of the epilogue-sized skew.  Deleted; git history holds it.)
// MFMA accumulators in the VGPR form (the 2-tile layout spilled to scratch with the default AGPR form)
// sdiar-build: -mllvm -amdgpu-mfma-vgpr-form=1
#include <cstring>
#include <vector>
#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {
namespace {

constexpr int kD = 384;
constexpr int kFT = kD / 16;          // 24 feature tiles of 16
constexpr int kKK = kD / 32;          // 12 k-steps over D
constexpr int kRows = 128;            // tokens per tile
constexpr int kFrag = 512;            // bf16 per fragment (64 lanes x 8)
constexpr int kPieceFrags = 24;
constexpr int kPiece = kPieceFrags * kFrag;   // 12288 bf16 = 24 KiB
constexpr int kNSlot = 5;
constexpr int kMaxHidden = 1024;
constexpr int kPD = 3;                // fragment reads in flight ahead of the MFMA that uses them
constexpr int kRefillAt = 8;          // the DMA refill is issued after this many MFMAs of a piece (round 6 sweep 0 / 3 / 8 / 16 / 22: 8)
// LDS parameter block (floats): b0 | per FFN: post_g post_b b2 (D each) b1 (kMaxHidden) | y_g y_b
constexpr int kPrmFfn = 3 * kD + kMaxHidden;
constexpr int kPrmB0 = 0, kPrmFfn0 = kD, kPrmY = kD + 2 * kPrmFfn;
constexpr int kPrmGn = kPrmY + 2 * kD;   // GroupNorm gamma | beta of the pre-GEMM's A transform
constexpr int kPrmFloats = (kPrmGn + 2 * kD + 255) / 256 * 256;   // padded to whole KiB
constexpr size_t kSmemBytes = sizeof(uint16_t) * (size_t)kNSlot * kPiece + sizeof(float) * kPrmFloats;
static_assert((kPrmFloats * 4) % 1024 == 0, "ring slots stay 1-KiB aligned");
static_assert(kSmemBytes <= 160 * 1024, "LDS budget");
typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// Piece g has landed once at most `younger` pieces' DMAs (DPW per wave each) are outstanding; any other
// VMEM operation issued after g's DMAs only makes the count conservative.
template <int DPW>
__device__ __forceinline__ void wait_piece(int younger) {
  static_assert(kNSlot == 5, "wait_piece counts");
  if (younger <= 0) wait_vm<0>();
  else if (younger == 1) wait_vm<DPW>();
  else if (younger == 2) wait_vm<2 * DPW>();
  else wait_vm<3 * DPW>();
}

__device__ __forceinline__ float silu(float v) { return v * sigmoid_rcp(v); }

// TT 16-token MFMA column tiles per wave; 8 / TT waves per 128-token tile.
template <int TT>
struct Ring {
  static constexpr int kWaves = 8 / TT;
  static constexpr int kDpw = kPieceFrags / kWaves;   // 1-KiB DMA instructions per wave and piece
  const uint16_t *w0, *wf0, *wf1;   // piece sources: pre-GEMM, FFN 0, FFN 1
  uint16_t* ring;
  int P;        // pieces per tile
  int n_pre;    // pre-GEMM pieces
  int n_f0;     // pieces of FFN 0
  int total;    // pieces this workgroup consumes
  int w, lane;
  bool dma;     // probe: false skips the weight stream

  __device__ __forceinline__ const uint16_t* src(int q) const {
    if (q < n_pre) return w0 + (size_t)q * kPiece;
    q -= n_pre;
    if (q < n_f0) return wf0 + (size_t)q * kPiece;
    return wf1 + (size_t)(q - n_f0) * kPiece;
  }
  __device__ __forceinline__ void issue(int g) const {
    if (g >= total || !dma) return;
    const uint16_t* s = src(g % P);
    uint16_t* slot = ring + (g % kNSlot) * kPiece;
#pragma unroll
    for (int j = 0; j < kDpw; ++j) {
      const int f = w + kWaves * j;
      dma_lds16(s + f * kFrag + lane * 8, (lds_ptr_t)(slot + f * kFrag));
    }
  }
  // Wait for piece g and make every wave's part visible; returns g's slot.  The slot of piece g - 1 is
  // free from here on: refill(g) (called a few MFMAs into the piece) streams piece g + kNSlot - 1 into it.
  __device__ __forceinline__ const uint16_t* wait(int g) const {
    wait_piece<kDpw>(min(kNSlot - 2, total - 1 - g));
    // plain s_barrier: __syncthreads()' workgroup fence waits for vmcnt(0) and would drain the ring
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    return ring + (g % kNSlot) * kPiece;
  }
  __device__ __forceinline__ void refill(int g) const { issue(g + kNSlot - 1); }
};

__device__ __forceinline__ bf16x8 frag(const uint16_t* slot, int f, int lane) {
  return *reinterpret_cast<const bf16x8*>(slot + f * kFrag + lane * 8);
}

template <bool ON>
__device__ __forceinline__ floatx4 mfma(const bf16x8& a, const bf16x8& b, const floatx4& c) {
  if constexpr (ON) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  else return c;
}

// LayerNorm statistics of this lane's token of column tile tt (two-pass, biased variance, as torch).
template <int TT>
__device__ __forceinline__ void ln_stats(const floatx4 (&acc)[kFT][TT], int tt, float eps, float& mean, float& rstd) {
  float s = 0.f;
#pragma unroll
  for (int ft = 0; ft < kFT; ++ft) s += (acc[ft][tt][0] + acc[ft][tt][1]) + (acc[ft][tt][2] + acc[ft][tt][3]);
  s += __shfl_xor(s, 16, 64);
  s += __shfl_xor(s, 32, 64);
  const float m = s * (1.f / kD);
  float q = 0.f;
#pragma unroll
  for (int ft = 0; ft < kFT; ++ft)
#pragma unroll
    for (int r = 0; r < 4; ++r) q += (acc[ft][tt][r] - m) * (acc[ft][tt][r] - m);
  q += __shfl_xor(q, 16, 64);
  q += __shfl_xor(q, 32, 64);
  mean = m;
  rstd = rsqrtf(q * (1.f / kD) + eps);
}

template <int TT>
__device__ __forceinline__ void add_bias(floatx4 (&acc)[kFT][TT], const float* b, int g4) {
#pragma unroll
  for (int ft = 0; ft < kFT; ++ft) {
    const float4 v = *reinterpret_cast<const float4*>(b + 16 * ft + g4);
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) {
      acc[ft][tt][0] += v.x; acc[ft][tt][1] += v.y; acc[ft][tt][2] += v.z; acc[ft][tt][3] += v.w;
    }
    asm volatile("" ::: "memory");   // parameter reads one tile at a time (register pressure)
  }
}

// PROG >= 0 fixes the program's structure at compile time (bit 0: pre-GEMM, bits 1-2: FFN count) so each
// program is its own symbol in rocprof traces / PMC passes and carries no structure branches; -1 reads it
// from the arguments (probe and 2-tile variants).
template <int TT, int PROBE, int PROG = -1>
__global__ __launch_bounds__(512 / TT) __attribute__((amdgpu_waves_per_eu(2 / TT, 2 / TT)))
void rowprog_kernel(RowProgArgs a) {
  constexpr int kWaves = 8 / TT, kThreads = 64 * kWaves;
  extern __shared__ __attribute__((aligned(1024))) uint16_t sm[];
  // parameters first: their addresses stay within ds_read's 16-bit immediate offset of one base register
  float* prm = reinterpret_cast<float*>(sm);
  uint16_t* ring = sm + 2 * kPrmFloats;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, g4 = (lane >> 4) * 4;
  constexpr bool do_mfma = !(PROBE & 1), do_lds = !(PROBE & 4);
  const bool has_pre = PROG >= 0 ? (PROG & 1) != 0 : a.w0 != nullptr;
  const int nffn = PROG >= 0 ? (PROG >> 1) : a.n_ffn;
  // odd workgroups start late, so their epilogue store bursts fall into the even ones' MFMA streaming
  // (delaying only the workgroups with a tile fewer, which have a tile of slack, measured no gain)
  if (blockIdx.x & 1)
    for (int i = 0; i < a.stagger; ++i) __builtin_amdgcn_s_sleep(64);

  // parameters -> LDS (before the first DMA, so the compiler's waits for these loads do not drain the ring)
  auto cp = [&](int off, const float* p, int n) {
    if (!p) return;
    for (int i = tid; i < n; i += kThreads) prm[off + i] = p[i];
  };
  cp(kPrmB0, a.b0, kD);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if (i >= nffn) break;
    const RowFfnArgs& f = a.ffn[i];
    const int o = kPrmFfn0 + i * kPrmFfn;
    cp(o, f.post_g, kD);
    cp(o + kD, f.post_b, kD);
    cp(o + 2 * kD, f.b2, kD);
    cp(o + 3 * kD, f.b1, f.hidden);
  }
  cp(kPrmY, a.y_g, kD);
  cp(kPrmY + kD, a.y_b, kD);
  cp(kPrmGn, a.gn_g, kD);
  cp(kPrmGn + kD, a.gn_b, kD);
  __syncthreads();

  const int ntiles = (a.M + kRows - 1) / kRows;
  const int my_tiles = blockIdx.x < ntiles ? (ntiles - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  Ring<TT> R;
  R.w0 = static_cast<const uint16_t*>(a.w0);
  R.wf0 = static_cast<const uint16_t*>(a.ffn[0].w);
  R.wf1 = static_cast<const uint16_t*>(a.ffn[1].w);
  R.ring = ring;
  R.n_pre = has_pre ? kKK : 0;
  R.n_f0 = nffn > 0 ? 2 * (a.ffn[0].hidden / 32) : 0;
  R.P = R.n_pre + R.n_f0 + (nffn > 1 ? 2 * (a.ffn[1].hidden / 32) : 0);
  R.total = my_tiles * R.P;
  R.w = w;
  R.lane = lane;
  R.dma = !(PROBE & 2);
  // PROBE & 8: phase cycles per wave (RowProgArgs::probe)
  constexpr bool kStamp = (PROBE & 8) != 0;
  unsigned long long st_acc[5] = {0, 0, 0, 0, 0};
  const unsigned long long st_t0 = kStamp ? __builtin_amdgcn_s_memtime() : 0;
  auto now = [&]() -> unsigned long long { return kStamp ? __builtin_amdgcn_s_memtime() : 0ull; };
  for (int g = 0; g < kNSlot - 1; ++g) R.issue(g);
  int g = 0;
  auto pwait = [&](int q) {
    if constexpr (kStamp) {
      const unsigned long long t = now();
      const uint16_t* r = R.wait(q);
      st_acc[1] += now() - t;
      return r;
    } else {
      return R.wait(q);
    }
  };
  auto prefill = [&](int q) {
    if constexpr (kStamp) {
      const unsigned long long t = now();
      R.refill(q);
      st_acc[2] += now() - t;
    } else {
      R.refill(q);
    }
  };
  // probe 4: fragments from registers instead of LDS
  const bf16x8 wconst = __builtin_bit_cast(bf16x8, make_uint4(0x3c003c00u, 0u, 0u, 0u));
  auto rd = [&](const uint16_t* slot, int f) {
    if constexpr (do_lds) return frag(slot, f, lane);
    else return wconst;
  };

  for (int it = 0; it < my_tiles; ++it) {
    const int tile = blockIdx.x + it * gridDim.x;
    unsigned long long t_ld = now();
    int64_t row[TT];
    bool live[TT];
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) {
      row[tt] = (int64_t)tile * kRows + w * 16 * TT + 16 * tt + l15;   // this lane's token of column tile tt
      live[tt] = row[tt] < a.M;
    }

    floatx4 acc[kFT][TT];
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) {
      if (a.x_ts) {
        // [ts_embed | mix] built on load (features 0..191 from the speaker's embedding, 192..383 from
        // the mixture frame), as build_speaker_input_kernel writes them
        constexpr int kSE = kD / 2;
        const int64_t sq = row[tt] / a.T_seq;
        const int t = (int)(row[tt] - sq * a.T_seq);
        const float* tsr = a.x_ts + sq * kSE + g4;
        const bool mv = live[tt] && t < a.x_Tmix;
        const float* mxr = a.x_mix + ((sq / a.x_NS) * a.x_Tmix + (mv ? t : 0)) * (int64_t)a.x_ldmix + g4 - kSE;
#pragma unroll
        for (int ft = 0; ft < kFT; ++ft) {
          const bool ts_half = 16 * ft < kSE;
          const float4 v = !live[tt] ? make_float4(0.f, 0.f, 0.f, 0.f)
                           : ts_half ? *reinterpret_cast<const float4*>(tsr + 16 * ft)
                           : mv      ? *reinterpret_cast<const float4*>(mxr + 16 * ft)
                                     : make_float4(0.f, 0.f, 0.f, 0.f);
          acc[ft][tt] = floatx4{v.x, v.y, v.z, v.w};
        }
      } else {
        // row-major: feature 16 ft + g4 of the row; tiled: run ft of the row's 16-row group, this lane's 16 B
        const float* xr = a.x_tiled ? a.X + (row[tt] - l15) * kD + lane * 4 : a.X + row[tt] * kD + g4;
        const int fs = a.x_tiled ? 256 : 16;
#pragma unroll
        for (int ft = 0; ft < kFT; ++ft) {
          const float4 v = live[tt] ? *reinterpret_cast<const float4*>(xr + fs * ft) : make_float4(0.f, 0.f, 0.f, 0.f);
          acc[ft][tt] = floatx4{v.x, v.y, v.z, v.w};
        }
      }
    }

    if constexpr (kStamp) st_acc[4] += now() - t_ld;
    // ---- pre-GEMM: acc += A · W0ᵀ + b0 (A rows in natural k order, 16 B per lane and k-step)
    if (has_pre) {
      bf16x8 af[TT][kKK];
#pragma unroll
      for (int tt = 0; tt < TT; ++tt) {
        // row-major: features 32 kk + 8 q of the row; tiled: fragment kk of the row's 16-row group, this lane's 16 B
        const uint16_t* ar = a.a_tiled ? static_cast<const uint16_t*>(a.A) + (row[tt] - l15) * kD + lane * 8
                                       : static_cast<const uint16_t*>(a.A) + row[tt] * kD + 2 * g4;
        const int ks = a.a_tiled ? 512 : 32;
#pragma unroll
        for (int kk = 0; kk < kKK; ++kk)
          af[tt][kk] = __builtin_bit_cast(
              bf16x8, live[tt] ? *reinterpret_cast<const uint4*>(ar + ks * kk) : make_uint4(0u, 0u, 0u, 0u));
      }
      if (a.gn_partial) {
        // A = silu(GroupNorm(A)): the conformer conv module's GroupNorm(1 group) + SiLU, applied on load
        // with groupnorm_silu_kernel's arithmetic (ops.hip: statistics in double from the dwconv partials)
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) {
          const int64_t sq = live[tt] ? row[tt] / a.gn_T : 0;
          double sum = 0.0, ssq = 0.0;
          for (int i = 0; i < a.gn_nblk; ++i) {
            sum += a.gn_partial[(sq * a.gn_nblk + i) * 2];
            ssq += a.gn_partial[(sq * a.gn_nblk + i) * 2 + 1];
          }
          const double n = (double)a.gn_T * kD;
          const double mean = sum / n;
          double var = ssq / n - mean * mean;
          if (var < 0) var = 0;
          const float fm = (float)mean;
          const float rstd = (float)(1.0 / sqrt(var + (double)a.eps));
#pragma unroll
          for (int kk = 0; kk < kKK; ++kk) {
            const int c = 32 * kk + 2 * g4;
            const float4 g0 = *reinterpret_cast<const float4*>(prm + kPrmGn + c);
            const float4 g1 = *reinterpret_cast<const float4*>(prm + kPrmGn + c + 4);
            const float4 b0 = *reinterpret_cast<const float4*>(prm + kPrmGn + kD + c);
            const float4 b1 = *reinterpret_cast<const float4*>(prm + kPrmGn + kD + c + 4);
            const float gg[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
            const float bb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
            const uint4 u = __builtin_bit_cast(uint4, af[tt][kk]);
            const uint32_t w4[4] = {u.x, u.y, u.z, u.w};
            uint32_t pk[4];
#pragma unroll
            for (int h = 0; h < 4; ++h) {
              float x0 = (__uint_as_float(w4[h] << 16) - fm) * rstd * gg[2 * h] + bb[2 * h];
              float x1 = (__uint_as_float(w4[h] & 0xffff0000u) - fm) * rstd * gg[2 * h + 1] + bb[2 * h + 1];
              x0 = x0 * sigmoid_rcp(x0);
              x1 = x1 * sigmoid_rcp(x1);
              pk[h] = pack_bf16x2(x0, x1);
            }
            af[tt][kk] = __builtin_bit_cast(bf16x8, make_uint4(pk[0], pk[1], pk[2], pk[3]));
            asm volatile("" ::: "memory");
          }
        }
      }
#pragma unroll
      for (int kk = 0; kk < kKK; ++kk) {
        const uint16_t* slot = pwait(g);
        bf16x8 wq[kPD];
#pragma unroll
        for (int q = 0; q < kPD; ++q) wq[q] = rd(slot, q);
#pragma unroll
        for (int ft = 0; ft < kFT; ++ft) {
          const bf16x8 wc = wq[ft % kPD];
          if (ft + kPD < kFT) wq[ft % kPD] = rd(slot, ft + kPD);
#pragma unroll
          for (int tt = 0; tt < TT; ++tt) acc[ft][tt] = mfma<do_mfma>(wc, af[tt][kk], acc[ft][tt]);
          if (ft == kRefillAt) prefill(g);
          asm volatile("" ::: "memory");   // kPD fragment reads ahead, not the whole piece
        }
        ++g;
      }
      add_bias<TT>(acc, prm + kPrmB0, g4);
    }

    // ---- FFN modules (torchaudio _FeedForwardModule, residual x * 0.5 folded into W2 / b2)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i >= nffn) break;
      const float* pf = prm + kPrmFfn0 + i * kPrmFfn;
      bf16x8 af[TT][kKK];
#pragma unroll
      for (int tt = 0; tt < TT; ++tt) {
        // the LayerNorm affine is folded into W1 / b1 (rowprog_pack_ffn): only (x - mean) * rstd here
        float mean, rstd;
        ln_stats<TT>(acc, tt, a.eps, mean, rstd);
        const float nm = -mean * rstd;
#pragma unroll
        for (int kk = 0; kk < kKK; ++kk) {
          uint32_t pk[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int j0 = 2 * u, j1 = 2 * u + 1;
            pk[u] = pack_bf16x2(fmaf(acc[2 * kk + (j0 >> 2)][tt][j0 & 3], rstd, nm),
                                fmaf(acc[2 * kk + (j1 >> 2)][tt][j1 & 3], rstd, nm));
          }
          af[tt][kk] = __builtin_bit_cast(bf16x8, make_uint4(pk[0], pk[1], pk[2], pk[3]));
        }
      }
      const int nch = a.ffn[i].hidden / 32;
      const float* b1 = pf + 3 * kD;
#pragma unroll 1
      for (int c = 0; c < nch; ++c) {
        // up projection: hidden features 32c + 16f + 4g + r
        const uint16_t* up = pwait(g);
        floatx4 u[2][TT];
#pragma unroll
        for (int f = 0; f < 2; ++f)
#pragma unroll
          for (int tt = 0; tt < TT; ++tt) u[f][tt] = floatx4{0.f, 0.f, 0.f, 0.f};
        // fragment order: step j = (k-step j / 2, up tile j % 2) at piece fragment (j % 2) * 12 + j / 2
        bf16x8 wq[kPD];
#pragma unroll
        for (int q = 0; q < kPD; ++q) wq[q] = rd(up, (q & 1) * kKK + (q >> 1));
#pragma unroll
        for (int j = 0; j < 2 * kKK; ++j) {
          const bf16x8 wc = wq[j % kPD];
          if (j + kPD < 2 * kKK) wq[j % kPD] = rd(up, ((j + kPD) & 1) * kKK + ((j + kPD) >> 1));
#pragma unroll
          for (int tt = 0; tt < TT; ++tt) u[j & 1][tt] = mfma<do_mfma>(wc, af[tt][j >> 1], u[j & 1][tt]);
          if (j == kRefillAt) prefill(g);
          asm volatile("" ::: "memory");
        }
        ++g;
        const float4 c0 = *reinterpret_cast<const float4*>(b1 + 32 * c + g4);
        const float4 c1 = *reinterpret_cast<const float4*>(b1 + 32 * c + 16 + g4);
        bf16x8 hf[TT];
#pragma unroll
        for (int tt = 0; tt < TT; ++tt)
          hf[tt] = __builtin_bit_cast(
              bf16x8, make_uint4(pack_bf16x2(silu(u[0][tt][0] + c0.x), silu(u[0][tt][1] + c0.y)),
                                 pack_bf16x2(silu(u[0][tt][2] + c0.z), silu(u[0][tt][3] + c0.w)),
                                 pack_bf16x2(silu(u[1][tt][0] + c1.x), silu(u[1][tt][1] + c1.y)),
                                 pack_bf16x2(silu(u[1][tt][2] + c1.z), silu(u[1][tt][3] + c1.w))));
        // down projection: k-step c of W2 for all 24 output tiles
        const uint16_t* dn = pwait(g);
#pragma unroll
        for (int q = 0; q < kPD; ++q) wq[q] = rd(dn, q);
#pragma unroll
        for (int ft = 0; ft < kFT; ++ft) {
          const bf16x8 wc = wq[ft % kPD];
          if (ft + kPD < kFT) wq[ft % kPD] = rd(dn, ft + kPD);
#pragma unroll
          for (int tt = 0; tt < TT; ++tt) acc[ft][tt] = mfma<do_mfma>(wc, hf[tt], acc[ft][tt]);
          if (ft == kRefillAt) prefill(g);
          asm volatile("" ::: "memory");
        }
        ++g;
      }
      add_bias<TT>(acc, pf + 2 * kD, g4);
      if (a.ffn[i].post_g) {
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) {
          float mean, rstd;
          ln_stats<TT>(acc, tt, a.eps, mean, rstd);
#pragma unroll
          for (int ft = 0; ft < kFT; ++ft) {
            const float4 gq = *reinterpret_cast<const float4*>(pf + 16 * ft + g4);
            const float4 bq = *reinterpret_cast<const float4*>(pf + kD + 16 * ft + g4);
            acc[ft][tt][0] = (acc[ft][tt][0] - mean) * rstd * gq.x + bq.x;
            acc[ft][tt][1] = (acc[ft][tt][1] - mean) * rstd * gq.y + bq.y;
            acc[ft][tt][2] = (acc[ft][tt][2] - mean) * rstd * gq.z + bq.z;
            acc[ft][tt][3] = (acc[ft][tt][3] - mean) * rstd * gq.w + bq.w;
            asm volatile("" ::: "memory");
          }
        }
      }
    }

    // ---- epilogue: Xo = acc; y = LN_y(acc)
    const unsigned long long t_ep = now();
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) {
      if (a.yt && live[tt]) {
        const int64_t sq = row[tt] / a.T_seq;
        const int64_t t = row[tt] - sq * a.T_seq;
        const int64_t b = sq / a.yt_NS, spk = sq - b * a.yt_NS;
        uint16_t* yo = static_cast<uint16_t*>(a.yt) + ((b * a.T_seq + t) * a.yt_NS + spk) * kD + g4;
#pragma unroll
        for (int ft = 0; ft < kFT; ++ft)
          *reinterpret_cast<uint2*>(yo + 16 * ft) = make_uint2(pack_bf16x2(acc[ft][tt][0], acc[ft][tt][1]),
                                                              pack_bf16x2(acc[ft][tt][2], acc[ft][tt][3]));
      }
      if (a.Xo && live[tt]) {
        float* xo = a.xo_tiled ? a.Xo + (row[tt] - l15) * kD + lane * 4 : a.Xo + row[tt] * kD + g4;
        const int fs = a.xo_tiled ? 256 : 16;
#pragma unroll
        for (int ft = 0; ft < kFT; ++ft)
          *reinterpret_cast<float4*>(xo + fs * ft) =
              make_float4(acc[ft][tt][0], acc[ft][tt][1], acc[ft][tt][2], acc[ft][tt][3]);
      }
      if (a.y) {
        float mean, rstd;
        ln_stats<TT>(acc, tt, a.eps, mean, rstd);
        if (live[tt]) {
          // row-major: features 16 ft + g4 of the row; tiled (a_tiled layout): fragment ft / 2 of the row's 16-row
          // group, lane l15 + 16 (2 (ft % 2) + g4 / 8), elements g4 % 8 .. + 3
          uint16_t* yo = a.y_tiled ? static_cast<uint16_t*>(a.y) + (row[tt] - l15) * kD + (l15 + 16 * (g4 >> 3)) * 8 + (g4 & 7)
                                   : static_cast<uint16_t*>(a.y) + row[tt] * kD + g4;
#pragma unroll
          for (int ft = 0; ft < kFT; ++ft) {
            const float4 gq = *reinterpret_cast<const float4*>(prm + kPrmY + 16 * ft + g4);
            const float4 bq = *reinterpret_cast<const float4*>(prm + kPrmY + kD + 16 * ft + g4);
            const int fo = a.y_tiled ? (ft >> 1) * 512 + (ft & 1) * 256 : 16 * ft;
            *reinterpret_cast<uint2*>(yo + fo) =
                make_uint2(pack_bf16x2((acc[ft][tt][0] - mean) * rstd * gq.x + bq.x,
                                       (acc[ft][tt][1] - mean) * rstd * gq.y + bq.y),
                           pack_bf16x2((acc[ft][tt][2] - mean) * rstd * gq.z + bq.z,
                                       (acc[ft][tt][3] - mean) * rstd * gq.w + bq.w));
            asm volatile("" ::: "memory");
          }
        }
      }
    }
    if constexpr (kStamp) st_acc[3] += now() - t_ep;
  }
  wait_vm<0>();   // no DMA into this workgroup's LDS outlives it (every issued piece was consumed)
  if constexpr (kStamp) {
    st_acc[0] = now() - st_t0;
    if (lane == 0 && a.probe) {   // launches on one stream add up (the tool runs the forward one-stream)
      a.probe[((size_t)blockIdx.x * kWaves + w) * 8 + 5] += (unsigned long long)my_tiles;
#pragma unroll
      for (int k = 0; k < 5; ++k) a.probe[((size_t)blockIdx.x * kWaves + w) * 8 + k] += st_acc[k];
    }
  }
}

// Host: k index of slot j (0..7) of lane group g in k-step kk.
inline int kslot(int kk, int g, int j, bool perm) {
  if (!perm) return 32 * kk + 8 * g + j;
  return 32 * kk + (j < 4 ? 4 * g + j : 16 + 4 * g + (j - 4));
}

uint16_t f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// Fragment (row tile rt, k-step kk) of W (N x K row-major) appended to out.
void put_frag(std::vector<uint16_t>& out, const std::vector<float>& W, int K, int rt, int kk, bool perm) {
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < 8; ++j)
      out.push_back(f2bf(W[(size_t)(16 * rt + (l & 15)) * K + kslot(kk, l >> 4, j, perm)]));
}

}  // namespace

bool rowprog_supported(int D, int hidden, bool bf16) {
  static const bool off = getenv("SDIAR_NO_ROWPROG") != nullptr;   // A/B switch: the unfused path
  return !off && bf16 && D == kD && hidden > 0 && hidden % 32 == 0 && hidden <= kMaxHidden;
}

std::vector<uint16_t> rowprog_pack_pre(const std::vector<float>& W, int N, int K) {
  SD_CHECK(N == kD && K == kD && (int64_t)W.size() == (int64_t)N * K, kErrInvalid, "rowprog_pack_pre: shape");
  std::vector<uint16_t> out;
  out.reserve(W.size());
  for (int kk = 0; kk < kKK; ++kk)
    for (int ft = 0; ft < kFT; ++ft) put_frag(out, W, K, ft, kk, false);
  return out;
}

std::vector<uint16_t> rowprog_pack_ffn(const std::vector<float>& W1in, const std::vector<float>& W2, int hidden,
                                       const std::vector<float>& ln_g, const std::vector<float>& ln_b,
                                       const std::vector<float>& b1, std::vector<float>& b1_folded) {
  SD_CHECK(hidden % 32 == 0 && (int64_t)W1in.size() == (int64_t)hidden * kD && (int64_t)W2.size() == (int64_t)kD * hidden &&
               (int)ln_g.size() == kD && (int)ln_b.size() == kD && (int)b1.size() == hidden,
           kErrInvalid, "rowprog_pack_ffn: shape");
  // Linear(LN(x)) = (W1 diag(g)) x_hat + (W1 b + b1): the LayerNorm affine folded into the up projection.
  std::vector<float> W1(W1in.size());
  b1_folded.assign(hidden, 0.f);
  for (int n = 0; n < hidden; ++n) {
    double acc = b1[n];
    for (int k = 0; k < kD; ++k) {
      W1[(size_t)n * kD + k] = W1in[(size_t)n * kD + k] * ln_g[k];
      acc += (double)W1in[(size_t)n * kD + k] * ln_b[k];
    }
    b1_folded[n] = (float)acc;
  }
  std::vector<uint16_t> out;
  out.reserve(W1.size() + W2.size());
  for (int c = 0; c < hidden / 32; ++c) {
    for (int f = 0; f < 2; ++f)
      for (int kk = 0; kk < kKK; ++kk) put_frag(out, W1, kD, 2 * c + f, kk, true);   // up piece
    for (int ft = 0; ft < kFT; ++ft) put_frag(out, W2, hidden, ft, c, true);        // down piece
  }
  return out;
}

static unsigned long long* g_rp_probe = nullptr;
void rowprog_set_probe(void* stamps) { g_rp_probe = static_cast<unsigned long long*>(stamps); }

void rowprog(const RowProgArgs& a, const char* name, hipStream_t st) {
  SD_CHECK(a.n_ffn >= 0 && a.n_ffn <= 2, kErrInvalid, "rowprog: n_ffn");
  for (int i = 0; i < a.n_ffn; ++i)
    SD_CHECK(rowprog_supported(kD, a.ffn[i].hidden, true) && a.ffn[i].w &&
                 a.ffn[i].b1 && a.ffn[i].b2 && (a.ffn[i].post_g != nullptr) == (a.ffn[i].post_b != nullptr),
             kErrInvalid, "rowprog: ffn arguments");
  SD_CHECK(!a.w0 || (a.A && a.b0), kErrInvalid, "rowprog: pre-GEMM arguments");
  SD_CHECK(!a.y || (a.y_g && a.y_b), kErrInvalid, "rowprog: y LayerNorm arguments");
  SD_CHECK((a.X || a.x_ts) && (a.Xo || a.yt) && (a.w0 || a.n_ffn > 0 || a.y), kErrInvalid, "rowprog: empty program");
  SD_CHECK(!a.x_ts || (a.x_mix && a.x_NS > 0 && a.T_seq > 0 && a.x_Tmix > 0 && a.x_ldmix % 4 == 0), kErrInvalid,
           "rowprog: speaker-input source arguments");
  SD_CHECK(!a.yt || (a.yt_NS > 0 && a.T_seq > 0), kErrInvalid, "rowprog: channel-layout output arguments");
  SD_CHECK(!(a.x_tiled || a.xo_tiled || a.a_tiled || a.y_tiled) || a.M % 16 == 0, kErrInvalid,
           "rowprog: the tiled X / A layouts need M % 16 == 0");
  if (a.M <= 0) return;
  static int grid_max = 0;
  if (!grid_max) {
    int dev = 0, cus = 0;
    SD_HIP(hipGetDevice(&dev));
    SD_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const void* ks[] = {reinterpret_cast<const void*>(rowprog_kernel<1, 0, 1>), reinterpret_cast<const void*>(rowprog_kernel<1, 0, 2>),
                        reinterpret_cast<const void*>(rowprog_kernel<1, 0, 3>), reinterpret_cast<const void*>(rowprog_kernel<1, 0, 5>),
                        reinterpret_cast<const void*>(rowprog_kernel<1, 0>), reinterpret_cast<const void*>(rowprog_kernel<1, 8, 5>)};
    for (const void* k : ks)
      SD_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSmemBytes));
    grid_max = cus > 0 ? cus : 256;
  }
  const int ntiles = (a.M + kRows - 1) / kRows;
  const int grid = ntiles < grid_max ? ntiles : grid_max;
  const double rows = (double)a.M;
  double flops = a.w0 ? 2.0 * rows * kD * kD : 0.0;
  double wbytes = a.w0 ? 2.0 * kD * kD : 0.0;
  for (int i = 0; i < a.n_ffn; ++i) {
    flops += 4.0 * rows * kD * a.ffn[i].hidden;
    wbytes += 4.0 * kD * a.ffn[i].hidden;
  }
  const double bytes =
      rows * kD * (4.0 + (a.Xo ? 4.0 : 0.0) + (a.w0 ? 2.0 : 0.0) + (a.y ? 2.0 : 0.0) + (a.yt ? 2.0 : 0.0)) + wbytes;
  ProfScope prof(name, flops, bytes, st);
  const dim3 g3(grid);
  {
    // Start offset of the odd workgroups per program, in s_sleep(64) units.  A/B on one box (C2, 3-4 rounds each, every round the
    // same way): pw2+FFN (prog 5, 76 pieces per tile) 6.06 -> 5.85 ms per step at 20 (12 less, 32 / 48 no
    // better); out_proj (prog 1, 12 pieces, HBM-bound) 2.53 -> 2.42 at 8 (4: 2.45; 16: 2.53); the one-launch
    // FFN programs (2, 3) get offsets in proportion to their tile length.
    const int prog = (a.w0 ? 1 : 0) | (a.n_ffn << 1);
    RowProgArgs b = a;
    const int base = prog == 5 ? 20 : prog == 3 ? 12 : 8;
    b.stagger = ntiles > grid ? base : 0;
    if (prog == 5 && g_rp_probe) {   // diagnostics: the pw2 + FFN program with phase stamps
      b.probe = g_rp_probe;
      hipLaunchKernelGGL((rowprog_kernel<1, 8, 5>), g3, dim3(512), kSmemBytes, st, b);
    } else if (prog == 1) hipLaunchKernelGGL((rowprog_kernel<1, 0, 1>), g3, dim3(512), kSmemBytes, st, b);
    else if (prog == 2) hipLaunchKernelGGL((rowprog_kernel<1, 0, 2>), g3, dim3(512), kSmemBytes, st, b);
    else if (prog == 3) hipLaunchKernelGGL((rowprog_kernel<1, 0, 3>), g3, dim3(512), kSmemBytes, st, b);
    else if (prog == 5) hipLaunchKernelGGL((rowprog_kernel<1, 0, 5>), g3, dim3(512), kSmemBytes, st, b);
    else hipLaunchKernelGGL((rowprog_kernel<1, 0>), g3, dim3(512), kSmemBytes, st, b);
  }
  SD_LAUNCH_CHECK();
}

}  // namespace sd
