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
// Layout (transposed MFMA, v_mfma_f32_16x16x32_bf16 with weights as the A operand): a workgroup is 4 waves
// (one per SIMD, ~350 VGPRs), a wave owns 32 tokens as two 16-token column tiles.  acc[ft][tt] holds
// features 16 ft + 4 g + r (g = lane / 16) of token 16 tt + lane % 16, i.e. a token's 384 features over the
// 4 lanes that share lane % 16 (LN statistics = 2 shuffles).  The B operand of the next GEMM is built from
// that layout without any data movement: k-step kk of a lane holds features 32 kk + 4 g + {0..3} (tile 2kk)
// and 32 kk + 16 + 4 g + {0..3} (tile 2kk + 1), and the weights are packed with the same k permutation
// (rowprog_pack_*).  The FFN hidden layer is produced 32 features at a time (2 up-projection tiles), SiLU'd
// in registers and consumed at once as one k-step of the down projection.
//
// Weights stream from L2 as 24-KiB pieces of 24 pre-packed 1-KiB MFMA fragments (lane-linear, so every
// ds_read_b128 is conflict-free) through a 5-slot LDS ring (global_load_lds, 4 pieces in flight, counted
// vmcnt waits, one barrier per piece).  The workgroups are persistent over tiles; the ring runs across tile
// boundaries, so the next tile's first weights are in flight during the current tile's epilogue.
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
constexpr int kWaves = 8;             // two per SIMD
constexpr int kThreads = 64 * kWaves;
constexpr int kRows = 16 * kWaves;    // tokens per tile (one 16-token MFMA column tile per wave)
constexpr int kFrag = 512;            // bf16 per fragment (64 lanes x 8)
constexpr int kPieceFrags = 24;
constexpr int kPiece = kPieceFrags * kFrag;   // 12288 bf16 = 24 KiB
constexpr int kNSlot = 5;
constexpr int kDmaPerWave = kPieceFrags / kWaves;   // 3 x 1 KiB per wave and piece
constexpr int kMaxHidden = 1024;
// LDS parameter block (floats): b0 | per FFN: ln_g ln_b post_g post_b b2 (D each) b1 (kMaxHidden) | y_g y_b
constexpr int kPrmFfn = 5 * kD + kMaxHidden;
constexpr int kPrmB0 = 0, kPrmFfn0 = kD, kPrmY = kD + 2 * kPrmFfn;
constexpr int kPrmFloats = (kPrmY + 2 * kD + 255) / 256 * 256;   // padded to whole KiB
constexpr size_t kSmemBytes = sizeof(uint16_t) * (size_t)kNSlot * kPiece + sizeof(float) * kPrmFloats;
static_assert((kPrmFloats * 4) % 1024 == 0, "ring slots stay 1-KiB aligned");
static_assert(kSmemBytes <= 160 * 1024, "LDS budget");
typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// Piece g has landed once at most `younger` pieces' DMAs (kDmaPerWave per wave each) are outstanding; any other
// VMEM operation issued after g's DMAs only makes the count conservative.
__device__ __forceinline__ void wait_piece(int younger) {
  static_assert(kNSlot == 5, "wait_piece counts");
  if (younger <= 0) wait_vm<0>();
  else if (younger == 1) wait_vm<kDmaPerWave>();
  else if (younger == 2) wait_vm<2 * kDmaPerWave>();
  else wait_vm<3 * kDmaPerWave>();
}

__device__ __forceinline__ float silu(float v) { return v / (1.f + __expf(-v)); }

struct Ring {
  const uint16_t *w0, *wf0, *wf1;   // piece sources: pre-GEMM, FFN 0, FFN 1
  uint16_t* ring;
  int P;        // pieces per tile
  int n_pre;    // pre-GEMM pieces
  int n_f0;     // pieces of FFN 0
  int total;    // pieces this workgroup consumes
  int w, lane;

  __device__ __forceinline__ const uint16_t* src(int q) const {
    if (q < n_pre) return w0 + (size_t)q * kPiece;
    q -= n_pre;
    if (q < n_f0) return wf0 + (size_t)q * kPiece;
    return wf1 + (size_t)(q - n_f0) * kPiece;
  }
  __device__ __forceinline__ void issue(int g) const {
    if (g >= total) return;
    const uint16_t* s = src(g % P);
    uint16_t* slot = ring + (g % kNSlot) * kPiece;
#pragma unroll
    for (int j = 0; j < kDmaPerWave; ++j) {
      const int f = w + kWaves * j;
      __builtin_amdgcn_global_load_lds((const void*)(s + f * kFrag + lane * 8), (lds_ptr_t)(slot + f * kFrag), 16,
                                       0, 0);
    }
  }
  // Wait for piece g, make every wave's part visible, refill the slot of piece g - 1, return g's slot.
  __device__ __forceinline__ const uint16_t* next(int& g) const {
    wait_piece(min(kNSlot - 2, total - 1 - g));
    __syncthreads();
    issue(g + kNSlot - 1);
    const uint16_t* slot = ring + (g % kNSlot) * kPiece;
    ++g;
    return slot;
  }
};

__device__ __forceinline__ bf16x8 frag(const uint16_t* slot, int f, int lane) {
  return *reinterpret_cast<const bf16x8*>(slot + f * kFrag + lane * 8);
}

// LayerNorm statistics of this lane's token (two-pass, biased variance, as torch).
__device__ __forceinline__ void ln_stats(const floatx4 (&acc)[kFT], float eps, float& mean, float& rstd) {
  float s = 0.f;
#pragma unroll
  for (int ft = 0; ft < kFT; ++ft) s += (acc[ft][0] + acc[ft][1]) + (acc[ft][2] + acc[ft][3]);
  s += __shfl_xor(s, 16, 64);
  s += __shfl_xor(s, 32, 64);
  const float m = s * (1.f / kD);
  float q = 0.f;
#pragma unroll
  for (int ft = 0; ft < kFT; ++ft)
#pragma unroll
    for (int r = 0; r < 4; ++r) q += (acc[ft][r] - m) * (acc[ft][r] - m);
  q += __shfl_xor(q, 16, 64);
  q += __shfl_xor(q, 32, 64);
  mean = m;
  rstd = rsqrtf(q * (1.f / kD) + eps);
}

__device__ __forceinline__ void add_bias(floatx4 (&acc)[kFT], const float* b, int g4) {
#pragma unroll
  for (int ft = 0; ft < kFT; ++ft) {
    const float4 v = *reinterpret_cast<const float4*>(b + 16 * ft + g4);
    acc[ft][0] += v.x; acc[ft][1] += v.y; acc[ft][2] += v.z; acc[ft][3] += v.w;
    asm volatile("" ::: "memory");   // parameter reads one tile at a time (register pressure)
  }
}

__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2, 2)))
void rowprog_kernel(RowProgArgs a) {
  extern __shared__ __attribute__((aligned(1024))) uint16_t sm[];
  // parameters first: their addresses stay within ds_read's 16-bit immediate offset of one base register
  float* prm = reinterpret_cast<float*>(sm);
  uint16_t* ring = sm + 2 * kPrmFloats;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, g4 = (lane >> 4) * 4;

  // parameters -> LDS (before the first DMA, so the compiler's waits for these loads do not drain the ring)
  auto cp = [&](int off, const float* p, int n) {
    if (!p) return;
    for (int i = tid; i < n; i += kThreads) prm[off + i] = p[i];
  };
  cp(kPrmB0, a.b0, kD);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if (i >= a.n_ffn) break;
    const RowFfnArgs& f = a.ffn[i];
    const int o = kPrmFfn0 + i * kPrmFfn;
    cp(o, f.ln_g, kD);
    cp(o + kD, f.ln_b, kD);
    cp(o + 2 * kD, f.post_g, kD);
    cp(o + 3 * kD, f.post_b, kD);
    cp(o + 4 * kD, f.b2, kD);
    cp(o + 5 * kD, f.b1, f.hidden);
  }
  cp(kPrmY, a.y_g, kD);
  cp(kPrmY + kD, a.y_b, kD);
  __syncthreads();

  const int ntiles = (a.M + kRows - 1) / kRows;
  const int my_tiles = blockIdx.x < ntiles ? (ntiles - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  Ring R;
  R.w0 = static_cast<const uint16_t*>(a.w0);
  R.wf0 = static_cast<const uint16_t*>(a.ffn[0].w);
  R.wf1 = static_cast<const uint16_t*>(a.ffn[1].w);
  R.ring = ring;
  R.n_pre = a.w0 ? kKK : 0;
  R.n_f0 = a.n_ffn > 0 ? 2 * (a.ffn[0].hidden / 32) : 0;
  R.P = R.n_pre + R.n_f0 + (a.n_ffn > 1 ? 2 * (a.ffn[1].hidden / 32) : 0);
  R.total = my_tiles * R.P;
  R.w = w;
  R.lane = lane;
  for (int g = 0; g < kNSlot - 1; ++g) R.issue(g);
  int g = 0;

  for (int it = 0; it < my_tiles; ++it) {
    const int tile = blockIdx.x + it * gridDim.x;
    const int64_t row = (int64_t)tile * kRows + w * 16 + l15;   // this lane's token
    const bool live = row < a.M;

    floatx4 acc[kFT];
    {
      const float* xr = a.X + row * kD + g4;
#pragma unroll
      for (int ft = 0; ft < kFT; ++ft) {
        const float4 v = live ? *reinterpret_cast<const float4*>(xr + 16 * ft) : make_float4(0.f, 0.f, 0.f, 0.f);
        acc[ft] = floatx4{v.x, v.y, v.z, v.w};
      }
    }

    // ---- pre-GEMM: acc += A · W0ᵀ + b0 (A rows in natural k order, 16 B per lane and k-step)
    if (a.w0) {
      bf16x8 af[kKK];
      const uint16_t* ar = static_cast<const uint16_t*>(a.A) + row * kD + 2 * g4;
#pragma unroll
      for (int kk = 0; kk < kKK; ++kk)
        af[kk] = __builtin_bit_cast(bf16x8, live ? *reinterpret_cast<const uint4*>(ar + 32 * kk) : make_uint4(0u, 0u, 0u, 0u));
#pragma unroll
      for (int kk = 0; kk < kKK; ++kk) {
        const uint16_t* slot = R.next(g);
        bf16x8 wc = frag(slot, 0, lane);
#pragma unroll
        for (int ft = 0; ft < kFT; ++ft) {
          const bf16x8 wn = ft + 1 < kFT ? frag(slot, ft + 1, lane) : wc;
          acc[ft] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wc, af[kk], acc[ft], 0, 0, 0);
          asm volatile("" ::: "memory");   // one fragment read ahead, not the whole piece
          wc = wn;
        }
      }
      add_bias(acc, prm + kPrmB0, g4);
    }

    // ---- FFN modules (torchaudio _FeedForwardModule, residual x * 0.5 folded into W2 / b2)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i >= a.n_ffn) break;
      const float* pf = prm + kPrmFfn0 + i * kPrmFfn;
      float mean, rstd;
      ln_stats(acc, a.eps, mean, rstd);
      bf16x8 af[kKK];
#pragma unroll
      for (int kk = 0; kk < kKK; ++kk) {
        const float4 ga = *reinterpret_cast<const float4*>(pf + 32 * kk + g4);
        const float4 gb = *reinterpret_cast<const float4*>(pf + 32 * kk + 16 + g4);
        const float4 ba = *reinterpret_cast<const float4*>(pf + kD + 32 * kk + g4);
        const float4 bb = *reinterpret_cast<const float4*>(pf + kD + 32 * kk + 16 + g4);
        const float gg[8] = {ga.x, ga.y, ga.z, ga.w, gb.x, gb.y, gb.z, gb.w};
        const float bv[8] = {ba.x, ba.y, ba.z, ba.w, bb.x, bb.y, bb.z, bb.w};
        uint32_t pk[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int j0 = 2 * u, j1 = 2 * u + 1;
          pk[u] = pack_bf16x2((acc[2 * kk + (j0 >> 2)][j0 & 3] - mean) * rstd * gg[j0] + bv[j0],
                              (acc[2 * kk + (j1 >> 2)][j1 & 3] - mean) * rstd * gg[j1] + bv[j1]);
        }
        af[kk] = __builtin_bit_cast(bf16x8, make_uint4(pk[0], pk[1], pk[2], pk[3]));
        asm volatile("" ::: "memory");
      }
      const int nch = a.ffn[i].hidden / 32;
      const float* b1 = pf + 5 * kD;
#pragma unroll 1
      for (int c = 0; c < nch; ++c) {
        // up projection: hidden features 32c + 16f + 4g + r
        const uint16_t* up = R.next(g);
        floatx4 u0 = {0.f, 0.f, 0.f, 0.f}, u1 = {0.f, 0.f, 0.f, 0.f};
        bf16x8 w0c = frag(up, 0, lane), w1c = frag(up, kKK, lane);
#pragma unroll
        for (int kk = 0; kk < kKK; ++kk) {
          const bf16x8 w0n = kk + 1 < kKK ? frag(up, kk + 1, lane) : w0c;
          const bf16x8 w1n = kk + 1 < kKK ? frag(up, kKK + kk + 1, lane) : w1c;
          u0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0c, af[kk], u0, 0, 0, 0);
          u1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1c, af[kk], u1, 0, 0, 0);
          asm volatile("" ::: "memory");
          w0c = w0n;
          w1c = w1n;
        }
        const float4 c0 = *reinterpret_cast<const float4*>(b1 + 32 * c + g4);
        const float4 c1 = *reinterpret_cast<const float4*>(b1 + 32 * c + 16 + g4);
        const bf16x8 hf = __builtin_bit_cast(
            bf16x8, make_uint4(pack_bf16x2(silu(u0[0] + c0.x), silu(u0[1] + c0.y)),
                               pack_bf16x2(silu(u0[2] + c0.z), silu(u0[3] + c0.w)),
                               pack_bf16x2(silu(u1[0] + c1.x), silu(u1[1] + c1.y)),
                               pack_bf16x2(silu(u1[2] + c1.z), silu(u1[3] + c1.w))));
        // down projection: k-step c of W2 for all 24 output tiles
        const uint16_t* dn = R.next(g);
        bf16x8 wc = frag(dn, 0, lane);
#pragma unroll
        for (int ft = 0; ft < kFT; ++ft) {
          const bf16x8 wn = ft + 1 < kFT ? frag(dn, ft + 1, lane) : wc;
          acc[ft] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wc, hf, acc[ft], 0, 0, 0);
          asm volatile("" ::: "memory");
          wc = wn;
        }
      }
      add_bias(acc, pf + 4 * kD, g4);
      if (a.ffn[i].post_g) {
        ln_stats(acc, a.eps, mean, rstd);
#pragma unroll
        for (int ft = 0; ft < kFT; ++ft) {
          const float4 gq = *reinterpret_cast<const float4*>(pf + 2 * kD + 16 * ft + g4);
          const float4 bq = *reinterpret_cast<const float4*>(pf + 3 * kD + 16 * ft + g4);
          acc[ft][0] = (acc[ft][0] - mean) * rstd * gq.x + bq.x;
          acc[ft][1] = (acc[ft][1] - mean) * rstd * gq.y + bq.y;
          acc[ft][2] = (acc[ft][2] - mean) * rstd * gq.z + bq.z;
          acc[ft][3] = (acc[ft][3] - mean) * rstd * gq.w + bq.w;
          asm volatile("" ::: "memory");
        }
      }
    }

    // ---- epilogue: Xo = acc; y = LN_y(acc)
    if (live) {
      float* xo = a.Xo + row * kD + g4;
#pragma unroll
      for (int ft = 0; ft < kFT; ++ft)
        *reinterpret_cast<float4*>(xo + 16 * ft) = make_float4(acc[ft][0], acc[ft][1], acc[ft][2], acc[ft][3]);
    }
    if (a.y) {
      float mean, rstd;
      ln_stats(acc, a.eps, mean, rstd);
      if (live) {
        uint16_t* yo = static_cast<uint16_t*>(a.y) + row * kD + g4;
#pragma unroll
        for (int ft = 0; ft < kFT; ++ft) {
          const float4 gq = *reinterpret_cast<const float4*>(prm + kPrmY + 16 * ft + g4);
          const float4 bq = *reinterpret_cast<const float4*>(prm + kPrmY + kD + 16 * ft + g4);
          *reinterpret_cast<uint2*>(yo + 16 * ft) =
              make_uint2(pack_bf16x2((acc[ft][0] - mean) * rstd * gq.x + bq.x, (acc[ft][1] - mean) * rstd * gq.y + bq.y),
                         pack_bf16x2((acc[ft][2] - mean) * rstd * gq.z + bq.z, (acc[ft][3] - mean) * rstd * gq.w + bq.w));
          asm volatile("" ::: "memory");
        }
      }
    }
  }
  wait_vm<0>();   // no DMA into this workgroup's LDS outlives it (every issued piece was consumed)
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

std::vector<uint16_t> rowprog_pack_ffn(const std::vector<float>& W1, const std::vector<float>& W2, int hidden) {
  SD_CHECK(hidden % 32 == 0 && (int64_t)W1.size() == (int64_t)hidden * kD && (int64_t)W2.size() == (int64_t)kD * hidden,
           kErrInvalid, "rowprog_pack_ffn: shape");
  std::vector<uint16_t> out;
  out.reserve(W1.size() + W2.size());
  for (int c = 0; c < hidden / 32; ++c) {
    for (int f = 0; f < 2; ++f)
      for (int kk = 0; kk < kKK; ++kk) put_frag(out, W1, kD, 2 * c + f, kk, true);   // up piece
    for (int ft = 0; ft < kFT; ++ft) put_frag(out, W2, hidden, ft, c, true);        // down piece
  }
  return out;
}

void rowprog(const RowProgArgs& a, const char* name, hipStream_t st) {
  SD_CHECK(a.n_ffn >= 0 && a.n_ffn <= 2, kErrInvalid, "rowprog: n_ffn");
  for (int i = 0; i < a.n_ffn; ++i)
    SD_CHECK(rowprog_supported(kD, a.ffn[i].hidden, true) && a.ffn[i].w && a.ffn[i].ln_g && a.ffn[i].ln_b &&
                 a.ffn[i].b1 && a.ffn[i].b2 && (a.ffn[i].post_g != nullptr) == (a.ffn[i].post_b != nullptr),
             kErrInvalid, "rowprog: ffn arguments");
  SD_CHECK(!a.w0 || (a.A && a.b0), kErrInvalid, "rowprog: pre-GEMM arguments");
  SD_CHECK(!a.y || (a.y_g && a.y_b), kErrInvalid, "rowprog: y LayerNorm arguments");
  SD_CHECK(a.X && a.Xo && (a.w0 || a.n_ffn > 0 || a.y), kErrInvalid, "rowprog: empty program");
  if (a.M <= 0) return;
  static int grid_max = 0;
  if (!grid_max) {
    int dev = 0, cus = 0;
    SD_HIP(hipGetDevice(&dev));
    SD_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(rowprog_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSmemBytes));
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
  const double bytes = rows * kD * (8.0 + (a.w0 ? 2.0 : 0.0) + (a.y ? 2.0 : 0.0)) + wbytes;
  ProfScope prof(name, flops, bytes, st);
  hipLaunchKernelGGL(rowprog_kernel, dim3(grid), dim3(kThreads), kSmemBytes, st, a);
  SD_LAUNCH_CHECK();
}

}  // namespace sd
