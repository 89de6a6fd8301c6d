// Conformer convolution module body fused for gfx950 (C2: torchaudio ConvolutionModule inside ConformerLayer,
// ts_vad2/model.py:259-267, restated in oracle/tsvad_ref.py conformer()): pointwise_conv1 (D -> 2D) + GLU
// and the depthwise conv (k taps, zero padding) of ONE sequence per workgroup, with the GLU output h kept
// in LDS.  Replaces gemm_areg (pw1 + GLU epilogue) + glu_dwconv, whose (S*T, D) bf16 h made an HBM round
// trip.  The GroupNorm statistics leave as the same per-(sequence, 64-channel block) partial sums
// glu_dwconv wrote (GroupNorm + SiLU are applied by the next row program as it loads this output).
//
// Workgroup: 5 waves, wave w owns tokens 32w .. 32w+31 as two 16-token MFMA column tiles; T <= 152.
//   prologue  the LayerNorm'd rows y (bf16) of the wave's tokens -> MFMA B-operand fragments (96 VGPRs);
//   pieces    pw1 weights as 48 pieces of 12 KiB = (GLU group n of 16 channels: value + gate tiles) x one
//             K half, pre-packed in fragment order (lane-linear: conflict-free ds_read_b128), through a
//             3-slot LDS-DMA ring, one piece in flight behind counted vmcnt waits; after a group's second
//             half: h = (v + bv) / (1 + exp(-(gate + bg))) (gemm_areg's GLU arithmetic) -> LDS h[t][c];
//   dwconv    lane = channel: a register window over the LDS column, 8 outputs per run, taps in registers
//             (glu_dwconv's fmaf order), bf16 stores; block-5 channels split over all waves by time.
#include <cstring>
#include <vector>
#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {
namespace {

constexpr int kD = 384;
constexpr int kTMax = 152;                 // h rows held in LDS
constexpr int kWaves = 5;
constexpr int kThreads = 64 * kWaves;
constexpr int kKK = kD / 32;               // 12 k-steps
constexpr int kGroups = kD / 16;           // 24 GLU groups
constexpr int kPieceFr = 12;               // fragments per piece: 2 tiles x 6 k-steps
constexpr int kPieceElems = kPieceFr * 512;
constexpr int kPieces = 2 * kGroups;       // 48
constexpr int kNSlot = 3;
constexpr int kHS = kD + 4;                // h row stride (bf16): 776 B, spreads 8-B epilogue writes over banks
constexpr int kRun = 8;                    // dwconv outputs per run
constexpr int kMaxK = 31;
constexpr int kCB = kD / 64;               // 64-channel blocks (GroupNorm partials per sequence)
constexpr size_t kSmemBytes = sizeof(uint16_t) * ((size_t)kNSlot * kPieceElems + (size_t)kTMax * kHS) +
                              sizeof(float) * (2 * kD + 2 * kCB * kWaves);
static_assert(kSmemBytes <= 160 * 1024, "LDS budget");
constexpr uint32_t kOOB = 0x80000000u;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__global__ __launch_bounds__(kThreads) void conv_block_kernel(ConvBlockArgs a) {
  extern __shared__ __attribute__((aligned(1024))) uint16_t sm[];
  uint16_t* ring = sm;                                        // [kNSlot][12 frags][512]
  uint16_t* hs = sm + kNSlot * kPieceElems;                   // [kTMax][kHS]
  float* s_bias = reinterpret_cast<float*>(hs + kTMax * kHS);  // [2D] interleaved pw1 bias
  float* s_stat = s_bias + 2 * kD;                            // [2][kCB][kWaves]
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, lk = lane >> 4;
  const int s = blockIdx.x, T = a.T;

  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w1), (short)0,
                                                                      (int)kOOB, 0x00020000);
  // 12 DMA instructions per piece: waves 0 and 1 issue three, the others two
  const int my_dma = w < 2 ? 3 : 2;
  auto issue = [&](int p) {
    uint16_t* slot = ring + (p % kNSlot) * kPieceElems;
    for (int j = w; j < kPieceFr; j += kWaves) {
      const uint32_t off = (uint32_t)(((p * kPieceFr + j) * 512 + lane * 8) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_ptr_t)(slot + j * 512), 16, off, 0, 0, 0);
    }
  };
  issue(0);
  issue(1);
  for (int i = tid; i < 2 * kD; i += kThreads) s_bias[i] = a.b1[i];

  // ---- prologue: B fragments of the wave's two token tiles (natural k order), zero past T
  bf16x8 af[2][kKK];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int t = 32 * w + 16 * tt + l15;
    const uint16_t* yr = static_cast<const uint16_t*>(a.y) + ((int64_t)s * T + t) * kD + 8 * lk;
#pragma unroll
    for (int kk = 0; kk < kKK; ++kk)
      af[tt][kk] = __builtin_bit_cast(bf16x8, t < T ? *reinterpret_cast<const uint4*>(yr + 32 * kk)
                                                    : make_uint4(0u, 0u, 0u, 0u));
  }

  // ---- pw1 + GLU into LDS h
  bool drain = true;   // the prologue's loads are younger than pieces 0 and 1
#pragma unroll 1
  for (int n = 0; n < kGroups; ++n) {
    floatx4 av[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    floatx4 ag[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int p = 2 * n + h;
      if (drain || p + 1 >= kPieces) wait_vm<0>();
      else if (my_dma == 3) wait_vm<3>();
      else wait_vm<2>();
      drain = false;
      __syncthreads();   // piece p landed for every wave; the slot of piece p - 1 is free
      if (p + 2 < kPieces) issue(p + 2);
      const uint16_t* slot = ring + (p % kNSlot) * kPieceElems;
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        const bf16x8 wv = *reinterpret_cast<const bf16x8*>(slot + q * 512 + lane * 8);
        const bf16x8 wg = *reinterpret_cast<const bf16x8*>(slot + (6 + q) * 512 + lane * 8);
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          av[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv, af[tt][6 * h + q], av[tt], 0, 0, 0);
          ag[tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wg, af[tt][6 * h + q], ag[tt], 0, 0, 0);
        }
      }
    }
    // lane: channels 16n + 4lk + r of token 32w + 16tt + l15; interleaved bias rows 32n + [0|16] + 4lk + r
    const float4 bv = *reinterpret_cast<const float4*>(s_bias + 32 * n + 4 * lk);
    const float4 bg = *reinterpret_cast<const float4*>(s_bias + 32 * n + 16 + 4 * lk);
    const float bvv[4] = {bv.x, bv.y, bv.z, bv.w}, bgg[4] = {bg.x, bg.y, bg.z, bg.w};
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int t = 32 * w + 16 * tt + l15;
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = av[tt][r] + bvv[r], gt = ag[tt][r] + bgg[r];
        o[r] = v / (1.f + __expf(-gt));
      }
      if (t < T)
        *reinterpret_cast<uint2*>(hs + t * kHS + 16 * n + 4 * lk) =
            make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]));
    }
  }
  __syncthreads();   // h complete

  // ---- depthwise conv: wave w runs channel block w over all runs, plus runs w, w+5, ... of block 5
  const int K = a.k, pad = (K - 1) / 2;
  const int nrun = (T + kRun - 1) / kRun;
  float lsum[2] = {0.f, 0.f}, lsq[2] = {0.f, 0.f};
  uint16_t* out = static_cast<uint16_t*>(a.out) + (int64_t)s * T * kD;
#pragma unroll
  for (int part = 0; part < 2; ++part) {   // unrolled: lsum / lsq stay in registers
    const int cb = part == 0 ? w : kCB - 1;
    const int c = cb * 64 + lane;
    float wr[kMaxK];
#pragma unroll
    for (int j = 0; j < kMaxK; ++j) wr[j] = j < K ? a.dw_w[c * K + j] : 0.f;
    const float bias = a.dw_b[c];
    const int r_first = part == 0 ? 0 : w, r_step = part == 0 ? 1 : kWaves;
#pragma unroll 1
    for (int run = r_first; run < nrun; run += r_step) {
      const int t0 = run * kRun;
      float win[kRun + kMaxK - 1];
#pragma unroll
      for (int i = 0; i < kRun + kMaxK - 1; ++i) {
        const int t = t0 - pad + i;
        win[i] = (i < kRun + K - 1 && t >= 0 && t < T) ? bf_bits2f(hs[t * kHS + c]) : 0.f;
      }
#pragma unroll
      for (int r = 0; r < kRun; ++r) {
        float acc = bias;
#pragma unroll
        for (int j = 0; j < kMaxK; ++j) acc = fmaf(wr[j], win[r + j], acc);
        const int t = t0 + r;
        if (t < T) {
          out[(int64_t)t * kD + c] = f2bf_bits(acc);
          lsum[part] += acc;
          lsq[part] += acc * acc;
        }
      }
    }
  }
  // GroupNorm partials per 64-channel block (glu_dwconv's layout): block w < 5 from wave w alone (part 0),
  // block 5 from every wave (part 1)
#pragma unroll
  for (int part = 0; part < 2; ++part) {
    const float ps = warp_sum(lsum[part]), pq = warp_sum(lsq[part]);
    const int cb = part == 0 ? w : kCB - 1;
    if (lane == 0) {
      s_stat[(0 * kCB + cb) * kWaves + w] = ps;
      s_stat[(1 * kCB + cb) * kWaves + w] = pq;
    }
  }
  __syncthreads();
  if (tid < kCB) {
    const int cb = tid;
    float sum = 0.f, sq = 0.f;
    for (int ww = 0; ww < kWaves; ++ww) {
      if (cb < kCB - 1 && ww != cb) continue;
      sum += s_stat[(0 * kCB + cb) * kWaves + ww];
      sq += s_stat[(1 * kCB + cb) * kWaves + ww];
    }
    a.partial[((int64_t)s * kCB + cb) * 2 + 0] = sum;
    a.partial[((int64_t)s * kCB + cb) * 2 + 1] = sq;
  }
}

}  // namespace

bool conv_block_supported(int D, int T, int k, bool bf16) {
  // Opt-in (SDIAR_CONV_BLOCK=1): correct (TS-VAD goldens) but slower on C2 than gemm_areg + glu_dwconv
  // (6.65 vs 3.3 ms per step): one sequence per CU (h fills the LDS) serialises the y load, the 48-piece
  // projection on 5 waves and the VALU depthwise conv with nothing to overlap them.
  static const bool on = getenv("SDIAR_CONV_BLOCK") && atoi(getenv("SDIAR_CONV_BLOCK")) == 1;
  return on && bf16 && D == kD && T >= 1 && T <= kTMax && k >= 1 && k <= kMaxK && k % 2 == 1;
}

std::vector<uint16_t> conv_block_pack_w1(const std::vector<float>& W, int N, int K) {
  // W: pointwise_conv1 (2D, D) in the ORIGINAL row order (values 0..D-1, gates D..2D-1)
  SD_CHECK(N == 2 * kD && K == kD && (int64_t)W.size() == (int64_t)N * K, kErrInvalid, "conv_block_pack_w1: shape");
  auto bf = [](float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
  };
  std::vector<uint16_t> out;
  out.reserve(W.size());
  for (int n = 0; n < kGroups; ++n)
    for (int h = 0; h < 2; ++h)
      for (int f = 0; f < kPieceFr; ++f) {
        const int part = f / 6, kk = 6 * h + f % 6;   // part 0: value rows, 1: gate rows
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j) {
            const int row = part * kD + 16 * n + (l & 15);
            out.push_back(bf(W[(size_t)row * K + 32 * kk + 8 * (l >> 4) + j]));
          }
      }
  return out;
}

void conv_block(const ConvBlockArgs& a, hipStream_t st) {
  SD_CHECK(conv_block_supported(kD, a.T, a.k, true) && a.y && a.w1 && a.b1 && a.dw_w && a.dw_b && a.out && a.partial,
           kErrInvalid, "conv_block: unsupported arguments");
  if (a.S <= 0) return;
  static bool attr = false;
  if (!attr) {
    SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(conv_block_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSmemBytes));
    attr = true;
  }
  const double rows = (double)a.S * a.T;
  const double flops = 2.0 * rows * 2 * kD * kD + 2.0 * rows * kD * a.k;
  const double bytes = rows * kD * 4.0 + 2.0 * 2 * kD * kD;
  ProfScope prof("conv_block", flops, bytes, st);
  hipLaunchKernelGGL(conv_block_kernel, dim3(a.S), dim3(kThreads), kSmemBytes, st, a);
  SD_LAUNCH_CHECK();
}

}  // namespace sd
