// Weight-resident streaming GEMM for the encoders' linears (bf16 A, K <= 768, row-major out).
//
// The conformer/transformer projections are tall-skinny: M = sequences x frames is
// 10^5..10^6 rows while K (384/512) and the weight matrix are small.  A classic
// 128x128 tile with a 2-stage k loop spends its life in prologue/epilogue latency
// (6 k-steps per tile).  Here each workgroup (8 waves, one per CU) keeps a BN x K
// weight panel resident in LDS for its whole life and streams row panels of A
// through a 4-deep LDS-DMA ring, walking a strided list of M tiles without ever
// draining the pipe: the DMA of the next tile's chunks is in flight while the
// current tile finishes and its epilogue stores leave straight from the MFMA
// accumulators.  HBM traffic is one pass over A and one over the output; the
// n-tiles of one M range are co-scheduled on one XCD (xcd_remap) so the re-reads
// of A hit that XCD's L2.
//
// LDS (bf16, 128-B rows, 16-B chunk c of row r stored at c ^ (r & 7)):
//   W panel  [K/64][BN][64]         BN * K * 2 bytes (<= 96 KiB)
//   A ring   [NST][128][64]         16 KiB per stage
#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {
namespace {

constexpr int SBM = 128;          // rows per M tile
constexpr int SBK = 64;           // k chunk
constexpr int NST = 4;            // A ring stages
constexpr int SD_ = NST - 1;      // prefetch distance
constexpr int kStreamThreads = 512;
constexpr int kGluEpi = 100;      // epilogue "activation" id of the GLU mode
constexpr uint32_t kOOB = 0x80000000u;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BN, int ACT>
__global__ __launch_bounds__(kStreamThreads) void gemm_stream_kernel(ConvGemmArgs p, int n_groups) {
  constexpr int WN = 2, WM = 4;                  // 8 waves: 4 along M x 2 along N
  constexpr int TM = SBM / WM, TN = BN / WN;     // 32 x 64 (BN 128) / 32 x 32 (BN 64)
  constexpr int MT = TM / 16, NT = TN / 16;
  constexpr int A_STAGE = SBM * SBK;             // bf16 elements
  extern __shared__ __attribute__((aligned(1024))) uint16_t sm[];
  const int K = p.K;
  const int KT = K / SBK;
  uint16_t* Ws = sm;                             // [KT][BN][64]
  uint16_t* As = sm + (size_t)KT * BN * SBK;     // [NST][128][64]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: keeps the accounting scalar
  const int wm = wid >> 1, wn = wid & 1;
  const int l15 = lane & 15, lk = lane >> 4;
  const int M = p.B * p.Ho * p.Wo;
  const int n_nt = (p.N + BN - 1) / BN;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int nt_id = lid % n_nt;
  const int grp = lid / n_nt;
  const int n0 = nt_id * BN;
  const int m_tiles = (M + SBM - 1) / SBM;
  if (grp >= n_groups) return;
  const int my_tiles = grp < m_tiles ? (m_tiles - 1 - grp) / n_groups + 1 : 0;
  const int total = my_tiles * KT;

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.A), (short)0,
                                                                      (int)kOOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.Wt), (short)0,
                                                                      (int)kOOB, 0x00020000);
  const int lrow = lane >> 3, lch = lane & 7;

  // ---- weight panel: BN/8 row groups x KT chunks, one 1-KiB DMA per (group, chunk)
  {
    const int n_inst = (BN / 8) * KT;
    for (int q = wid; q < n_inst; q += 8) {
      const int kc = q / (BN / 8), rg = q % (BN / 8);
      const int r = rg * 8 + lrow;
      const int n = n0 + r;
      const int src = lch ^ (r & 7);
      const uint32_t off = n < p.N ? (uint32_t)(((int64_t)n * K + kc * SBK + src * 8) * 2) : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr_t)(Ws + ((size_t)kc * BN + rg * 8) * SBK), 16, off,
                                               0, 0, 0);
    }
  }
  // ---- A ring.  Prefetch cursor: tile pj, chunk pkc, ring slot pslot.  a_off holds the
  // per-lane byte offsets of this wave's two 8-row groups in the cursor's tile; the
  // chunk advances through the scalar soffset, so a stage costs no VALU.
  uint32_t a_off[2];
  auto set_tile = [&](int jj) {
    const int m0 = (grp + jj * n_groups) * SBM;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = (wid * 2 + i) * 8 + lrow;
      const int m = m0 + r;
      const int src = lch ^ (r & 7);
      a_off[i] = m < M ? (uint32_t)(((int64_t)m * p.lda + p.a_coff + src * 8) * 2) : kOOB;
    }
  };
  int pj = 0, pkc = 0, pslot = 0;
  set_tile(0);
  auto issue_next = [&]() {
    uint16_t* dst = As + (size_t)pslot * A_STAGE;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)(dst + (wid * 2 + i) * 8 * SBK), 16, a_off[i],
                                               pkc * SBK * 2, 0, 0);
    if (++pkc == KT) {
      pkc = 0;
      set_tile(++pj);
    }
    pslot = pslot == NST - 1 ? 0 : pslot + 1;
  };

  // The MFMA computes the transposed tile (W fragment as the A operand): lane l holds
  // rows m = .. + (l & 15) and 4 CONSECUTIVE columns n = .. + 4*(l >> 4) + r, so the
  // epilogue writes 8 B (bf16) / 16 B (f32) per lane and store instead of 4 scattered
  // 2-B stores.  Per-lane epilogue constants for those columns:
  float al[NT][4], be[NT][4];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + wn * TN + nt * 16 + lk * 4 + r;
      al[nt][r] = (p.alpha && n < p.N) ? p.alpha[n] : 1.f;
      be[nt][r] = (p.beta && n < p.N) ? p.beta[n] : 0.f;
    }

  // VMEM accounting (vmcnt counts loads, stores and LDS-DMA together, in issue order;
  // every op is issued unconditionally — masked elements use an out-of-range offset —
  // so counts are exact).  At the end of step s, "stage s+1 landed" is vmcnt <= the
  // ops issued after it: 2 per later stage already issued, plus the epilogue stores
  // of a tile that ended within the SD_ steps since stage s+1 was issued (KT >= SD_,
  // so at most one).
  int pro = 0;
  for (; pro < SD_ && pro < total; ++pro) issue_next();
  if (total > 0) {   // weight panel + stage 0 landed
    if (pro == 3) wait_vm<4>();
    else if (pro == 2) wait_vm<2>();
    else wait_vm<0>();
  }
  asm volatile("s_barrier" ::: "memory");

  floatx4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};

  const bool out_bf = p.out_bf16;
  const int64_t out_bytes = (int64_t)M * p.o_sw * (out_bf ? 2 : 4);
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(p.out, (short)0, (int)out_bytes, 0x00020000);
  int slot = 0;
  for (int j = 0, s = 0; j < my_tiles; ++j) {
    const int m0 = (grp + j * n_groups) * SBM;
    const int mb = m0 + wm * TM + l15;               // epilogue rows mb + mt*16
    const int nb = n0 + wn * TN + lk * 4;            // epilogue columns nb + nt*16 + r
  for (int kc = 0; kc < KT; ++kc, ++s) {
    if (s + SD_ < total) issue_next();
    const uint16_t* Ast = As + (size_t)slot * A_STAGE;
    const uint16_t* Wst = Ws + (size_t)kc * BN * SBK;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[MT], bfr[NT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int r = wm * TM + mt * 16 + l15;
        af[mt] = *reinterpret_cast<const bf16x8*>(Ast + r * SBK + (((ks * 4 + lk) ^ (r & 7)) * 8));
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int r = wn * TN + nt * 16 + l15;
        bfr[nt] = *reinterpret_cast<const bf16x8*>(Wst + r * SBK + (((ks * 4 + lk) ^ (r & 7)) * 8));
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[nt], af[mt], acc[mt][nt], 0, 0, 0);
    }
    if (kc == KT - 1 && ACT == kGluEpi) {
      // ---- GLU epilogue: value tile nt (even) and gate tile nt + 1 hold the same
      // 4 channels ((n0 + wn*TN + nt*16) / 32) * 16 + 4*lk + r; bf16 output N/2 wide.
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; nt += 2) {
          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float a = fmaf(acc[mt][nt][r], al[nt][r], be[nt][r]);
            const float gt = fmaf(acc[mt][nt + 1][r], al[nt + 1][r], be[nt + 1][r]);
            o[r] = a * sigmoid_rcp(gt);
          }
          const int m = mb + mt * 16;
          const int ch = ((n0 + wn * TN + nt * 16) >> 5) * 16 + lk * 4;
          const uint32_t off = (m < M && 2 * ch < p.N) ? (uint32_t)(((int64_t)m * p.o_sw + ch) * 2) : kOOB;
          const u32x2_t v = {pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])};
          __builtin_amdgcn_raw_buffer_store_b64(v, ro, off, 0, 0);
        }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = floatx4{0.f, 0.f, 0.f, 0.f};
    } else if (kc == KT - 1) {
      // ---- epilogue of tile j straight from the accumulators
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          float x[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            x[r] = fmaf(acc[mt][nt][r], al[nt][r], be[nt][r]);
            if constexpr (ACT == kActRelu) x[r] = fmaxf(x[r], 0.f);
            if constexpr (ACT == kActSigmoid) x[r] = sigmoid_rcp(x[r]);
            if constexpr (ACT == kActSilu) x[r] = x[r] * sigmoid_rcp(x[r]);
          }
          const int m = mb + mt * 16, n = nb + nt * 16;
          const bool ok = m < M && n < p.N;
          if (out_bf) {
            const uint32_t off = ok ? (uint32_t)(((int64_t)m * p.o_sw + n) * 2) : kOOB;
            const u32x2_t v = {pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3])};
            __builtin_amdgcn_raw_buffer_store_b64(v, ro, off, 0, 0);
          } else {
            const uint32_t off = ok ? (uint32_t)(((int64_t)m * p.o_sw + n) * 4) : kOOB;
            const u32x4_t v = {__float_as_uint(x[0]), __float_as_uint(x[1]), __float_as_uint(x[2]),
                               __float_as_uint(x[3])};
            __builtin_amdgcn_raw_buffer_store_b128(v, ro, off, 0, 0);
          }
        }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = floatx4{0.f, 0.f, 0.f, 0.f};
    }
    if (s + 1 < total) {
      const int later = (s + SD_ < total - 1 ? s + SD_ : total - 1) - (s + 1);   // stages issued after s+1
      const bool st = kc == KT - 1 || (j > 0 && kc < SD_ - 1);
      constexpr int ST = ACT == kGluEpi ? MT * NT / 2 : MT * NT;
      if (st) {
        if (later == 2) wait_vm<4 + ST>();
        else if (later == 1) wait_vm<2 + ST>();
        else wait_vm<ST>();
      } else {
        if (later == 2) wait_vm<4>();
        else if (later == 1) wait_vm<2>();
        else wait_vm<0>();
      }
      // plain s_barrier: __syncthreads()' workgroup fence would add vmcnt(0) and drain the ring
      asm volatile("s_barrier" ::: "memory");
    }
    slot = slot == NST - 1 ? 0 : slot + 1;
  }
  }
}

int g_num_cu = 0;

template <int BN, int ACT>
void launch_stream(const ConvGemmArgs& p, hipStream_t st) {
  const int M = p.B * p.Ho * p.Wo;
  const int n_nt = cdiv(p.N, BN);
  const int m_tiles = cdiv(M, SBM);
  int groups = std::max(1, g_num_cu / n_nt);
  groups = std::min(groups, m_tiles);
  const size_t smem = sizeof(uint16_t) * ((size_t)(p.K / SBK) * BN * SBK + (size_t)NST * SBM * SBK);
  static bool attr = false;
  if (!attr) {
    SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_stream_kernel<BN, ACT>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL((gemm_stream_kernel<BN, ACT>), dim3(n_nt * groups), dim3(kStreamThreads), smem, st, p, groups);
}

int stream_bn(const ConvGemmArgs& p) {
  const size_t ring = (size_t)NST * SBM * SBK * 2;
  if ((size_t)128 * p.K * 2 + ring <= 160 * 1024 && p.N >= 128) return 128;
  if ((size_t)64 * p.K * 2 + ring <= 160 * 1024) return 64;
  return 0;
}

}  // namespace

bool gemm_stream_supported(const ConvGemmArgs& p) {
  static const bool disabled = getenv("SDIAR_NO_STREAM_GEMM") != nullptr;
  if (disabled) return false;
  const int M = p.B * p.Ho * p.Wo;
  const bool row_major = p.o_sn == 1 && out_rows_linear(p) && a_rows_linear(p);
  return p.a_bf16 && !p.pre_scale && !p.gate && !p.res && p.kh * p.kw == 1 && p.K % SBK == 0 && p.lda % 8 == 0 &&
         p.N % 4 == 0 && p.o_sw % 4 == 0 &&   // 4-column vector stores
         p.K >= SD_ * SBK &&                  // KT >= SD_ (store accounting)
         p.a_coff % 8 == 0 && row_major && stream_bn(p) > 0 && M >= 16 * SBM &&
         (int64_t)M * p.lda * 2 < (int64_t)kOOB && (int64_t)p.N * p.K * 2 < (int64_t)kOOB &&
         (int64_t)M * p.o_sw * 4 < (int64_t)kOOB && (!p.res || (int64_t)M * p.res_ld * 4 < (int64_t)kOOB);
}

void conv_gemm_stream(const ConvGemmArgs& p, hipStream_t st) {
  if (!g_num_cu) {
    int dev = 0;
    SD_HIP(hipGetDevice(&dev));
    SD_HIP(hipDeviceGetAttribute(&g_num_cu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const bool wide = stream_bn(p) == 128;
  if (p.glu) {
    SD_CHECK(p.act == kActNone && p.out_bf16 && p.N % 32 == 0, kErrInvalid,
             "GLU epilogue: bf16 output, no activation, N % 32 == 0");
    wide ? launch_stream<128, kGluEpi>(p, st) : launch_stream<64, kGluEpi>(p, st);
    SD_LAUNCH_CHECK();
    return;
  }
  switch (p.act) {
    case kActRelu: wide ? launch_stream<128, kActRelu>(p, st) : launch_stream<64, kActRelu>(p, st); break;
    case kActSigmoid: wide ? launch_stream<128, kActSigmoid>(p, st) : launch_stream<64, kActSigmoid>(p, st); break;
    case kActSilu: wide ? launch_stream<128, kActSilu>(p, st) : launch_stream<64, kActSilu>(p, st); break;
    default: wide ? launch_stream<128, kActNone>(p, st) : launch_stream<64, kActNone>(p, st); break;
  }
  SD_LAUNCH_CHECK();
}

}  // namespace sd
