// Register-resident-A GEMM for the encoders' wide linears (bf16 A, K in {192, 256, 384},
// N % 64 == 0, N >= 768).
//
// The weight-resident streaming kernel (gemm_stream.hip) keeps a BN-column weight panel in
// LDS, so an N = 384..1152 projection is split over 3..9 column tiles and every one of them
// streams the same A rows again: its intake per CU, not HBM, bounds it (measured: time grows
// with the column-tile count; a single-tile N = 128 problem runs at 4.7 TB/s, N = 1152 at
// 1.9 TB/s).  Here A is read exactly once: each workgroup (8 waves, one per CU) owns a
// 256-row tile whose MFMA B-operand fragments sit in VGPRs for the whole tile (32 rows x K
// per wave), and the weights stream through a 3-slot LDS-DMA ring as 64-column chunks
// (64 x K bf16, <= 48 KiB), two chunks in flight.  Every chunk is a complete 256 x 64
// output block: its epilogue stores leave straight from the accumulators (transposed MFMA:
// 4 consecutive columns per lane -> 8-B bf16 / 16-B fp32 stores), optionally through the
// conformer GLU.  The weights (<= 864 KiB) stay L2-resident; per 256-row tile a CU reads
// 192 KiB of A from HBM and N x K x 2 bytes of weights from L2.  The next tile's A
// fragments are loaded during the tile's last chunk, each right after its final use.
//
// LDS (one array): W ring [3][K/64][64][64] bf16 (16-B chunk c of row r at c ^ (r & 7)),
// then alpha / beta for all N columns.
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {
namespace {

constexpr int RB = 256;            // rows per tile (32 per wave)
constexpr int NB = 64;             // columns per weight chunk
constexpr int NSLOT = 3;           // ring slots (2 chunks in flight)
constexpr int kMaxN = 1536;        // alpha/beta staged in LDS
constexpr int kGlu = 100;
constexpr uint32_t kOOB = 0x80000000u;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// vmcnt at the end of step s ("chunk s+1 landed"): the ops this wave issued after chunk s+1's
// pieces are, in order, the previous step's A reloads and stores (s > 0), this step's
// chunk-(s+2) pieces (more), its A reloads and its stores.  A reloads happen in at most one
// of the two steps (rl).
// vmcnt at the end of step s ("chunk s+1 landed"; its DMA went out at the start of step s-1).  Chunk c's
// epilogue runs during step c+1's k-steps 1.., after that step's chunk DMA, so the ops younger than chunk
// s+1's DMA are: step s-1's stores (of chunk s-2, s >= 2) and A reloads, then step s's chunk-(s+2) DMA
// (more), its stores (of chunk s-1, s >= 1) and its A reloads (rl: reloads in either step).
template <int P, int ST, int AL>
__device__ __forceinline__ void wait_chunk(int s, bool more, bool rl) {
  if (s == 0) {
    if (more) { if (rl) wait_vm<P + AL>(); else wait_vm<P>(); }
    else { if (rl) wait_vm<AL>(); else wait_vm<0>(); }
  } else if (s == 1) {
    if (more) { if (rl) wait_vm<P + ST + AL>(); else wait_vm<P + ST>(); }
    else { if (rl) wait_vm<ST + AL>(); else wait_vm<ST>(); }
  } else {
    if (more) { if (rl) wait_vm<2 * ST + P + AL>(); else wait_vm<2 * ST + P>(); }
    else { if (rl) wait_vm<2 * ST + AL>(); else wait_vm<2 * ST>(); }
  }
}

template <int KT32, int ACT>
__global__ __launch_bounds__(512) void gemm_areg_kernel(ConvGemmArgs p) {
  constexpr int K = KT32 * 32;
  constexpr int KC = K / 64;                       // 64-k blocks per chunk
  constexpr int SLOT = NB * K;                     // bf16 elements per slot
  constexpr int PIECES = KC;                       // 1-KiB DMA pieces per wave per chunk
  constexpr int MT = 2, NT = NB / 16;
  constexpr int ST = ACT == kGlu ? MT * NT / 2 : MT * NT;   // epilogue stores per wave
  constexpr int AL = MT * KT32;                              // A fragment loads per wave
  extern __shared__ __attribute__((aligned(1024))) uint16_t sm[];
  uint16_t* Ws = sm;                                               // [NSLOT][KC][64][64]
  float* s_al = reinterpret_cast<float*>(sm + (size_t)NSLOT * SLOT);
  float* s_be = s_al + kMaxN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, lk = lane >> 4;
  const int M = p.B * p.Ho * p.Wo;
  const int n_chunks = p.N / NB;
  const int n_tiles = (M + RB - 1) / RB;
  const int grid = gridDim.x;
  const int tile0 = blockIdx.x;
  const int my_tiles = tile0 < n_tiles ? (n_tiles - 1 - tile0) / grid + 1 : 0;
  const int total = my_tiles * n_chunks;
  if (total == 0) return;

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.A), (short)0,
                                                                      (int)kOOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.Wt), (short)0,
                                                                      (int)kOOB, 0x00020000);
  const bool out_bf = p.out_bf16;
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
      p.out, (short)0, (int)((int64_t)M * p.o_sw * (out_bf ? 2 : 4)), 0x00020000);

  // Epilogue constants for all N columns, staged once (LDS reads keep the vmcnt count exact).
  for (int n = tid; n < p.N; n += 512) {
    s_al[n] = p.alpha ? p.alpha[n] : 1.f;
    s_be[n] = p.beta ? p.beta[n] : 0.f;
  }

  // ---- weight chunk DMA: chunk c = columns [64c, 64c+64), all K.  Wave wid loads rows
  // 8*wid .. 8*wid+7 of every 64-k block (one 1-KiB piece per block).
  const int lrow = lane >> 3, lch = lane & 7;
  const int wr = wid * 8 + lrow;
  const int wsrc = (lch ^ (wr & 7)) * 8;
  // Workgroups walk the chunks from different starting points: in lockstep every CU of an XCD
  // would request the same 48 KiB of weights at once and serialize on a few L2 channels.
  const int rot = tile0 % n_chunks;
  auto chunk_of = [&](int step) {
    const int c = step % n_chunks + rot;
    return c >= n_chunks ? c - n_chunks : c;
  };
  auto issue_chunk = [&](int step) {
    const int c = chunk_of(step);
    uint16_t* dst = Ws + (size_t)(step % NSLOT) * SLOT + wid * 8 * 64;
    const uint32_t base = (uint32_t)(((int64_t)(c * NB + wr) * K + wsrc) * 2);
#pragma unroll
    for (int kc = 0; kc < PIECES; ++kc)
      dma_lds16_buf(rw, base + kc * 128, (lds_ptr_t)(dst + (size_t)kc * NB * 64));
  };

  // ---- A fragments of this wave's 32 rows: af[mt][kk] = row tile*256 + 32*wid + 16*mt + l15,
  // k = 32*kk + 8*lk .. +7 (the MFMA B operand).
  bf16x8 af[MT][KT32];
  auto load_a = [&](int tile, int mt, int kk) {
    const int m = tile * RB + wid * 32 + mt * 16 + l15;
    // tiled: fragment kk of row m's 16-row group, lane l15 + 16 lk (one contiguous 1-KiB run per instruction)
    const int64_t e = p.a_tiled ? ((int64_t)((m >> 4) * KT32 + kk) * 64 + l15 + 16 * lk) * 8
                                : (int64_t)m * p.lda + p.a_coff + kk * 32 + lk * 8;
    const uint32_t off = m < M ? (uint32_t)(e * 2) : kOOB;
    const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0);
    af[mt][kk] = __builtin_bit_cast(bf16x8, v);
  };
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int kk = 0; kk < KT32; ++kk) load_a(tile0, mt, kk);

  issue_chunk(0);
  if (total > 1) issue_chunk(1);
  if (total > 1) wait_vm<PIECES>(); else wait_vm<0>();
  __syncthreads();   // chunk 0 and alpha/beta visible to every wave

  // Two accumulator sets: chunk s accumulates into set s & 1 while chunk s-1's epilogue (GLU / act,
  // stores) is interleaved with its k-steps — the epilogue's VALU work issues in the MFMAs' shadow
  // instead of after a barrier where every wave of the CU would run it at once with the MFMA pipe idle.
  floatx4 acc[2][MT][NT];
  constexpr int G = ACT == kGlu ? MT * NT / 2 : MT * NT;   // epilogue groups (one 8/16-B store each)
  // epilogue group gi of set SET: chunk column block ccol of tile ptile
  auto epi_group = [&](auto SETC, int ptile, int ccol, int gi) {
    constexpr int SET = decltype(SETC)::value;
    const int mb = ptile * RB + wid * 32 + l15;
    const int n0 = ccol * NB;
    if constexpr (ACT == kGlu) {
      const int mt = gi / (NT / 2), nt = (gi % (NT / 2)) * 2;
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int nv = n0 + nt * 16 + lk * 4 + r, ng = nv + 16;
        const float av = fmaf(acc[SET][mt][nt][r], s_al[nv], s_be[nv]);
        const float gt = fmaf(acc[SET][mt][nt + 1][r], s_al[ng], s_be[ng]);
        o[r] = av * sigmoid_rcp(gt);
      }
      const int m = mb + mt * 16;
      const int ch = ((n0 + nt * 16) >> 5) * 16 + lk * 4;
      const uint32_t off = m < M ? (uint32_t)(((int64_t)m * p.o_sw + ch) * 2) : kOOB;
      const u32x2_t v = {pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])};
      __builtin_amdgcn_raw_buffer_store_b64(v, ro, off, 0, 0);
    } else {
      const int mt = gi / NT, nt = gi % NT;
      const int n = n0 + nt * 16 + lk * 4;
      float x[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        x[r] = fmaf(acc[SET][mt][nt][r], s_al[n + r], s_be[n + r]);
        if constexpr (ACT == kActRelu) x[r] = fmaxf(x[r], 0.f);
        if constexpr (ACT == kActSigmoid) x[r] = sigmoid_rcp(x[r]);
        if constexpr (ACT == kActSilu) x[r] = x[r] * sigmoid_rcp(x[r]);
      }
      const int m = mb + mt * 16;
      if (out_bf) {
        const uint32_t off = m < M ? (uint32_t)(((int64_t)m * p.o_sw + n) * 2) : kOOB;
        const u32x2_t v = {pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3])};
        __builtin_amdgcn_raw_buffer_store_b64(v, ro, off, 0, 0);
      } else {
        const uint32_t off = m < M ? (uint32_t)(((int64_t)m * p.o_sw + n) * 4) : kOOB;
        const u32x4_t v = {__float_as_uint(x[0]), __float_as_uint(x[1]), __float_as_uint(x[2]), __float_as_uint(x[3])};
        __builtin_amdgcn_raw_buffer_store_b128(v, ro, off, 0, 0);
      }
    }
  };

  bool rl_prev = false;
  int p_tile = 0, p_col = 0;   // the chunk whose epilogue is pending (set (s - 1) & 1)
  auto step = [&](auto CURC, int s) {
    constexpr int CUR = decltype(CURC)::value, PRV = 1 - CUR;
    const int j = s / n_chunks, c = s - j * n_chunks;
    const int tile = tile0 + j * grid;
    const bool reload = c == n_chunks - 1 && j + 1 < my_tiles;   // next tile's A during the last chunk
    const bool more = s + 2 < total;
    const bool pend = s > 0;
    const uint16_t* Wst = Ws + (size_t)(s % NSLOT) * SLOT;
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < NT; ++b) acc[CUR][a][b] = floatx4{0.f, 0.f, 0.f, 0.f};
    // W fragments of step kk+1 are read while the MFMAs of step kk run (double-buffered).
    auto read_w = [&](int kk, bf16x8* bfr) {
      const int sb = kk >> 1;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int r = nt * 16 + l15;
        const int ch = ((kk & 1) * 4 + lk) ^ (r & 7);
        bfr[nt] = *reinterpret_cast<const bf16x8*>(Wst + ((size_t)sb * NB + r) * 64 + ch * 8);
      }
    };
    bf16x8 wbuf[2][NT];
    read_w(0, wbuf[0]);
#pragma unroll
    for (int kk = 0; kk < KT32; ++kk) {
      if (kk + 1 < KT32) read_w(kk + 1, wbuf[(kk + 1) & 1]);
      const bf16x8* bfr = wbuf[kk & 1];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[CUR][mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[nt], af[mt][kk], acc[CUR][mt][nt], 0, 0, 0);
      if (kk == 0) {
        // The chunk-(s+2) DMA goes out after the first MFMAs: on a tile's first chunk those wait
        // for the A fragments loaded during the previous chunk, and a DMA issued before them
        // would be drained by that wait.
        __builtin_amdgcn_sched_barrier(0);
        if (more) issue_chunk(s + 2);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (reload) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) load_a(tile + grid, mt, kk);
      }
      // the pending epilogue's groups over k-steps 1 .. KT32-1 (after this step's chunk DMA)
      if (pend && kk >= 1) {
#pragma unroll
        for (int gi = 0; gi < G; ++gi)
          if (1 + gi * (KT32 - 1) / G == kk) epi_group(std::integral_constant<int, PRV>{}, p_tile, p_col, gi);
      }
    }
    p_tile = tile;
    p_col = chunk_of(s);
    if (s + 1 < total) {
      wait_chunk<PIECES, ST, AL>(s, more, reload || rl_prev);
      // plain s_barrier: __syncthreads()' fence would add vmcnt(0) and drain the ring
      asm volatile("s_barrier" ::: "memory");
    }
    rl_prev = reload;
  };
  int s = 0;
  for (; s + 1 < total; s += 2) {
    step(std::integral_constant<int, 0>{}, s);
    step(std::integral_constant<int, 1>{}, s + 1);
  }
  if (s < total) step(std::integral_constant<int, 0>{}, s);
  // the last chunk's epilogue (set (total - 1) & 1)
  if ((total - 1) & 1) {
#pragma unroll
    for (int gi = 0; gi < G; ++gi) epi_group(std::integral_constant<int, 1>{}, p_tile, p_col, gi);
  } else {
#pragma unroll
    for (int gi = 0; gi < G; ++gi) epi_group(std::integral_constant<int, 0>{}, p_tile, p_col, gi);
  }
}

int g_cu = 0;

template <int KT32, int ACT>
void launch_areg(const ConvGemmArgs& p, hipStream_t st) {
  const int M = p.B * p.Ho * p.Wo;
  const int tiles = cdiv(M, RB);
  const int grid = std::min(tiles, g_cu);
  const size_t smem = sizeof(uint16_t) * (size_t)NSLOT * NB * KT32 * 32 + 2 * kMaxN * sizeof(float);
  static bool attr = false;
  if (!attr) {
    SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_areg_kernel<KT32, ACT>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL((gemm_areg_kernel<KT32, ACT>), dim3(grid), dim3(512), smem, st, p);
}

template <int ACT>
void launch_act(const ConvGemmArgs& p, hipStream_t st) {
  switch (p.K) {
    case 384: launch_areg<12, ACT>(p, st); break;
    case 256: launch_areg<8, ACT>(p, st); break;
    default: launch_areg<6, ACT>(p, st); break;   // 192
  }
}

}  // namespace

bool gemm_areg_supported(const ConvGemmArgs& p) {
  static const bool disabled = getenv("SDIAR_NO_AREG_GEMM") != nullptr;
  if (disabled) return false;
  const int M = p.B * p.Ho * p.Wo;
  const bool row_major = p.o_sn == 1 && out_rows_linear(p) && a_rows_linear(p);
  return p.a_bf16 && !p.pre_scale && !p.gate && !p.res && p.kh * p.kw == 1 &&
         // measured against gemm_stream on the C2 shapes (M = 360000, K = 384): faster from
         // N = 768 (GLU pw1 768: 318 vs 355 us; QKV 1152: 508 vs 586 us), slower at N = 384 / 512
         // K 256 (FS-EEND decoder in-projections, M 36000, N 768): gemm_stream 132 vs 167 us, so not here
         (p.K == 384 || p.K == 192) && p.N % NB == 0 && p.N >= 768 && p.N <= kMaxN &&
         p.lda % 8 == 0 && p.a_coff % 8 == 0 && p.o_sw % 4 == 0 && row_major && M >= 64 * RB &&
         (int64_t)M * p.lda * 2 < (int64_t)kOOB && (int64_t)p.N * p.K * 2 < (int64_t)kOOB &&
         (int64_t)M * p.o_sw * 4 < (int64_t)kOOB && (!p.glu || (p.out_bf16 && p.act == kActNone && p.N % 32 == 0));
}

void conv_gemm_areg(const ConvGemmArgs& p, hipStream_t st) {
  if (!g_cu) {
    int dev = 0;
    SD_HIP(hipGetDevice(&dev));
    SD_HIP(hipDeviceGetAttribute(&g_cu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  if (p.glu) {
    launch_act<kGlu>(p, st);
  } else {
    switch (p.act) {
      case kActRelu: launch_act<kActRelu>(p, st); break;
      case kActSigmoid: launch_act<kActSigmoid>(p, st); break;
      case kActSilu: launch_act<kActSilu>(p, st); break;
      default: launch_act<kActNone>(p, st); break;
    }
  }
  SD_LAUNCH_CHECK();
}

}  // namespace sd
