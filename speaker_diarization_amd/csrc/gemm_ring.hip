// Tall bf16 GEMM with an optional BN-ReLU prologue on A, fed by a 3-stage LDS-DMA
// ring: the CAM++ dense-block bottlenecks (nonlinear1 -> linear1 -> nonlinear2:
// M = windows x frames ~ 1.8e5 rows, N = 128, K = 32 * layer = 256..1024, A a
// channel slice of the growing concat buffer) and the transit layers.
//
// These GEMMs are HBM-bound (A is read once, ~K*2 bytes per row, for 128 output
// columns), so the kernel is built to keep A in flight: one 512-thread workgroup per
// CU owns a 256 x 128 output tile; while the MFMAs consume k-tile kt, the DMAs of
// k-tiles kt+1 and kt+2 are outstanding (3 x 48 KiB ring).  The prologue
// a' = relu(a * s + h) is applied in place on the landed A stage (each element once
// per workgroup), reading the per-channel s/h staged in LDS at kernel start — no
// global loads inside the loop, so the vmcnt accounting of the ring stays exact.
// The MFMA computes the transposed tile (weights as the A operand) so each lane ends
// with 4 consecutive output columns: 8-B bf16 stores straight from the accumulators.
//
// LDS (bf16, 128-B rows, 16-B chunk c of row r stored at c ^ (r & 7)):
//   ring   [3][A 256 x 64 | B 128 x 64]   3 x 48 KiB
//   s/h    [2][K] f32                      8 KiB at K = 1024
#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {
namespace {

constexpr int RBM = 256, RBN = 128, RBK = 64;
constexpr int RST = 3;                         // ring stages
constexpr int kRingThreads = 512;
constexpr int kRingMaxK = 1024;
constexpr int A_ELEMS = RBM * RBK, B_ELEMS = RBN * RBK, STAGE_ELEMS = A_ELEMS + B_ELEMS;
constexpr uint32_t kOOB = 0x80000000u;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <bool PRE, int ACT>
__global__ __launch_bounds__(kRingThreads) void gemm_ring_kernel(ConvGemmArgs p) {
  constexpr int WM = 4, WN = 2;                 // 8 waves: 4 along M x 2 along N
  constexpr int TM = RBM / WM, TN = RBN / WN;   // 64 x 64 per wave
  constexpr int MT = TM / 16, NT = TN / 16;
  extern __shared__ __attribute__((aligned(1024))) uint16_t sm[];
  float* s_scale = reinterpret_cast<float*>(sm + RST * STAGE_ELEMS);
  float* s_shift = s_scale + kRingMaxK;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int l15 = lane & 15, lk = lane >> 4;
  const int M = p.B * p.Ho * p.Wo;
  const int K = p.K;
  const int KT = (K + RBK - 1) / RBK;
  const int n_nt = (p.N + RBN - 1) / RBN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (tile / n_nt) * RBM;
  const int n0 = (tile % n_nt) * RBN;

  // Per-channel prologue constants -> LDS; per-lane epilogue constants -> registers.
  if constexpr (PRE) {
    for (int k = tid; k < KT * RBK; k += kRingThreads) {
      s_scale[k] = k < K ? p.pre_scale[k] : 0.f;   // K tail: a*0 + 0 (its weights are 0 too)
      s_shift[k] = k < K ? p.pre_shift[k] : 0.f;
    }
  }
  float al[NT][4], be[NT][4];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + wn * TN + nt * 16 + lk * 4 + r;
      al[nt][r] = (p.alpha && n < p.N) ? p.alpha[n] : 1.f;
      be[nt][r] = (p.beta && n < p.N) ? p.beta[n] : 0.f;
    }

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.A), (short)0,
                                                                      (int)kOOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.Wt), (short)0,
                                                                      (int)kOOB, 0x00020000);
  // DMA pieces of this wave: A rows wid*32 + i*8 + (lane>>3) (i < 4), B rows wid*16 + i*8 + .. (i < 2);
  // lane fills physical chunk lane&7 of its row from logical chunk src = (lane&7) ^ (row&7).
  const int lrow = lane >> 3, lch = lane & 7;
  const int src = lch ^ lrow;                  // every piece starts at a multiple of 8 rows
  uint32_t a_off[4], b_off[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wid * 32 + i * 8 + lrow;
    a_off[i] = m < M ? (uint32_t)(((int64_t)m * p.lda + p.a_coff + src * 8) * 2) : kOOB;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int n = n0 + wid * 16 + i * 8 + lrow;
    b_off[i] = n < p.N ? (uint32_t)(((int64_t)n * K + src * 8) * 2) : kOOB;
  }
  auto issue = [&](int kt) {
    uint16_t* As = sm + (kt % RST) * STAGE_ELEMS;
    uint16_t* Bs = As + A_ELEMS;
    const bool ok = kt * RBK + src * 8 < K;    // K tail chunks read as zeros
    const int soff = kt * RBK * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)(As + (wid * 32 + i * 8) * RBK), 16,
                                               ok ? a_off[i] : kOOB, soff, 0, 0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr_t)(Bs + (wid * 16 + i * 8) * RBK), 16,
                                               ok ? b_off[i] : kOOB, soff, 0, 0);
  };
  constexpr int PIECES = 6;                    // VMEM ops per wave per stage

  // Prologue transform mapping: thread i touches rows (i >> 3) + 64 j and physical chunk
  // i & 7; (row & 7) is fixed, so its logical chunk (8 consecutive k) is fixed too.
  const int pre_pc = tid & 7;
  const int pre_lc = pre_pc ^ ((tid >> 3) & 7);

  issue(0);
  if (KT > 1) issue(1);
  if (KT > 1) wait_vm<PIECES>();
  else wait_vm<0>();
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // stage 0 + s/h visible

  floatx4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};

  for (int kt = 0; kt < KT; ++kt) {
    if (kt + 2 < KT) issue(kt + 2);
    uint16_t* As = sm + (kt % RST) * STAGE_ELEMS;
    const uint16_t* Bs = As + A_ELEMS;
    if constexpr (PRE) {
      const int k = kt * RBK + pre_lc * 8;
      // s/h read through inline asm for the same reason as the write-back below: a
      // compiler-visible LDS read here gets a full vmcnt(0) drain of the ring in front.
      u32x4_t s0, s1, h0, h1;
      asm volatile(
          "ds_read_b128 %0, %4\n\t"
          "ds_read_b128 %1, %4 offset:16\n\t"
          "ds_read_b128 %2, %5\n\t"
          "ds_read_b128 %3, %5 offset:16\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(s0), "=&v"(s1), "=&v"(h0), "=&v"(h1)
          : "v"((uint32_t)reinterpret_cast<uintptr_t>((lds_ptr_t)(s_scale + k))),
            "v"((uint32_t)reinterpret_cast<uintptr_t>((lds_ptr_t)(s_shift + k)))
          : "memory");
      const float sc[8] = {__uint_as_float(s0.x), __uint_as_float(s0.y), __uint_as_float(s0.z),
                           __uint_as_float(s0.w), __uint_as_float(s1.x), __uint_as_float(s1.y),
                           __uint_as_float(s1.z), __uint_as_float(s1.w)};
      const float sh[8] = {__uint_as_float(h0.x), __uint_as_float(h0.y), __uint_as_float(h0.z),
                           __uint_as_float(h0.w), __uint_as_float(h1.x), __uint_as_float(h1.y),
                           __uint_as_float(h1.z), __uint_as_float(h1.w)};
      // Thread rows (tid >> 3) + 64 j, j < 4: 8 KiB apart.  All LDS traffic of the transform
      // goes through inline asm: compiler-visible LDS accesses here get a full vmcnt(0)
      // drain of the ring in front (it cannot tell this slot from the DMA targets).
      static_assert(RBM == 256, "transform unrolled for 4 x 64 rows");
      const uint32_t la = (uint32_t)reinterpret_cast<uintptr_t>(
          (lds_ptr_t)(As + (tid >> 3) * RBK + pre_pc * 8));
      u32x4_t v[4];
      asm volatile(
          "ds_read_b128 %0, %4\n\t"
          "ds_read_b128 %1, %4 offset:8192\n\t"
          "ds_read_b128 %2, %4 offset:16384\n\t"
          "ds_read_b128 %3, %4 offset:24576\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])
          : "v"(la)
          : "memory");
      u32x4_t o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t w = v[j][u];
          const float x0 = fmaxf(fmaf(__uint_as_float(w << 16), sc[2 * u], sh[2 * u]), 0.f);
          const float x1 = fmaxf(fmaf(__uint_as_float(w & 0xffff0000u), sc[2 * u + 1], sh[2 * u + 1]), 0.f);
          o[j][u] = pack_bf16x2(x0, x1);
        }
      asm volatile(
          "ds_write_b128 %0, %1\n\t"
          "ds_write_b128 %0, %2 offset:8192\n\t"
          "ds_write_b128 %0, %3 offset:16384\n\t"
          "ds_write_b128 %0, %4 offset:24576"
          ::"v"(la), "v"(o[0]), "v"(o[1]), "v"(o[2]), "v"(o[3])
          : "memory");
      // LDS writes visible; plain barrier (a __syncthreads() fence would add vmcnt(0))
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[MT], bfr[NT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int r = wm * TM + mt * 16 + l15;
        af[mt] = *reinterpret_cast<const bf16x8*>(As + r * RBK + (((ks * 4 + lk) ^ (r & 7)) * 8));
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int r = wn * TN + nt * 16 + l15;
        bfr[nt] = *reinterpret_cast<const bf16x8*>(Bs + r * RBK + (((ks * 4 + lk) ^ (r & 7)) * 8));
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[nt], af[mt], acc[mt][nt], 0, 0, 0);
    }
    if (kt + 1 < KT) {
      // stage kt+1 landed (kt+2 may stay in flight); the barrier also retires this
      // stage's slot before step kt+1 issues k-tile kt+3 into it.
      if (kt + 2 < KT) wait_vm<PIECES>();
      else wait_vm<0>();
      asm volatile("s_barrier" ::: "memory");
    }
  }

  // ---- epilogue: lane holds rows m0 + wm*TM + mt*16 + l15, columns n .. n+3 (bf16: 8-B stores; fp32 out,
  // e.g. the TS-VAD LSTM input projection: 16-B stores)
  const int eb = p.out_bf16 ? 2 : 4;
  const int64_t out_bytes = (int64_t)M * p.o_sw * eb;
  const __amdgpu_buffer_rsrc_t ro =
      __builtin_amdgcn_make_buffer_rsrc(p.out, (short)0, (int)(out_bytes < (int64_t)kOOB ? out_bytes : kOOB - 1),
                                        0x00020000);
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
      const int m = m0 + wm * TM + mt * 16 + l15;
      const int n = n0 + wn * TN + nt * 16 + lk * 4;
      const uint32_t off = (m < M && n < p.N) ? (uint32_t)(((int64_t)m * p.o_sw + n) * eb) : kOOB;
      if (p.out_bf16) {
        const u32x2_t v = {pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3])};
        __builtin_amdgcn_raw_buffer_store_b64(v, ro, off, 0, 0);
      } else {
        const u32x4_t v = {__float_as_uint(x[0]), __float_as_uint(x[1]), __float_as_uint(x[2]), __float_as_uint(x[3])};
        __builtin_amdgcn_raw_buffer_store_b128(v, ro, off, 0, 0);
      }
    }
}

// Persistent variant for a single N tile (N <= 128: the dense-block bottlenecks): one workgroup per CU walks
// M tiles b, b + grid, ... and the 3-stage ring runs across tile boundaries, so the next tile's first two
// k-tiles are in flight during the current tile's last MFMAs and epilogue (the one-tile-per-workgroup
// kernel exposed a ring fill and a drain per 256-row tile: at K = 256 that is 2 of its 4 k-steps).
template <bool PRE, int ACT>
__global__ __launch_bounds__(kRingThreads) void gemm_ring_persist_kernel(ConvGemmArgs p) {
  constexpr int WM = 4, WN = 2;
  constexpr int TM = RBM / WM, TN = RBN / WN;
  constexpr int MT = TM / 16, NT = TN / 16;
  constexpr int STORES = MT * NT;              // epilogue VMEM ops per wave per tile
  extern __shared__ __attribute__((aligned(1024))) uint16_t sm[];
  float* s_scale = reinterpret_cast<float*>(sm + RST * STAGE_ELEMS);
  float* s_shift = s_scale + kRingMaxK;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int l15 = lane & 15, lk = lane >> 4;
  const int M = p.B * p.Ho * p.Wo;
  const int K = p.K;
  const int KT = (K + RBK - 1) / RBK;
  const int ntiles = (M + RBM - 1) / RBM;
  const int my_tiles = (int)blockIdx.x < ntiles ? (ntiles - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int total = my_tiles * KT;
  if constexpr (PRE) {
    for (int k = tid; k < KT * RBK; k += kRingThreads) {
      s_scale[k] = k < K ? p.pre_scale[k] : 0.f;
      s_shift[k] = k < K ? p.pre_shift[k] : 0.f;
    }
  }
  float al[NT][4], be[NT][4];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = wn * TN + nt * 16 + lk * 4 + r;
      al[nt][r] = (p.alpha && n < p.N) ? p.alpha[n] : 1.f;
      be[nt][r] = (p.beta && n < p.N) ? p.beta[n] : 0.f;
      // consume them here, before the ring starts: a first use inside the tile loop would get a
      // compiler vmcnt wait that also drains the k-tiles in flight
      asm volatile("" ::"v"(al[nt][r]), "v"(be[nt][r]));
    }
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.A), (short)0,
                                                                      (int)kOOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.Wt), (short)0,
                                                                      (int)kOOB, 0x00020000);
  const int64_t out_bytes = (int64_t)M * p.o_sw * 2;
  const __amdgpu_buffer_rsrc_t ro =
      __builtin_amdgcn_make_buffer_rsrc(p.out, (short)0, (int)(out_bytes < (int64_t)kOOB ? out_bytes : kOOB - 1),
                                        0x00020000);
  const int lrow = lane >> 3, lch = lane & 7;
  const int src = lch ^ lrow;
  uint32_t b_off[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int n = wid * 16 + i * 8 + lrow;
    b_off[i] = n < p.N ? (uint32_t)(((int64_t)n * K + src * 8) * 2) : kOOB;
  }
  // global k-step g = (tile iteration g / KT, k-tile g % KT)
  auto issue = [&](int g) {
    if (g >= total) return;
    const int it = g / KT, kt = g - it * KT;
    const int m0 = ((int)blockIdx.x + it * (int)gridDim.x) * RBM;
    uint16_t* As = sm + (g % RST) * STAGE_ELEMS;
    uint16_t* Bs = As + A_ELEMS;
    const bool ok = kt * RBK + src * 8 < K;
    const int soff = kt * RBK * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wid * 32 + i * 8 + lrow;
      const uint32_t off = (ok && m < M) ? (uint32_t)(((int64_t)m * p.lda + p.a_coff + src * 8) * 2) : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)(As + (wid * 32 + i * 8) * RBK), 16, off,
                                               off == kOOB ? 0 : soff, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr_t)(Bs + (wid * 16 + i * 8) * RBK), 16,
                                               ok ? b_off[i] : kOOB, ok ? soff : 0, 0, 0);
  };
  constexpr int PIECES = 6;
  const int pre_pc = tid & 7;
  const int pre_lc = pre_pc ^ ((tid >> 3) & 7);

  issue(0);
  issue(1);
  if (total > 1) wait_vm<PIECES>();
  else wait_vm<0>();
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // stage 0 + s/h visible

  int g = 0;
  for (int it = 0; it < my_tiles; ++it) {
    floatx4 acc[MT][NT];
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b2 = 0; b2 < NT; ++b2) acc[a][b2] = floatx4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < KT; ++kt, ++g) {
      issue(g + 2);
      uint16_t* As = sm + (g % RST) * STAGE_ELEMS;
      const uint16_t* Bs = As + A_ELEMS;
      if constexpr (PRE) {
        const int k = kt * RBK + pre_lc * 8;
        u32x4_t s0, s1, h0, h1;
        asm volatile(
            "ds_read_b128 %0, %4\n\t"
            "ds_read_b128 %1, %4 offset:16\n\t"
            "ds_read_b128 %2, %5\n\t"
            "ds_read_b128 %3, %5 offset:16\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(s0), "=&v"(s1), "=&v"(h0), "=&v"(h1)
            : "v"((uint32_t)reinterpret_cast<uintptr_t>((lds_ptr_t)(s_scale + k))),
              "v"((uint32_t)reinterpret_cast<uintptr_t>((lds_ptr_t)(s_shift + k)))
            : "memory");
        const float sc[8] = {__uint_as_float(s0.x), __uint_as_float(s0.y), __uint_as_float(s0.z),
                             __uint_as_float(s0.w), __uint_as_float(s1.x), __uint_as_float(s1.y),
                             __uint_as_float(s1.z), __uint_as_float(s1.w)};
        const float sh[8] = {__uint_as_float(h0.x), __uint_as_float(h0.y), __uint_as_float(h0.z),
                             __uint_as_float(h0.w), __uint_as_float(h1.x), __uint_as_float(h1.y),
                             __uint_as_float(h1.z), __uint_as_float(h1.w)};
        const uint32_t la = (uint32_t)reinterpret_cast<uintptr_t>(
            (lds_ptr_t)(As + (tid >> 3) * RBK + pre_pc * 8));
        u32x4_t v[4];
        asm volatile(
            "ds_read_b128 %0, %4\n\t"
            "ds_read_b128 %1, %4 offset:8192\n\t"
            "ds_read_b128 %2, %4 offset:16384\n\t"
            "ds_read_b128 %3, %4 offset:24576\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])
            : "v"(la)
            : "memory");
        u32x4_t o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const uint32_t w = v[j][u];
            const float x0 = fmaxf(fmaf(__uint_as_float(w << 16), sc[2 * u], sh[2 * u]), 0.f);
            const float x1 = fmaxf(fmaf(__uint_as_float(w & 0xffff0000u), sc[2 * u + 1], sh[2 * u + 1]), 0.f);
            o[j][u] = pack_bf16x2(x0, x1);
          }
        asm volatile(
            "ds_write_b128 %0, %1\n\t"
            "ds_write_b128 %0, %2 offset:8192\n\t"
            "ds_write_b128 %0, %3 offset:16384\n\t"
            "ds_write_b128 %0, %4 offset:24576"
            ::"v"(la), "v"(o[0]), "v"(o[1]), "v"(o[2]), "v"(o[3])
            : "memory");
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 af[MT], bfr[NT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const int r = wm * TM + mt * 16 + l15;
          af[mt] = *reinterpret_cast<const bf16x8*>(As + r * RBK + (((ks * 4 + lk) ^ (r & 7)) * 8));
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int r = wn * TN + nt * 16 + l15;
          bfr[nt] = *reinterpret_cast<const bf16x8*>(Bs + r * RBK + (((ks * 4 + lk) ^ (r & 7)) * 8));
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[nt], af[mt], acc[mt][nt], 0, 0, 0);
      }
      if (kt + 1 == KT) {
        // epilogue of this tile: its stores go out while the next tile's first k-tiles are in flight
        const int m0 = ((int)blockIdx.x + it * (int)gridDim.x) * RBM;
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
            const int m = m0 + wm * TM + mt * 16 + l15;
            const int n = wn * TN + nt * 16 + lk * 4;
            const uint32_t off = (m < M && n < p.N) ? (uint32_t)(((int64_t)m * p.o_sw + n) * 2) : kOOB;
            const u32x2_t v = {pack_bf16x2(x[0], x[1]), pack_bf16x2(x[2], x[3])};
            __builtin_amdgcn_raw_buffer_store_b64(v, ro, off, 0, 0);
          }
      }
      if (g + 1 < total) {
        // stage g+1 landed: younger ops are stage g+2's DMAs (if issued) and, after a tile's last k-step,
        // that tile's STORES epilogue stores; the barrier also retires stage g's slot before g+3 reuses it
        const bool more = g + 2 < total;
        if (kt + 1 == KT) {
          if (more) wait_vm<PIECES + STORES>();
          else wait_vm<STORES>();
        } else {
          if (more) wait_vm<PIECES>();
          else wait_vm<0>();
        }
        asm volatile("s_barrier" ::: "memory");
      }
    }
  }
  wait_vm<0>();
}

template <bool PRE, int ACT>
void launch_ring_persist(const ConvGemmArgs& p, hipStream_t st) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    SD_HIP(hipGetDevice(&dev));
    SD_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const int M = p.B * p.Ho * p.Wo;
  const size_t smem = sizeof(uint16_t) * RST * STAGE_ELEMS + (PRE ? 2 * kRingMaxK * sizeof(float) : 0);
  static bool attr = false;
  if (!attr) {
    SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_ring_persist_kernel<PRE, ACT>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const int tiles = cdiv(M, RBM);
  hipLaunchKernelGGL((gemm_ring_persist_kernel<PRE, ACT>), dim3(tiles < cus ? tiles : cus), dim3(kRingThreads),
                     smem, st, p);
}

template <bool PRE, int ACT>
void launch_ring(const ConvGemmArgs& p, hipStream_t st) {
  if (p.N <= RBN) {
    launch_ring_persist<PRE, ACT>(p, st);
    return;
  }
  const int M = p.B * p.Ho * p.Wo;
  const size_t smem = sizeof(uint16_t) * RST * STAGE_ELEMS + (PRE ? 2 * kRingMaxK * sizeof(float) : 0);
  static bool attr = false;
  if (!attr) {
    SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(gemm_ring_kernel<PRE, ACT>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL((gemm_ring_kernel<PRE, ACT>), dim3(cdiv(M, RBM) * cdiv(p.N, RBN)), dim3(kRingThreads), smem,
                     st, p);
}

template <bool PRE>
void launch_ring_act(const ConvGemmArgs& p, hipStream_t st) {
  switch (p.act) {
    case kActRelu: launch_ring<PRE, kActRelu>(p, st); break;
    case kActSigmoid: launch_ring<PRE, kActSigmoid>(p, st); break;
    case kActSilu: launch_ring<PRE, kActSilu>(p, st); break;
    default: launch_ring<PRE, kActNone>(p, st); break;
  }
}

}  // namespace

bool gemm_ring_supported(const ConvGemmArgs& p) {
  static const bool disabled = getenv("SDIAR_NO_RING_GEMM") != nullptr;
  if (disabled) return false;
  const int M = p.B * p.Ho * p.Wo;
  const bool row_major = p.o_sn == 1 && out_rows_linear(p) && a_rows_linear(p);
  const int64_t a_bytes = ((int64_t)p.B * p.H * p.W) * p.lda * 2;
  // fp32 output: the one-tile-per-workgroup kernel only (N > RBN); K > kRingMaxK: no prologue (the s/h
  // staging in LDS is what bounds K)
  return p.a_bf16 && (p.out_bf16 || p.N > RBN) && !p.gate && !p.res && !p.glu && p.kh * p.kw == 1 &&
         (!p.pre_scale || p.pre_shift) && (!p.pre_scale || p.K <= kRingMaxK) && p.K % 8 == 0 && p.lda % 8 == 0 &&
         p.a_coff % 8 == 0 && p.N >= 96 && p.N % 4 == 0 && p.o_sw % 4 == 0 && row_major && M >= 8 * RBM &&
         a_bytes < (int64_t)kOOB && (int64_t)p.N * p.K * 2 < (int64_t)kOOB;
}

void conv_gemm_ring(const ConvGemmArgs& p, hipStream_t st) {
  if (p.pre_scale) launch_ring_act<true>(p, st);
  else launch_ring_act<false>(p, st);
  SD_LAUNCH_CHECK();
}

}  // namespace sd
