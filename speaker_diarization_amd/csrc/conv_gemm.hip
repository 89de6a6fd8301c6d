// Implicit-GEMM convolution / linear layer on gfx950 MFMA.
//
// One kernel family serves every dense contraction on the diarization path:
//   * nn.Linear                     (kh=kw=1, H=1, W=rows)
//   * nn.Conv1d over time           (H=1, W=T, kw taps, stride/pad/dilation)
//   * nn.Conv2d over (freq, time)   (FCM head of CAM++, cam_pplus_wespeaker.py:236-308)
// Activations are channel-last: element (b, h, w, c) lives at
//   A[((b*H + h)*W + w)*lda + a_coff + c]
// so a 1x1 conv is a plain GEMM and a k-tap conv reads k shifted rows.  Weights
// are packed on the host as Wt[N][K] with K = (kh*kw)*Cin ordered tap-major.
//
// Fused prologue:  a' = relu(a*pre_scale[c] + pre_shift[c])   (pre-activation
//                  BatchNorm+ReLU of CAM++ dense/transit layers); padded taps
//                  read as exact zeros, like the reference's zero padding.
// Fused epilogue:  v = acc*alpha[n] + beta[n]   (bias + folded eval BatchNorm)
//                  v += res[m*res_ld + n]       (residual)
//                  v = act(v)                   (ReLU / sigmoid / SiLU)
//                  v *= gate[b, w/seg, n]       (CAMLayer context gate)
//                  out[b*o_sb + h*o_sh + w*o_sw + n*o_sn] = v
//
// Tiles: BM x BN per 256-thread workgroup (2x2 waves), BK = 32, register-staged
// global->LDS double buffer (one barrier per k-step).  bf16 mode converts the
// fp32 activations to bf16 while staging and runs v_mfma_f32_16x16x32_bf16;
// fp32 mode runs the exact-f32 v_mfma_f32_16x16x4_f32; bf16x3 mode (round 6, the
// fp32-equivalent fast path: conv_gemm_x3_kernel) keeps fp32 tensors and splits every
// staged element into bf16 hi + lo: acc += lo·hi + hi·lo + hi·hi on
// v_mfma_f32_16x16x32_bf16 (the lo·lo term and the lo part's own rounding leave
// ~2^-16 relative error per product; 3 MFMAs of 16 cycles per 32-k step against
// 8 f32 MFMAs of 32).
#include <string>

#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {

namespace {

constexpr int kBK = 32;
constexpr int kLdsBf = kBK + 8;   // bf16 row stride (80 B: 16-B aligned, conflict-light)
constexpr int kLdsF = kBK + 2;    // fp32 row stride (34 words: conflict-free 16x16x4 reads)

thread_local bool t_gemm_x3 = false;

// LDS-staged fp32 epilogue (round 6): the accumulator tile goes to LDS (BM x (BN + 4) floats), then each thread
// owns one 4-column group of rows r0, r0 + 256 / (BN / 4), ...: per-channel alpha / beta loaded once, the rows'
// residuals fetched before any store (res may alias out: the in-place residual adds), float4 stores along the
// output rows.  The per-element form it replaces (a 64-B piece per 16 lanes, a divide chain per row, a scalar
// alpha / beta load per element) took 45 % of the bf16x3 GEMM time on C2.
// General outputs (strided, gated) keep a per-element loop over the staged tile.
template <int BM, int BN, int MT, int NT>
__device__ __forceinline__ void staged_epilogue_f32(const ConvGemmArgs& p, const floatx4 (&acc)[MT][NT], float* Cs,
                                                    int m0, int n0, int M) {
  constexpr int TM = BM / 2, TN = BN / 2, CLD = BN + 4, CPR = BN / 4;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1, lrow = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) Cs[(wm * TM + mt * 16 + lk * 4 + r) * CLD + wn * TN + nt * 16 + lrow] = acc[mt][nt][r];
  __syncthreads();
  float* const outp = reinterpret_cast<float*>(p.out);
  const bool lin = out_rows_linear(p);
  // float4 rows: unit column stride, 4-float row strides and 16-B aligned base pointers
  if (lin && p.o_sn == 1 && (p.o_sw & 3) == 0 && (reinterpret_cast<uintptr_t>(p.out) & 15) == 0 && !p.gate &&
      (!p.res || ((p.res_ld & 3) == 0 && (reinterpret_cast<uintptr_t>(p.res) & 15) == 0))) {
    constexpr int RPI = 256 / CPR, ITER = BM / RPI;
    const int cg = tid % CPR, r0 = tid / CPR, n = n0 + cg * 4;
    if (n >= p.N) return;
    const bool full = n + 3 < p.N;
    float al[4], be[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool ok = full || n + u < p.N;
      al[u] = (p.alpha && ok) ? p.alpha[n + u] : 1.f;
      be[u] = (p.beta && ok) ? p.beta[n + u] : 0.f;
    }
    float4 rv[ITER];
    if (p.res) {
      const float* rbase = reinterpret_cast<const float*>(p.res);
#pragma unroll
      for (int i = 0; i < ITER; ++i) {
        const int m = m0 + r0 + i * RPI;
        rv[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (m < M) {
          const float* r = rbase + (int64_t)m * p.res_ld + n;
          if (full) rv[i] = *reinterpret_cast<const float4*>(r);
          else {
            rv[i].x = r[0];
            if (n + 1 < p.N) rv[i].y = r[1];
            if (n + 2 < p.N) rv[i].z = r[2];
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < ITER; ++i) {
      const int row = r0 + i * RPI, m = m0 + row;
      if (m >= M) break;
      const float4 c4 = *reinterpret_cast<const float4*>(Cs + row * CLD + cg * 4);
      float v[4] = {c4.x, c4.y, c4.z, c4.w};
      const float r4[4] = {p.res ? rv[i].x : 0.f, p.res ? rv[i].y : 0.f, p.res ? rv[i].z : 0.f, p.res ? rv[i].w : 0.f};
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = apply_act(v[u] * al[u] + be[u] + r4[u], p.act);
      const int64_t o = (int64_t)m * p.o_sw + n;
      if (full) *reinterpret_cast<float4*>(outp + o) = make_float4(v[0], v[1], v[2], v[3]);
      else
        for (int u = 0; u < 4 && n + u < p.N; ++u) outp[o + u] = v[u];
    }
    return;
  }
  for (int q = tid; q < BM * BN; q += 256) {
    const int row = q / BN, col = q % BN, m = m0 + row, n = n0 + col;
    if (m >= M || n >= p.N) continue;
    const int wo = m % p.Wo, t = m / p.Wo, ho = t % p.Ho, b = t / p.Ho;
    float v = Cs[row * CLD + col];
    if (p.alpha) v *= p.alpha[n];
    if (p.beta) v += p.beta[n];
    if (p.res) v += reinterpret_cast<const float*>(p.res)[(int64_t)m * p.res_ld + n];
    v = apply_act(v, p.act);
    if (p.gate) v *= p.gate[((int64_t)b * p.gate_nseg + wo / p.gate_seg) * p.N + n];
    outp[(int64_t)b * p.o_sb + (int64_t)ho * p.o_sh + (int64_t)wo * p.o_sw + (int64_t)n * p.o_sn] = v;
  }
}

// MODE 0: exact f32 MFMA, 1: bf16 (fp32 activations converted on staging); bf16x3: conv_gemm_x3_kernel
template <int BM, int BN, int MODE>
__global__ __launch_bounds__(256) void conv_gemm_kernel(ConvGemmArgs p) {
  constexpr bool BF16 = MODE == 1;
  constexpr int TM = BM / 2, TN = BN / 2;
  constexpr int MT = TM / 16, NT = TN / 16;
  constexpr int APASS = BM / 32;
  using LdsT = typename std::conditional<BF16, uint16_t, float>::type;
  constexpr int LDS_STRIDE = BF16 ? kLdsBf : kLdsF;
  // one array (As then Bs) so the exact-f32 epilogue can stage its tile over both
  __shared__ __attribute__((aligned(16))) LdsT smem[2 * (BM + BN) * LDS_STRIDE];
  LdsT (*const As)[BM * LDS_STRIDE] = reinterpret_cast<LdsT (*)[BM * LDS_STRIDE]>(smem);
  LdsT (*const Bs)[BN * LDS_STRIDE] = reinterpret_cast<LdsT (*)[BN * LDS_STRIDE]>(smem + 2 * BM * LDS_STRIDE);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int M = p.B * p.Ho * p.Wo;
  // 1-D grid, XCD-grouped (xcd_remap): the column tiles of one row block are consecutive tiles and run on one
  // XCD, so its L2 fetches the block's A rows once instead of every XCD fetching them (A is the large operand)
  const int n_nt = (p.N + BN - 1) / BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (tile / n_nt) * BM;
  const int n0 = (tile % n_nt) * BN;

  // Per-thread A rows (fixed across the k loop).
  int rbh[APASS], rh[APASS], rw[APASS];
  const int kq = (tid & 7) * 4;
#pragma unroll
  for (int i = 0; i < APASS; ++i) {
    int m = m0 + i * 32 + (tid >> 3);
    if (m < M) {
      int wo = m % p.Wo;
      int t = m / p.Wo;
      int ho = t % p.Ho;
      int b = t / p.Ho;
      rbh[i] = b * p.H;
      rh[i] = ho * p.sh - p.ph;
      rw[i] = wo * p.sw - p.pw;
    } else {
      rbh[i] = 0;
      rh[i] = -(1 << 28);
      rw[i] = 0;
    }
  }

  const int KT = (p.K + kBK - 1) / kBK;
  // raw loads only: the BN-ReLU prologue is applied in store_tile, after the k-step's MFMAs, so no wait for a
  // load sits between a k-step's loads and its MFMAs (applied at load time, the compiler waited for each load)
  float4 areg[APASS], s4, h4;
  uint32_t avalid = 0;
  // B staging registers.
  constexpr int BCHUNK = BF16 ? (BN * 4) : (BN * 8);   // 16-B chunks per tile
  constexpr int BPASS = (BCHUNK + 255) / 256;
  uint4 breg[BPASS];

  auto load_tile = [&](int kt) {
    const int k0 = kt * kBK;
    const int tap = k0 / p.Cin;
    const int c0 = k0 - tap * p.Cin;
    const int ti = tap / p.kw;
    const int tj = tap - ti * p.kw;
    const int c = c0 + kq;
    if (p.pre_scale && k0 + kq < p.K) {
      s4 = *reinterpret_cast<const float4*>(p.pre_scale + c);
      h4 = *reinterpret_cast<const float4*>(p.pre_shift + c);
    }
    avalid = 0;
#pragma unroll
    for (int i = 0; i < APASS; ++i) {
      int hi = rh[i] + ti * p.dh;
      int wi = rw[i] + tj * p.dw;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if ((unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W && k0 + kq < p.K) {
        const float* src = reinterpret_cast<const float*>(p.A) + ((int64_t)(rbh[i] + hi) * p.W + wi) * p.lda + p.a_coff + c;
        v = *reinterpret_cast<const float4*>(src);
        avalid |= 1u << i;
      }
      areg[i] = v;
    }
#pragma unroll
    for (int i = 0; i < BPASS; ++i) {
      int ch = tid + i * 256;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (ch < BCHUNK) {
        if (BF16) {
          int n = ch >> 2, kc = (ch & 3) * 8;
          if (n0 + n < p.N && k0 + kc < p.K)
            v = *reinterpret_cast<const uint4*>(
                reinterpret_cast<const uint16_t*>(p.Wt) + (int64_t)(n0 + n) * p.K + k0 + kc);
        } else {
          int n = ch >> 3, kc = (ch & 7) * 4;
          if (n0 + n < p.N && k0 + kc < p.K)
            v = *reinterpret_cast<const uint4*>(
                reinterpret_cast<const float*>(p.Wt) + (int64_t)(n0 + n) * p.K + k0 + kc);
        }
      }
      breg[i] = v;
    }
  };

  auto store_tile = [&](int buf) {
#pragma unroll
    for (int i = 0; i < APASS; ++i) {
      int row = i * 32 + (tid >> 3);
      if (p.pre_scale && (avalid >> i & 1u)) {   // padded taps stay exact zeros
        areg[i].x = fmaxf(areg[i].x * s4.x + h4.x, 0.f);
        areg[i].y = fmaxf(areg[i].y * s4.y + h4.y, 0.f);
        areg[i].z = fmaxf(areg[i].z * s4.z + h4.z, 0.f);
        areg[i].w = fmaxf(areg[i].w * s4.w + h4.w, 0.f);
      }
      if (BF16) {
        uint2 pk;
        pk.x = (uint32_t)f2bf_bits(areg[i].x) | ((uint32_t)f2bf_bits(areg[i].y) << 16);
        pk.y = (uint32_t)f2bf_bits(areg[i].z) | ((uint32_t)f2bf_bits(areg[i].w) << 16);
        *reinterpret_cast<uint2*>(&As[buf][row * LDS_STRIDE + kq]) = pk;
      } else {
        float* d = reinterpret_cast<float*>(&As[buf][row * LDS_STRIDE + kq]);
        *reinterpret_cast<float2*>(d) = make_float2(areg[i].x, areg[i].y);
        *reinterpret_cast<float2*>(d + 2) = make_float2(areg[i].z, areg[i].w);
      }
    }
#pragma unroll
    for (int i = 0; i < BPASS; ++i) {
      int ch = tid + i * 256;
      if (ch < BCHUNK) {
        if (BF16) {
          int n = ch >> 2, kc = (ch & 3) * 8;
          *reinterpret_cast<uint4*>(&Bs[buf][n * LDS_STRIDE + kc]) = breg[i];
        } else {
          int n = ch >> 3, kc = (ch & 7) * 4;
          float* d = reinterpret_cast<float*>(&Bs[buf][n * LDS_STRIDE + kc]);
          *reinterpret_cast<uint2*>(d) = make_uint2(breg[i].x, breg[i].y);
          *reinterpret_cast<uint2*>(d + 2) = make_uint2(breg[i].z, breg[i].w);
        }
      }
    }
  };

  floatx4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};

  load_tile(0);
  store_tile(0);
  __syncthreads();

  const int lrow = lane & 15;
  const int lk = lane >> 4;
  for (int kt = 0; kt < KT; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < KT) load_tile(kt + 1);
    if (BF16) {
      bf16x8 af[MT], bfr[NT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        af[mt] = *reinterpret_cast<const bf16x8*>(
            &As[buf][(wm * TM + mt * 16 + lrow) * LDS_STRIDE + lk * 8]);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        bfr[nt] = *reinterpret_cast<const bf16x8*>(
            &Bs[buf][(wn * TN + nt * 16 + lrow) * LDS_STRIDE + lk * 8]);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bfr[nt], acc[mt][nt], 0, 0, 0);
    } else {
      const float* Af = reinterpret_cast<const float*>(As[buf]);
      const float* Bf = reinterpret_cast<const float*>(Bs[buf]);
#pragma unroll
      for (int kk = 0; kk < kBK / 4; ++kk) {
        float af[MT], bfr[NT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          af[mt] = Af[(wm * TM + mt * 16 + lrow) * LDS_STRIDE + kk * 4 + lk];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          bfr[nt] = Bf[(wn * TN + nt * 16 + lrow) * LDS_STRIDE + kk * 4 + lk];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt)
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[mt], bfr[nt], acc[mt][nt], 0, 0, 0);
      }
    }
    if (kt + 1 < KT) store_tile(buf ^ 1);
    __syncthreads();
  }

  // Epilogue: staged through LDS in exact-f32 mode (the tile fits the fp32 operand buffers)
  if constexpr (!BF16 && (int)sizeof(smem) >= BM * (BN + 4) * 4) {
    staged_epilogue_f32<BM, BN, MT, NT>(p, acc, reinterpret_cast<float*>(smem), m0, n0, M);
    return;
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * TM + mt * 16 + lk * 4 + r;
      if (m >= M) continue;
      const int wo = m % p.Wo;
      const int t = m / p.Wo;
      const int ho = t % p.Ho;
      const int b = t / p.Ho;
      const int64_t obase = (int64_t)b * p.o_sb + (int64_t)ho * p.o_sh + (int64_t)wo * p.o_sw;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int n = n0 + wn * TN + nt * 16 + lrow;
        if (n >= p.N) continue;
        float v = acc[mt][nt][r];
        if (p.alpha) v *= p.alpha[n];
        if (p.beta) v += p.beta[n];
        if (p.res) v += reinterpret_cast<const float*>(p.res)[(int64_t)m * p.res_ld + n];
        v = apply_act(v, p.act);
        if (p.gate) v *= p.gate[((int64_t)b * p.gate_nseg + wo / p.gate_seg) * p.N + n];
        reinterpret_cast<float*>(p.out)[obase + (int64_t)n * p.o_sn] = v;
      }
    }
  }
}

// 4 fp32 -> bf16 hi (round to nearest even) and lo = bf16(v - hi) (v - hi is exact in fp32), 2 words each
__device__ __forceinline__ void split_bf16x4(const float4& v, uint2& hi, uint2& lo) {
  hi.x = pack_bf16x2(v.x, v.y);
  hi.y = pack_bf16x2(v.z, v.w);
  lo.x = pack_bf16x2(v.x - __uint_as_float(hi.x << 16), v.y - __uint_as_float(hi.x & 0xffff0000u));
  lo.y = pack_bf16x2(v.z - __uint_as_float(hi.y << 16), v.w - __uint_as_float(hi.y & 0xffff0000u));
}

// LDS offset (bf16 elements) of 16-B chunk c (k 8c .. 8c + 7) of tile row r in the bf16x3 tiles: 64-B rows,
// chunk XOR (r >> 1) & 3.  Conflict-free for both accesses (MI355X_MICROARCH.md LDS table): the stores
// (ds_write_b64, 16 contiguous lanes = 2 rows x 64 B, banks mod 32) and the fragment reads (ds_read_b128 in
// its 4 x 16-lane groups, banks mod 64), where the 80-B padded rows left a 2-way conflict on both.
__device__ __forceinline__ int x3_chunk(int r, int c) { return r * kBK + ((c ^ ((r >> 1) & 3)) << 3); }

// bf16x3 GEMM (round 6).  Every fp32 element is split ONCE, by the thread that stages it, into bf16 hi (RNE)
// and lo = bf16(x - hi), written to hi / lo LDS tiles (64-B rows, x3_chunk swizzle); the waves read ready bf16
// fragments with ds_read_b128.  Per 32-deep k-step a wave issues, per 16x16 output tile, lo_A·hi_B, hi_A·lo_B,
// hi_A·hi_B (fp32 accumulate, that order for every accumulator).  The loads are unconditional (out-of-range
// rows / taps read chunk 0 and are zeroed when staged) and the BN-ReLU prologue is applied at staging, so the
// k-step's MFMAs never wait for its own loads.  LDS: hi + lo tiles of A and B, double-buffered =
// 2 * 2 * (BM + BN) * 64 B (64 KiB at 128 x 128: two workgroups per CU).
// Measured on C2 (bf16x3 line): the first form, each wave re-splitting the fp32
// fragments it read from fp32 tiles, 153 ms; this form 126 ms.  Also measured, no better: an LDS-DMA-fed form
// (raw fp32 stages converted in place, 2-4 stage ring: 142-214 ms), every row tile's MFMAs interleaved for the
// wide tiles too (126.3 ms), the XCD-grouped 1-D grid (127.0 ms; kept: neutral here, it keeps a row block's
// A reads in one XCD's L2).
template <int BM, int BN>
__global__ __launch_bounds__(256) void conv_gemm_x3_kernel(ConvGemmArgs p) {
  constexpr int TM = BM / 2, TN = BN / 2;
  constexpr int MT = TM / 16, NT = TN / 16;
  constexpr int APASS = BM / 32;
  constexpr int S = kBK;   // 64-B rows, 16-B chunks XOR-swizzled by x3_chunk (no padding)
  constexpr int ABUF = 2 * BM * S, BBUF = 2 * BN * S;   // hi tile then lo tile
  extern __shared__ __attribute__((aligned(16))) uint16_t smx[];
  uint16_t* const As = smx;                 // [2][ABUF]
  uint16_t* const Bs = smx + 2 * ABUF;      // [2][BBUF]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int M = p.B * p.Ho * p.Wo;
  // 1-D grid, XCD-grouped (xcd_remap): the column tiles of one row block are consecutive tiles and run on one
  // XCD, so its L2 fetches the block's A rows once instead of every XCD fetching them (A is the large operand)
  const int n_nt = (p.N + BN - 1) / BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (tile / n_nt) * BM;
  const int n0 = (tile % n_nt) * BN;

  int rbh[APASS], rh[APASS], rw[APASS];
  const int kq = (tid & 7) * 4;
#pragma unroll
  for (int i = 0; i < APASS; ++i) {
    int m = m0 + i * 32 + (tid >> 3);
    if (m < M) {
      int wo = m % p.Wo;
      int t = m / p.Wo;
      int ho = t % p.Ho;
      int b = t / p.Ho;
      rbh[i] = b * p.H;
      rh[i] = ho * p.sh - p.ph;
      rw[i] = wo * p.sw - p.pw;
    } else {
      rbh[i] = 0;
      rh[i] = -(1 << 28);
      rw[i] = 0;
    }
  }

  const int KT = (p.K + kBK - 1) / kBK;
  constexpr int BPASS = (BN * 8 + 255) / 256;   // 16-B fp32 chunks of the B tile
  // raw loads only: the BN-ReLU prologue is applied in store_tile, after the MFMAs, so no wait for a load
  // sits between a k-step's loads and its MFMAs (applied at load time, the compiler waited for each load).
  // (two register stages, each k-step's loads issued two compute phases ahead, measured 127 -> 186 ms on C2:
  // the second stage's registers cost the second workgroup per CU)
  struct Stage {
    float4 a[APASS], b[BPASS], s4, h4;
    uint32_t av, bv;
  };
  Stage st;

  auto load_tile = [&](int kt, Stage& sg) {
    const int k0 = kt * kBK;
    const int tap = k0 / p.Cin;
    const int c0 = k0 - tap * p.Cin;
    const int ti = tap / p.kw;
    const int tj = tap - ti * p.kw;
    const int c = c0 + kq;
    if (p.pre_scale && k0 + kq < p.K) {
      sg.s4 = *reinterpret_cast<const float4*>(p.pre_scale + c);
      sg.h4 = *reinterpret_cast<const float4*>(p.pre_shift + c);
    }
    sg.av = 0;
#pragma unroll
    for (int i = 0; i < APASS; ++i) {
      int hi = rh[i] + ti * p.dh;
      int wi = rw[i] + tj * p.dw;
      // unconditional load (an out-of-range tap reads the tensor's first chunk, zeroed in store_tile): with
      // exec-masked loads the compiler copied every loaded register at the top of the MFMA phase, i.e.
      // waited for the loads there
      const bool ok = (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W && k0 + kq < p.K;
      const int64_t off = ok ? ((int64_t)(rbh[i] + hi) * p.W + wi) * p.lda + p.a_coff + c : 0;
      sg.a[i] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p.A) + off);
      sg.av |= (ok ? 1u : 0u) << i;
    }
    sg.bv = 0;
#pragma unroll
    for (int i = 0; i < BPASS; ++i) {
      const int ch = tid + i * 256;
      const int n = ch >> 3, kc = (ch & 7) * 4;
      const bool ok = ch < BN * 8 && n0 + n < p.N && k0 + kc < p.K;
      sg.b[i] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p.Wt) +
                                                 (ok ? (int64_t)(n0 + n) * p.K + k0 + kc : 0));
      sg.bv |= (ok ? 1u : 0u) << i;
    }
  };

  auto store_tile = [&](int buf, const Stage& sg) {
    uint16_t* a = As + buf * ABUF;
    uint16_t* b = Bs + buf * BBUF;
#pragma unroll
    for (int i = 0; i < APASS; ++i) {
      const int row = i * 32 + (tid >> 3);
      float4 v = sg.a[i];
      if (!(sg.av >> i & 1u)) {
        v = make_float4(0.f, 0.f, 0.f, 0.f);    // padded taps are exact zeros
      } else if (p.pre_scale) {
        v.x = fmaxf(v.x * sg.s4.x + sg.h4.x, 0.f);
        v.y = fmaxf(v.y * sg.s4.y + sg.h4.y, 0.f);
        v.z = fmaxf(v.z * sg.s4.z + sg.h4.z, 0.f);
        v.w = fmaxf(v.w * sg.s4.w + sg.h4.w, 0.f);
      }
      uint2 h, l;
      split_bf16x4(v, h, l);
      const int o = x3_chunk(row, kq >> 3) + (kq & 4);
      *reinterpret_cast<uint2*>(a + o) = h;
      *reinterpret_cast<uint2*>(a + BM * S + o) = l;
    }
#pragma unroll
    for (int i = 0; i < BPASS; ++i) {
      const int ch = tid + i * 256;
      if (ch < BN * 8) {
        const int n = ch >> 3, kc = (ch & 7) * 4;
        uint2 h, l;
        split_bf16x4((sg.bv >> i & 1u) ? sg.b[i] : make_float4(0.f, 0.f, 0.f, 0.f), h, l);
        const int o = x3_chunk(n, kc >> 3) + (kc & 4);
        *reinterpret_cast<uint2*>(b + o) = h;
        *reinterpret_cast<uint2*>(b + BN * S + o) = l;
      }
    }
  };

  floatx4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int lrow = lane & 15;
  const int lk = lane >> 4;
  auto compute = [&](int buf) {
    const uint16_t* a = As + buf * ABUF;
    const uint16_t* b = Bs + buf * BBUF;
    bf16x8 bh[NT], bl[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int o = x3_chunk(wn * TN + nt * 16 + lrow, lk);
      bh[nt] = *reinterpret_cast<const bf16x8*>(b + o);
      bl[nt] = *reinterpret_cast<const bf16x8*>(b + BN * S + o);
    }
    if constexpr (NT >= 4) {
      // per row tile, term-major over the NT column tiles: NT - 1 independent MFMAs between two on the same
      // accumulator, which sums al·bh, ah·bl, ah·bh in that order
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int o = x3_chunk(wm * TM + mt * 16 + lrow, lk);
        const bf16x8 ah = *reinterpret_cast<const bf16x8*>(a + o);
        const bf16x8 al = *reinterpret_cast<const bf16x8*>(a + BM * S + o);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[nt], acc[mt][nt], 0, 0, 0);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[nt], acc[mt][nt], 0, 0, 0);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[nt], acc[mt][nt], 0, 0, 0);
      }
    } else {
      // narrow tiles (NT 1-2): term-major over every (mt, nt), so MT x NT - 1 independent MFMAs separate two
      // on one accumulator (per row tile they were back to back: 128 x 32 waited on each MFMA's result)
      bf16x8 ah[MT], al[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int o = x3_chunk(wm * TM + mt * 16 + lrow, lk);
        ah[mt] = *reinterpret_cast<const bf16x8*>(a + o);
        al[mt] = *reinterpret_cast<const bf16x8*>(a + BM * S + o);
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[mt], bh[nt], acc[mt][nt], 0, 0, 0);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[mt], bl[nt], acc[mt][nt], 0, 0, 0);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[mt], bh[nt], acc[mt][nt], 0, 0, 0);
    }
  };

  load_tile(0, st);
  store_tile(0, st);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < KT) load_tile(kt + 1, st);
    compute(buf);
    if (kt + 1 < KT) store_tile(buf ^ 1, st);
    __syncthreads();
  }
  staged_epilogue_f32<BM, BN, MT, NT>(p, acc, reinterpret_cast<float*>(smx), m0, n0, M);
}

template <int BM, int BN>
void launch_x3(const ConvGemmArgs& p, dim3 grid, hipStream_t st) {
  constexpr int kRing = 2 * (2 * BM + 2 * BN) * kBK * (int)sizeof(uint16_t);   // 2 buffers x (hi+lo of A, B)
  constexpr int kEpi = BM * (BN + 4) * (int)sizeof(float);                      // the staged epilogue tile
  constexpr int kBytes = kRing > kEpi ? kRing : kEpi;
  static bool attr = [] {
    SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_gemm_x3_kernel<BM, BN>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, kBytes));
    return true;
  }();
  (void)attr;
  hipLaunchKernelGGL((conv_gemm_x3_kernel<BM, BN>), grid, dim3(256), kBytes, st, p);
}

template <int BM, int BN>
void launch_tile(const ConvGemmArgs& p, bool bf16, hipStream_t st) {
  SD_CHECK(!p.a_bf16 && !p.out_bf16 && !p.res_bf16, kErrInvalid, "fp32 conv_gemm takes fp32 tensors");
  const int M = p.B * p.Ho * p.Wo;
  dim3 grid(cdiv(p.N, BN) * cdiv(M, BM));
  if (bf16)
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, 1>), grid, dim3(256), 0, st, p);
  else if (t_gemm_x3)
    launch_x3<BM, BN>(p, grid, st);
  else
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, 0>), grid, dim3(256), 0, st, p);
}

}  // namespace

bool gemm_x3() { return t_gemm_x3; }
GemmX3Scope::GemmX3Scope(bool on) : prev(t_gemm_x3) { t_gemm_x3 = on; }
GemmX3Scope::~GemmX3Scope() { t_gemm_x3 = prev; }

void conv_gemm(const ConvGemmArgs& p, bool bf16, hipStream_t st) {
  SD_CHECK(p.K == p.kh * p.kw * p.Cin, kErrInvalid, "conv_gemm: K != kh*kw*Cin");
  SD_CHECK(p.K % 4 == 0, kErrInvalid, "conv_gemm: K must be a multiple of 4");
  SD_CHECK(p.Cin % kBK == 0 || (p.kh * p.kw == 1), kErrInvalid,
           "conv_gemm: multi-tap conv needs Cin % 32 == 0");
  SD_CHECK(p.lda % 4 == 0 && p.a_coff % 4 == 0, kErrInvalid, "conv_gemm: lda/a_coff must be multiples of 4");
  SD_CHECK(p.N > 0 && p.B > 0 && p.Ho > 0 && p.Wo > 0, kErrInvalid, "conv_gemm: empty problem");
  SD_CHECK(!p.gate || p.gate_seg > 0, kErrInvalid, "conv_gemm: gate_seg must be > 0");
  SD_CHECK(!p.glu || (bf16 && gemm_stream_supported(p)), kErrInvalid,
           "conv_gemm: the GLU epilogue exists on the bf16 streaming path only");
  SD_CHECK(!p.a_tiled || (bf16 && p.a_bf16 && p.lda == p.K && p.a_coff == 0 && (p.B * p.Ho * p.Wo) % 16 == 0 &&
                           gemm_areg_supported(p)),
           kErrInvalid, "conv_gemm: the tiled A layout exists on the register-A GEMM only");
  if (gemm_skinny_supported(p)) {   // <= 16 rows: weight streaming (streaming FS-EEND chunks)
    conv_gemm_skinny(p, bf16, st);
    return;
  }
  SD_CHECK(!p.ln_g && !p.kv_out && !p.pro_mode, kErrInvalid,
           "conv_gemm: LN / other prologues and the K-V epilogue exist on the skinny path only");
  if (bf16) {
    conv_gemm_bf16(p, st);
    return;
  }
  const int M = p.B * p.Ho * p.Wo;
  // Algorithmic work: 2*M*N*K flops; bytes = input activation once + weights + output (+res).
  const double flops = 2.0 * M * p.N * (double)p.K;
  const double bytes = 4.0 * p.B * p.H * p.W * p.Cin + (bf16 ? 2.0 : 4.0) * p.N * p.K +
                       4.0 * M * p.N * (p.res ? 2.0 : 1.0);
  static const bool detail = getenv("SDIAR_PROF_DETAIL") != nullptr;
  std::string key = bf16 ? "conv_gemm_bf16" : t_gemm_x3 ? "conv_gemm_bf16x3" : "conv_gemm_f32";
  if (detail && prof_enabled())
    key += " M=" + std::to_string(M) + " N=" + std::to_string(p.N) + " K=" + std::to_string(p.K) +
           " taps=" + std::to_string(p.kh * p.kw) + (p.pre_scale ? " pre" : "");
  ProfScope prof(key.c_str(), flops, bytes, st);
  const int bn = p.N >= 128 ? 128 : (p.N >= 64 ? 64 : 32);
  const int tiles128 = cdiv(M, 128) * cdiv(p.N, bn);
  const bool big = tiles128 >= 512;
  if (bn == 128) {
    if (big) launch_tile<128, 128>(p, bf16, st); else launch_tile<64, 128>(p, bf16, st);
  } else if (bn == 64) {
    if (big) launch_tile<128, 64>(p, bf16, st); else launch_tile<64, 64>(p, bf16, st);
  } else {
    if (big) launch_tile<128, 32>(p, bf16, st); else launch_tile<64, 32>(p, bf16, st);
  }
  SD_LAUNCH_CHECK();
}

}  // namespace sd
