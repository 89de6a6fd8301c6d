// CAM++ FCM 3x3 convolutions (32 -> 32 channels, pad 1, freq stride 1 or 2) for gfx950.
//
// cam_pplus_wespeaker.py BasicResBlock / FCM.conv2 (:240-308) are 3x3 convs over
// (freq, time) maps with only 32 channels: as a GEMM, K = 288 and N = 32, so a
// generic tile kernel re-reads every input pixel 9 times and spends its time on
// address arithmetic.  Here a persistent workgroup walks output tiles of one row
// (b, ho) x 128 frames: the 3 input rows a tile needs (+1 halo frame each side) are
// staged in LDS once (16-B loads, the NEXT tile's rows prefetched into registers
// while the current one computes), the 9 x 2 weight fragments are loaded into
// registers once per workgroup, and each wave runs 9 taps x (2 x 2)
// v_mfma_f32_16x16x32_bf16 per 32 output frames.  The epilogue (folded BN,
// residual, ReLU) is staged through LDS so stores leave as 16-B vectors (or
// per-element for the transposed FCM output layout).
#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {
namespace {

constexpr int kPx = 128;          // output frames per tile
constexpr int kPS = 40;           // LDS pixel stride in bf16 (32 channels + 8 pad: 80 B)
constexpr int kRowPx = kPx + 2;   // staged frames per input row
constexpr int kHaloVec = 3 * kRowPx * 4;           // 16-B vectors per tile (1560)
constexpr int kHaloPer = (kHaloVec + 255) / 256;   // per thread (7)
constexpr int kCS = 33;           // epilogue LDS row stride (floats)

__global__ __launch_bounds__(256) void fcm_conv3x3_kernel(ConvGemmArgs p, int n_tiles) {
  __shared__ __attribute__((aligned(16))) uint16_t xs[3 * kRowPx * kPS];   // 31.2 KiB
  __shared__ float cs[kPx * kCS];                                          // 16.5 KiB
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int l15 = lane & 15, q = lane >> 4;
  const int n_wt = (p.Wo + kPx - 1) / kPx;
  const uint16_t* A = reinterpret_cast<const uint16_t*>(p.A);

  // weights: Wt[n][tap*32 + c] -> fragment (tap, nt) = W[nt*16 + l15][tap*32 + 8q .. +8]
  bf16x8 wf[9][2];
  {
    const uint16_t* W = reinterpret_cast<const uint16_t*>(p.Wt);
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        wf[t][nt] = *reinterpret_cast<const bf16x8*>(W + (nt * 16 + l15) * 288 + t * 32 + q * 8);
  }
  // epilogue channel group of this thread is fixed: c0 = (tid & 3) * 8
  const int ec0 = (tid & 3) * 8;
  float al[8], be[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    al[u] = p.alpha ? p.alpha[ec0 + u] : 1.f;
    be[u] = p.beta ? p.beta[ec0 + u] : 0.f;
  }
  const bool nhwc = p.o_sn == 1 && p.o_sw == 32 && p.o_sh == (int64_t)p.Wo * 32;

  auto load_halo = [&](int tile, uint4* v) {
    const int wt = tile % n_wt;
    const int bh = tile / n_wt;
    const int ho = bh % p.Ho, b = bh / p.Ho;
    const int wo0 = wt * kPx;
#pragma unroll
    for (int k = 0; k < kHaloPer; ++k) {
      const int i = tid + k * 256;
      const int ch = (i & 3) * 8;
      const int px = (i >> 2) % kRowPx;
      const int dh = (i >> 2) / kRowPx;
      const int hi = ho * p.sh - 1 + dh;
      const int wi = wo0 - 1 + px;
      v[k] = make_uint4(0u, 0u, 0u, 0u);
      if (i < kHaloVec && (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W)
        v[k] = *reinterpret_cast<const uint4*>(A + (((int64_t)b * p.H + hi) * p.W + wi) * p.lda + p.a_coff + ch);
    }
  };

  uint4 hv[kHaloPer];
  int tile = blockIdx.x;
  if (tile < n_tiles) load_halo(tile, hv);
  for (; tile < n_tiles; tile += gridDim.x) {
#pragma unroll
    for (int k = 0; k < kHaloPer; ++k) {
      const int i = tid + k * 256;
      if (i < kHaloVec) {
        const int ch = (i & 3) * 8, px = (i >> 2) % kRowPx, dh = (i >> 2) / kRowPx;
        *reinterpret_cast<uint4*>(xs + (dh * kRowPx + px) * kPS + ch) = hv[k];
      }
    }
    __syncthreads();
    const int next = tile + gridDim.x;
    if (next < n_tiles) load_halo(next, hv);   // in flight during the MFMAs and epilogue

    floatx4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 2; ++c) acc[a][c] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dh = 0; dh < 3; ++dh)
#pragma unroll
      for (int dw = 0; dw < 3; ++dw) {
        const int t = dh * 3 + dw;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
          const int px = wv * 32 + mt * 16 + l15 + dw;   // staged frame of output (wv*32 + mt*16 + l15)
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(xs + (dh * kRowPx + px) * kPS + q * 8);
#pragma unroll
          for (int nt = 0; nt < 2; ++nt)
            acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, wf[t][nt], acc[mt][nt], 0, 0, 0);
        }
      }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) cs[(wv * 32 + mt * 16 + q * 4 + r) * kCS + nt * 16 + l15] = acc[mt][nt][r];
    __syncthreads();   // xs free for the next tile, cs complete

    const int wt = tile % n_wt;
    const int bh = tile / n_wt;
    const int ho = bh % p.Ho, b = bh / p.Ho;
    const int wo0 = wt * kPx;
#pragma unroll
    for (int k = 0; k < kPx * 4 / 256; ++k) {
      const int px = (tid >> 2) + k * 64;
      const int wo = wo0 + px;
      if (wo >= p.Wo) continue;
      float rv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (p.res) {
        const int64_t ro = (((int64_t)b * p.Ho + ho) * p.Wo + wo) * p.res_ld + ec0;
        if (p.res_bf16) {
          const uint4 r4 = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(p.res) + ro);
          const uint32_t rw[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            rv[2 * u] = __uint_as_float(rw[u] << 16);
            rv[2 * u + 1] = __uint_as_float(rw[u] & 0xffff0000u);
          }
        } else {
          const float* rf = reinterpret_cast<const float*>(p.res) + ro;
#pragma unroll
          for (int u = 0; u < 8; ++u) rv[u] = rf[u];
        }
      }
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = apply_act(fmaf(cs[px * kCS + ec0 + u], al[u], be[u]) + rv[u], p.act);
      const int64_t ob = (int64_t)b * p.o_sb + (int64_t)ho * p.o_sh + (int64_t)wo * p.o_sw;
      if (nhwc && p.out_bf16) {
        uint4 o;
        o.x = (uint32_t)f2bf_bits(v[0]) | ((uint32_t)f2bf_bits(v[1]) << 16);
        o.y = (uint32_t)f2bf_bits(v[2]) | ((uint32_t)f2bf_bits(v[3]) << 16);
        o.z = (uint32_t)f2bf_bits(v[4]) | ((uint32_t)f2bf_bits(v[5]) << 16);
        o.w = (uint32_t)f2bf_bits(v[6]) | ((uint32_t)f2bf_bits(v[7]) << 16);
        *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(p.out) + ob + ec0) = o;
      } else {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int64_t o = ob + (int64_t)(ec0 + u) * p.o_sn;
          if (p.out_bf16) reinterpret_cast<uint16_t*>(p.out)[o] = f2bf_bits(v[u]);
          else reinterpret_cast<float*>(p.out)[o] = v[u];
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------
// Row-band variant (the production path when the whole time axis fits in LDS).
//
// The tile above (one output row x 128 frames) reads every input row three times
// (once per kernel row) and pads W = 598 frames to 640.  Here a persistent
// 512-thread workgroup owns bands of R output rows x one time tile (the fewest tiles
// of <= 19 16-frame blocks covering W: 2 x 304 for W = 598): the
// NR = (R-1)*sh + 3 input rows of a band (+1 halo frame each side) are staged in LDS
// once (input read (R+2)/R times instead of 3), the next band's rows are loaded into
// registers (16-B buffer loads, zeros out of range) while the current band computes,
// and the MFMA runs transposed (weights as the A operand) so each lane ends with 4
// consecutive channels of one frame: 8-B bf16 stores / residual loads straight from
// the accumulators, no LDS epilogue.
constexpr int kBandThreads = 512;
constexpr int kBandVecPer = 15;     // 16-B vectors per thread per band (NR * (W+2) * 4 <= 7680)
constexpr uint32_t kFcmOOB = 0x80000000u;

// Output channel held by accumulator row i of MFMA tile nt.  Rows are permuted so that
// lane group q (rows 4q..4q+3 of both tiles) owns the 8 contiguous channels 8q..8q+7:
// one 16-B bf16 store per lane writes a whole 64-B frame row with its 3 neighbours.
__host__ __device__ inline int band_channel(int i, int nt) { return 8 * (i >> 2) + 4 * nt + (i & 3); }

// Fused variants (FcmFuse, campp.cpp FCM head):
//   SC    the block's shortcut (1x1 conv, same freq stride, folded BN) as two more MFMAs on the centre tap's
//         fragment, stored to f.sc_out: the shortcut never re-reads the input map;
//   STEM  the staged input rows are head.conv1 (1 -> 32, 3x3, pad 1) + BN + ReLU computed in LDS from the
//         fbank rows they need (cam_pplus_wespeaker.py:277-301), so the 80-bin 32-channel stem map (1.84 GB
//         for a 10-min C2 meeting) is never written.  Same fmaf order as fcm_conv1_kernel (bit-identical).
// TOUT: FCM head.conv2, whose output is the TDNN input (B, T, 32 * Ho) with channel c * Ho + h: a band is
// ALL Ho = R output rows of kToutBlk 16-frame blocks, so its output is one contiguous run of whole
// 640-B frame rows.  The epilogue scatters into an LDS image of those rows and the band leaves as 16-B
// stores (per-element stores of R-row bands left every frame row to be assembled from 2-B pieces by
// five different bands).
// SMF: the band barriers are LDS-only (`lgkmcnt(0)` + `s_barrier`): a __syncthreads() fence also waits for the
// next band's prefetch and this band's output stores; with STEM also the MFMA stem (see the stem block below).
constexpr int kToutBlk = 4;
constexpr int kToutRow = 328;   // LDS frame-row stride in bf16 (656 B: 16-B aligned, rows 36 banks apart)

template <int R, int SH, bool STEM = false, bool SC = false, bool TOUT = false, bool SMF = false>
__global__ __launch_bounds__(kBandThreads) void fcm_conv3x3_band_kernel(ConvGemmArgs p, FcmFuse f, int n_bands,
                                                                       int n_blk) {
  // A band: (image b, R output rows from ho0, time tile tt of n_blk 16-frame blocks).
  static_assert(!STEM || SMF, "the stem runs on the MFMA with LDS-only band barriers (the fp32 VALU stem: round 5)");
  constexpr int NR = (R - 1) * SH + 3;
  // staged 16-B vectors per thread: NR rows x (at most 19 x 16 + 2 = 306 frames) x 4 (band_fits checks it)
  constexpr int kVP = (NR * (TOUT ? kToutBlk * 16 + 2 : 306) * 4 + kBandThreads - 1) / kBandThreads;
  extern __shared__ __attribute__((aligned(16))) uint16_t xs[];   // [NR][TW+2][kPS] (+ STEM: fbank tile)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int l15 = lane & 15, q = lane >> 4;
  const int W = p.W, Wp = n_blk * 16 + 2;
  const int n_rb = (p.Ho + R - 1) / R;
  const int n_tt = (W + n_blk * 16 - 1) / (n_blk * 16);
  const int n_vec = NR * Wp * 4;

  bf16x8 wf[9][2];
  // STEM: the conv weights are re-read per band (L1/L2 hits) behind a laundered pointer so that they and the
  // stem's 72 weights are not live at the same time (register pressure)
  auto load_wf = [&](const uint16_t* Wt) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        wf[t][nt] = *reinterpret_cast<const bf16x8*>(Wt + band_channel(l15, nt) * 288 + t * 32 + q * 8);
  };
  if constexpr (!STEM || SMF) load_wf(reinterpret_cast<const uint16_t*>(p.Wt));
  bf16x8 wsc[2];
  float sal[2][4], sbe[2][4];
  if constexpr (SC) {
    const uint16_t* Ws = reinterpret_cast<const uint16_t*>(f.sc_w);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      wsc[nt] = *reinterpret_cast<const bf16x8*>(Ws + band_channel(l15, nt) * 32 + q * 8);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = band_channel(4 * q + r, nt);
        sal[nt][r] = f.sc_alpha[c];
        sbe[nt][r] = f.sc_beta[c];
      }
    }
  }
  // Per lane: accumulator (nt, r) is channel 8q + 4nt + r, i.e. channels 8q .. 8q+7.
  float al[2][4], be[2][4];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = band_channel(4 * q + r, nt);
      al[nt][r] = p.alpha ? p.alpha[c] : 1.f;
      be[nt][r] = p.beta ? p.beta[c] : 0.f;
    }
  const bool nhwc = p.o_sn == 1 && p.o_sw == 32 && p.o_sh == (int64_t)p.Wo * 32;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.A), (short)0,
                                                                      (int)kFcmOOB, 0x00020000);

  // Vector i = tid + k*512 of a band: staged pixel i >> 2 (row rr, frame px), channel
  // group i & 3.  (i >> 2) advances by 128 per k and Wp > 128, so px wraps at most once.
  const int px_base = (tid >> 2) % Wp, rr_base = (tid >> 2) / Wp;
  auto load_band = [&](int band, uint4* v) {
    const int tt = band % n_tt, bh = band / n_tt;
    const int b = bh / n_rb, hb = (bh % n_rb) * R * SH - 1;   // first staged input row
    const int w0 = tt * n_blk * 16 - 1;                      // first staged input frame
    const int64_t img = (int64_t)b * p.H * W;
    int px = px_base, rr = rr_base;
#pragma unroll
    for (int k = 0; k < kVP; ++k) {
      const int i = tid + k * kBandThreads;
      const int ch = (i & 3) * 8;
      const int hi = hb + rr, wi = w0 + px;
      const bool ok = i < n_vec && (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)W;
      const uint32_t off = ok ? (uint32_t)(((img + (int64_t)hi * W + wi) * p.lda + p.a_coff + ch) * 2) : kFcmOOB;
      const u32x4_t x = __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0);
      v[k] = make_uint4(x.x, x.y, x.z, x.w);
      px += 128;
      if constexpr (TOUT) {   // Wp < 128: the frame index can wrap twice
        while (px >= Wp) {
          px -= Wp;
          ++rr;
        }
      } else if (px >= Wp) {
        px -= Wp;
        ++rr;
      }
    }
  };

  // STEM: fbank tile [NR + 2 bins][Wp + 2 frames] (fp32) after the staged rows; this thread's 8 stem
  // channels (channel group tid & 3, fixed because 512 % 4 == 0) keep their 72 weights in registers.
  float* fbs = reinterpret_cast<float*>(xs + NR * Wp * kPS);
  const int fb_n = (NR + 2) * (Wp + 2);
  constexpr int kFbPer = 5;   // fbank tile floats per thread (<= 2560)
  // MFMA stem: v_mfma_f32_32x32x16_bf16 with the 32 channels as rows and 32 staged pixels as
  // columns; k = the 9 taps (dh, dw) in order, then beta's bf16 hi and lo parts against a constant 1 (BN
  // folded: A = bf16(alpha_c * w_c), so a pixel is relu(sum + beta) with no epilogue FMAs).  A row m is
  // channel 16 ((m >> 2) & 1) + 4 (m >> 3) + (m & 3), so accumulator i of lane half h is channel 16 h + i
  // and a lane stores its pixel's 16 contiguous channels as two 16-B LDS writes.
  bf16x8 stem_a;
  if constexpr (STEM) {
    {
      const int m = lane & 31, h = lane >> 5;
      const int c = 16 * ((m >> 2) & 1) + 4 * (m >> 3) + (m & 3);
      const float al = f.stem_alpha[c], be = f.stem_beta[c];
      float e[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) e[j] = al * f.stem_w[c * 9 + min(8 * h + j, 8)];
      const float bh = __uint_as_float(f2bf_bits(be) << 16);
      if (h) {
        e[1] = bh;
        e[2] = __uint_as_float(f2bf_bits(be - bh) << 16);
#pragma unroll
        for (int j = 3; j < 8; ++j) e[j] = 0.f;
      }
      const uint32_t w4[4] = {pack_bf16x2(e[0], e[1]), pack_bf16x2(e[2], e[3]), pack_bf16x2(e[4], e[5]),
                              pack_bf16x2(e[6], e[7])};
      stem_a = *reinterpret_cast<const bf16x8*>(w4);
    }
  }
  // fbank value (bin hb - 1 + j, frame w0 - 1 + x) of a band, j < NR + 2, x < Wp + 2; zero outside the map
  auto load_fb = [&](int band, float* v) {
    const int tt = band % n_tt, bh = band / n_tt;
    const int b = bh / n_rb, hb = (bh % n_rb) * R * SH - 1;
    const int w0 = tt * n_blk * 16 - 1;
#pragma unroll
    for (int k = 0; k < kFbPer; ++k) {
      const int i = tid + k * kBandThreads;   // frame-major: a frame's NR + 2 bins are contiguous in the fbank
      const int x = i / (NR + 2), j = i - x * (NR + 2);
      const int bin = hb - 1 + j, fr = w0 - 1 + x;
      v[k] = (i < fb_n && (unsigned)bin < (unsigned)f.fb_F && (unsigned)fr < (unsigned)W)
                 ? f.fbank[((int64_t)b * W + fr) * f.fb_F + bin]
                 : 0.f;
    }
  };

  uint4 hv[STEM ? 1 : kVP];
  float fv[STEM ? kFbPer : 1];
  int band = blockIdx.x;
  if (band < n_bands) {
    if constexpr (STEM) load_fb(band, fv);
    else load_band(band, hv);
  }
  for (; band < n_bands; band += gridDim.x) {
    if constexpr (STEM) {
#pragma unroll
      for (int k = 0; k < kFbPer; ++k) {
        const int i = tid + k * kBandThreads;
        const int x = i / (NR + 2), j = i - x * (NR + 2);
        if (i < fb_n) fbs[j * (Wp + 2) + x] = fv[k];   // LDS tile [bin][frame]
      }
      if constexpr (SMF) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else __syncthreads();
      const int next = band + gridDim.x;
      if (next < n_bands) load_fb(next, fv);
      // stem: staged pixel (rr, px) = conv1 row hb + rr, frame w0 + px; zero outside (next conv's padding)
      const int tt = band % n_tt, bh = band / n_tt;
      const int hb = (bh % n_rb) * R * SH - 1, w0 = tt * n_blk * 16 - 1;
      {
        const int n = lane & 31, h = lane >> 5;
        const int ngr = (Wp + 31) >> 5;   // 32-pixel groups per staged row (reads past Wp hit the tile's pad)
        for (int g = wv; g < NR * ngr; g += kBandThreads / 64) {
          const int rr = g / ngr, px = (g - rr * ngr) * 32 + n;
          const float* t0 = fbs + rr * (Wp + 2) + px;
          float tp[9];
#pragma unroll
          for (int k = 0; k < 9; ++k) tp[k] = t0[(k / 3) * (Wp + 2) + k % 3];
          float e[8];
          e[0] = h ? tp[8] : tp[0];
          e[1] = h ? 1.f : tp[1];
          e[2] = h ? 1.f : tp[2];
#pragma unroll
          for (int j = 3; j < 8; ++j) e[j] = h ? 0.f : tp[j];
          const uint32_t b4[4] = {pack_bf16x2(e[0], e[1]), pack_bf16x2(e[2], e[3]), pack_bf16x2(e[4], e[5]),
                                  pack_bf16x2(e[6], e[7])};
          typedef float floatx16 __attribute__((ext_vector_type(16)));
          floatx16 acc = {};
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(stem_a, *reinterpret_cast<const bf16x8*>(b4), acc, 0, 0, 0);
          if (px < Wp) {
            const bool ok = (unsigned)(hb + rr) < (unsigned)p.H && (unsigned)(w0 + px) < (unsigned)W;
            uint32_t o[8];
#pragma unroll
            for (int u = 0; u < 8; ++u)
              o[u] = ok ? pack_bf16x2(fmaxf(acc[2 * u], 0.f), fmaxf(acc[2 * u + 1], 0.f)) : 0u;
            uint16_t* dst = xs + (rr * Wp + px) * kPS + 16 * h;
            *reinterpret_cast<uint4*>(dst) = make_uint4(o[0], o[1], o[2], o[3]);
            *reinterpret_cast<uint4*>(dst + 8) = make_uint4(o[4], o[5], o[6], o[7]);
          }
        }
      }
      // SMF: LDS-only barriers (a __syncthreads() fence would also drain the next band's fbank prefetch
      // and this band's output stores)
      if constexpr (SMF) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else __syncthreads();
    } else {
#pragma unroll
      for (int k = 0; k < kVP; ++k) {
        const int i = tid + k * kBandThreads;
        if (i < n_vec) *reinterpret_cast<uint4*>(xs + (i >> 2) * kPS + (i & 3) * 8) = hv[k];
      }
      if constexpr (SMF) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else __syncthreads();
      const int next = band + gridDim.x;
      if (next < n_bands) load_band(next, hv);   // in flight while this band computes
    }

    const int tt = band % n_tt, bh = band / n_tt;
    const int b = bh / n_rb, ho0 = (bh % n_rb) * R;
    const int wo0 = tt * n_blk * 16;
    // Work items: (output row r, 16-frame block) round-robin over the 8 waves.
    for (int it = wv; it < R * n_blk; it += kBandThreads / 64) {
      const int r = it / n_blk, blk = it - r * n_blk;
      const int ho = ho0 + r;
      if (ho >= p.Ho) break;
      floatx4 acc[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
      floatx4 sacc[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int dh = 0; dh < 3; ++dh)
#pragma unroll
        for (int dw = 0; dw < 3; ++dw) {
          const int px = blk * 16 + l15 + dw;   // staged frame of output frame blk*16 + l15
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(xs + ((r * SH + dh) * Wp + px) * kPS + q * 8);
#pragma unroll
          for (int nt = 0; nt < 2; ++nt)
            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[dh * 3 + dw][nt], af, acc[nt], 0, 0, 0);
          if constexpr (SC) {
            if (dh == 1 && dw == 1)   // input row SH * ho, frame wo: the 1x1 shortcut's operand
#pragma unroll
              for (int nt = 0; nt < 2; ++nt)
                sacc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wsc[nt], af, sacc[nt], 0, 0, 0);
          }
        }
      const int wo = wo0 + blk * 16 + l15;
      if (wo >= p.Wo) continue;
      const int64_t pix = ((int64_t)b * p.Ho + ho) * p.Wo + wo;
      const int c0 = q * 8;
      if constexpr (SC) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = fmaf(sacc[u >> 2][u & 3], sal[u >> 2][u & 3], sbe[u >> 2][u & 3]);
        *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(f.sc_out) + pix * 32 + c0) =
            make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                       pack_bf16x2(v[6], v[7]));
      }
      float rv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (p.res) {
        const int64_t ro = pix * p.res_ld + c0;
        if (p.res_bf16) {
          const uint4 r4 = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(p.res) + ro);
          const uint32_t rw[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            rv[2 * u] = __uint_as_float(rw[u] << 16);
            rv[2 * u + 1] = __uint_as_float(rw[u] & 0xffff0000u);
          }
        } else {
          const float4 a4 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p.res) + ro);
          const float4 b4 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p.res) + ro + 4);
          rv[0] = a4.x; rv[1] = a4.y; rv[2] = a4.z; rv[3] = a4.w;
          rv[4] = b4.x; rv[5] = b4.y; rv[6] = b4.z; rv[7] = b4.w;
        }
      }
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = apply_act(fmaf(acc[u >> 2][u & 3], al[u >> 2][u & 3], be[u >> 2][u & 3]) + rv[u], p.act);
      if constexpr (TOUT) {   // output row r of frame wo -> its LDS frame row, channel c at c * R + r
        uint16_t* so = xs + NR * Wp * kPS + (blk * 16 + l15) * kToutRow + r;
#pragma unroll
        for (int u = 0; u < 8; ++u) so[(c0 + u) * R] = f2bf_bits(v[u]);
      } else if (nhwc && p.out_bf16) {
        *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(p.out) + pix * 32 + c0) =
            make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]),
                       pack_bf16x2(v[6], v[7]));
      } else {
        const int64_t ob = (int64_t)b * p.o_sb + (int64_t)ho * p.o_sh + (int64_t)wo * p.o_sw;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int64_t o = ob + (int64_t)(c0 + u) * p.o_sn;
          if (p.out_bf16) reinterpret_cast<uint16_t*>(p.out)[o] = f2bf_bits(v[u]);
          else reinterpret_cast<float*>(p.out)[o] = v[u];
        }
      }
    }
    if constexpr (TOUT) {   // the band's frame rows are contiguous in the output: 16-B copies
      if constexpr (SMF) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else __syncthreads();
      const int nfr = min(n_blk * 16, p.Wo - wo0), cpr = R * 4;
      uint16_t* ob = reinterpret_cast<uint16_t*>(p.out) + ((int64_t)b * p.Wo + wo0) * 32 * R;
      const uint16_t* so = xs + NR * Wp * kPS;
      for (int i = tid; i < nfr * cpr; i += kBandThreads) {
        const int fr = i / cpr, ck = i - fr * cpr;
        *reinterpret_cast<uint4*>(ob + (int64_t)fr * 32 * R + ck * 8) =
            *reinterpret_cast<const uint4*>(so + fr * kToutRow + ck * 8);
      }
    }
    if constexpr (SMF) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // xs free
    else __syncthreads();   // xs free for the next band
  }
}

int g_fcm_cu = 0;

// ---------------------------------------------------------------------------------
// Ring variant of the stride-1 band conv (the production path for FCM's stride-1 3x3 convs, bf16 NHWC
// in and out).  The band kernel above keeps ONE band's rows in flight (register prefetch, drained by the
// band-end barrier), so every band paid an HBM latency that its 2-3 us of MFMA work did not cover, and
// the residual load of each output tile waited behind the next band's prefetch (in-order vmcnt).  Here
// bands are small (4 output rows x 64 frames) and arrive by LDS-DMA through a 3-slot ring, two bands
// ahead of the one being computed; the band's residual tile rides in the same slot, so the epilogue
// reads it from LDS.  Conv zero padding, the frames past W and the unused DMA lanes are out-of-range
// buffer offsets (the DMA writes zeros, no memory traffic).  The 16-B chunks of a pixel are rotated by
// (frame >> 2) in LDS so the 16 frames of an MFMA B fragment hit 16 distinct bank slots.  Same MFMA
// and epilogue arithmetic, in the same order, as the band kernel: bit-identical outputs.
constexpr int kRR = 4;                                   // output rows per band
constexpr int kRB = 4;                                   // 16-frame blocks per band
constexpr int kRPx = kRB * 16 + 2;                       // staged frames per input row
constexpr int kRInChunks = (kRR + 2) * kRPx * 4;         // 16-B chunks of staged input (1584)
constexpr int kRInInstr = (kRInChunks + 63) / 64;        // DMA instructions for them (25)
constexpr int kRResChunks = kRR * kRB * 16 * 4;          // residual tile chunks (1024)
constexpr int kRResBase = kRInInstr * 64;                // slot position of the residual tile
template <bool RES>
constexpr int ring_dma_per_wave() { return (kRInInstr + (RES ? kRResChunks / 64 : 0) + 7) / 8; }
constexpr int kRNSlot = 3;
template <bool RES>
constexpr int ring_slot_bytes() { return ring_dma_per_wave<RES>() * 8 * 64 * 16; }

__device__ __forceinline__ int ring_pos(int row, int px, int q, int row_px) {
  return (row * row_px + px) * 4 + ((q + (px >> 2)) & 3);
}

template <bool RES, bool RELU>
__global__ __launch_bounds__(kBandThreads) void fcm_conv3x3_ring_kernel(ConvGemmArgs p, int n_bands, int n_tt) {
  constexpr int kDma = ring_dma_per_wave<RES>();
  constexpr int kSlot = ring_slot_bytes<RES>();
  extern __shared__ __attribute__((aligned(1024))) uint16_t xs[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l15 = lane & 15, q = lane >> 4;
  const int H = p.H, W = p.W;
  const int n_rb = (p.Ho + kRR - 1) / kRR;
  bf16x8 wf[9][2];
  {
    const uint16_t* Wt = reinterpret_cast<const uint16_t*>(p.Wt);
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        wf[t][nt] = *reinterpret_cast<const bf16x8*>(Wt + band_channel(l15, nt) * 288 + t * 32 + q * 8);
  }
  float al[2][4], be[2][4];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = band_channel(4 * q + r, nt);
      al[nt][r] = p.alpha ? p.alpha[c] : 1.f;
      be[nt][r] = p.beta ? p.beta[c] : 0.f;
    }
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.A), (short)0,
                                                                      (int)kFcmOOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(RES ? p.res : p.A), (short)0,
                                                                      (int)kFcmOOB, 0x00020000);
  // this lane's chunk of each of the wave's DMAs: DMA k writes slot positions (k * 8 + wv) * 64 + lane
  int d_row[kDma], d_px[kDma], d_q[kDma];
#pragma unroll
  for (int k = 0; k < kDma; ++k) {
    const int gi = k * 8 + wv;
    int pos = gi * 64 + lane, row_px = kRPx;
    if (gi >= kRInInstr) pos -= kRResBase, row_px = kRB * 16;
    const int row = pos / (row_px * 4), rem = pos - row * row_px * 4, px = rem >> 2;
    d_row[k] = row;
    d_px[k] = px;
    d_q[k] = ((rem & 3) - (px >> 2)) & 3;
  }
  // XCD-aware band order: the workgroups of one XCD (blockIdx % 8) take consecutive bands, so a band and
  // its row neighbours (which re-read two of its input rows) are served by the same L2
  const int G = gridDim.x;
  const int vb = (G % 8 == 0) ? (blockIdx.x % 8) * (G / 8) + blockIdx.x / 8 : blockIdx.x;
  auto issue = [&](int band, int slot) {
    const int tt = band % n_tt, bh = band / n_tt;
    const int b = bh / n_rb, ho0 = (bh % n_rb) * kRR, w0 = tt * kRB * 16;
#pragma unroll
    for (int k = 0; k < kDma; ++k) {
      const int gi = k * 8 + wv;
      const auto* lds = (const __attribute__((address_space(3))) void*)(xs + (slot * kSlot + gi * 1024) / 2);
      if (gi < kRInInstr) {
        const int h = ho0 - 1 + d_row[k], w = w0 - 1 + d_px[k];
        const bool ok = gi * 64 + lane < kRInChunks && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
        const uint32_t off =
            ok ? (uint32_t)(((((int64_t)b * H + h) * W + w) * p.lda + p.a_coff + d_q[k] * 8) * 2) : kFcmOOB;
        dma_lds16_buf(ra, off, lds);
      } else {
        const int ho = ho0 + d_row[k], wo = w0 + d_px[k];
        const bool ok = RES && gi * 64 + lane - kRResBase < kRResChunks && ho < p.Ho && wo < p.Wo;
        const uint32_t off =
            ok ? (uint32_t)(((((int64_t)b * p.Ho + ho) * p.Wo + wo) * p.res_ld + d_q[k] * 8) * 2) : kFcmOOB;
        dma_lds16_buf(rr, off, lds);
      }
    }
  };
  auto barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  const int nb_mine = n_bands > vb ? (n_bands - vb + G - 1) / G : 0;   // bands of this workgroup
  if (nb_mine > 0) issue(vb, 0);
  if (nb_mine > 1) issue(vb + G, 1);
  for (int i = 0; i < nb_mine; ++i) {
    // band i landed: only band i + 1's DMAs (and this wave's stores) are younger; outstanding <= kDma
    // then implies all of band i's DMAs are done (loads complete in order)
    if (i + 1 < nb_mine) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kDma) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();   // every wave's part of band i is in LDS; every wave is done with band i - 1's slot
    if (i + 2 < nb_mine) issue(vb + (i + 2) * G, (i + 2) % kRNSlot);
    const int band = vb + i * G;
    const int tt = band % n_tt, bh = band / n_tt;
    const int b = bh / n_rb, ho0 = (bh % n_rb) * kRR, w0 = tt * kRB * 16;
    const uint16_t* sx = xs + (i % kRNSlot) * (kSlot / 2);
#pragma unroll
    for (int j = 0; j < kRR * kRB / 8; ++j) {
      const int it = wv + 8 * j, r = it / kRB, blk = it % kRB;
      const int ho = ho0 + r;
      if (ho >= p.Ho) break;
      floatx4 acc[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int dh = 0; dh < 3; ++dh)
#pragma unroll
        for (int dw = 0; dw < 3; ++dw) {
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(sx + ring_pos(r + dh, blk * 16 + l15 + dw, q, kRPx) * 8);
#pragma unroll
          for (int nt = 0; nt < 2; ++nt)
            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[dh * 3 + dw][nt], af, acc[nt], 0, 0, 0);
        }
      const int wo = w0 + blk * 16 + l15;
      float rv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if constexpr (RES) {
        const u32x4_t r4 = *reinterpret_cast<const u32x4_t*>(sx + (kRResBase + ring_pos(r, blk * 16 + l15, q, kRB * 16)) * 8);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          rv[2 * u] = __uint_as_float(r4[u] << 16);
          rv[2 * u + 1] = __uint_as_float(r4[u] & 0xffff0000u);
        }
      }
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        v[u] = fmaf(acc[u >> 2][u & 3], al[u >> 2][u & 3], be[u >> 2][u & 3]) + rv[u];
        if (RELU) v[u] = fmaxf(v[u], 0.f);   // apply_act(., kActRelu)
      }
      if (wo < p.Wo)
        *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(p.out) + (((int64_t)b * p.Ho + ho) * p.Wo + wo) * 32 +
                                  q * 8) = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                                                      pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
    }
  }
}

bool ring_ok(const ConvGemmArgs& p) {
  const int64_t in_bytes = (int64_t)p.B * p.H * p.W * p.lda * 2;
  const int64_t res_bytes = p.res ? (int64_t)p.B * p.Ho * p.Wo * p.res_ld * 2 : 0;
  return p.sh == 1 && (p.act == kActRelu || p.act == kActNone) && p.out_bf16 && p.o_sn == 1 && p.o_sw == 32 && p.o_sh == (int64_t)p.Wo * 32 &&
         p.o_sb == (int64_t)p.Ho * p.o_sh && (!p.res || (p.res_bf16 && p.res_ld % 8 == 0)) &&
         in_bytes < (int64_t)kFcmOOB && res_bytes < (int64_t)kFcmOOB;
}

template <bool RES, bool RELU>
void launch_ring(const ConvGemmArgs& p, hipStream_t st) {
  const int n_tt = cdiv(p.Wo, kRB * 16);
  const int64_t bands = (int64_t)p.B * cdiv(p.Ho, kRR) * n_tt;
  SD_CHECK(bands < (1ll << 31), kErrInvalid, "fcm conv: too many bands");
  constexpr size_t smem = (size_t)kRNSlot * ring_slot_bytes<RES>();
  static_assert(smem <= 160 * 1024, "LDS budget");
  static bool attr = false;
  if (!attr) {
    SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(fcm_conv3x3_ring_kernel<RES, RELU>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
    attr = true;
  }
  const int grid = (int)std::min<int64_t>(bands, (int64_t)g_fcm_cu);
  hipLaunchKernelGGL((fcm_conv3x3_ring_kernel<RES, RELU>), dim3(grid), dim3(kBandThreads), smem, st, p, (int)bands, n_tt);
}

// Time tiling: the fewest tiles whose 16-frame blocks (at most kBandMaxBlk, so a
// staged row stays <= 306 frames) cover W, blocks spread evenly over them.
constexpr int kBandMaxBlk = 19;
inline int band_blocks(int W) {
  const int nb = (W + 15) / 16;
  const int n_tt = (nb + kBandMaxBlk - 1) / kBandMaxBlk;
  return (nb + n_tt - 1) / n_tt;
}

template <int R, int SH, bool STEM = false>
size_t band_lds(int n_blk) {
  constexpr int nr = (R - 1) * SH + 3;
  // STEM: fbank tile + 32 floats of pad (the MFMA stem's last 32-pixel group reads up to 31 past the tile)
  const size_t fb = STEM ? (size_t)(nr + 2) * (n_blk * 16 + 4) * 4 + 128 : 0;
  return (size_t)nr * (n_blk * 16 + 2) * kPS * 2 + fb;
}

template <int R, int SH, bool STEM = false>
bool band_fits(const ConvGemmArgs& p) {
  const int nr = (R - 1) * SH + 3;
  const int nb = band_blocks(p.W);
  // (n_blk*16 + 2) > 128 keeps the loader's frame index wrapping at most once per step.
  return nb >= 8 && nb <= kBandMaxBlk && band_lds<R, SH, STEM>(nb) <= 156 * 1024 &&
         nr * (nb * 16 + 2) * 4 <= kBandVecPer * kBandThreads &&
         (!STEM || (nr + 2) * (nb * 16 + 4) <= 5 * kBandThreads) &&
         (int64_t)p.B * p.H * p.W * p.lda * 2 < (int64_t)kFcmOOB &&
         (!p.res || (p.res_ld % 8 == 0)) && (p.o_sn != 1 || p.o_sw % 8 == 0);
}

template <int R, int SH, bool STEM = false, bool SC = false, bool SMF = false>
void launch_band(const ConvGemmArgs& p, hipStream_t st, const FcmFuse& f = FcmFuse{}) {
  const int nb = band_blocks(p.W);
  const int64_t bands = (int64_t)p.B * cdiv(p.Ho, R) * cdiv(p.W, nb * 16);
  SD_CHECK(bands < (1ll << 31), kErrInvalid, "fcm conv: too many bands");
  static bool attr = false;
  if (!attr) {
    SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(fcm_conv3x3_band_kernel<R, SH, STEM, SC, false, SMF>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const int grid = (int)std::min<int64_t>(bands, (int64_t)g_fcm_cu);
  const size_t smem = band_lds<R, SH, STEM>(nb);
  hipLaunchKernelGGL((fcm_conv3x3_band_kernel<R, SH, STEM, SC, false, SMF>), dim3(grid), dim3(kBandThreads), smem, st, p, f,
                     (int)bands, nb);
}

}  // namespace

// FCM head.conv2 (stride 2 to Ho = 10 rows) into the TDNN's (B, T, 32 * Ho) layout: see TOUT above
bool tout_ok(const ConvGemmArgs& p) {
  return p.sh == 2 && p.Ho == 10 && p.out_bf16 && !p.res && p.o_sn == p.Ho && p.o_sh == 1 &&
         p.o_sw == 32 * p.Ho && p.o_sb == (int64_t)p.Wo * 32 * p.Ho &&
         (int64_t)p.B * p.H * p.W * p.lda * 2 < (int64_t)kFcmOOB;
}

void launch_tout(const ConvGemmArgs& p, hipStream_t st) {
  constexpr int R = 10, NR = (R - 1) * 2 + 3;
  const int n_tt = cdiv(p.Wo, kToutBlk * 16);
  const int64_t bands = (int64_t)p.B * n_tt;
  SD_CHECK(bands < (1ll << 31), kErrInvalid, "fcm conv: too many bands");
  const size_t smem = (size_t)NR * (kToutBlk * 16 + 2) * kPS * 2 + (size_t)kToutBlk * 16 * kToutRow * 2;
  static_assert((size_t)NR * (kToutBlk * 16 + 2) * kPS * 2 + (size_t)kToutBlk * 16 * kToutRow * 2 <= 160 * 1024,
                "LDS budget");
  static bool attr = false;
  if (!attr) {
    SD_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(fcm_conv3x3_band_kernel<R, 2, false, false, true, true>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem));
    attr = true;
  }
  const int grid = (int)std::min<int64_t>(bands, (int64_t)g_fcm_cu);
  hipLaunchKernelGGL((fcm_conv3x3_band_kernel<R, 2, false, false, true, true>), dim3(grid), dim3(kBandThreads), smem, st,
                     p, FcmFuse{}, (int)bands, kToutBlk);
}

bool fcm_conv_supported(const ConvGemmArgs& p) {
  return p.a_bf16 && !p.pre_scale && !p.gate && p.kh == 3 && p.kw == 3 && p.Cin == 32 && p.N == 32 &&
         p.K == 288 && p.ph == 1 && p.pw == 1 && p.sw == 1 && (p.sh == 1 || p.sh == 2) && p.dh == 1 &&
         p.dw == 1 && p.lda % 8 == 0 && p.a_coff % 8 == 0 && (!p.res || p.res_ld % 8 == 0) &&
         p.Ho == (p.H + 2 - 3) / p.sh + 1 && p.Wo == p.W;
}

void conv_fcm3x3(const ConvGemmArgs& p, hipStream_t st) {
  if (!g_fcm_cu) {
    int dev = 0;
    SD_HIP(hipGetDevice(&dev));
    SD_HIP(hipDeviceGetAttribute(&g_fcm_cu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  if (ring_ok(p)) {
    const bool relu = p.act == kActRelu;
    if (p.res) relu ? launch_ring<true, true>(p, st) : launch_ring<true, false>(p, st);
    else relu ? launch_ring<false, true>(p, st) : launch_ring<false, false>(p, st);
    SD_LAUNCH_CHECK();
    return;
  }
  if (p.sh == 1 && band_fits<4, 1>(p)) {
    launch_band<4, 1>(p, st);
    SD_LAUNCH_CHECK();
    return;
  }
  if (tout_ok(p)) {
    launch_tout(p, st);
    SD_LAUNCH_CHECK();
    return;
  }
  if (p.sh == 2 && band_fits<2, 2>(p)) {
    launch_band<2, 2>(p, st);
    SD_LAUNCH_CHECK();
    return;
  }
  const int n_wt = cdiv(p.Wo, kPx);
  const int64_t tiles = (int64_t)p.B * p.Ho * n_wt;
  SD_CHECK(tiles < (1ll << 31), kErrInvalid, "fcm conv: too many tiles");
  const int grid = (int)std::min<int64_t>(tiles, (int64_t)g_fcm_cu * 4);
  hipLaunchKernelGGL(fcm_conv3x3_kernel, dim3(grid), dim3(256), 0, st, p, (int)tiles);
  SD_LAUNCH_CHECK();
}

bool fcm_fused_supported(const ConvGemmArgs& p, const FcmFuse& f) {
  if (p.sh != 2 || !p.out_bf16 || p.res || p.o_sn != 1 || p.o_sw != 32) return false;
  if (f.sc_w && !(f.sc_alpha && f.sc_beta && f.sc_out)) return false;
  if (f.fbank) {
    if (!(f.stem_w && f.stem_alpha && f.stem_beta && f.fb_F == p.H)) return false;
    ConvGemmArgs q = p;
    q.a_bf16 = true;
    q.lda = 32;
    return fcm_conv_supported(q) && band_fits<2, 2, true>(q);
  }
  return fcm_conv_supported(p) && band_fits<2, 2>(p);
}

void conv_fcm3x3_fused(const ConvGemmArgs& p, const FcmFuse& f, hipStream_t st) {
  SD_CHECK(fcm_fused_supported(p, f), kErrInvalid, "fcm fused conv: unsupported arguments");
  if (!g_fcm_cu) {
    int dev = 0;
    SD_HIP(hipGetDevice(&dev));
    SD_HIP(hipDeviceGetAttribute(&g_fcm_cu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const double px = (double)p.B * p.Ho * p.Wo;
  const double in_px = f.fbank ? 0.0 : (double)p.B * p.H * p.W;
  double flops = 2.0 * px * 32 * 288 + (f.sc_w ? 2.0 * px * 32 * 32 : 0.0);
  if (f.fbank) flops += 2.0 * (double)p.B * p.H * p.W * 32 * 9;
  const double bytes = in_px * 64 + (f.fbank ? 4.0 * p.B * p.W * f.fb_F : 0.0) + px * 64 * (f.sc_w ? 2 : 1);
  ProfScope prof(f.fbank ? "fcm_stem" : "fcm_conv3x3_band", flops, bytes, st);
  if (f.fbank && f.sc_w) launch_band<2, 2, true, true, true>(p, st, f);
  else if (f.fbank) launch_band<2, 2, true, false, true>(p, st, f);
  else if (f.sc_w) launch_band<2, 2, false, true, true>(p, st, f);
  else launch_band<2, 2>(p, st);
  SD_LAUNCH_CHECK();
}

}  // namespace sd
