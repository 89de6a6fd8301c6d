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

int g_fcm_cu = 0;

}  // namespace

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
  const int n_wt = cdiv(p.Wo, kPx);
  const int64_t tiles = (int64_t)p.B * p.Ho * n_wt;
  SD_CHECK(tiles < (1ll << 31), kErrInvalid, "fcm conv: too many tiles");
  const int grid = (int)std::min<int64_t>(tiles, (int64_t)g_fcm_cu * 4);
  hipLaunchKernelGGL(fcm_conv3x3_kernel, dim3(grid), dim3(256), 0, st, p, (int)tiles);
  SD_LAUNCH_CHECK();
}

}  // namespace sd
