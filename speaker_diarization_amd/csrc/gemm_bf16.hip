// bf16 implicit-GEMM conv / linear on gfx950 (v_mfma_f32_16x16x32_bf16, fp32 accumulate).
//
// Same contract as conv_gemm (kernels.h ConvGemmArgs); this is the production
// path of precision=bf16.  Differences from the exact-f32 kernel:
//  * BK = 64, register-staged double buffer, one barrier per k-tile;
//  * every thread owns one 8-element k-chunk; its (tap, channel) position is
//    advanced incrementally, so the k-loop has no integer division;
//  * activations may be bf16 (16-B loads) or fp32 (converted while staging);
//    the BN-ReLU prologue is applied in fp32 on the staged chunk;
//  * the epilogue goes through LDS so bias/BN/residual/activation/gate are
//    applied on row-contiguous 4-column groups and stored with 8/16-B stores,
//    as fp32 or bf16.
#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {
namespace {

constexpr int BK = 64;
constexpr int LROW = BK + 8;   // bf16 elements per LDS row: 144 B (16-B aligned)

__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  return (uint32_t)f2bf_bits(a) | ((uint32_t)f2bf_bits(b) << 16);
}

__device__ __forceinline__ void unpack_bf8(const uint4& v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

template <int BM, int BN, bool ABF>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(ConvGemmArgs p) {
  constexpr int TM = BM / 2, TN = BN / 2;
  constexpr int MT = TM / 16, NT = TN / 16;
  constexpr int APT = BM / 32;                 // A chunks per thread
  constexpr int BPT = (BN + 31) / 32;          // B chunks per thread
  constexpr int STAGE = (BM + BN) * LROW;      // uint16 per stage
  constexpr int CLD = BN + 4;                  // fp32 epilogue row stride
  constexpr int EPI = BM * CLD * 2;            // in uint16 units
  constexpr int SMEM = (2 * STAGE > EPI) ? 2 * STAGE : EPI;
  __shared__ __attribute__((aligned(16))) uint16_t sm[SMEM];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int M = p.B * p.Ho * p.Wo;
  const int n_nt = (p.N + BN - 1) / BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (tile / n_nt) * BM;
  const int n0 = (tile % n_nt) * BN;
  const int kc = (tid & 7) * 8;
  const int rsub = tid >> 3;

  int rbh[APT], rh[APT], rw[APT];
#pragma unroll
  for (int i = 0; i < APT; ++i) {
    const int m = m0 + rsub + 32 * i;
    if (m < M) {
      const int wo = m % p.Wo;
      const int t = m / p.Wo;
      const int ho = t % p.Ho;
      rbh[i] = (t / p.Ho) * p.H;
      rh[i] = ho * p.sh - p.ph;
      rw[i] = wo * p.sw - p.pw;
    } else {
      rbh[i] = 0;
      rh[i] = -(1 << 28);
      rw[i] = 0;
    }
  }
  int kpos = kc;
  int tap = kc / p.Cin;
  int c = kc - tap * p.Cin;
  int ti = tap / p.kw;
  int tj = tap - ti * p.kw;

  const uint16_t* __restrict__ Wt = reinterpret_cast<const uint16_t*>(p.Wt);
  uint4 areg[APT], breg[BPT];

  auto load = [&]() {
    const bool kv = kpos < p.K;
    const bool pre = p.pre_scale != nullptr;
    float s[8], h[8];
    if (pre && kv) {
      const float4* ps = reinterpret_cast<const float4*>(p.pre_scale + c);
      const float4* ph = reinterpret_cast<const float4*>(p.pre_shift + c);
      float4 a0 = ps[0], a1 = ps[1], b0 = ph[0], b1 = ph[1];
      s[0] = a0.x; s[1] = a0.y; s[2] = a0.z; s[3] = a0.w; s[4] = a1.x; s[5] = a1.y; s[6] = a1.z; s[7] = a1.w;
      h[0] = b0.x; h[1] = b0.y; h[2] = b0.z; h[3] = b0.w; h[4] = b1.x; h[5] = b1.y; h[6] = b1.z; h[7] = b1.w;
    }
    const int dho = ti * p.dh, dwo = tj * p.dw;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const int hi = rh[i] + dho, wi = rw[i] + dwo;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (kv && (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W) {
        const int64_t off = ((int64_t)(rbh[i] + hi) * p.W + wi) * p.lda + p.a_coff + c;
        float f[8];
        if constexpr (ABF) {
          v = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(p.A) + off);
          if (pre) unpack_bf8(v, f);
        } else {
          const float4* src = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(p.A) + off);
          float4 x0 = src[0], x1 = src[1];
          f[0] = x0.x; f[1] = x0.y; f[2] = x0.z; f[3] = x0.w; f[4] = x1.x; f[5] = x1.y; f[6] = x1.z; f[7] = x1.w;
        }
        if (pre) {
#pragma unroll
          for (int u = 0; u < 8; ++u) f[u] = fmaxf(fmaf(f[u], s[u], h[u]), 0.f);
        }
        if (!ABF || pre)
          v = make_uint4(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]), pack_bf2(f[4], f[5]), pack_bf2(f[6], f[7]));
      }
      areg[i] = v;
    }
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int nr = rsub + 32 * j;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (nr < BN && kv && n0 + nr < p.N)
        v = *reinterpret_cast<const uint4*>(Wt + (int64_t)(n0 + nr) * p.K + kpos);
      breg[j] = v;
    }
  };
  auto advance = [&]() {
    kpos += BK;
    c += BK;
    while (c >= p.Cin) {
      c -= p.Cin;
      if (++tj == p.kw) { tj = 0; ++ti; }
    }
  };
  auto store = [&](int stg) {
    uint16_t* As = sm + stg * STAGE;
    uint16_t* Bs = As + BM * LROW;
#pragma unroll
    for (int i = 0; i < APT; ++i)
      *reinterpret_cast<uint4*>(As + (rsub + 32 * i) * LROW + kc) = areg[i];
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int nr = rsub + 32 * j;
      if (nr < BN) *reinterpret_cast<uint4*>(Bs + nr * LROW + kc) = breg[j];
    }
  };

  floatx4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int KT = (p.K + BK - 1) / BK;
  load();
  store(0);
  __syncthreads();
  const int l15 = lane & 15, lk = lane >> 4;
  for (int kt = 0; kt < KT; ++kt) {
    const int stg = kt & 1;
    if (kt + 1 < KT) {
      advance();
      load();
    }
    const uint16_t* As = sm + stg * STAGE;
    const uint16_t* Bs = As + BM * LROW;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[MT], bfr[NT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        af[mt] = *reinterpret_cast<const bf16x8*>(As + (wm * TM + mt * 16 + l15) * LROW + ks * 32 + lk * 8);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        bfr[nt] = *reinterpret_cast<const bf16x8*>(Bs + (wn * TN + nt * 16 + l15) * LROW + ks * 32 + lk * 8);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bfr[nt], acc[mt][nt], 0, 0, 0);
    }
    if (kt + 1 < KT) store(stg ^ 1);
    __syncthreads();
  }

  // ---- epilogue through LDS: C tile (fp32) -> row-contiguous 4-column groups.
  float* Cs = reinterpret_cast<float*>(sm);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Cs[(wm * TM + mt * 16 + lk * 4 + r) * CLD + wn * TN + nt * 16 + l15] = acc[mt][nt][r];
  __syncthreads();

  const bool lin = out_rows_linear(p);
  const bool vec = lin && p.o_sn == 1 && (p.o_sw & 3) == 0;
  constexpr int CPR = BN / 4;
  for (int q = tid; q < BM * CPR; q += 256) {
    const int row = q / CPR;
    const int cc = (q % CPR) * 4;
    const int m = m0 + row;
    const int n = n0 + cc;
    if (m >= M || n >= p.N) continue;
    const float4 c4 = *reinterpret_cast<const float4*>(Cs + row * CLD + cc);
    float v[4] = {c4.x, c4.y, c4.z, c4.w};
    int b = 0, ho = 0, wo = m;
    if (!lin || p.gate) {
      wo = m % p.Wo;
      const int t = m / p.Wo;
      ho = t % p.Ho;
      b = t / p.Ho;
    }
    const bool full = n + 3 < p.N;
    float rv[4] = {0.f, 0.f, 0.f, 0.f};
    if (p.res) {
      const int64_t ro = (int64_t)m * p.res_ld + n;
      if (p.res_bf16) {
        const uint16_t* r = reinterpret_cast<const uint16_t*>(p.res) + ro;
#pragma unroll
        for (int u = 0; u < 4; ++u) rv[u] = (full || n + u < p.N) ? bf_bits2f(r[u]) : 0.f;
      } else {
        const float* r = reinterpret_cast<const float*>(p.res) + ro;
#pragma unroll
        for (int u = 0; u < 4; ++u) rv[u] = (full || n + u < p.N) ? r[u] : 0.f;
      }
    }
    const float* gr = p.gate ? p.gate + ((int64_t)b * p.gate_nseg + wo / p.gate_seg) * p.N : nullptr;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int nn = n + u;
      if (!full && nn >= p.N) break;
      float x = v[u];
      if (p.alpha) x *= p.alpha[nn];
      if (p.beta) x += p.beta[nn];
      x += rv[u];
      x = apply_act(x, p.act);
      if (gr) x *= gr[nn];
      v[u] = x;
    }
    if (vec && full) {
      const int64_t o = (int64_t)m * p.o_sw + n;
      if (p.out_bf16) {
        uint2 pk = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(p.out) + o) = pk;
      } else {
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.out) + o) = make_float4(v[0], v[1], v[2], v[3]);
      }
    } else {
      const int64_t ob = lin ? (int64_t)m * p.o_sw
                             : (int64_t)b * p.o_sb + (int64_t)ho * p.o_sh + (int64_t)wo * p.o_sw;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (n + u >= p.N) break;
        const int64_t o = ob + (int64_t)(n + u) * p.o_sn;
        if (p.out_bf16) reinterpret_cast<uint16_t*>(p.out)[o] = f2bf_bits(v[u]);
        else reinterpret_cast<float*>(p.out)[o] = v[u];
      }
    }
  }
}

template <int BM, int BN>
void launch(const ConvGemmArgs& p, hipStream_t st) {
  const int M = p.B * p.Ho * p.Wo;
  dim3 grid(cdiv(p.N, BN) * cdiv(M, BM));
  if (p.a_bf16)
    hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, true>), grid, dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL((gemm_bf16_kernel<BM, BN, false>), grid, dim3(256), 0, st, p);
}

}  // namespace

void conv_gemm_bf16(const ConvGemmArgs& p, hipStream_t st) {
  SD_CHECK(p.K == p.kh * p.kw * p.Cin, kErrInvalid, "conv_gemm: K != kh*kw*Cin");
  SD_CHECK(p.Cin % 8 == 0 && p.K % 8 == 0, kErrInvalid, "conv_gemm(bf16): Cin must be a multiple of 8");
  SD_CHECK(p.a_bf16 ? (p.lda % 8 == 0 && p.a_coff % 8 == 0) : (p.lda % 4 == 0 && p.a_coff % 4 == 0),
           kErrInvalid, "conv_gemm(bf16): misaligned activation rows");
  SD_CHECK(p.N > 0 && p.B > 0 && p.Ho > 0 && p.Wo > 0, kErrInvalid, "conv_gemm: empty problem");
  SD_CHECK(!p.gate || p.gate_seg > 0, kErrInvalid, "conv_gemm: gate_seg must be > 0");
  SD_CHECK(!p.pre_scale || p.Cin % 8 == 0, kErrInvalid, "conv_gemm: prologue needs Cin % 8 == 0");
  const int M = p.B * p.Ho * p.Wo;
  const double ab = p.a_bf16 ? 2.0 : 4.0, ob = p.out_bf16 ? 2.0 : 4.0;
  const double flops = 2.0 * M * p.N * (double)p.K;
  const double bytes = ab * p.B * p.H * p.W * p.Cin + 2.0 * p.N * p.K + ob * M * p.N +
                       (p.res ? (p.res_bf16 ? 2.0 : 4.0) * M * p.N : 0.0);
  // Path selection first, so the live timer (bench.py roofline) is keyed by the kernel that runs.
  enum Path { kFcm, kAreg, kRing, kStream, kDma, kReg } path = kReg;
  if (fcm_conv_supported(p))              // CAM++ FCM 3x3 32->32 convs (fcm_conv.hip)
    path = kFcm;
  else if (gemm_areg_supported(p))        // A read once, weights streamed (gemm_areg.hip)
    path = kAreg;
  else if (p.K > 384 && p.N >= 256 && gemm_ring_supported(p))   // stream would split N into 64-col panels
    path = kRing;
  else if (gemm_stream_supported(p))      // weight-resident streaming path (gemm_stream.hip)
    path = kStream;
  else if (gemm_ring_supported(p))        // 3-stage ring, BN-ReLU prologue (gemm_ring.hip)
    path = kRing;
  else if (gemm_dma_supported(p))         // LDS-DMA fast path (gemm_dma.hip)
    path = kDma;
  static const char* kNames[] = {"fcm_conv3x3_band", "gemm_areg", "gemm_ring", "gemm_stream", "gemm_dma",
                                 "gemm_bf16_reg"};
  static const bool detail = getenv("SDIAR_PROF_DETAIL") != nullptr;
  std::string key = kNames[path];
  if (detail && prof_enabled())
    key += " M=" + std::to_string(M) + " N=" + std::to_string(p.N) + " K=" + std::to_string(p.K) +
           " taps=" + std::to_string(p.kh * p.kw) + (p.a_bf16 ? " Abf" : " Af32") + (p.pre_scale ? " pre" : "");
  ProfScope prof(key.c_str(), flops, bytes, st);
  switch (path) {
    case kFcm: conv_fcm3x3(p, st); return;
    case kAreg: conv_gemm_areg(p, st); return;
    case kRing: conv_gemm_ring(p, st); return;
    case kStream: conv_gemm_stream(p, st); return;
    case kDma: conv_gemm_dma(p, st); return;
    case kReg: break;
  }
  const int bn = p.N >= 128 ? 128 : (p.N >= 64 ? 64 : 32);
  const bool big = (int64_t)cdiv(M, 128) * cdiv(p.N, bn) >= 512;
  if (bn == 128) {
    if (big) launch<128, 128>(p, st); else launch<64, 128>(p, st);
  } else if (bn == 64) {
    if (big) launch<128, 64>(p, st); else launch<64, 64>(p, st);
  } else {
    if (big) launch<128, 32>(p, st); else launch<64, 32>(p, st);
  }
  SD_LAUNCH_CHECK();
}

}  // namespace sd
