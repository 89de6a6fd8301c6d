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
// fp32-equivalent fast path) stages fp32 like fp32 mode and splits each operand
// fragment in registers into bf16 hi + lo: acc += hi·hi + hi·lo + lo·hi on
// v_mfma_f32_16x16x32_bf16 (the lo·lo term and the lo part's own rounding leave
// ~2^-16 relative error per product; 3 MFMAs of 16 cycles per 32-k step against
// 8 f32 MFMAs of 32).
#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {

namespace {

constexpr int kBK = 32;
constexpr int kLdsBf = kBK + 8;   // bf16 row stride (80 B: 16-B aligned, conflict-light)
constexpr int kLdsF = kBK + 2;    // fp32 row stride (34 words: conflict-free 16x16x4 reads)

thread_local bool t_gemm_x3 = false;

// 8 fp32 values -> bf16 hi (round to nearest even) and lo = bf16(v - hi)
__device__ __forceinline__ void split_bf16x8(const float (&v)[8], bf16x8& hi, bf16x8& lo) {
  uint32_t h[4], l[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    h[j] = pack_bf16x2(v[2 * j], v[2 * j + 1]);
    const float h0 = __uint_as_float(h[j] << 16), h1 = __uint_as_float(h[j] & 0xffff0000u);
    l[j] = pack_bf16x2(v[2 * j] - h0, v[2 * j + 1] - h1);
  }
  hi = __builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
  lo = __builtin_bit_cast(bf16x8, make_uint4(l[0], l[1], l[2], l[3]));
}

// 8 consecutive fp32 of an LDS row (8-B aligned: the fp32 stride of 34 words) as 4 x 8-B reads
__device__ __forceinline__ void lds_f32x8(const float* p, float (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float2 t = *reinterpret_cast<const float2*>(p + 2 * j);
    v[2 * j] = t.x;
    v[2 * j + 1] = t.y;
  }
}

// MODE 0: exact f32 MFMA, 1: bf16 (fp32 activations converted on staging), 2: bf16x3 on fp32 tiles
template <int BM, int BN, int MODE>
__global__ __launch_bounds__(256) void conv_gemm_kernel(ConvGemmArgs p) {
  constexpr bool BF16 = MODE == 1;
  constexpr int TM = BM / 2, TN = BN / 2;
  constexpr int MT = TM / 16, NT = TN / 16;
  constexpr int APASS = BM / 32;
  using LdsT = typename std::conditional<BF16, uint16_t, float>::type;
  constexpr int LDS_STRIDE = BF16 ? kLdsBf : kLdsF;
  __shared__ __attribute__((aligned(16))) LdsT As[2][BM * LDS_STRIDE];
  __shared__ __attribute__((aligned(16))) LdsT Bs[2][BN * LDS_STRIDE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int M = p.B * p.Ho * p.Wo;
  const int m0 = blockIdx.y * BM;
  const int n0 = blockIdx.x * BN;

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
  float4 areg[APASS];
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
    float4 s4, h4;
    if (p.pre_scale && k0 + kq < p.K) {
      s4 = *reinterpret_cast<const float4*>(p.pre_scale + c);
      h4 = *reinterpret_cast<const float4*>(p.pre_shift + c);
    }
#pragma unroll
    for (int i = 0; i < APASS; ++i) {
      int hi = rh[i] + ti * p.dh;
      int wi = rw[i] + tj * p.dw;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if ((unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W && k0 + kq < p.K) {
        const float* src = reinterpret_cast<const float*>(p.A) + ((int64_t)(rbh[i] + hi) * p.W + wi) * p.lda + p.a_coff + c;
        v = *reinterpret_cast<const float4*>(src);
        if (p.pre_scale) {
          v.x = fmaxf(v.x * s4.x + h4.x, 0.f);
          v.y = fmaxf(v.y * s4.y + h4.y, 0.f);
          v.z = fmaxf(v.z * s4.z + h4.z, 0.f);
          v.w = fmaxf(v.w * s4.w + h4.w, 0.f);
        }
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
    } else if constexpr (MODE == 2) {
      // one 16x16x32 k-step per BK = 32: lane (row lrow, k 8 lk .. 8 lk + 7) of every fragment, split hi / lo
      const float* Af = reinterpret_cast<const float*>(As[buf]);
      const float* Bf = reinterpret_cast<const float*>(Bs[buf]);
      bf16x8 bh[NT], bl[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        float v[8];
        lds_f32x8(Bf + (wn * TN + nt * 16 + lrow) * LDS_STRIDE + lk * 8, v);
        split_bf16x8(v, bh[nt], bl[nt]);
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        float v[8];
        lds_f32x8(Af + (wm * TM + mt * 16 + lrow) * LDS_STRIDE + lk * 8, v);
        bf16x8 ah, al;
        split_bf16x8(v, ah, al);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[nt], acc[mt][nt], 0, 0, 0);
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[nt], acc[mt][nt], 0, 0, 0);
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[nt], acc[mt][nt], 0, 0, 0);
        }
      }
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

  // Epilogue.
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

template <int BM, int BN>
void launch_tile(const ConvGemmArgs& p, bool bf16, hipStream_t st) {
  SD_CHECK(!p.a_bf16 && !p.out_bf16 && !p.res_bf16, kErrInvalid, "fp32 conv_gemm takes fp32 tensors");
  const int M = p.B * p.Ho * p.Wo;
  dim3 grid(cdiv(p.N, BN), cdiv(M, BM));
  if (bf16)
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, 1>), grid, dim3(256), 0, st, p);
  else if (t_gemm_x3)
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, 2>), grid, dim3(256), 0, st, p);
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
  ProfScope prof(bf16 ? "conv_gemm_bf16" : t_gemm_x3 ? "conv_gemm_bf16x3" : "conv_gemm_f32", flops, bytes, st);
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
