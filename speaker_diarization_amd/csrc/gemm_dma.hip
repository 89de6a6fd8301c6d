// bf16 implicit GEMM fed by LDS-DMA (buffer_load_dwordx4 ... lds) — the fast path
// of conv_gemm for bf16 activations without a BN-ReLU prologue.
//
// * A (activations) and B (packed weights) tiles go global -> LDS directly, 16 B
//   per lane; each wave instruction fills 8 rows x 128 B.  Out-of-range rows
//   (conv zero padding, M/N/K tails) use an out-of-range buffer offset, which
//   the buffer unit returns as zeros: no branches in the k loop.
// * LDS rows are 128 B (BK = 64 bf16) unpadded; the 16-B chunk c of row r is
//   stored at chunk c ^ (r & 7) (swizzle applied on the SOURCE address, the
//   DMA destination stays lane-linear), which makes the MFMA fragment reads
//   (ds_read_b128, 16 rows x one chunk) bank-conflict free.
// * NS-stage LDS ring: the DMAs of k-tiles k+1 .. k+NS-1 are in flight while tile k is consumed; the
//   DMAs are inline asm (invisible to the compiler's wait-count pass), so each k-tile costs one counted
//   vmcnt wait + one barrier.  The BN-ReLU prologue's per-channel scale / shift live in LDS, so no
//   compiler-visible global load sits in the loop either (its wait would drain the ring).
// * Epilogue identical to gemm_bf16.hip (LDS-staged, coalesced, bf16/fp32 out).
// Handles taps == 1 (linear / 1x1 conv) and multi-tap convs with Cin % 64 == 0.
#include <string>

#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {
namespace {

constexpr int BK = 64;
constexpr uint32_t kOOB = 0x80000000u;   // >= num_records -> hardware returns zeros
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  return (uint32_t)f2bf_bits(a) | ((uint32_t)f2bf_bits(b) << 16);
}

constexpr int kPreMax = 1024;   // prologue channels staged in LDS

template <int BM, int BN, int NS>
__global__ __launch_bounds__(256) void gemm_dma_kernel(ConvGemmArgs p) {
  constexpr int TM = BM / 2, TN = BN / 2;
  constexpr int MT = TM / 16, NT = TN / 16;
  constexpr int AI = BM / 32;        // A DMA instructions per wave per k-tile (8 rows each)
  constexpr int BI = BN / 32;
  constexpr int STAGE = (BM + BN) * BK;   // bf16 elements per stage
  constexpr int CLD = BN + 4;
  constexpr int EPI = BM * CLD * 2;
  constexpr int SMEM = (NS * STAGE > EPI) ? NS * STAGE : EPI;
  constexpr int DPW = AI + BI;       // DMA instructions per wave per k-tile
  __shared__ __attribute__((aligned(1024))) uint16_t sm[SMEM];
  __shared__ float pre_ss[2 * kPreMax];   // prologue scale | shift per input channel

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int M = p.B * p.Ho * p.Wo;
  const int n_nt = (p.N + BN - 1) / BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (tile / n_nt) * BM;
  const int n0 = (tile % n_nt) * BN;
  const int taps = p.kh * p.kw;
  // split-K share [kb, ke) of this workgroup (blockIdx.y); whole K without a split
  const int z = blockIdx.y;
  int kb = 0, ke = p.K;
  if (p.ksplit > 1) {
    const int kc = ((p.K + BK - 1) / BK + p.ksplit - 1) / p.ksplit * BK;
    kb = min(p.K, z * kc);
    ke = min(p.K, kb + kc);
  }

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.A), (short)0,
                                                                      (int)kOOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.Wt), (short)0,
                                                                      (int)kOOB, 0x00020000);
  // Per-lane A rows handled by this wave's DMA instructions.
  const int lrow = lane >> 3;          // row within an 8-row group
  const int lch = lane & 7;            // physical chunk this lane fills
  int a_bh[AI], a_h[AI], a_w[AI], a_lc[AI];
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    const int r = wid * (BM / 4) + j * 8 + lrow;
    const int m = m0 + r;
    a_lc[j] = lch ^ (r & 7);
    if (m < M) {
      const int wo = m % p.Wo;
      const int t = m / p.Wo;
      const int ho = t % p.Ho;
      a_bh[j] = (t / p.Ho) * p.H;
      a_h[j] = ho * p.sh - p.ph;
      a_w[j] = wo * p.sw - p.pw;
    } else {
      a_bh[j] = 0;
      a_h[j] = -(1 << 28);
      a_w[j] = 0;
    }
  }
  int b_row[BI], b_lc[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int r = wid * (BN / 4) + j * 8 + lrow;
    b_row[j] = n0 + r;
    b_lc[j] = lch ^ (r & 7);
  }

  auto issue = [&](int kt, int stg) {
    const int k0 = kb + kt * BK;
    int tap = 0, c0 = k0;
    if (taps > 1) {
      tap = k0 / p.Cin;
      c0 = k0 - tap * p.Cin;
    }
    const int ti = tap / p.kw, tj = tap - (tap / p.kw) * p.kw;
    const int dho = ti * p.dh, dwo = tj * p.dw;
    uint16_t* As = sm + stg * STAGE;
    uint16_t* Bs = As + BM * BK;
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int hi = a_h[j] + dho, wi = a_w[j] + dwo;
      const int c = c0 + a_lc[j] * 8;
      const bool ok = (unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W && (k0 + a_lc[j] * 8) < ke;
      const uint32_t off = ok ? (uint32_t)((((int64_t)(a_bh[j] + hi) * p.W + wi) * p.lda + p.a_coff + c) * 2)
                              : kOOB;
      lds_ptr_t dst = (lds_ptr_t)(As + (wid * (BM / 4) + j * 8) * BK);
      dma_lds16_buf(ra, off, dst);
    }
#pragma unroll
    for (int j = 0; j < BI; ++j) {
      const int k = k0 + b_lc[j] * 8;
      const bool ok = b_row[j] < p.N && k < ke;
      const uint32_t off = ok ? (uint32_t)(((int64_t)b_row[j] * p.K + k) * 2) : kOOB;
      lds_ptr_t dst = (lds_ptr_t)(Bs + (wid * (BN / 4) + j * 8) * BK);
      dma_lds16_buf(rb, off, dst);
    }
  };

  floatx4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int KT = (ke - kb + BK - 1) / BK;
  const int l15 = lane & 15, lk = lane >> 4;
  // Optional BN-ReLU prologue (CAM dense layers: nonlinear1 before linear1): applied
  // in place on the landed A stage, 16 B per thread-step, before the MFMAs read it.
  // Zero-filled K-tail columns stay harmless: their weight rows are zero-filled too.
  // Thread i always touches rows r = i/8 + 32j (r & 7 fixed) and physical chunk i & 7, so
  // its logical chunk, hence its 8 k columns, are fixed: 2 x 2 float4 loads per k-tile.
  const int pre_pc = tid & 7;
  const int pre_lc = pre_pc ^ ((tid >> 3) & 7);
  // Multi-tap convs: a prologue row whose input position is conv zero padding for the k-tile's tap must
  // stay 0 (BN-ReLU is applied before the padding); the rows a thread transforms are fixed (r = tid/8 + 32j),
  // so their input offsets are computed once.
  constexpr int PRJ = BM / 32;
  int pr_h[PRJ], pr_w[PRJ];
#pragma unroll
  for (int j = 0; j < PRJ; ++j) {
    const int m = m0 + (tid >> 3) + 32 * j;
    if (m < M) {
      const int wo = m % p.Wo, t = m / p.Wo;
      pr_h[j] = (t % p.Ho) * p.sh - p.ph;
      pr_w[j] = wo * p.sw - p.pw;
    } else {
      pr_h[j] = -(1 << 28);
      pr_w[j] = 0;
    }
  }
  auto prologue = [&](int kt, int stg) {
    uint16_t* As = sm + stg * STAGE;
    const int kg = kb + kt * BK;                    // first k of the tile (one tap: Cin % BK == 0)
    const int tap = taps > 1 ? kg / p.Cin : 0;
    const int ti = tap / p.kw, tj = tap - ti * p.kw;
    const int k = kg + pre_lc * 8;                  // this thread's 8 k columns
    const int c = k - tap * p.Cin;                  // their channel (k itself for one tap)
    float sc[8], sh[8];
    if (k + 8 <= ke) {
      const float4 s0 = *reinterpret_cast<const float4*>(pre_ss + c);
      const float4 s1 = *reinterpret_cast<const float4*>(pre_ss + c + 4);
      const float4 h0 = *reinterpret_cast<const float4*>(pre_ss + kPreMax + c);
      const float4 h1 = *reinterpret_cast<const float4*>(pre_ss + kPreMax + c + 4);
      sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w; sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
      sh[0] = h0.x; sh[1] = h0.y; sh[2] = h0.z; sh[3] = h0.w; sh[4] = h1.x; sh[5] = h1.y; sh[6] = h1.z; sh[7] = h1.w;
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u) { sc[u] = 0.f; sh[u] = 0.f; }   // K tail: A*0 + 0 (weights are 0 too)
    }
#pragma unroll
    for (int j = 0; j < PRJ; ++j) {
      const int i = tid + 256 * j;
      uint4* ptr = reinterpret_cast<uint4*>(As + (i >> 3) * BK + pre_pc * 8);
      if (taps > 1 && !((unsigned)(pr_h[j] + ti * p.dh) < (unsigned)p.H && (unsigned)(pr_w[j] + tj * p.dw) < (unsigned)p.W)) {
        *ptr = make_uint4(0u, 0u, 0u, 0u);   // zero padding stays zero
        continue;
      }
      uint4 v = *ptr;
      uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float x0 = fmaxf(fmaf(__uint_as_float(w[u] << 16), sc[2 * u], sh[2 * u]), 0.f);
        const float x1 = fmaxf(fmaf(__uint_as_float(w[u] & 0xffff0000u), sc[2 * u + 1], sh[2 * u + 1]), 0.f);
        w[u] = pack_bf2(x0, x1);
      }
      *ptr = make_uint4(w[0], w[1], w[2], w[3]);
    }
  };
  const bool pre = p.pre_scale != nullptr;
  if (pre) {
    const int cin = taps > 1 ? p.Cin : p.K;
    for (int i = tid; i < cin; i += 256) {
      pre_ss[i] = p.pre_scale[i];
      pre_ss[kPreMax + i] = p.pre_shift[i];
    }
  }
  // a plain barrier (LDS writes done): a __syncthreads() fence would add vmcnt(0) and drain the ring
  auto barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < KT) issue(s, s);
  for (int kt = 0; kt < KT; ++kt) {
    const int stg = kt % NS;
    // k-tile kt landed: only the tiles issued after it (kt + 1 .. kt + NS - 2, DPW DMAs each) are younger
    const int younger = min(KT - 1, kt + NS - 2) - kt;
    if (NS >= 4 && younger >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * DPW) : "memory");
    else if (NS >= 3 && younger >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();   // tile kt visible to every wave; every wave is done with tile kt - 1's stage
    if (pre) {
      prologue(kt, stg);
      barrier();
    }
    if (kt + NS - 1 < KT) issue(kt + NS - 1, (kt + NS - 1) % NS);
    const uint16_t* As = sm + stg * STAGE;
    const uint16_t* Bs = As + BM * BK;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[MT], bfr[NT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int r = wm * TM + mt * 16 + l15;
        af[mt] = *reinterpret_cast<const bf16x8*>(As + r * BK + (((ks * 4 + lk) ^ (r & 7)) * 8));
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int r = wn * TN + nt * 16 + l15;
        bfr[nt] = *reinterpret_cast<const bf16x8*>(Bs + r * BK + (((ks * 4 + lk) ^ (r & 7)) * 8));
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bfr[nt], acc[mt][nt], 0, 0, 0);
    }
  }
  barrier();   // every wave is done with the ring: the epilogue tile takes over its LDS

  // ---- epilogue (LDS-staged, row-contiguous 4-column groups)
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
  // 4-column vector stores: unit column stride, 4-element row strides, base pointers aligned for the vector width
  // (16 B fp32, 8 B bf16; split-K slabs are whole allocations)
  const bool vec = lin && p.o_sn == 1 && (p.o_sw & 3) == 0 &&
                   (reinterpret_cast<uintptr_t>(p.out) & (p.out_bf16 ? 7 : 15)) == 0;
  constexpr int CPR = BN / 4;
  if (vec && !p.gate &&
      (!p.res || (!p.res_bf16 && (p.res_ld & 3) == 0 && (reinterpret_cast<uintptr_t>(p.res) & 15) == 0))) {
    // Fast epilogue (row-major output): each thread owns one 4-column group, so the
    // per-channel alpha/beta are loaded once, and all residual rows are fetched before
    // any store (res may alias out: the in-place residual add of the encoders).
    constexpr int RPI = 256 / CPR;      // rows per pass
    constexpr int ITER = BM / RPI;
    const int cg = tid % CPR, r0 = tid / CPR;
    const int n = n0 + cg * 4;
    if (n >= p.N) return;
    const bool full = n + 3 < p.N;
    float al[4], be[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool ok = full || n + u < p.N;
      al[u] = (p.alpha && ok) ? p.alpha[n + u] : 1.f;
      be[u] = (p.beta && ok && z == 0) ? p.beta[n + u] : 0.f;   // split-K: bias once, in slab 0
    }
    void* const outp = p.ksplit > 1 ? static_cast<void*>(reinterpret_cast<float*>(p.out) + z * p.split_stride) : p.out;
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
      const int row = r0 + i * RPI;
      const int m = m0 + row;
      if (m >= M) break;
      const float4 c4 = *reinterpret_cast<const float4*>(Cs + row * CLD + cg * 4);
      float v[4] = {c4.x, c4.y, c4.z, c4.w};
      const float r4[4] = {p.res ? rv[i].x : 0.f, p.res ? rv[i].y : 0.f, p.res ? rv[i].z : 0.f,
                           p.res ? rv[i].w : 0.f};
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = apply_act(fmaf(v[u], al[u], be[u]) + r4[u], p.act);
      const int64_t o = (int64_t)m * p.o_sw + n;
      if (full) {
        if (p.out_bf16)
          *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(outp) + o) =
              make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
        else
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(outp) + o) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        for (int u = 0; u < 4 && n + u < p.N; ++u) {
          if (p.out_bf16) reinterpret_cast<uint16_t*>(outp)[o + u] = f2bf_bits(v[u]);
          else reinterpret_cast<float*>(outp)[o + u] = v[u];
        }
      }
    }
    return;
  }
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
        if (full && (p.res_ld & 3) == 0) {
          const float4 r4 = *reinterpret_cast<const float4*>(r);
          rv[0] = r4.x; rv[1] = r4.y; rv[2] = r4.z; rv[3] = r4.w;
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u) rv[u] = (full || n + u < p.N) ? r[u] : 0.f;
        }
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
      if (p.out_bf16)
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(p.out) + o) =
            make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
      else
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(p.out) + o) = make_float4(v[0], v[1], v[2], v[3]);
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

// ring depth 2: two 64-KiB workgroups per CU overlap one's BN-ReLU prologue pass with the other's MFMAs;
// a 4-stage ring at one workgroup per CU measured slower (C2 gemm_dma 0.60 -> 0.90 ms; 2 stages: 0.56)
template <int BM, int BN>
constexpr int dma_stages() {
  return 2;
}

template <int BM, int BN>
void launch(const ConvGemmArgs& p, hipStream_t st) {
  const int M = p.B * p.Ho * p.Wo;
  dim3 grid(cdiv(p.N, BN) * cdiv(M, BM), p.ksplit > 1 ? p.ksplit : 1);
  hipLaunchKernelGGL((gemm_dma_kernel<BM, BN, dma_stages<BM, BN>()>), grid, dim3(256), 0, st, p);
}

}  // namespace

bool gemm_dma_supported(const ConvGemmArgs& p) {
  const int taps = p.kh * p.kw;
  const int64_t a_bytes = ((int64_t)p.B * p.H * p.W) * p.lda * 2;
  const int64_t w_bytes = (int64_t)p.N * p.K * 2;
  return p.a_bf16 && (!p.pre_scale || (p.pre_shift && (taps == 1 || p.Cin % BK == 0) &&
                                       (taps > 1 ? p.Cin : p.K) <= kPreMax)) && (taps == 1 || p.Cin % BK == 0) && p.K % 8 == 0 && p.lda % 8 == 0 &&
         p.a_coff % 8 == 0 && a_bytes < (int64_t)kOOB && w_bytes < (int64_t)kOOB;
}

void conv_gemm_dma(const ConvGemmArgs& p, hipStream_t st) {
  const int M = p.B * p.Ho * p.Wo;
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

// Split-K for the short-M, long-K GEMMs (the post-LN FFN down-projections: M 6000, K 2048, N 256 is 188
// 64x128 tiles, one per CU, each walking 32 k-tiles at one DMA latency apiece): ksplit workgroups per tile.
int gemm_splitk_count(const ConvGemmArgs& p) {
  const int M = p.B * p.Ho * p.Wo;
  if (!gemm_dma_supported(p) || p.pre_scale || p.alpha || p.res || p.gate || p.glu ||
      p.act != kActNone || p.o_sn != 1 || p.K < 1024 || p.N % 4)
    return 1;
  // enough 256x128 tiles for one per CU: the ring GEMM (3-stage DMA ring) beats the split (FS-EEND decoder
  // FFN-down, M 36000: 163 vs 243 us for 2 launches; at M 6000 the split wins, 96 vs 141 us for 4)
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    SD_HIP(hipGetDevice(&dev));
    SD_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  if (gemm_ring_supported(p) && (int64_t)cdiv(M, 256) * cdiv(p.N, 128) >= n_cu) return 1;
  const int bn = p.N >= 128 ? 128 : (p.N >= 64 ? 64 : 32);
  const int64_t tiles = (int64_t)cdiv(M, 128) * cdiv(p.N, bn);
  const int64_t tiles_launched = tiles >= 512 ? tiles : (int64_t)cdiv(M, 64) * cdiv(p.N, bn);
  int ks = 1;
  while (ks < 4 && tiles_launched * ks < 768 && p.K / (2 * ks) >= 512) ks *= 2;
  return ks;
}

void conv_gemm_splitk(const ConvGemmArgs& p_in, int ksplit, float* slabs, hipStream_t st) {
  SD_CHECK(ksplit >= 1 && ksplit <= 8, kErrInvalid, "splitk: bad split count");
  ConvGemmArgs p = p_in;
  const int M = p.B * p.Ho * p.Wo;
  p.ksplit = ksplit;
  p.split_stride = (int64_t)M * p.N;
  p.out = slabs;
  p.out_bf16 = false;
  p.o_sb = (int64_t)p.Ho * p.Wo * p.N; p.o_sh = (int64_t)p.Wo * p.N; p.o_sw = p.N; p.o_sn = 1;
  static const bool detail = getenv("SDIAR_PROF_DETAIL") != nullptr;
  std::string key = "gemm_dma_splitk";
  if (detail && prof_enabled()) key += " M=" + std::to_string(M) + " K=" + std::to_string(p.K) + " ks=" + std::to_string(ksplit);
  ProfScope prof(key.c_str(), 2.0 * M * p.N * (double)p.K,
                 2.0 * M * (double)p.K + 2.0 * p.N * p.K + 4.0 * ksplit * M * p.N, st);
  conv_gemm_dma(p, st);
}

}  // namespace sd
