// Streaming (KV-cache) kernels for the chunked FS-EEND forward on gfx950.
//
// The reference computes OnlineTransformerDADiarization.test() (fs_eend.py:79-96) over a
// whole recording with causal masks (mask_delay 0 in every shipped config,
// fs_eend/config/*.yaml).  Causality makes the forward incremental: frame t of every
// encoder layer depends on frames <= t only, the look-ahead Conv1d (k 19, pad 9,
// fs_eend.py:41,85) needs 9 frames of encoder output past t, and the decoder's time
// attention (fs_eend.py:456-467) is causal again.  The streaming runner keeps, per
// layer, the K|V rows of every frame already seen and runs each new chunk of `c` frames
// against them.  Every position-dependent argument is read from a device-resident
// cursor so a chunk's whole kernel sequence can be captured once into a hipGraph and
// replayed (no host arguments change between chunks).
//
//   kv_append       copy `rows` rows (width bytes) of a staging buffer into a history
//                   buffer at row cursor*mult (the K|V half of the in-projection, or the
//                   encoder output)
//   attn_decode     softmax(q·kᵀ·scale)·v for nq (≤ 32) queries at absolute positions
//                   cursor + i against all cached keys j <= cursor + i + delay:
//                   a fixed grid of <= 32 blocks per (sequence, head) whose waves stride
//                   over 64-key tiles with an online softmax, block-merged partials, one
//                   combine wave per query (fixed grid: replayable for any cursor).
//                   fp32 arithmetic; K/V/Q/O fp32 or bf16 (the dtype of the cache).
//                   HBM-bound: each cached key row is read once per (sequence, head).
//   gather_window   rows [cursor - pad, cursor + c + pad) of the encoder-output history,
//                   zero outside [0, n_valid) (the conv's zero padding and the
//                   emb[:ilen] re-pad of fs_eend.py:83-84)
//   cursor_advance  cursor[i] += c (+ optional mirror), the graph's last node
#include <algorithm>
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {
namespace {

constexpr int kMaxQ = 32;
constexpr int kHD = 64;
constexpr int kMaxBlk = 32;   // partials per (sequence, head): attn_decode_blocks' cap
typedef float f32x2 __attribute__((ext_vector_type(2)));

// 16-B row copy; rows of `width16` uint4 units.
__global__ __launch_bounds__(256) void kv_append_kernel(const uint4* __restrict__ src, int64_t ld_src16, int rows,
                                                        int width16, uint4* __restrict__ dst, int64_t ld_dst16,
                                                        const int* __restrict__ cursor, int mult) {
  const int64_t r0 = (int64_t)(*cursor) * mult;
  const int64_t n = (int64_t)rows * width16;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / width16;
    const int c = (int)(i - r * width16);
    dst[(r0 + r) * ld_dst16 + c] = src[r * ld_src16 + c];
  }
}

template <bool IOBF>
__device__ __forceinline__ void load_row64(const act_t<IOBF>* p, float* v) {
  if constexpr (IOBF) {
#pragma unroll
    for (int j = 0; j < kHD; j += 8) {
      const uint4 u = *reinterpret_cast<const uint4*>(p + j);
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[j + 2 * e] = __uint_as_float(w[e] << 16);
        v[j + 2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < kHD; j += 4) {
      const float4 u = *reinterpret_cast<const float4*>(p + j);
      v[j] = u.x; v[j + 1] = u.y; v[j + 2] = u.z; v[j + 3] = u.w;
    }
  }
}

// Weight rows as 16-B vectors: 8 bf16 or 4 fp32 values per vector.  The fused slot block below issues a thread's
// whole weight slice as one batch before it needs any of it (one memory latency per slice, not one per vector).
template <bool WBF>
struct WVec {
  static constexpr int VE = WBF ? 8 : 4;
  __device__ __forceinline__ static uint4 load(const void* w, int64_t elem) {
    if constexpr (WBF) return *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(w) + elem);
    else return *reinterpret_cast<const uint4*>(static_cast<const float*>(w) + elem);
  }
  __device__ __forceinline__ static float at(const uint4& u, int e) {
    const uint32_t w = e < (WBF ? 2 : 1) ? u.x : e < (WBF ? 4 : 2) ? u.y : e < (WBF ? 6 : 3) ? u.z : u.w;
    if constexpr (WBF) return __uint_as_float((e & 1) ? (w & 0xffff0000u) : (w << 16));
    else return __uint_as_float(w);
  }
  // weights 2p, 2p + 1 of the vector as an f32 pair (one v_pk_fma_f32 operand)
  __device__ __forceinline__ static f32x2 pair(const uint4& u, int p) { return f32x2{at(u, 2 * p), at(u, 2 * p + 1)}; }
};

// The nblk partials of one (sequence, head), merged: wave -> query, lane -> head dim (lane-parallel max /
// weights, shuffled weights for o).  SC1: the partials were handed over inside this launch (write-through
// stores, read back with L1-bypassing sc1 loads).
template <bool SC1>
__device__ __forceinline__ float combine_value(const DecodeAttnArgs& a, int sh, int qi, int lane, int nblk) {
  const int64_t bstride = (int64_t)a.nq * (2 + kHD);
  const int64_t base = (int64_t)sh * nblk * bstride + qi * (2 + kHD);
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(a.ws, (short)0, 0x7fffffff, 0x00020000);
  auto ld = [&](int64_t i) {
    if constexpr (SC1) return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rw, (uint32_t)(i * 4), 0, 16));
    else return a.ws[i];
  };
  // every load issued before the first use: one memory round trip for the whole merge (nblk <= 32 by
  // attn_decode_blocks; rows past nblk re-read the last partial and get weight 0)
  const float mv0 = ld(base + min(lane, nblk - 1) * bstride);
  const float lv0 = ld(base + min(lane, nblk - 1) * bstride + 1);
  float ov[kMaxBlk];
#pragma unroll
  for (int b = 0; b < kMaxBlk; ++b) ov[b] = ld(base + min(b, nblk - 1) * bstride + 2 + lane);
  const float mv = lane < nblk ? mv0 : -INFINITY;
  const float lv = lane < nblk ? lv0 : 0.f;
  const float M = warp_max(mv);
  const float w = (mv == -INFINITY) ? 0.f : __expf(mv - M);
  const float L = warp_sum(w * lv);
  float o = 0.f;
#pragma unroll
  for (int b = 0; b < kMaxBlk; ++b) o = fmaf(__shfl(w, b, 64), ov[b], o);
  return o / L;
}

template <bool IOBF, bool SC1>
__device__ __forceinline__ void combine_partials(const DecodeAttnArgs& a, int sh, int qi, int lane, int nblk) {
  using io_t = act_t<IOBF>;
  const int s = sh / a.nh, h = sh % a.nh;
  const float o = combine_value<SC1>(a, sh, qi, lane, nblk);
  io_t* ob = reinterpret_cast<io_t*>(a.out) + (int64_t)qi * a.o_tok + (int64_t)s * a.o_seq + h * kHD;
  st_act(ob, lane, o);
}

// grid (nblk, nseq*nh), 256 threads.  Wave w of block b walks the 64-key tiles
// t = 4b + w, 4b + w + 4*nblk, ... below the device cursor's key count with an online
// softmax per query (lane = key for q·k; lane = (key parity, head-dim pair) for p·v, so
// each lane issues 32 independent 4/8-B V loads per tile), the 4 waves merge in LDS and
// the block writes one (m, l, o[64]) partial per query.  FUSED (a.cnt set): the partials are
// stored write-through, every block counts itself on its (sequence, head)'s counter, and the
// block whose add completes the launch's nblk merges them (MI355X guide hand-off row 1) -- the
// separate combine launch (a dependent kernel boundary + its own ramp per attention) is gone.
// The counters are monotonic: each launch adds exactly nblk per (sequence, head).
template <bool IOBF, int QMAX, bool FUSED, bool OP = false>
__global__ __launch_bounds__(256) void attn_decode_kernel(DecodeAttnArgs a) {
  using io_t = act_t<IOBF>;
  __shared__ float qs[QMAX][kHD];
  __shared__ float ps[4][QMAX][64];
  __shared__ float wm[4][QMAX], wl[4][QMAX];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int sh = blockIdx.y, s = sh / a.nh, h = sh % a.nh;
  const int nq = a.nq;
  const int pos = *a.pos;
  const int total = pos + nq;                           // keys present after this chunk's append
  const io_t* qb = reinterpret_cast<const io_t*>(a.q) + (int64_t)s * a.q_seq + h * kHD;
  const io_t* kb = reinterpret_cast<const io_t*>(a.k) + (int64_t)s * a.kv_seq + h * kHD;
  const io_t* vb = reinterpret_cast<const io_t*>(a.v) + (int64_t)s * a.kv_seq + h * kHD;
  const int half = lane >> 5, d2 = (lane & 31) * 2;
  // K row (lane = key) and V operands (keys k0 + 2i + half, dims d2, d2 + 1) of tile t
  float kr[kHD], v0[32], v1[32];
  auto load_tile = [&](int t) {
    const int k0 = t * 64;
    load_row64<IOBF>(kb + (int64_t)min(k0 + lane, total - 1) * a.kv_tok, kr);
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const int key = min(k0 + 2 * i + half, total - 1);
      const io_t* vr = vb + (int64_t)key * a.kv_tok + d2;
      if constexpr (IOBF) {
        const uint32_t u = *reinterpret_cast<const uint32_t*>(vr);
        v0[i] = __uint_as_float(u << 16);
        v1[i] = __uint_as_float(u & 0xffff0000u);
      } else {
        const float2 u = *reinterpret_cast<const float2*>(vr);
        v0[i] = u.x;
        v1[i] = u.y;
      }
    }
  };
  // the wave's first tile is in flight while the queries are staged (at short histories a wave has one tile)
  int t = blockIdx.x * 4 + wid;
  if (t * 64 < total) load_tile(t);
  for (int i = tid; i < nq * kHD; i += 256) {
    const int qi = i / kHD, d = i % kHD;
    qs[qi][d] = ld_act(qb, (int64_t)qi * a.q_tok + d) * a.scale;
  }
  __syncthreads();
  float m_run[QMAX], l_run[QMAX], o0[QMAX], o1[QMAX];
#pragma unroll
  for (int qi = 0; qi < QMAX; ++qi) { m_run[qi] = -INFINITY; l_run[qi] = 0.f; o0[qi] = 0.f; o1[qi] = 0.f; }
  while (t * 64 < total) {
    const int j = t * 64 + lane;
    const bool kv = j < total;
#pragma unroll
    for (int qi = 0; qi < QMAX; ++qi) {
      if (qi < nq) {
        float sc = 0.f;
#pragma unroll
        for (int d = 0; d < kHD; ++d) sc = fmaf(qs[qi][d], kr[d], sc);
        const bool vis = kv && j <= pos + qi + a.delay;
        sc = vis ? sc : -INFINITY;
        const float mn = fmaxf(m_run[qi], warp_max(sc));
        const float p = (!vis || mn == -INFINITY) ? 0.f : __expf(sc - mn);
        const float corr = (m_run[qi] == -INFINITY) ? 0.f : __expf(m_run[qi] - mn);
        l_run[qi] = l_run[qi] * corr + warp_sum(p);
        o0[qi] *= corr;
        o1[qi] *= corr;
        m_run[qi] = mn;
        ps[wid][qi][lane] = p;   // read back by the same wave only (a wave's LDS ops stay in order)
      }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int qi = 0; qi < QMAX; ++qi) {
      if (qi < nq) {
#pragma unroll
        for (int i = 0; i < 32; ++i) {
          const float p = ps[wid][qi][2 * i + half];
          o0[qi] = fmaf(p, v0[i], o0[qi]);
          o1[qi] = fmaf(p, v1[i], o1[qi]);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    t += gridDim.x * 4;
    if (t * 64 < total) load_tile(t);
  }
  // merge the two key-parity halves, park the wave's partial in LDS
#pragma unroll
  for (int qi = 0; qi < QMAX; ++qi) {
    if (qi < nq) {
      o0[qi] += __shfl_xor(o0[qi], 32, 64);
      o1[qi] += __shfl_xor(o1[qi], 32, 64);
      if (half == 0) {
        ps[wid][qi][d2] = o0[qi];
        ps[wid][qi][d2 + 1] = o1[qi];
      }
      if (lane == 0) {
        wm[wid][qi] = m_run[qi];
        wl[wid][qi] = l_run[qi];
      }
    }
  }
  __syncthreads();
  const int64_t poff = ((int64_t)sh * gridDim.x + blockIdx.x) * nq * (2 + kHD);
  float* part = a.ws + poff;
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(a.ws, (short)0, 0x7fffffff, 0x00020000);
  auto put = [&](int64_t i, float v) {   // i: index within this block's partial
    if constexpr (FUSED) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rw, (uint32_t)((poff + i) * 4), 0, 16);
    else part[i] = v;
  };
  for (int i = tid; i < nq * kHD; i += 256) {
    const int qi = i / kHD, d = i % kHD;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, wm[w][qi]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float e = (wm[w][qi] == -INFINITY) ? 0.f : __expf(wm[w][qi] - M);
      L = fmaf(e, wl[w][qi], L);
      O = fmaf(e, ps[w][qi][d], O);
    }
    put(qi * (2 + kHD) + 2 + d, O);
    if (d == 0) {
      put(qi * (2 + kHD), M);
      put(qi * (2 + kHD) + 1, L);
    }
  }
  if constexpr (FUSED) {
    __shared__ int last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      // wrapping increment (old >= n-1 -> 0): the counter runs 0..n-1 and is back at 0 after every launch,
      // whatever n is and however many launches ran (a free-running u32 % n loses the merge at the 2^32 wrap
      // unless n divides 2^32)
      const unsigned n = gridDim.x;
      last = __builtin_amdgcn_atomic_inc32(a.cnt + sh, n - 1, __ATOMIC_RELAXED, "agent") == n - 1;
    }
    __syncthreads();
    if (!last) return;
    if constexpr (!OP) {
      for (int qi = wid; qi < nq; qi += 4) combine_partials<IOBF, true>(a, sh, qi, lane, gridDim.x);
    } else {
      // OP: the out-projection as a second hand-off.  The (sequence, head)'s merged output stays in LDS (qs), the
      // thread's slice of W_out (row tid, the head's 64 inputs) is loaded in the same round trip as the
      // partials, the head's out-projection partial of feature tid is published write-through, and the last
      // head of the sequence to count itself sums the nh partials in head order + b_out (slot block pattern).
      using V = WVec<IOBF>;
      constexpr int NWV = kHD / V::VE;
      const int D = a.nh * kHD;
      uint4 wv[NWV];
      const int64_t wrow = (int64_t)min(tid, D - 1) * D + h * kHD;
#pragma unroll
      for (int v = 0; v < NWV; ++v) wv[v] = V::load(a.wo, wrow + v * V::VE);
      for (int qi = wid; qi < nq; qi += 4) qs[qi][lane] = combine_value<true>(a, sh, qi, lane, gridDim.x);
      __syncthreads();
      float pr[QMAX];
#pragma unroll
      for (int qi = 0; qi < QMAX; ++qi) pr[qi] = 0.f;
#pragma unroll
      for (int v = 0; v < NWV; ++v)
#pragma unroll
        for (int e = 0; e < V::VE; ++e) {
          const float w = V::at(wv[v], e);
#pragma unroll
          for (int qi = 0; qi < QMAX; ++qi) pr[qi] = fmaf(qs[qi][v * V::VE + e], w, pr[qi]);
        }
      const __amdgpu_buffer_rsrc_t r2 = __builtin_amdgcn_make_buffer_rsrc(a.ws2, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
      for (int qi = 0; qi < QMAX; ++qi)   // rows >= nq and threads >= D: dropped (offset past the range)
        __builtin_amdgcn_raw_buffer_store_b32(
            __float_as_uint(pr[qi]), r2,
            qi < nq && tid < D ? (uint32_t)((((int64_t)sh * nq + qi) * D + tid) * 4) : 0xfffffff0u, 0, 16);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const unsigned nh = a.nh;
        last = __builtin_amdgcn_atomic_inc32(a.cnt2 + s, nh - 1, __ATOMIC_RELAXED, "agent") == nh - 1;
      }
      __syncthreads();
      if (!last || tid >= D) return;
      const float bo = a.bo[tid];
      using io_t = act_t<IOBF>;
      for (int qi = 0; qi < nq; ++qi) {
        float hv[4];
#pragma unroll
        for (int hh = 0; hh < 4; ++hh)   // nh <= 4 (D = nh * 64 <= 256); heads past nh re-read head nh - 1
          hv[hh] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
              r2, (uint32_t)((((int64_t)(s * a.nh + min(hh, a.nh - 1))) * nq + qi) * D + tid) * 4, 0, 16));
        float v = 0.f;
#pragma unroll
        for (int hh = 0; hh < 4; ++hh)
          if (hh < a.nh) v += hv[hh];
        io_t* ob = reinterpret_cast<io_t*>(a.o2) + (int64_t)qi * a.o_tok + (int64_t)s * a.o_seq;
        st_act(ob, tid, v + bo);
      }
    }
  }
}

// grid (nseq*nh, cdiv(nq, 4)), 256 threads: wave -> query, lane -> head dim; merges the
// nblk (<= 64) block partials (lane-parallel max / weights, shuffled weights for o).
template <bool IOBF>
__global__ __launch_bounds__(256) void attn_combine_kernel(DecodeAttnArgs a, int nblk) {
  const int qi = blockIdx.y * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (qi >= a.nq) return;
  combine_partials<IOBF, false>(a, blockIdx.x, qi, lane, nblk);
}

__global__ __launch_bounds__(256) void gather_window_kernel(const float* __restrict__ hist, int D,
                                                            const int* __restrict__ cursor,
                                                            const int* __restrict__ n_valid, int pad, int rows,
                                                            float* __restrict__ dst) {
  const int base = *cursor - pad, nv = *n_valid;
  const int64_t n = (int64_t)rows * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / D), d = (int)(i - (int64_t)r * D);
    const int src = base + r;
    dst[i] = (src >= 0 && src < nv) ? hist[(int64_t)src * D + d] : 0.f;
  }
}

// One wave per row: v = LN(x + t)*g + b over D (D % 256 == 0, <= 1024); 4 floats per lane per 256.
__device__ __forceinline__ void ln_row(const float* xr, const void* t, bool t_bf16, int64_t toff, const float* g,
                                       const float* b, float eps, int D, int lane, float4 (&y)[4]) {
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = i * 256 + lane * 4;
    if (c < D) {
      float4 a = *reinterpret_cast<const float4*>(xr + c);
      if (t) {
        if (t_bf16) {
          const uint2 u = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(t) + toff + c);
          a.x += __uint_as_float(u.x << 16); a.y += __uint_as_float(u.x & 0xffff0000u);
          a.z += __uint_as_float(u.y << 16); a.w += __uint_as_float(u.y & 0xffff0000u);
        } else {
          const float4 u = *reinterpret_cast<const float4*>(static_cast<const float*>(t) + toff + c);
          a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
        }
      }
      y[i] = a;
      sum += (a.x + a.y) + (a.z + a.w);
    }
  }
  const float mean = warp_sum(sum) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i * 256 + lane * 4 < D) {
      const float dx = y[i].x - mean, dy = y[i].y - mean, dz = y[i].z - mean, dw = y[i].w - mean;
      q += (dx * dx + dy * dy) + (dz * dz + dw * dw);
    }
  }
  const float rstd = rsqrtf(warp_sum(q) / (float)D + eps);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = i * 256 + lane * 4;
    if (c < D) {
      const float4 gg = *reinterpret_cast<const float4*>(g + c);
      const float4 bb = *reinterpret_cast<const float4*>(b + c);
      y[i].x = (y[i].x - mean) * rstd * gg.x + bb.x;
      y[i].y = (y[i].y - mean) * rstd * gg.y + bb.y;
      y[i].z = (y[i].z - mean) * rstd * gg.z + bb.z;
      y[i].w = (y[i].w - mean) * rstd * gg.w + bb.w;
    }
  }
}

// Single workgroup: every wave reads the cursor before the barrier, thread 0 advances it after.
__global__ __launch_bounds__(256) void enc_finish_kernel(const float* __restrict__ x, const void* t, int t_bf16,
                                                         const float* __restrict__ g, const float* __restrict__ b,
                                                         float eps, int c, int D, float* __restrict__ hist,
                                                         int* cursor, int* mirror) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int cur = *cursor;
  for (int r = wid; r < c; r += 4) {
    float4 y[4];
    ln_row(x + (int64_t)r * D, t, t_bf16, (int64_t)r * D, g, b, eps, D, lane, y);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = i * 256 + lane * 4;
      if (col < D) *reinterpret_cast<float4*>(hist + (int64_t)(cur + r) * D + col) = y[i];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    *cursor = cur + c;
    if (mirror) *mirror = cur + c;
  }
}

// One wave per (frame, slot) row; workgroup 0 / thread 0 advances the decoder cursor (no
// thread of this kernel reads it).
__global__ __launch_bounds__(256) void dec_finish_kernel(const float* __restrict__ x, const void* t, int t_bf16,
                                                         const float* __restrict__ g, const float* __restrict__ b,
                                                         float eps, int c, int C, int D, const float* __restrict__ emb,
                                                         float* __restrict__ scores, int* cursor) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blockIdx.x == 0 && threadIdx.x == 0) *cursor += c;
  if (r >= c * C) return;
  float4 y[4];
  ln_row(x + (int64_t)r * D, t, t_bf16, (int64_t)r * D, g, b, eps, D, lane, y);
  const float* e = emb + (int64_t)(r / C) * D;
  float dot = 0.f, sq = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int col = i * 256 + lane * 4;
    if (col < D) {
      const float4 ev = *reinterpret_cast<const float4*>(e + col);
      dot += (ev.x * y[i].x + ev.y * y[i].y) + (ev.z * y[i].z + ev.w * y[i].w);
      sq += (y[i].x * y[i].x + y[i].y * y[i].y) + (y[i].z * y[i].z + y[i].w * y[i].w);
    }
  }
  dot = warp_sum(dot);
  sq = warp_sum(sq);
  if (lane == 0) scores[r] = dot / sqrtf(sq);
}

// acc += w . y over VE consecutive inputs as VE / 2 packed-pair FMAs (even / odd inputs in the pair's halves)
template <int VE>
__device__ __forceinline__ f32x2 fma_pairs(const f32x2 (&w2)[VE / 2], const float* y, f32x2 acc) {
#pragma unroll
  for (int e = 0; e < VE; e += 4) {
    const float4 q = *reinterpret_cast<const float4*>(y + e);
    acc = __builtin_elementwise_fma(w2[e / 2], f32x2{q.x, q.y}, acc);
    acc = __builtin_elementwise_fma(w2[e / 2 + 1], f32x2{q.z, q.w}, acc);
  }
  return acc;
}

// stream_slot_block (kernels.h).  grid nh, 512 threads; workgroup h = head h.  The two projections run
// weight-vector outer, row inner: a vector is unpacked once for all NR (>= n, padded) rows, and each row's dot
// is a chain of packed-pair FMAs (rows n..NR-1 read unused LDS rows and are never stored).
constexpr int kSlotRows = 16, kSlotD = 256;
template <bool WBF, int NR>
__global__ __launch_bounds__(512) void slot_block_kernel(SlotBlockArgs a) {
  using V = WVec<WBF>;
  constexpr int D = kSlotD, VE = V::VE;
  constexpr int NIN = D / 2 / VE;    // vectors of a half in-projection row
  constexpr int NOUT = kHD / VE;     // vectors of the head's slice of an out-projection row
  __shared__ float ys[kSlotRows][D];
  __shared__ float qs[kSlotRows][kHD], ks[kSlotRows][kHD], vs[kSlotRows][kHD], os[kSlotRows][kHD];
  __shared__ float sc[kSlotRows][8];
  __shared__ int last;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int h = blockIdx.x, n = a.c * a.C, C = a.C;
#ifdef SDIAR_SLOT_STAMPS   // probe build only: phase stamps (100 MHz), printed by thread 0 every 997th launch
  unsigned long long stv[8];
  int nst = 0;
  auto stamp = [&] { stv[nst++] = __builtin_amdgcn_s_memrealtime(); };
#else
  auto stamp = [] {};
#endif
  stamp();
  // thread t < 384: in-projection row (t / 2 / 64) * D + h * 64 + (t / 2) % 64, K half t % 2;
  // thread t < 256: out-projection row t, the head's 64 inputs
  // (unconditional, clamped loads: arrays filled under a branch end up in scratch)
  // this wave's first LN row (x + t) and the LN affine issued ahead of the weights: the LN waits on these
  // alone while the weight slices stream on behind it (loads return in issue order)
  // (no load behind a branch and no use of them before the weights are issued: both t dtypes are read through
  // bounded buffer descriptors, out-of-range and absent t read as 0, and the dtype is picked afterwards)
  const int r0 = min(wid, n - 1);
  const uint32_t eoff = (uint32_t)(r0 * D + lane * 4);
  const float4 xr0 = *reinterpret_cast<const float4*>(a.ln_x + eoff);
  const uint32_t tbytes = a.ln_t ? (uint32_t)(n * D * (a.t_bf16 ? 2 : 4)) : 0u;
  const __amdgpu_buffer_rsrc_t rt =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.ln_t ? a.ln_t : static_cast<const void*>(a.ln_x)), (short)0,
                                        tbytes, 0x00020000);
  const u32x2_t tb = __builtin_amdgcn_raw_buffer_load_b64(rt, eoff * 2, 0, 0);
  const u32x4_t tf = __builtin_amdgcn_raw_buffer_load_b128(rt, eoff * 4, 0, 0);
  const float4 lg = *reinterpret_cast<const float4*>(a.ln_g + lane * 4);
  const float4 lb = *reinterpret_cast<const float4*>(a.ln_b + lane * 4);
  __builtin_amdgcn_sched_barrier(0);   // these loads stay ahead of the weight slices
  const int r2 = min(tid, 6 * kHD - 1) >> 1, kh = tid & 1, sel = r2 / kHD, d2 = r2 % kHD;
  const int64_t rin = ((int64_t)sel * D + h * kHD + d2) * D + kh * (D / 2);
  const int64_t rout = (int64_t)(tid & (D - 1)) * D + h * kHD;
  uint4 win[NIN], wout[NOUT];
#pragma unroll
  for (int v = 0; v < NIN; ++v) win[v] = V::load(a.w_in, rin + v * VE);
#pragma unroll
  for (int v = 0; v < NOUT; ++v) wout[v] = V::load(a.w_out, rout + v * VE);
  __builtin_amdgcn_sched_barrier(0);   // ... and all are issued before the LN's first wait
  // the LN operands enter here (an empty asm that may change them): no LN arithmetic is hoisted above the
  // weight loads, so the wait for its inputs leaves the weights in flight
  float4 xa0 = xr0;
  u32x2_t tbv = tb;
  u32x4_t tfv = tf;
  asm volatile("" : "+v"(xa0.x), "+v"(xa0.y), "+v"(xa0.z), "+v"(xa0.w), "+v"(tbv), "+v"(tfv));
  // y = LN(x + t): one wave per row (every workgroup; workgroup 0 stores the residual stream); ln_row's
  // arithmetic on the prefetched first row, ln_row itself for rows past the 8 waves
  {   // every wave (waves past n redo row n - 1 and store the same values again)
    // x + t with t's dtype selected (not branched on); an absent t reads as zeros
    const bool tb16 = a.t_bf16;
    float4 xa = xa0;
    xa.x += tb16 ? __uint_as_float(tbv[0] << 16) : __uint_as_float(tfv[0]);
    xa.y += tb16 ? __uint_as_float(tbv[0] & 0xffff0000u) : __uint_as_float(tfv[1]);
    xa.z += tb16 ? __uint_as_float(tbv[1] << 16) : __uint_as_float(tfv[2]);
    xa.w += tb16 ? __uint_as_float(tbv[1] & 0xffff0000u) : __uint_as_float(tfv[3]);
    const float mean = warp_sum((xa.x + xa.y) + (xa.z + xa.w)) / (float)D;
    const float dx = xa.x - mean, dy = xa.y - mean, dz = xa.z - mean, dw = xa.w - mean;
    const float rstd = rsqrtf(warp_sum((dx * dx + dy * dy) + (dz * dz + dw * dw)) / (float)D + a.eps);
    float4 y;
    y.x = (xa.x - mean) * rstd * lg.x + lb.x;
    y.y = (xa.y - mean) * rstd * lg.y + lb.y;
    y.z = (xa.z - mean) * rstd * lg.z + lb.z;
    y.w = (xa.w - mean) * rstd * lg.w + lb.w;
    *reinterpret_cast<float4*>(&ys[r0][lane * 4]) = y;
    if (h == 0) *reinterpret_cast<float4*>(a.ln_out + eoff) = y;
  }
  for (int r = wid + 8; r < n; r += 8) {
    float4 y[4];
    ln_row(a.ln_x + (int64_t)r * D, a.ln_t, a.t_bf16, (int64_t)r * D, a.ln_g, a.ln_b, a.eps, D, lane, y);
    *reinterpret_cast<float4*>(&ys[r][lane * 4]) = y[0];
    if (h == 0) *reinterpret_cast<float4*>(a.ln_out + (int64_t)r * D + lane * 4) = y[0];
  }
  // LDS-only barrier: __syncthreads()' workgroup fence would also wait for the weight slices still in flight
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  stamp();
  if (wid < 6) {   // 384 threads: (q|k|v column, K half); waves 6, 7 have no column
    const float b = a.b_in[(int64_t)sel * D + h * kHD + d2];
    float(*dst)[kHD] = sel == 0 ? qs : sel == 1 ? ks : vs;
    const float mul = sel == 0 ? a.scale : 1.f;
    f32x2 acc[NR];
#pragma unroll
    for (int m = 0; m < NR; ++m) acc[m] = f32x2{0.f, 0.f};
#pragma unroll
    for (int v = 0; v < NIN; ++v) {
      f32x2 w2[VE / 2];
#pragma unroll
      for (int e = 0; e < VE / 2; ++e) w2[e] = V::pair(win[v], e);
#pragma unroll
      for (int m = 0; m < NR; ++m) acc[m] = fma_pairs<VE>(w2, &ys[m][kh * (D / 2) + v * VE], acc[m]);
      asm volatile("" ::: "memory");   // keeps each vector's LDS reads in its own iteration (else they are all hoisted and spill)
    }
    // every row stored by every lane (rows n..NR-1 of qs/ks/vs are never read): a store under `m < n` or
    // `kh == 0` lets the compiler sink the row's whole FMA chain behind the branch and spill the LDS operands
#pragma unroll
    for (int m = 0; m < NR; ++m) {
      float t = acc[m].x + acc[m].y;
      t += __shfl_xor(t, 1, 64);   // the two K halves (both lanes of a pair hold the same sum and store it)
      dst[m][d2] = (t + b) * mul;
    }
  }
  __syncthreads();
  stamp();
  // scores of row m = f * C + i against the C slots of frame f, softmax per row
  for (int t = tid; t < n * C; t += 512) {
    const int m = t / C, j = t % C, kr = (m / C) * C + j;
    float s = 0.f;
#pragma unroll 16
    for (int d = 0; d < kHD; ++d) s = fmaf(qs[m][d], ks[kr][d], s);
    sc[m][j] = s;
  }
  __syncthreads();
  if (tid < n) {
    float mx = -INFINITY;
    for (int j = 0; j < C; ++j) mx = fmaxf(mx, sc[tid][j]);
    float l = 0.f;
    for (int j = 0; j < C; ++j) {
      const float e = __expf(sc[tid][j] - mx);
      sc[tid][j] = e;
      l += e;
    }
    const float inv = 1.f / l;
    for (int j = 0; j < C; ++j) sc[tid][j] *= inv;
  }
  __syncthreads();
  for (int t = tid; t < n * kHD; t += 512) {
    const int m = t / kHD, d = t % kHD, f0 = (m / C) * C;
    float o = 0.f;
    for (int j = 0; j < C; ++j) o = fmaf(sc[m][j], vs[f0 + j][d], o);
    os[m][d] = o;
  }
  __syncthreads();
  stamp();
  // out-projection partial of head h for output feature tid, published write-through
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(a.ws, (short)0, 0x7fffffff, 0x00020000);
  if (tid < D) {
    f32x2 acc[NR];
#pragma unroll
    for (int m = 0; m < NR; ++m) acc[m] = f32x2{0.f, 0.f};
#pragma unroll
    for (int v = 0; v < NOUT; ++v) {
      f32x2 w2[VE / 2];
#pragma unroll
      for (int e = 0; e < VE / 2; ++e) w2[e] = V::pair(wout[v], e);
#pragma unroll
      for (int m = 0; m < NR; ++m) acc[m] = fma_pairs<VE>(w2, &os[m][v * VE], acc[m]);
      asm volatile("" ::: "memory");
    }
#pragma unroll
    for (int m = 0; m < NR; ++m)   // rows >= n: an offset past the buffer's range, the store is dropped (no branch)
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[m].x + acc[m].y), rw,
                                            m < n ? (uint32_t)((((int64_t)h * n + m) * D + tid) * 4) : 0xfffffff0u,
                                            0, 16);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  stamp();
  unsigned arrival = 0;
  if (tid == 0) {
    const unsigned nh = gridDim.x;
    arrival = __builtin_amdgcn_atomic_inc32(a.cnt, nh - 1, __ATOMIC_RELAXED, "agent");   // wraps to 0 per launch
    last = arrival == nh - 1;
  }
  __syncthreads();
  stamp();
#ifdef SDIAR_SLOT_STAMPS
  auto report = [&] {
    if (tid == 0 && (arrival / gridDim.x) % 997 == 5)
      printf("SLOTSTAMP h %d last %d ln %llu inproj %llu attn %llu outproj %llu arrive %llu merge %llu\n", h, (int)last,
             stv[1] - stv[0], stv[2] - stv[1], stv[3] - stv[2], stv[4] - stv[3], stv[5] - stv[4],
             nst > 6 ? stv[6] - stv[5] : 0ull);
  };
  if (!last) { report(); return; }
#else
  (void)arrival;
#endif
  if (!last || tid >= D) {
#ifdef SDIAR_SLOT_STAMPS
    if (tid == 0) { stamp(); report(); }
#endif
    return;
  }
  const float bo = a.b_out[tid];
  const int nh = gridDim.x;
  // every row's head partials loaded before the first sum (one round trip);
  // rows past n re-read row n - 1 and store its value again (no load behind a branch)
  constexpr int NHM = kSlotD / kHD;   // = nh (the launch requires nh * 64 == D == kSlotD)
  float pv[NR][NHM];
#pragma unroll
  for (int m = 0; m < NR; ++m)
#pragma unroll
    for (int hh = 0; hh < NHM; ++hh)
      pv[m][hh] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
          rw, (uint32_t)((((int64_t)min(hh, nh - 1) * n + min(m, n - 1)) * D + tid) * 4), 0, 16));
#pragma unroll
  for (int m = 0; m < NR; ++m) {
    float v = 0.f;
#pragma unroll
    for (int hh = 0; hh < NHM; ++hh)
      if (hh < nh) v += pv[m][hh];
    v += bo;
    const int64_t o = (int64_t)min(m, n - 1) * D + tid;
    if (a.out_bf16) static_cast<uint16_t*>(a.out)[o] = f2bf_bits(v);
    else static_cast<float*>(a.out)[o] = v;
  }
#ifdef SDIAR_SLOT_STAMPS
  if (tid == 0) { stamp(); report(); }
#endif
}

// stream_ffn_pair (kernels.h).  grid G = F / FC, 256 threads; workgroup g owns hidden units [g FC, (g + 1) FC):
//   y = LN(x + t) (every workgroup; workgroup 0 stores it as the next residual), h_u = relu(y . W1[u] + b1[u]) for
//   its FC units (LPU = 256 / FC lanes per unit, packed K pieces of 4 so the LDS reads are conflict-free), then
//   thread j's partial of output feature j over those units, published write-through; the last workgroup to count
//   itself sums the G partials in workgroup order (4 g-parts per column quad, then the parts in order) + b2.
// One launch per FFN instead of two: the hidden layer never leaves the workgroup (fp32; the two-launch path
// stores it as the activation dtype), and the down-projection's split-K seam is a last-arriver merge.
template <bool WBF, int NR, int FC, int G>
__global__ __launch_bounds__(256) void ffn_pair_kernel(FfnPairArgs a) {
  using V = WVec<WBF>;
  constexpr int D = kSlotD, VE = V::VE;
  constexpr int LPU = 256 / FC;          // lanes per hidden unit
  constexpr int NJ = D / 4 / LPU;        // K pieces of 4 per lane
  constexpr int W2V = FC / VE;           // 16-B vectors of a thread's W2 slice
  constexpr int GP = G / 4;              // partials per thread and row in the merge
  constexpr int RB = GP >= 48 ? 1 : 48 / GP;   // rows merged per round trip (<= 48 loads in flight)
  static_assert(FC * LPU == 256 && NJ * LPU * 4 == D && W2V * VE == FC && G % 4 == 0, "ffn_pair geometry");
  typedef std::conditional_t<WBF, uint2, uint4> P4;
  __shared__ float ys[NR][D];
  __shared__ float hs[NR][FC];
  __shared__ float4 red[4][RB][64];
  __shared__ int last;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = blockIdx.x, n = a.n;
  const int u = tid / LPU, kp = tid % LPU;
  // the thread's weights first, as one batch: W1 pieces (unit u, K = 4 (kp + j LPU) ..) and its W2 slice (row tid)
  const int64_t urow = (int64_t)(g * FC + u) * D;
  P4 w1[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
    w1[j] = *reinterpret_cast<const P4*>(static_cast<const char*>(a.w1) + (urow + 4 * (kp + j * LPU)) * (WBF ? 2 : 4));
  uint4 w2[W2V];
#pragma unroll
  for (int v = 0; v < W2V; ++v) w2[v] = V::load(a.w2, (int64_t)tid * a.F + g * FC + v * VE);
  const float b1u = a.b1[g * FC + u];
  __builtin_amdgcn_sched_barrier(0);
  // y = LN(x + t), one wave per row (rows n..NR-1 repeat row n - 1: no uninitialised LDS is ever read)
  for (int r = wid; r < NR; r += 4) {
    const int rr = min(r, n - 1);
    float4 y[4];
    ln_row(a.ln_x + (int64_t)rr * D, a.ln_t, a.t_bf16, (int64_t)rr * D, a.ln_g, a.ln_b, a.eps, D, lane, y);
    *reinterpret_cast<float4*>(&ys[r][lane * 4]) = y[0];
    if (g == 0 && r < n) *reinterpret_cast<float4*>(a.ln_out + (int64_t)r * D + lane * 4) = y[0];
  }
  __syncthreads();
  // hidden units of the chunk
  float acc[NR];
#pragma unroll
  for (int m = 0; m < NR; ++m) acc[m] = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    float wv[4];
    if constexpr (WBF) {
      wv[0] = __uint_as_float(w1[j].x << 16); wv[1] = __uint_as_float(w1[j].x & 0xffff0000u);
      wv[2] = __uint_as_float(w1[j].y << 16); wv[3] = __uint_as_float(w1[j].y & 0xffff0000u);
    } else {
      wv[0] = __uint_as_float(w1[j].x); wv[1] = __uint_as_float(w1[j].y);
      wv[2] = __uint_as_float(w1[j].z); wv[3] = __uint_as_float(w1[j].w);
    }
    const int k = 4 * (kp + j * LPU);
#pragma unroll
    for (int m = 0; m < NR; ++m) {
      const float4 y = *reinterpret_cast<const float4*>(&ys[m][k]);
      acc[m] = fmaf(y.x, wv[0], acc[m]);
      acc[m] = fmaf(y.y, wv[1], acc[m]);
      acc[m] = fmaf(y.z, wv[2], acc[m]);
      acc[m] = fmaf(y.w, wv[3], acc[m]);
    }
  }
#pragma unroll
  for (int m = 0; m < NR; ++m) {
#pragma unroll
    for (int o = 1; o < LPU; o <<= 1) acc[m] += __shfl_xor(acc[m], o, 64);
    if (kp == 0) hs[m][u] = fmaxf(acc[m] + b1u, 0.f);
  }
  __syncthreads();
  // partial of output feature tid over the chunk's units, published write-through
  float pr[NR];
#pragma unroll
  for (int m = 0; m < NR; ++m) pr[m] = 0.f;
#pragma unroll
  for (int v = 0; v < W2V; ++v)
#pragma unroll
    for (int e = 0; e < VE; ++e) {
      const float w = V::at(w2[v], e);
#pragma unroll
      for (int m = 0; m < NR; ++m) pr[m] = fmaf(hs[m][v * VE + e], w, pr[m]);
    }
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(a.ws, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int m = 0; m < NR; ++m)   // rows >= n: an offset past the buffer's range, the store is dropped (no branch)
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(pr[m]), rw,
                                          m < n ? (uint32_t)((((int64_t)g * n + m) * D + tid) * 4) : 0xfffffff0u, 0, 16);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0)   // wrapping increment: back at 0 after every complete launch
    last = __builtin_amdgcn_atomic_inc32(a.cnt, (unsigned)G - 1, __ATOMIC_RELAXED, "agent") == (unsigned)G - 1;
  __syncthreads();
  if (!last) return;
  // merge: thread (gp, q) sums column quad q over workgroups [gp GP, (gp + 1) GP) for RB rows per round trip
  const int q = tid & 63, gp = tid >> 6;
  for (int m0 = 0; m0 < n; m0 += RB) {
    u32x4_t pv[RB][GP];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int mr = min(m0 + r, n - 1);
#pragma unroll
      for (int i = 0; i < GP; ++i)
        pv[r][i] = __builtin_amdgcn_raw_buffer_load_b128(
            rw, (uint32_t)((((int64_t)(gp * GP + i) * n + mr) * D + q * 4) * 4), 0, 16);
    }
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int i = 0; i < GP; ++i) {
        s.x += __uint_as_float(pv[r][i][0]); s.y += __uint_as_float(pv[r][i][1]);
        s.z += __uint_as_float(pv[r][i][2]); s.w += __uint_as_float(pv[r][i][3]);
      }
      red[gp][r][q] = s;
    }
    __syncthreads();
    if (tid < 64 * RB) {
      const int r = tid >> 6, m = m0 + r;
      if (m < n) {
        const float4 bb = *reinterpret_cast<const float4*>(a.b2 + q * 4);
        float4 v = red[0][r][q];
#pragma unroll
        for (int k = 1; k < 4; ++k) {
          const float4 t = red[k][r][q];
          v.x += t.x; v.y += t.y; v.z += t.z; v.w += t.w;
        }
        v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w;
        const int64_t o = (int64_t)m * D + q * 4;
        if (a.out_bf16) {
          uint2 hv;
          hv.x = (uint32_t)f2bf_bits(v.x) | ((uint32_t)f2bf_bits(v.y) << 16);
          hv.y = (uint32_t)f2bf_bits(v.z) | ((uint32_t)f2bf_bits(v.w) << 16);
          *reinterpret_cast<uint2*>(static_cast<uint16_t*>(a.out) + o) = hv;
        } else {
          *reinterpret_cast<float4*>(static_cast<float*>(a.out) + o) = v;
        }
      }
    }
    __syncthreads();
  }
}

__global__ void cursor_advance_kernel(int* cursor, int by, int* mirror) {
  if (threadIdx.x == 0) {
    const int v = *cursor + by;
    *cursor = v;
    if (mirror) *mirror = v;
  }
}

}  // namespace

void kv_append(const void* src, int64_t ld_src_bytes, int rows, int width_bytes, void* dst, int64_t ld_dst_bytes,
               const int* cursor, int mult, hipStream_t st) {
  SD_CHECK(width_bytes % 16 == 0 && ld_src_bytes % 16 == 0 && ld_dst_bytes % 16 == 0, kErrInvalid,
           "kv_append: rows must be 16-byte multiples");
  SD_CHECK(((uintptr_t)src | (uintptr_t)dst) % 16 == 0, kErrInvalid, "kv_append: unaligned buffers");
  if (rows <= 0) return;
  const int w16 = width_bytes / 16;
  const int64_t n = (int64_t)rows * w16;
  ProfScope prof("kv_append", 0.0, 2.0 * rows * width_bytes, st);
  const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(kv_append_kernel, dim3(blocks), dim3(256), 0, st, static_cast<const uint4*>(src),
                     ld_src_bytes / 16, rows, w16, static_cast<uint4*>(dst), ld_dst_bytes / 16, cursor, mult);
  SD_LAUNCH_CHECK();
}

int attn_decode_blocks(int max_keys) {
  return std::min(cdiv(max_keys, 256), kMaxBlk);
}

template <bool IOBF, bool FUSED>
static void launch_decode_q(const DecodeAttnArgs& a, dim3 g1, hipStream_t st) {
  if (a.nq == 1) hipLaunchKernelGGL((attn_decode_kernel<IOBF, 1, FUSED>), g1, dim3(256), 0, st, a);
  else if (a.nq <= 8) hipLaunchKernelGGL((attn_decode_kernel<IOBF, 8, FUSED>), g1, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((attn_decode_kernel<IOBF, 32, FUSED>), g1, dim3(256), 0, st, a);
  SD_LAUNCH_CHECK();
}

template <bool IOBF>
static bool launch_decode(const DecodeAttnArgs& a, int nblk, hipStream_t st) {
  const int nsh = a.nseq * a.nh;
  const dim3 g1(nblk, nsh), g2(nsh, cdiv(a.nq, 4));
  if (a.cnt) {
    // the out-projection merge for one query per sequence (the 1-frame chunks of the latency mode; with more
    // queries its per-query partials push the kernel past the register budget)
    const bool op = a.nq == 1 && a.wo && a.bo && a.o2 && a.ws2 && a.cnt2 && a.nh * kHD <= 256 &&
                    reinterpret_cast<uintptr_t>(a.wo) % 16 == 0;
    if (op) {
      hipLaunchKernelGGL((attn_decode_kernel<IOBF, 1, true, true>), g1, dim3(256), 0, st, a);
      SD_LAUNCH_CHECK();
    } else {
      launch_decode_q<IOBF, true>(a, g1, st);
    }
    return op;
  }
  launch_decode_q<IOBF, false>(a, g1, st);
  hipLaunchKernelGGL(attn_combine_kernel<IOBF>, g2, dim3(256), 0, st, a, nblk);
  SD_LAUNCH_CHECK();
  return false;
}

bool attn_decode(const DecodeAttnArgs& a, hipStream_t st) {
  SD_CHECK(a.hd == kHD, kErrInvalid, "attn_decode: head dim must be 64");
  SD_CHECK(a.nq >= 1 && a.nq <= kMaxQ, kErrInvalid, "attn_decode: 1..32 queries per sequence");
  const int nblk = attn_decode_blocks(a.max_keys);
  SD_CHECK(a.n_blocks >= nblk, kErrInvalid, "attn_decode: workspace too small");
  const int nsh = a.nseq * a.nh;
  // bytes: upper bound (full history), the graph does not know the cursor
  ProfScope prof("attn_decode", 4.0 * a.max_keys * kHD * nsh * a.nq,
                 2.0 * a.max_keys * kHD * nsh * (a.io_bf16 ? 2 : 4), st);
  return a.io_bf16 ? launch_decode<true>(a, nblk, st) : launch_decode<false>(a, nblk, st);
}

template <int NR>
static void launch_slot_block(const SlotBlockArgs& a, hipStream_t st) {
  if (a.w_bf16) hipLaunchKernelGGL((slot_block_kernel<true, NR>), dim3(a.nh), dim3(512), 0, st, a);
  else hipLaunchKernelGGL((slot_block_kernel<false, NR>), dim3(a.nh), dim3(512), 0, st, a);
  SD_LAUNCH_CHECK();
}

bool stream_slot_block(const SlotBlockArgs& a, hipStream_t st) {
  const int n = a.c * a.C;
  if (a.D != kSlotD || a.nh * kHD != a.D || a.nh > 8 || n < 1 || n > kSlotRows || a.C > 8 || !a.ws || !a.cnt)
    return false;
  ProfScope prof("slot_block", 2.0 * n * a.D * 4.0 * a.D + 4.0 * n * a.C * a.D, (a.w_bf16 ? 2.0 : 4.0) * 4 * a.D * a.D, st);
  if (n <= 2) launch_slot_block<2>(a, st);
  else if (n <= 4) launch_slot_block<4>(a, st);
  else if (n <= 6) launch_slot_block<6>(a, st);
  else if (n <= 8) launch_slot_block<8>(a, st);
  else launch_slot_block<kSlotRows>(a, st);
  return true;
}

template <bool WBF, int NR, int FC, int G>
static void launch_ffn_pair_t(const FfnPairArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((ffn_pair_kernel<WBF, NR, FC, G>), dim3(G), dim3(256), 0, st, a);
  SD_LAUNCH_CHECK();
}

template <int NR, int FC, int G>
static void launch_ffn_pair(const FfnPairArgs& a, hipStream_t st) {
  if (a.w_bf16) launch_ffn_pair_t<true, NR, FC, G>(a, st);
  else launch_ffn_pair_t<false, NR, FC, G>(a, st);
}

bool stream_ffn_pair(const FfnPairArgs& a, hipStream_t st) {
  if (a.D != kSlotD || a.F != 2048 || a.n < 1 || a.n > 8 || !a.ws || !a.cnt || !a.ln_g || !a.ln_b || !a.ln_out)
    return false;
  auto al = [](const void* p) { return reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  if (!al(a.w1) || !al(a.w2) || !al(a.ln_x) || !al(a.ln_out) || !al(a.out) || !al(a.ws) || !al(a.b2)) return false;
  ProfScope prof("ffn_pair", 4.0 * a.n * a.D * a.F, (a.w_bf16 ? 2.0 : 4.0) * 2 * a.D * a.F, st);
  // one row (the encoder's chunk of 1): 128 workgroups of 16 units; more rows: 64 of 32 (half the partials to merge)
  if (a.n == 1) launch_ffn_pair<1, 16, 128>(a, st);
  else launch_ffn_pair<8, 32, 64>(a, st);
  return true;
}

void gather_window(const float* hist, int D, const int* cursor, const int* n_valid, int pad, int rows, float* dst,
                   hipStream_t st) {
  const int64_t n = (int64_t)rows * D;
  ProfScope prof("gather_window", 0.0, 8.0 * n, st);
  const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(gather_window_kernel, dim3(blocks), dim3(256), 0, st, hist, D, cursor, n_valid, pad, rows, dst);
  SD_LAUNCH_CHECK();
}

void stream_enc_finish(const float* x, const void* t, bool t_bf16, const float* g, const float* b, float eps, int c,
                       int D, float* hist, int* cursor, int* mirror, hipStream_t st) {
  SD_CHECK(D % 256 == 0 && D <= 1024, kErrInvalid, "stream_enc_finish: D must be 256/512/768/1024");
  ProfScope prof("stream_finish", 8.0 * c * D, 12.0 * c * D, st);
  hipLaunchKernelGGL(enc_finish_kernel, dim3(1), dim3(256), 0, st, x, t, (int)t_bf16, g, b, eps, c, D, hist, cursor,
                     mirror);
  SD_LAUNCH_CHECK();
}

void stream_dec_finish(const float* x, const void* t, bool t_bf16, const float* g, const float* b, float eps, int c,
                       int C, int D, const float* emb, float* scores, int* cursor, hipStream_t st) {
  SD_CHECK(D % 256 == 0 && D <= 1024, kErrInvalid, "stream_dec_finish: D must be 256/512/768/1024");
  ProfScope prof("stream_finish", 12.0 * c * C * D, 8.0 * c * C * D, st);
  hipLaunchKernelGGL(dec_finish_kernel, dim3(cdiv(c * C, 4)), dim3(256), 0, st, x, t, (int)t_bf16, g, b, eps, c, C, D,
                     emb, scores, cursor);
  SD_LAUNCH_CHECK();
}

void cursor_advance(int* cursor, int by, int* mirror, hipStream_t st) {
  hipLaunchKernelGGL(cursor_advance_kernel, dim3(1), dim3(64), 0, st, cursor, by, mirror);
  SD_LAUNCH_CHECK();
}

}  // namespace sd
