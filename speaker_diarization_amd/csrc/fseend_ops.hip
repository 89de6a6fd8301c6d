// FS-EEND glue kernels for gfx950 (speaker_diarization/fs_eend/fs_eend.py).
//   row_l2norm   emb / torch.norm(emb, dim=-1)                 :87 (and attractors, :89)
//   slot_init    convert(cat(emb repeated over C, slot PE))    :129-130, decomposed as
//                emb·W_embᵀ (one GEMM over T rows) + (pe_c·W_peᵀ + b) (C rows, per launch)
//   slot_scores  emb · (att / |att|)ᵀ per frame                 :89-90
// One wavefront per row; D = 256 -> 4 floats per lane.
#include "common.h"
#include "kernels.h"
#include "prof.h"

namespace sd {
namespace {

// slabs > 1: x is the sum of `slabs` split-K partial slabs x + k * rows * D (summed in slab order).
__global__ __launch_bounds__(256) void row_l2norm_kernel(const float* __restrict__ x, int rows, int D,
                                                         float* __restrict__ y, int slabs) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const float* xr = x + (int64_t)r * D;
  constexpr int kMaxPer = 8;   // D <= 512
  float v[kMaxPer];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < kMaxPer; ++j) {
    const int i = lane + 64 * j;
    float a = 0.f;
    if (i < D) {
      a = xr[i];
      for (int k = 1; k < slabs; ++k) a += xr[(int64_t)k * rows * D + i];
    }
    v[j] = a;
    s = fmaf(a, a, s);
  }
  s = warp_sum(s);
  const float n = sqrtf(s);
#pragma unroll
  for (int j = 0; j < kMaxPer; ++j) {
    const int i = lane + 64 * j;
    if (i < D) y[(int64_t)r * D + i] = v[j] / n;
  }
}

// out[(t*C + c), :] = g[t, :] + p[c, :]
__global__ __launch_bounds__(256) void slot_init_kernel(const float* __restrict__ g, int T, int C, int D,
                                                        const float* __restrict__ p, float* __restrict__ out) {
  const int64_t n = (int64_t)T * C * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int d = (int)(i % D);
    const int64_t tc = i / D;
    const int c = (int)(tc % C);
    const int64_t t = tc / C;
    out[i] = g[t * D + d] + p[(int64_t)c * D + d];
  }
}

// One wave per frame: scores[t, c] = emb[t]·att[t,c] / |att[t,c]|; optionally the
// normalised attractors are written back in place.
__global__ __launch_bounds__(256) void slot_scores_kernel(const float* __restrict__ emb, float* __restrict__ att,
                                                          int T, int C, int D, float* __restrict__ scores,
                                                          int write_norm) {
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (t >= T) return;
  const float* e = emb + (int64_t)t * D;
  for (int c = 0; c < C; ++c) {
    float* a = att + ((int64_t)t * C + c) * D;
    float dot = 0.f, sq = 0.f;
    for (int i = lane; i < D; i += 64) {
      dot = fmaf(e[i], a[i], dot);
      sq = fmaf(a[i], a[i], sq);
    }
    dot = warp_sum(dot);
    sq = warp_sum(sq);
    const float n = sqrtf(sq);
    if (lane == 0) scores[(int64_t)t * C + c] = dot / n;
    if (write_norm)
      for (int i = lane; i < D; i += 64) a[i] = a[i] / n;
  }
}

}  // namespace

void row_l2norm(const float* x, int rows, int D, float* y, hipStream_t st, int slabs) {
  if (rows <= 0) return;
  SD_CHECK(D <= 512 && slabs >= 1, kErrInvalid, "row_l2norm: D > 512");
  ProfScope prof("row_l2norm", 3.0 * rows * D, 4.0 * (slabs + 1) * rows * D, st);
  hipLaunchKernelGGL(row_l2norm_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, st, x, rows, D, y, slabs);
  SD_LAUNCH_CHECK();
}

void slot_init(const float* g, int T, int C, int D, const float* p, float* out, hipStream_t st) {
  const int64_t n = (int64_t)T * C * D;
  if (n <= 0) return;
  ProfScope prof("slot_init", (double)n, 4.0 * ((double)T * D + n), st);
  const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(slot_init_kernel, dim3(blocks), dim3(256), 0, st, g, T, C, D, p, out);
  SD_LAUNCH_CHECK();
}

void slot_scores(const float* emb, float* att, int T, int C, int D, float* scores, bool write_norm,
                 hipStream_t st) {
  if (T <= 0) return;
  ProfScope prof("slot_scores", 4.0 * T * C * D, 4.0 * ((double)T * D + (double)T * C * D * (write_norm ? 2 : 1)),
                 st);
  hipLaunchKernelGGL(slot_scores_kernel, dim3(cdiv(T, 4)), dim3(256), 0, st, emb, att, T, C, D, scores,
                     (int)write_norm);
  SD_LAUNCH_CHECK();
}

}  // namespace sd
