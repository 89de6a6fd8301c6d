// Shared helpers for the gfx950 diarization kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include <type_traits>

namespace sd {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

// Status codes (mirrored in include/sdiar.h).
enum Status : int {
  kOk = 0,
  kErrInvalid = -1,   // ValueError in the reference (unknown type / bad argument)
  kErrShape = -2,     // AssertionError in the reference (length mismatch)
  kErrParam = -3,     // load_state_dict missing / unexpected key or wrong size
  kErrHip = -4,       // HIP runtime failure
  kErrState = -5,     // handle used before finalize / after destroy
};

void set_error(const std::string& msg);
const char* last_error();

struct Error {
  int code;
  std::string msg;
};

#define SD_HIP(expr)                                                              \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess) {                                                       \
      throw ::sd::Error{::sd::kErrHip, std::string(#expr) + ": " + hipGetErrorString(_e)}; \
    }                                                                             \
  } while (0)

#define SD_CHECK(cond, code, msg)                                                 \
  do {                                                                            \
    if (!(cond)) throw ::sd::Error{(code), (msg)};                                \
  } while (0)

#define SD_LAUNCH_CHECK() SD_HIP(hipGetLastError())

__host__ __device__ inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// Round-to-nearest-even fp32 -> bf16 bits (finite inputs; NaN kept NaN by the
// explicit check so a poisoned activation stays visible).
__device__ __forceinline__ uint16_t f2bf_bits(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// Two fp32 -> packed bf16 pair with v_cvt_pk_bf16_f32 (round-to-nearest-even, the
// same bits as f2bf_bits for finite inputs; NaN stays NaN).
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  bf16x2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

// 16-B-per-lane global -> LDS DMA (global_load_lds_dwordx4): lane i's 16 B land at lds + 16 i.  Issued as
// inline asm rather than __builtin_amdgcn_global_load_lds on purpose: the compiler's wait-count pass knows
// about a builtin LDS DMA in flight and then puts s_waitcnt vmcnt(0) in front of EVERY later LDS access it
// cannot prove disjoint (all of one dynamic LDS array) - draining a multi-stage DMA ring at each fragment
// read.  Callers own the ordering: a counted s_waitcnt vmcnt(N) + barrier before the slot is read.
// `lds` must be wave-uniform (it goes to M0).
__device__ __forceinline__ void dma_lds16(const void* g, const void __attribute__((address_space(3)))* lds) {
  const uint32_t m0v = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>(lds));
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m0v), "v"(g) : "memory", "m0");
}

// The buffer form (bounds-checked by the resource: out-of-range lanes land as zeros), same contract.
__device__ __forceinline__ void dma_lds16_buf(__amdgpu_buffer_rsrc_t rsrc, uint32_t voff,
                                              const void __attribute__((address_space(3)))* lds) {
  const uint32_t m0v = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>(lds));
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m0v), "v"(voff),
               "s"(rsrc)
               : "memory", "m0");
}

__device__ __forceinline__ float bf_bits2f(uint16_t b) {
  return __uint_as_float(((uint32_t)b) << 16);
}

// Element access for activations stored as fp32 or bf16 (uint16 bits).
__device__ __forceinline__ float ld_act(const float* p, int64_t i) { return p[i]; }
__device__ __forceinline__ float ld_act(const uint16_t* p, int64_t i) { return bf_bits2f(p[i]); }
__device__ __forceinline__ void st_act(float* p, int64_t i, float v) { p[i] = v; }
__device__ __forceinline__ void st_act(uint16_t* p, int64_t i, float v) { p[i] = f2bf_bits(v); }

template <bool BF>
using act_t = typename std::conditional<BF, uint16_t, float>::type;

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }
// Sigmoid with the hardware reciprocal (v_rcp_f32, <= 1 ulp) instead of an IEEE division (about ten
// instructions: div_scale / rcp / fma chain / div_fmas / div_fixup) - for the GLU / SiLU epilogues of
// the hot GEMM and conv kernels.  sigmoid_rcp(-inf) = 0, (+inf) = 1, NaN stays NaN.
__device__ __forceinline__ float sigmoid_rcp(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

// XCD-aware tile order (cdna_hip_programming.md T1, bijective form): workgroups
// are dealt round-robin over the 8 XCDs, so remap the linear id such that
// consecutive logical tiles (the N-tiles sharing one A row panel) run on the
// same XCD and hit its L2.  Returns the logical tile id.
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

enum Act : int { kActNone = 0, kActRelu = 1, kActSigmoid = 2, kActSilu = 3 };

__device__ __forceinline__ float apply_act(float v, int act) {
  switch (act) {
    case kActRelu: return fmaxf(v, 0.f);
    case kActSigmoid: return 1.f / (1.f + expf(-v));
    case kActSilu: return v / (1.f + expf(-v));
    default: return v;
  }
}

}  // namespace sd
