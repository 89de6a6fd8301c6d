// Probe for the open attn_long select-form failure: the select form computes each
// key's mask as the sequence below, 16 times per tile, and the GPU run gave all-masked rows.  This replays that
// exact instruction sequence (copied from the disassembly of attn_long_kernel<64, 1>'s select form) on MI355X,
// back to back as in the kernel, and compares every lane's mask bit with the host's answer:
//   v_cmp_gt_i32_e32 vcc, klen, key          key < klen
//   s_and_saveexec_b64 s[4:5], vcc
//   v_cmp_le_i32_e32 vcc, key, q              key <= q   (only lanes with key < klen active)
//   s_or_b64 s[0:1], notcausal, vcc           VALU-written VCC read by the very next SALU instruction
//   s_and_b64 s[0:1], s[0:1], exec
//   s_or_b64 exec, exec, s[4:5]
//   v_cndmask_b32 out, 0, 1, s[0:1]
// Variant 1 puts `s_nop 4` between the v_cmp and the s_or (a wait-state control).
//   hipcc -O3 --offload-arch=gfx950 tools/probe/vcc_salu.hip -o /tmp/vcc_salu && /tmp/vcc_salu
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

template <int NOP>
__global__ __launch_bounds__(64) void probe(int* out, int nq) {
  const int lane = threadIdx.x;
  const int cfg = blockIdx.x;              // klen = cfg % 80, q = (cfg / 80) % 80 - 8, notcausal = cfg / 6400
  const int klen = __builtin_amdgcn_readfirstlane(cfg % 80);
  const int qv = (cfg / 80) % 80 - 8;
  const int nc = __builtin_amdgcn_readfirstlane(cfg / 6400);
  int acc = 0;
#pragma unroll
  for (int rep = 0; rep < 16; ++rep) {     // 16 masks per tile, keys lane + rep
    const int key = lane + rep;
    int bit;
    if (NOP)
      asm volatile(
          "s_cmp_lg_u32 %4, 0\n\t"
          "s_cselect_b64 s[2:3], -1, 0\n\t"
          "v_cmp_gt_i32_e32 vcc, %1, %3\n\t"
          "s_and_saveexec_b64 s[4:5], vcc\n\t"
          "v_cmp_le_i32_e32 vcc, %3, %2\n\t"
          "s_nop 4\n\t"
          "s_or_b64 s[0:1], s[2:3], vcc\n\t"
          "s_and_b64 s[0:1], s[0:1], exec\n\t"
          "s_or_b64 exec, exec, s[4:5]\n\t"
          "v_cndmask_b32_e64 %0, 0, 1, s[0:1]"
          : "=v"(bit)
          : "s"(klen), "v"(qv), "v"(key), "s"(nc)
          : "s0", "s1", "s2", "s3", "s4", "s5", "vcc", "exec", "scc");
    else
      asm volatile(
          "s_cmp_lg_u32 %4, 0\n\t"
          "s_cselect_b64 s[2:3], -1, 0\n\t"
          "v_cmp_gt_i32_e32 vcc, %1, %3\n\t"
          "s_and_saveexec_b64 s[4:5], vcc\n\t"
          "v_cmp_le_i32_e32 vcc, %3, %2\n\t"
          "s_or_b64 s[0:1], s[2:3], vcc\n\t"
          "s_and_b64 s[0:1], s[0:1], exec\n\t"
          "s_or_b64 exec, exec, s[4:5]\n\t"
          "v_cndmask_b32_e64 %0, 0, 1, s[0:1]"
          : "=v"(bit)
          : "s"(klen), "v"(qv), "v"(key), "s"(nc)
          : "s0", "s1", "s2", "s3", "s4", "s5", "vcc", "exec", "scc");
    acc |= bit << rep;
  }
  out[cfg * 64 + lane] = acc;
}

int main() {
  const int n = 2 * 6400;
  int* d;
  hipMalloc(&d, sizeof(int) * n * 64);
  std::vector<int> h(n * 64);
  int bad_total = 0;
  for (int v = 0; v < 2; ++v) {
    hipMemset(d, 0xff, sizeof(int) * n * 64);
    for (int rep = 0; rep < 20; ++rep) {
      if (v == 0) hipLaunchKernelGGL(probe<0>, dim3(n), dim3(64), 0, 0, d, n);
      else hipLaunchKernelGGL(probe<1>, dim3(n), dim3(64), 0, 0, d, n);
    }
    hipMemcpy(h.data(), d, sizeof(int) * n * 64, hipMemcpyDeviceToHost);
    long bad = 0, lanes = 0;
    for (int cfg = 0; cfg < n; ++cfg) {
      const int klen = cfg % 80, q = (cfg / 80) % 80 - 8, nc = cfg / 6400;
      for (int lane = 0; lane < 64; ++lane) {
        int want = 0;
        for (int rep = 0; rep < 16; ++rep) {
          const int key = lane + rep;
          want |= (key < klen && (nc || key <= q)) << rep;
        }
        ++lanes;
        if (h[cfg * 64 + lane] != want) {
          if (bad < 5)
            printf("variant %d cfg %d (klen %d q %d notcausal %d) lane %d: got %04x want %04x\n", v, cfg, klen, q, nc,
                   lane, h[cfg * 64 + lane], want);
          ++bad;
        }
      }
    }
    printf("variant %d (%s): %ld of %ld lanes wrong\n", v, v ? "s_nop 4 after v_cmp" : "as compiled", bad, lanes);
    bad_total += bad;
  }
  hipFree(d);
  return 0;
}
