// Host-side parameter store: state_dict tensors by their reference key names,
// eval-BatchNorm folding and packing of weights into the conv_gemm layout.
#pragma once
#include <map>
#include <memory>
#include <string>
#include <vector>
#include "common.h"

namespace sd {

struct HostTensor {
  std::vector<int64_t> shape;
  std::vector<float> data;
  int64_t numel() const { return (int64_t)data.size(); }
};

// Device allocation owned by a model handle.
class DeviceArena {
 public:
  ~DeviceArena() { release(); }
  void* alloc(size_t bytes) {
    void* p = nullptr;
    if (bytes == 0) bytes = 4;
    SD_HIP(hipMalloc(&p, bytes));
    ptrs_.push_back(p);
    total_ += bytes;
    return p;
  }
  float* upload(const std::vector<float>& v) {
    float* p = static_cast<float*>(alloc(v.size() * sizeof(float)));
    SD_HIP(hipMemcpy(p, v.data(), v.size() * sizeof(float), hipMemcpyHostToDevice));
    return p;
  }
  void release() {
    for (void* p : ptrs_) (void)hipFree(p);
    ptrs_.clear();
    total_ = 0;
  }
  size_t total() const { return total_; }

 private:
  std::vector<void*> ptrs_;
  size_t total_ = 0;
};

// Pinned, device-mapped host ints per handle, one slot per persistent LSTM recurrence of a forward.  A
// launch that lost co-residency stores 1 into its slot from the kernel (system scope); nothing on the
// device ever stores 0, so reports accumulate across forwards until take() reads and clears every slot
// (callers use it once the stream has completed, in the same call, or on the next call).
class PinnedFlags {
 public:
  static constexpr int kSlots = 4;
  PinnedFlags() {
    SD_HIP(hipHostMalloc(reinterpret_cast<void**>(&p_), kSlots * sizeof(int), hipHostMallocMapped));
    for (int i = 0; i < kSlots; ++i) p_[i] = 0;
    SD_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_), p_, 0));
  }
  ~PinnedFlags() { if (p_) (void)hipHostFree(p_); }
  PinnedFlags(const PinnedFlags&) = delete;
  PinnedFlags& operator=(const PinnedFlags&) = delete;
  int* get(int slot) const { return d_ + slot; }   // device address of the slot (kernel argument)
  int take() {
    int any = 0;
    for (int i = 0; i < kSlots; ++i) any |= __atomic_exchange_n(p_ + i, 0, __ATOMIC_ACQ_REL);
    return any;
  }
  // kErrHip if a recurrence of an earlier launch on the handle timed out (its outputs are NaN)
  void raise_if_set(const char* what = "lstm: a persistent LSTM launch lost workgroup co-residency "
                                       "(its outputs were poisoned with NaN)") {
    SD_CHECK(take() == 0, kErrHip, what);
  }

 private:
  int* p_ = nullptr;
  int* d_ = nullptr;
};

struct Folded {        // per-channel affine y = x*scale + shift
  const float* scale = nullptr;
  const float* shift = nullptr;
};

struct PackedW {       // Wt[N][K] for conv_gemm (bf16 bits or fp32)
  const void* w = nullptr;
  int N = 0, K = 0, Cin = 0, kh = 1, kw = 1;
};

class ParamStore {
 public:
  void set(const std::string& name, const float* data, const int64_t* shape, int ndim);
  bool has(const std::string& name) const { return t_.count(name) > 0; }
  const HostTensor& get(const std::string& name) const;
  void mark(const std::string& name) const { used_[name] = true; }
  // Keys that were provided but never consumed (reference "unexpected keys"),
  // ignoring BatchNorm num_batches_tracked counters.
  std::vector<std::string> unused() const;

  // Eval BatchNorm (eps 1e-5) as scale/shift; optional preceding conv bias folded in.
  void bn_fold(const std::string& prefix, std::vector<float>& scale, std::vector<float>& shift,
               const std::string& conv_bias = "", float eps = 1e-5f) const;

  // Pack a Conv1d (N, Cin, k) / Conv2d (N, Cin, kh, kw) / Linear (N, K) weight
  // into Wt[N][(tap)*Cin + c]; `mult` scales the weight (exact powers of two only).
  std::vector<float> pack(const std::string& name, int& N, int& Cin, int& kh, int& kw,
                          float mult = 1.f) const;

 private:
  std::map<std::string, HostTensor> t_;
  mutable std::map<std::string, bool> used_;
};

// Converts a packed fp32 weight to the device layout (bf16 bits when bf16).
PackedW upload_packed(DeviceArena& arena, const std::vector<float>& w, int N, int Cin, int kh,
                      int kw, bool bf16);
// bf16(w - bf16(w)) element for element (same layout): the lo part of the bf16x3 split, hi = upload_packed(bf16)
const void* upload_bf16_lo(DeviceArena& arena, const std::vector<float>& w);

}  // namespace sd
