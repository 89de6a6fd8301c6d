#include "params.h"

#include <cmath>
#include <cstring>

namespace sd {

void ParamStore::set(const std::string& name, const float* data, const int64_t* shape, int ndim) {
  HostTensor t;
  int64_t n = 1;
  for (int i = 0; i < ndim; ++i) {
    SD_CHECK(shape[i] >= 0, kErrParam, "negative dim for " + name);
    t.shape.push_back(shape[i]);
    n *= shape[i];
  }
  t.data.assign(data, data + n);
  t_[name] = std::move(t);
}

const HostTensor& ParamStore::get(const std::string& name) const {
  auto it = t_.find(name);
  SD_CHECK(it != t_.end(), kErrParam, "Missing key(s) in state_dict: \"" + name + "\"");
  used_[name] = true;
  return it->second;
}

std::vector<std::string> ParamStore::unused() const {
  std::vector<std::string> out;
  for (auto& kv : t_) {
    const std::string& k = kv.first;
    if (used_.count(k)) continue;
    if (k.size() >= 19 && k.compare(k.size() - 19, 19, "num_batches_tracked") == 0) continue;
    out.push_back(k);
  }
  return out;
}

void ParamStore::bn_fold(const std::string& p, std::vector<float>& scale, std::vector<float>& shift,
                         const std::string& conv_bias, float eps) const {
  const HostTensor& mean = get(p + ".running_mean");
  const HostTensor& var = get(p + ".running_var");
  const int64_t C = mean.numel();
  SD_CHECK(var.numel() == C, kErrParam, "BatchNorm size mismatch at " + p);
  const HostTensor* w = has(p + ".weight") ? &get(p + ".weight") : nullptr;
  const HostTensor* b = has(p + ".bias") ? &get(p + ".bias") : nullptr;
  const HostTensor* cb = conv_bias.empty() ? nullptr : &get(conv_bias);
  scale.resize(C);
  shift.resize(C);
  for (int64_t c = 0; c < C; ++c) {
    double s = 1.0 / std::sqrt((double)var.data[c] + (double)eps);
    double g = w ? w->data[c] : 1.0;
    double bb = b ? b->data[c] : 0.0;
    double cbias = cb ? cb->data[c] : 0.0;
    scale[c] = (float)(g * s);
    shift[c] = (float)((cbias - mean.data[c]) * g * s + bb);
  }
}

std::vector<float> ParamStore::pack(const std::string& name, int& N, int& Cin, int& kh, int& kw,
                                    float mult) const {
  const HostTensor& t = get(name);
  const auto& s = t.shape;
  SD_CHECK(s.size() >= 2 && s.size() <= 4, kErrParam, "unexpected weight rank for " + name);
  N = (int)s[0];
  Cin = (int)s[1];
  kh = s.size() == 4 ? (int)s[2] : 1;
  kw = s.size() == 4 ? (int)s[3] : (s.size() == 3 ? (int)s[2] : 1);
  const int taps = kh * kw;
  std::vector<float> out((size_t)N * taps * Cin);
  for (int n = 0; n < N; ++n)
    for (int c = 0; c < Cin; ++c)
      for (int tp = 0; tp < taps; ++tp)
        out[((size_t)n * taps + tp) * Cin + c] = t.data[((size_t)n * Cin + c) * taps + tp] * mult;
  return out;
}

static uint16_t f2bf_host(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

PackedW upload_packed(DeviceArena& arena, const std::vector<float>& w, int N, int Cin, int kh, int kw,
                      bool bf16) {
  PackedW p;
  p.N = N;
  p.Cin = Cin;
  p.kh = kh;
  p.kw = kw;
  p.K = kh * kw * Cin;
  if (bf16) {
    std::vector<uint16_t> h(w.size());
    for (size_t i = 0; i < w.size(); ++i) h[i] = f2bf_host(w[i]);
    void* d = arena.alloc(h.size() * 2);
    SD_HIP(hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    p.w = d;
  } else {
    p.w = arena.upload(w);
  }
  return p;
}

const void* upload_bf16_lo(DeviceArena& arena, const std::vector<float>& w) {
  std::vector<uint16_t> lo(w.size());
  for (size_t i = 0; i < w.size(); ++i) {
    const uint32_t hb = (uint32_t)f2bf_host(w[i]) << 16;
    float hi;
    std::memcpy(&hi, &hb, 4);
    lo[i] = f2bf_host(w[i] - hi);
  }
  void* d = arena.alloc(lo.size() * 2);
  SD_HIP(hipMemcpy(d, lo.data(), lo.size() * 2, hipMemcpyHostToDevice));
  return d;
}

}  // namespace sd
