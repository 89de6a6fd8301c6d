#include "prof.h"

#include <map>
#include <mutex>
#include <vector>

namespace sd {
namespace {

struct Rec {
  std::string name;
  hipEvent_t a, b;
  double flops, bytes, steps;
};
struct Agg {
  long long launches = 0;
  double flops = 0, bytes = 0, ms = 0, steps = 0;
};

std::mutex g_mu;
bool g_on = false;
std::vector<Rec> g_pending;
std::map<std::string, Agg> g_agg;

void drain_locked() {
  for (auto& r : g_pending) {
    float ms = 0.f;
    (void)hipEventSynchronize(r.b);
    (void)hipEventElapsedTime(&ms, r.a, r.b);
    Agg& a = g_agg[r.name];
    a.launches += 1;
    a.flops += r.flops;
    a.bytes += r.bytes;
    a.ms += ms;
    a.steps += r.steps;
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  g_pending.clear();
}

}  // namespace

bool prof_enabled() { return g_on; }
void prof_enable(bool on) { g_on = on; }

void prof_reset() {
  std::lock_guard<std::mutex> l(g_mu);
  drain_locked();
  g_agg.clear();
}

bool prof_query(int i, std::string& name, long long& launches, double& flops, double& bytes, double& ms) {
  std::lock_guard<std::mutex> l(g_mu);
  drain_locked();
  if (i < 0 || i >= (int)g_agg.size()) return false;
  auto it = g_agg.begin();
  std::advance(it, i);
  name = it->first;
  launches = it->second.launches;
  flops = it->second.flops;
  bytes = it->second.bytes;
  ms = it->second.ms;
  return true;
}

double prof_query_steps(int i) {
  std::lock_guard<std::mutex> l(g_mu);
  drain_locked();
  if (i < 0 || i >= (int)g_agg.size()) return 0;
  auto it = g_agg.begin();
  std::advance(it, i);
  return it->second.steps;
}

ProfScope::ProfScope(const char* name, double flops, double bytes, hipStream_t st)
    : name_(name), flops_(flops), bytes_(bytes), st_(st) {
  if (!g_on) return;
  // Kernels captured into a hipGraph (FS-EEND streaming) are timed per replay by the caller.
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st_, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return;
  on_ = true;
  SD_HIP(hipEventCreate(&a_));
  SD_HIP(hipEventCreate(&b_));
  SD_HIP(hipEventRecord(a_, st_));
}

ProfScope::~ProfScope() {
  if (!on_) return;
  (void)hipEventRecord(b_, st_);
  std::lock_guard<std::mutex> l(g_mu);
  g_pending.push_back(Rec{name_, a_, b_, flops_, bytes_, steps_});
}

}  // namespace sd
