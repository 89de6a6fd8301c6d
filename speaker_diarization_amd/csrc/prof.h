// Opt-in per-kernel-family timing with HIP events on the launch stream, plus
// algorithmic FLOP/byte accounting — feeds bench.py's live roofline numbers.
#pragma once
#include <string>
#include "common.h"

namespace sd {

bool prof_enabled();
void prof_enable(bool on);
void prof_reset();
// Aggregated stats of family i (after synchronising its events); false past the end.
bool prof_query(int i, std::string& name, long long& launches, double& flops, double& bytes, double& ms);
// Dependent sequential steps accumulated by family i (latency-bound kernels such as the LSTM recurrence set
// them: a launch's time / its steps is its per-step latency); 0 past the end or when none were set.
double prof_query_steps(int i);

class ProfScope {
 public:
  ProfScope(const char* name, double flops, double bytes, hipStream_t st);
  ~ProfScope();
  void set_steps(double steps) { steps_ = steps; }

 private:
  bool on_ = false;
  const char* name_;
  double flops_, bytes_, steps_ = 0;
  hipStream_t st_;
  hipEvent_t a_ = nullptr, b_ = nullptr;
};

}  // namespace sd
