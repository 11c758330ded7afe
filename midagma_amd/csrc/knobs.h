// Experiment knobs (MIDAGMA_EXP_*): measured alternatives of the product paths, kept so that a
// measurement can be repeated (DESIGN.md section 8 lists each with its result).
//
// The product library (`make`, libmidagma_hip.so) compiles every knob to its default: it reads
// no MIDAGMA_EXP_* variable, and rejected paths (the one-launch inverse of dfinv.hip, the 512
// block, the look-ahead residual, the 64-tile GEMM, ...) cannot be selected.  `make exp` builds
// libmidagma_hip_exp.so with -DMIDAGMA_EXPERIMENTS, where the knobs read the environment
// (tools/probe_perf.py, `pytest -m experiment` with MIDAGMA_LIB pointing at that library).
#pragma once

#include <cstdlib>

namespace midagma {

#ifdef MIDAGMA_EXPERIMENTS
constexpr bool kExperiments = true;
// the variable is set (any value)
inline bool knob_set(const char* name) { return std::getenv(name) != nullptr; }
// the variable's integer value, or dflt when unset
inline long knob(const char* name, long dflt) {
  const char* e = std::getenv(name);
  return e ? std::atol(e) : dflt;
}
inline double knob_f(const char* name, double dflt) {
  const char* e = std::getenv(name);
  return e ? std::atof(e) : dflt;
}
#else
constexpr bool kExperiments = false;
constexpr bool knob_set(const char*) { return false; }
constexpr long knob(const char*, long dflt) { return dflt; }
constexpr double knob_f(const char*, double dflt) { return dflt; }
#endif

}  // namespace midagma
