// Phase stamps of the cov slot's latency-bound kernels (diagnostic build only: `make kstamps`,
// -DMIDAGMA_KSTAMPS; tools/kstamps.py).  Wave 0 of every workgroup reads the shader clock
// (s_memtime) at the kernel's phase points; lane 0 adds the phase lengths into per-kind sums
// (device-scope atomics), so a run yields the mean per-workgroup time of each phase.
//   nm_resid:   entry -> operands + warm start loaded -> MFMA + split-K sum -> stores drained
//   nm_pass:    entry -> rho (previous pass's row partials reduced) -> MFMAs + split-K sums -> stores drained
//   binv_panel / binv_trail: entry -> tile product (operand chunks + MFMA) -> stores drained
// Without MIDAGMA_KSTAMPS every macro is empty.
#pragma once

#include <hip/hip_runtime.h>

namespace midagma {

enum KStampKind : int { KS_RESID = 0, KS_PASS = 1, KS_PANEL = 2, KS_TRAIL = 3, KS_KINDS = 4 };
constexpr int KS_POINTS = 6;  // phase slots per kind; [KS_POINTS] = workgroups, [KS_POINTS + 1] = real-time span

#ifdef MIDAGMA_KSTAMPS
__device__ unsigned long long g_kstamps[KS_KINDS][KS_POINTS + 2];

struct KStamp {
  unsigned long long t[KS_POINTS];
  unsigned long long rt0;
  int n;
};
__device__ __forceinline__ unsigned long long ks_clock() { return __builtin_amdgcn_s_memtime(); }
#define KS_DECL(ks) \
  KStamp ks;        \
  ks.n = 0;         \
  ks.rt0 = __builtin_amdgcn_s_memrealtime(); \
  ks.t[ks.n++] = ks_clock()
#define KS_MARK(ks) \
  if (ks.n < KS_POINTS) ks.t[ks.n++] = ks_clock()
// drain this wave's stores, stamp, and add the phases (lane 0 of wave 0)
#define KS_END(ks, kind)                                                                       \
  do {                                                                                         \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                           \
    KS_MARK(ks);                                                                               \
    if (threadIdx.x == 0) {                                                                    \
      for (int p_ = 0; p_ + 1 < ks.n; ++p_) atomicAdd(&g_kstamps[kind][p_], ks.t[p_ + 1] - ks.t[p_]); \
      atomicAdd(&g_kstamps[kind][KS_POINTS], 1ull);                                            \
      atomicAdd(&g_kstamps[kind][KS_POINTS + 1], __builtin_amdgcn_s_memrealtime() - ks.rt0);  \
    }                                                                                          \
  } while (0)
#else
#define KS_DECL(ks) \
  do {              \
  } while (0)
#define KS_MARK(ks) \
  do {              \
  } while (0)
#define KS_END(ks, kind) \
  do {                   \
  } while (0)
#endif

}  // namespace midagma
