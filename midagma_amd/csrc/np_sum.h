// numpy's float32 sum, bit for bit: the `np.abs(W).sum()` of the reference's checkpoint objective
// (linear.py:127) on a float32 W (DagmaLinear(dtype=np.float32), linear.py:29, 429).
//
// np.add.reduce over a contiguous float32 array walks it in buffer-sized chunks (8192 elements,
// np.getbufsize()) and adds each chunk's pairwise sum to the running total, all in float32:
//   total = ((0 + pw(chunk 0)) + pw(chunk 1)) + ...
// pw (numpy's pairwise_sum for FLOAT): n < 8 -> a sequential sum from 0; n <= 128 -> eight
// accumulators over the multiple-of-8 prefix, combined as ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)),
// then the rest added in order; larger n -> pw(first n2) + pw(rest), n2 = n/2 rounded down to a
// multiple of 8.  tests/test_np_sum.py pins this restatement against numpy on the CPU.
#pragma once

#include <stdint.h>

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define MIDAGMA_HD __host__ __device__
#else  // plain C++ (tests/test_np_sum.py builds the host form with g++)
#include <cmath>
#define MIDAGMA_HD
#endif

namespace midagma {

constexpr int64_t NP_SUM_CHUNK = 8192;  // numpy's default buffer size (elements)
constexpr int64_t NP_PW_BLOCK = 128;    // numpy's PW_BLOCKSIZE

// one pairwise leaf (n <= 128) of the elements ld(off) .. ld(off + n - 1)
template <class L>
MIDAGMA_HD inline float np_pw_leaf(const L& ld, int64_t off, int64_t n) {
  if (n < 8) {
    float res = 0.f;
    for (int64_t i = 0; i < n; ++i) res += ld(off + i);
    return res;
  }
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = ld(off + j);
  int64_t i = 8;
  for (; i < n - (n % 8); i += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += ld(off + i + j);
  }
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += ld(off + i);
  return res;
}

// numpy's pairwise sum of ld(off) .. ld(off + n - 1), its recursion unrolled onto a small stack
// (depth <= log2(8192 / 128) + 2 within a chunk)
template <class L>
MIDAGMA_HD inline float np_pairwise(const L& ld, int64_t f0, int64_t n) {
  constexpr int kDepth = 24;
  int64_t off[kDepth], len[kDepth];
  int stage[kDepth];
  float left[kDepth];
  int sp = 0;
  off[0] = f0;
  len[0] = n;
  stage[0] = 0;
  float ret = 0.f;
  bool returning = false;
  while (sp >= 0) {
    if (!returning) {
      if (len[sp] <= NP_PW_BLOCK) {
        ret = np_pw_leaf(ld, off[sp], len[sp]);
        returning = true;
        --sp;
        continue;
      }
      int64_t n2 = len[sp] / 2;
      n2 -= n2 % 8;
      stage[sp] = 1;
      off[sp + 1] = off[sp];
      len[sp + 1] = n2;
      ++sp;
      continue;
    }
    if (stage[sp] == 1) {  // the left half is done: descend into the right half
      left[sp] = ret;
      stage[sp] = 2;
      int64_t n2 = len[sp] / 2;
      n2 -= n2 % 8;
      off[sp + 1] = off[sp] + n2;
      len[sp + 1] = len[sp] - n2;
      ++sp;
      returning = false;
      continue;
    }
    ret = left[sp] + ret;  // both halves done
    --sp;
  }
  return ret;
}

// |W| (float32 values held in float64) of the d x d matrix at W with leading dimension D, in
// numpy's flat (row-major, unpadded) order
struct AbsW32 {
  const double* W;
  int64_t d, D;
  MIDAGMA_HD float operator()(int64_t f) const { return fabsf((float)W[(f / d) * D + f % d]); }
};

// numpy's np.abs(W).sum() of a float32 W, serially (host, or one device thread)
MIDAGMA_HD inline float np_abs_sum32(const double* W, int64_t d, int64_t D) {
  const AbsW32 ld{W, d, D};
  const int64_t n = d * d;
  float total = 0.f;
  for (int64_t c = 0; c < n; c += NP_SUM_CHUNK) total += np_pairwise(ld, c, n - c < NP_SUM_CHUNK ? n - c : NP_SUM_CHUNK);
  return total;
}

}  // namespace midagma
