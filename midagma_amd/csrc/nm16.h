// Compute pieces of the product-form diagonal-block inverse shared by the launch-per-phase
// blocked inverse (blockinv.hip) and the one-launch dataflow inverse (dfinv.hip): the 16 x 16
// split-K tile product over the 4 waves, its fixed-order wave sum, the row sums of |Q| and the
// domain flags.  Both files run the same arithmetic in the same order, so their results are
// bit-identical; they differ only in how operands reach the registers.
#pragma once

#include "tile32.h"

namespace midagma {

// This wave's quarter of K for a 16 x 16 output tile: lane (r, kq) runs k = kb + kq L + q,
// q < L, kb = w * 4L (L = K / 16), so each lane streams L contiguous values of its A row.
// The MFMA chains: q even / odd, summed at the end.
template <int L>
__device__ __forceinline__ void splitk_mfma(const double (&a)[L], const double (&b)[L], dbl4& acc) {
  dbl4 c1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int q = 0; q < L; q += 2) {
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q], b[q], acc, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q + 1], b[q + 1], c1, 0, 0, 0);
  }
  acc = acc + c1;
}

// first k of this lane's run (see splitk_mfma)
template <int L>
__device__ __forceinline__ int splitk_k0() {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  return w * 4 * L + (lane >> 4) * L;
}

// Sum the 4 waves' partials of one 16 x 16 tile in a fixed order: thread e of the workgroup
// returns element e (t = e >> 6 register, lane e & 63 of the accumulator layout).
__device__ __forceinline__ double splitk_sum(const dbl4& part, double* red) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll
  for (int t = 0; t < 4; ++t) red[w * 256 + t * 64 + lane] = part[t];
  __syncthreads();
  return ((red[tid] + red[256 + tid]) + red[512 + tid]) + red[768 + tid];
}

// The same for NW waves splitting K (NW x 256 doubles of red); NW = 4 sums in splitk_sum's
// order.  Threads >= 256 return 0 (the tile has 256 elements); every thread passes the barrier.
template <int NW>
__device__ __forceinline__ double splitk_sum_w(const dbl4& part, double* red) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
#pragma unroll
  for (int t = 0; t < 4; ++t) red[w * 256 + t * 64 + lane] = part[t];
  __syncthreads();
  if (tid >= 256) return 0.0;
  double s = red[tid];
#pragma unroll
  for (int k = 1; k < NW; ++k) s += red[k * 256 + tid];
  return s;
}

__device__ __forceinline__ void tile_elem(int e, int& row, int& col) {
  const int t = e >> 6, lane = e & 63;
  row = acc_row(lane, t);
  col = acc_col(lane);
}

// max over the workgroup of one non-negative float per thread -> red4 (4 floats), all threads
__device__ __forceinline__ float block_max(float v, float* red4) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = v;
  __syncthreads();
  return fmaxf(fmaxf(red4[0], red4[1]), fmaxf(red4[2], red4[3]));
}
// the same over NW waves (redn: NW floats)
template <int NW>
__device__ __forceinline__ float block_max_w(float v, float* redn) {
  if (NW == 4) return block_max(v, redn);
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) redn[threadIdx.x >> 6] = v;
  __syncthreads();
  float m = redn[0];
#pragma unroll
  for (int k = 1; k < NW; ++k) m = fmaxf(m, redn[k]);
  return m;
}

__device__ __forceinline__ double abs_or_inf(double v) { return isfinite(v) ? fabs(v) : INFINITY; }

// The domain flags of reduce_check (linear.py:226-230: any(inv + 1e-16 < 0); non-finite),
// taken on the last outer step's outputs so the fast slot needs no extra pass over Mt.
__device__ __forceinline__ int domain_flag(double v) { return (v + 1e-16 < 0.0 ? 1 : 0) | (isfinite(v) ? 0 : 2); }

template <int CTRL>
__device__ __forceinline__ double dpp_add(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
  return v + __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Row sum over a tile's 16 columns: thread e holds tile element (row, col); the 16 threads of
// a row are one DPP row of a wave.  Every thread of the row returns the sum.
__device__ __forceinline__ double row_sum16(double a) {
  a = dpp_add<0xB1>(a);   // quad_perm [1,0,3,2]
  a = dpp_add<0x4E>(a);   // quad_perm [2,3,0,1]
  a = dpp_add<0x141>(a);  // row_half_mirror
  a = dpp_add<0x140>(a);  // row_mirror
  return a;
}

// ||Q||_inf from the row partials (row r's NT = B2 / 16 tile partials at rowpart[r NT + t]),
// one row per thread (B2 = 512: two); load(i) returns rowpart[i].  Non-finite propagates as
// inf/nan; widened by 1e-6 against the float max.
template <int B2, int NTH = NTHREADS, class Load>
__device__ __forceinline__ double inf_norm_rows(Load&& load, float* red4) {
  constexpr int NT = B2 / 16;
  constexpr int RPT = B2 > NTH ? B2 / NTH : 1;  // rows per thread
  float f = 0.0f;
#pragma unroll
  for (int h = 0; h < RPT; ++h) {
    const int row = (int)threadIdx.x + h * NTH;
    double r = 0.0;
    if (row < B2) {
      constexpr int CH = NT < 16 ? NT : 16;  // loads in flight per chunk (registers)
#pragma unroll
      for (int c0 = 0; c0 < NT; c0 += CH) {
        double v[CH];  // a chunk's loads in flight before its (ordered) sum
#pragma unroll
        for (int t = 0; t < CH; ++t) v[t] = load(row * NT + c0 + t);
#pragma unroll
        for (int t = 0; t < CH; ++t) r += v[t];
      }
    }
    f = fmaxf(f, isfinite(r) ? (float)(r * (1.0 + 1e-6)) : INFINITY);
  }
  return (double)block_max_w<NTH / 64>(f, red4);
}

}  // namespace midagma
