// 32 x 32 tile products of the two-level blocked inverse (blockinv.hip) shared with the launch
// that runs the cov score GEMM beside the last trailing update (gemm.hip, gemm_trail_kernel).
#pragma once

#include "kstamps.h"
#include "nm16.h"

namespace midagma {

// consecutive jobs (which share operand panels) onto one XCD: blocks b, b+8 share an XCD
__device__ __forceinline__ int xcd_spread(int w, int nwg) {
  const int q = nwg / 8, r = nwg % 8, x = w % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + w / 8;
}

// acc += A[0:32, 0:K] B[0:K, 0:32] (global operands, K = 32 NK), 32-deep chunks through double-
// buffered LDS images; the register loads run PF chunks ahead of the MFMAs (the operands were
// written by the previous launch on other XCDs: each chunk is a MALL round trip).  One barrier
// per chunk; SB (As0 == As1, Bs0 == Bs1: one image each) adds the barrier after the MFMAs that
// double buffering saves, for half the LDS.
template <int PF, int NK, bool SB = false>
__device__ __forceinline__ void tile32_gemm_pf(const double* __restrict__ A, int64_t lda,
                                               const double* __restrict__ B, int64_t ldb, dbl4& acc,
                                               double* As0, double* As1, double* Bs0, double* Bs1) {
  const int tid = threadIdx.x;
  const int r0 = tid >> 4, c0 = (tid & 15) * 2;  // items tid and tid + 256: rows r0, r0 + 16
  double2 a0[PF], a1[PF], b0[PF], b1[PF];
  constexpr int nk = NK;
#define T32_LOAD(slot, kc)                                                                 \
  do {                                                                                     \
    const double* ap = A + (int64_t)r0 * lda + (kc) * 32 + c0;                             \
    const double* bp = B + ((int64_t)(kc) * 32 + r0) * ldb + c0;                           \
    a0[slot] = *reinterpret_cast<const double2*>(ap);                                      \
    a1[slot] = *reinterpret_cast<const double2*>(ap + 16 * lda);                           \
    b0[slot] = *reinterpret_cast<const double2*>(bp);                                      \
    b1[slot] = *reinterpret_cast<const double2*>(bp + 16 * ldb);                           \
  } while (0)
#pragma unroll
  for (int p = 0; p < PF; ++p)
    if (p < nk) T32_LOAD(p, p);
  // slot 0 holds chunk kc; the queue shifts by one each chunk (constant register indices:
  // the loop need not be unrolled for the arrays to stay in registers)
  for (int kc = 0; kc < nk; ++kc) {
    double* As = (kc & 1) ? As1 : As0;
    double* Bs = (kc & 1) ? Bs1 : Bs0;
    *reinterpret_cast<double2*>(As + r0 * ST + c0) = a0[0];
    *reinterpret_cast<double2*>(As + (r0 + 16) * ST + c0) = a1[0];
    *reinterpret_cast<double2*>(Bs + r0 * ST + c0) = b0[0];
    *reinterpret_cast<double2*>(Bs + (r0 + 16) * ST + c0) = b1[0];
    __syncthreads();
#pragma unroll
    for (int p = 0; p + 1 < PF; ++p) {
      a0[p] = a0[p + 1];
      a1[p] = a1[p + 1];
      b0[p] = b0[p + 1];
      b1[p] = b1[p + 1];
    }
    if (kc + PF < nk) T32_LOAD(PF - 1, kc + PF);
    mma32(As, Bs, acc);
    if (SB) __syncthreads();
  }
#undef T32_LOAD
}

// SBPF > 0: single-buffered at a fixed prefetch depth SBPF, K = 256 (the panel variant; one
// instantiation, so the kernel holds only that depth's registers)
template <int SBPF = 0>
__device__ __forceinline__ void tile32_gemm_any(int pf, const double* __restrict__ A, int64_t lda,
                                                const double* __restrict__ B, int64_t ldb, int K, dbl4& acc,
                                                double* As0, double* As1, double* Bs0, double* Bs1) {
  if constexpr (SBPF > 0) {
    tile32_gemm_pf<SBPF, 8, true>(A, lda, B, ldb, acc, As0, As1, Bs0, Bs1);
  } else if (K == 128) {
    if (pf >= 2)
      tile32_gemm_pf<2, 4>(A, lda, B, ldb, acc, As0, As1, Bs0, Bs1);
    else
      tile32_gemm_pf<1, 4>(A, lda, B, ldb, acc, As0, As1, Bs0, Bs1);
  } else if (K == 512) {  // 512-wide outer blocks
    tile32_gemm_pf<3, 16>(A, lda, B, ldb, acc, As0, As1, Bs0, Bs1);
  } else if (pf == 3) {
    tile32_gemm_pf<3, 8>(A, lda, B, ldb, acc, As0, As1, Bs0, Bs1);
  } else if (pf == 2) {
    tile32_gemm_pf<2, 8>(A, lda, B, ldb, acc, As0, As1, Bs0, Bs1);
  } else {
    tile32_gemm_pf<1, 8>(A, lda, B, ldb, acc, As0, As1, Bs0, Bs1);
  }
}

// Trailing update of outer step g: Aout[i, j] = Ain[i, j] - Ain[i, G] Aout[G, j] for i, j
// outside G (Aout[G, j] = P Ain[G, j] from the panel launch).
__device__ __forceinline__ void binv_trail_tile(int job, const double* __restrict__ Ain, double* __restrict__ Aout,
                                                int64_t D, int B2, int g, int check, State* __restrict__ st, int pf,
                                                double* img0, double* img1, double* img2, double* img3) {
  const int nb = (int)(D / NB), gb = B2 / NB, g0 = g * gb, mb = nb - gb;
  const int iq = job / mb, jq = job % mb;
  const int i = iq < g0 ? iq : iq + gb, j = jq < g0 ? jq : jq + gb;
  const int64_t G0 = (int64_t)g0 * NB;
  const double* Ci = Ain + (int64_t)i * NB * D + (int64_t)j * NB;
  dbl4 c_old;
  acc_foreach(c_old, [&](int row, int col, double& v) { v = Ci[(int64_t)row * D + col]; });
  dbl4 acc = {0.0, 0.0, 0.0, 0.0};
  tile32_gemm_any(pf, Ain + (int64_t)i * NB * D + G0, D, Aout + G0 * D + (int64_t)j * NB, D, B2, acc, img0, img1,
                  img2, img3);
  double* out = Aout + (int64_t)i * NB * D + (int64_t)j * NB;
  const int lane = threadIdx.x & 63, m0 = q_m0(), n0 = q_n0();
  int flag = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int row = m0 + acc_row(lane, t), col = n0 + acc_col(lane);
    const double v = c_old[t] - acc[t];
    st_wt(out + (int64_t)row * D + col, v);
    flag |= domain_flag(v);
  }
  if (check && flag) atomicOr(&st->flags, flag);
}


// One job of the panels of outer step g (one 32 x 32 tile; binv_panel_kernel's grid, or a job
// claimed by the trailing update that runs the next block's panel, gemm.hip trail_panel_kernel):
//   U  Aout[G, j] = P Ain[G, j]         (j outside G)           jobs [0, nu)
//   V  Aout[i, G] = -Ain[i, G] P        (i outside G)           jobs [nu, 2 nu)
//   P  Aout[G, G] = P, Pst = P          (next slot's warm start) jobs [2 nu, 2 nu + gb^2)
//   look-ahead LPZ = P LZ                                        jobs past those
// i0..i3: the LDS images (SBPF > 0: i0 == i1, i2 == i3)
template <int SBPF>
__device__ __forceinline__ void binv_panel_job(int job, const double* __restrict__ Ain, double* __restrict__ Aout,
                                               int64_t D, int B2, int g, const double* __restrict__ P, int64_t ldp,
                                               double* __restrict__ Pe, double* __restrict__ Po, int check,
                                               State* __restrict__ st, int pf, const double* __restrict__ LZ,
                                               double* __restrict__ LPZ, double* i0, double* i1, double* i2,
                                               double* i3) {
  const int nb = (int)(D / NB), gb = B2 / NB, g0 = g * gb, mb = nb - gb;
  const int nu = gb * mb;
  const int64_t G0 = (int64_t)g0 * NB;
  dbl4 acc = {0.0, 0.0, 0.0, 0.0};
  KS_DECL(ks);
  if (job < nu) {
    const int a = job / mb, cq = job % mb, c = cq < g0 ? cq : cq + gb;
    tile32_gemm_any<SBPF>(pf, P + (int64_t)a * NB * ldp, ldp, Ain + G0 * D + (int64_t)c * NB, D, B2, acc, i0, i1, i2,
                        i3);
    KS_MARK(ks);
    double* out = Aout + (G0 + (int64_t)a * NB) * D + (int64_t)c * NB;
    int flag = 0;
    acc_foreach(acc, [&](int row, int col, double& v) {
      st_wt(out + (int64_t)row * D + col, v);
      flag |= domain_flag(v);
    });
    if (check && flag) atomicOr(&st->flags, flag);
    KS_END(ks, KS_PANEL);
  } else if (job < 2 * nu) {
    const int j2 = job - nu, iq = j2 / gb, c = j2 % gb, i = iq < g0 ? iq : iq + gb;
    tile32_gemm_any<SBPF>(pf, Ain + (int64_t)i * NB * D + G0, D, P + (int64_t)c * NB, ldp, B2, acc, i0, i1, i2, i3);
    KS_MARK(ks);
    double* out = Aout + (int64_t)i * NB * D + G0 + (int64_t)c * NB;
    int flag = 0;
    acc_foreach(acc, [&](int row, int col, double& v) {
      st_wt(out + (int64_t)row * D + col, -v);
      flag |= domain_flag(-v);
    });
    if (check && flag) atomicOr(&st->flags, flag);
    KS_END(ks, KS_PANEL);
  } else if (job >= 2 * nu + gb * gb) {  // look-ahead: LPZ = P LZ (next block's residual)
    const int j4 = job - 2 * nu - gb * gb, a = j4 / gb, c = j4 % gb;
    tile32_gemm_any<SBPF>(pf, P + (int64_t)a * NB * ldp, ldp, LZ + (int64_t)c * NB, B2, B2, acc, i0, i1, i2, i3);
    double* out = LPZ + (int64_t)a * NB * B2 + (int64_t)c * NB;
    acc_foreach(acc, [&](int row, int col, double& v) { st_wt(out + (int64_t)row * B2 + col, v); });
  } else {
    const int j3 = job - 2 * nu, a = j3 / gb, c = j3 % gb;
    const double* src = P + (int64_t)a * NB * ldp + (int64_t)c * NB;
    double* out = Aout + (G0 + (int64_t)a * NB) * D + G0 + (int64_t)c * NB;
    double* Pst = (st && (st->slots & 1)) ? Po : Pe;  // this slot's store (parity of k)
    double* ps = Pst + (int64_t)a * NB * B2 + (int64_t)c * NB;
    int flag = 0;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int e = it * NTHREADS + threadIdx.x, row = e >> 5, col = e & 31;
      const double v = src[(int64_t)row * ldp + col];
      st_wt(out + (int64_t)row * D + col, v);
      st_wt(ps + (int64_t)row * B2 + col, v);
      flag |= domain_flag(v);
    }
    if (check && flag) atomicOr(&st->flags, flag);
  }
}

}  // namespace midagma
