// The product-form series of one B2 x B2 diagonal block (the fast blocked inverse's outer blocks,
// blockinv.hip; the DagmaMLP log-det's warm-started inverse): the split-K operand loads, the
// residual and pass tile bodies and their tile placement.  Shared by the series launches
// (blockinv.hip) and the trailing-update launch that also runs the next block's series
// (gemm.hip, trail_series_kernel), so both compute the same tiles in the same order.
#pragma once

#include "kstamps.h"
#include "launch.h"
#include "nm16.h"

namespace midagma {

template <int L>
__device__ __forceinline__ void splitk_load_a(const double* __restrict__ A, int64_t lda, int m0, double (&a)[L]) {
  const double* ap = A + (int64_t)(m0 + (threadIdx.x & 15)) * lda + splitk_k0<L>();
#pragma unroll
  for (int q = 0; q < L; ++q) a[q] = ap[q];
}
template <int L>
__device__ __forceinline__ void splitk_load_b(const double* __restrict__ B, int64_t ldb, int n0, double (&b)[L]) {
  const double* bp = B + (int64_t)splitk_k0<L>() * ldb + n0 + (threadIdx.x & 15);
#pragma unroll
  for (int q = 0; q < L; ++q) b[q] = bp[(int64_t)q * ldb];
}

// splitk_load_a of S = (sI - W∘W)^T[0:B2, 0:B2] (outer block 0) computed from W itself:
// S[i][k] = (k == i ? s : 0) - W[k][i]^2, identity in the padding -- build_at's values, bit for bit
// (build_at_tile), so block 0's residual can run in build_at's launch (build_resid0_kernel)
template <int L>
__device__ __forceinline__ void splitk_load_a_w(const double* __restrict__ W, int64_t ldw, int64_t d, double s,
                                                int m0, double (&a)[L], bool w32) {
  const int64_t i = m0 + (threadIdx.x & 15), k0 = splitk_k0<L>();
#pragma unroll
  for (int q = 0; q < L; ++q) {
    const int64_t k = k0 + q;
    if (i < d && k < d) {
      a[q] = sw_entry(k == i, s, W[k * ldw + i], w32);
    } else {
      a[q] = (k == i) ? 1.0 : 0.0;
    }
  }
}

// splitk_load_a of S = (sI - A)^T (the DagmaMLP log-det's fast path, B2 x B2 with identity
// padding) computed from A itself: S[i][k] = (k == i ? s : 0) - A[k][i], the values the former S
// launch stored, bit for bit, so the fast step's residual needs no launch before it
// (ldfast_resid_kernel)
template <int L>
__device__ __forceinline__ void splitk_load_a_at(const double* __restrict__ A, int64_t lda, int64_t d, double s,
                                                 int m0, double (&a)[L]) {
  const int64_t i = m0 + (threadIdx.x & 15), k0 = splitk_k0<L>();
#pragma unroll
  for (int q = 0; q < L; ++q) {
    const int64_t k = k0 + q;
    if (i < d && k < d)
      a[q] = (k == i ? s : 0.0) - A[k * lda + i];
    else
      a[q] = (k == i) ? 1.0 : 0.0;
  }
}

// Row partial of |Q| over this tile's 16 columns -> rowpart[(m0 + row) * NT + tile column]
__device__ __forceinline__ void store_row_partial(double a, double* __restrict__ rowpart, int m0, int n0, int NT) {
  a = row_sum16(a);
  int row, col;
  tile_elem(threadIdx.x, row, col);
  if (col == 0) st_wt(rowpart + (int64_t)(m0 + row) * NT + n0 / 16, a);  // write-through: handed to other CUs
}

template <int B2, int NTH = NTHREADS>
__device__ __forceinline__ double inf_norm(const double* __restrict__ rowpart, float* red4) {
  return inf_norm_rows<B2, NTH>([&](int i) { return rowpart[i]; }, red4);
}

// The warm start X0 of a block (see nm_resid_kernel) as the B operand of a split-K tile
template <int L>
__device__ __forceinline__ void load_x0_b(const double* __restrict__ Pe, const double* __restrict__ Po,
                                          const State* __restrict__ st, int n0, double (&b)[L]) {
  constexpr int B2 = 16 * L;
  const bool odd = (st->slots & 1) != 0;
  splitk_load_b<L>(odd ? Pe : Po, B2, n0, b);
  if (st->warm_run >= 2) {
    double b2[L];
    splitk_load_b<L>(odd ? Po : Pe, B2, n0, b2);
#pragma unroll
    for (int q = 0; q < L; ++q) b[q] = 2.0 * b[q] - b2[q];
  }
}

// Tile of workgroup wg in a series launch over an nt x nt grid of 16 x 16 tiles.  xmap (256-wide
// blocks, nt = 16): the 32 workgroups the dispatcher puts on one XCD (wg, wg + 8, ...) take a
// 4 x 8 block of tiles, so that XCD's L2 serves 4 row bands and 8 column bands of the operands
// instead of all 16 row bands (row-major order: every XCD read the whole of Y and Q)
__device__ __forceinline__ void nm_tile(int wg, int nt, int xmap, int& m0, int& n0) {
  int t = wg;
  if (xmap && nt == 16) {
    const int x = wg & 7, l = wg >> 3;
    t = (4 * (x >> 1) + (l >> 3)) * 16 + 8 * (x & 1) + (l & 7);
  }
  m0 = (t / nt) * 16;
  n0 = (t % nt) * 16;
}

// X0 = the warm start of this block: with two consecutive stored slots (st->warm_run >= 2)
// the linear extrapolation 2 P1 - P2 of the last two inverses (P1 = slot k-1's, P2 = slot
// k-2's, by the parity of k = st->slots), else P1.  Adam moves W smoothly (beta1 = 0.99), so
// the extrapolation leaves a residual ~100x smaller than P1 alone (2 product-form passes
// instead of 3 at d = 1000, measured on the default fit).
// R = I - S X0 (tile (m0, n0) of the B2 x B2 block), row partials of |R| -> part0; the
// workgroup also writes its tile of X0 -> Y0 (the first pass's iterate).
// NW waves split K (B2 = 4 NW L): NW = 4 for B2 <= 256; B2 = 512 runs NW = 8 with L = 16, so
// the per-lane operand runs and registers stay those of the 256-wide kernel
// Body of the residual launch for workgroup wg; FROM_W: S from W (outer block 0, SW = {W, ldw,
// d, s}) instead of the At block S (lds); FROM_A (sw.pr null): S = (sI - A)^T from A = sw.W with
// s = sw.s.  slot_bias: added to st->slots for the warm start's parity (1: the step's opening
// increment is still to come, ldfast_resid_kernel)
struct SFromW {
  const double* W;
  int64_t ldw, d;
  const Params* pr;
  double s = 0.0;
};
template <int L, int NW, bool FROM_W, bool FROM_A = false>
__device__ __forceinline__ void nm_resid_body(int wg, const double* __restrict__ S, int64_t lds, const SFromW& sw,
                                              const double* __restrict__ Pe, const double* __restrict__ Po,
                                              double* __restrict__ Y0, double* __restrict__ Q0,
                                              double* __restrict__ part0, int* __restrict__ done,
                                              State* __restrict__ st, int xmap, double* red, int slot_bias = 0) {
  if (st->ckpt_pending) {  // a log-det is due: pivots come from the slow path only
    if (wg == 0 && threadIdx.x == 0) st->status = ST_NEED_GJ;
    return;
  }
  constexpr int B2 = 4 * NW * L;
  const int nt = B2 / 16;
  KS_DECL(ks);
  int m0, n0;
  nm_tile(wg, nt, xmap, m0, n0);
  if (wg == 0 && threadIdx.x == 0) *done = 0;
  const bool odd = ((st->slots + slot_bias) & 1) != 0;
  const double* P1 = odd ? Pe : Po;  // slot k-1
  const double* P2 = odd ? Po : Pe;  // slot k-2
  const bool extrap = st->warm_run >= 2;
  double a[L], b[L];
  if (FROM_A)
    splitk_load_a_at<L>(sw.W, sw.ldw, sw.d, sw.s, m0, a);
  else if (FROM_W)
    splitk_load_a_w<L>(sw.W, sw.ldw, sw.d, sw.pr->s, m0, a, sw.pr->w32 != 0);
  else
    splitk_load_a<L>(S, lds, m0, a);
  splitk_load_b<L>(P1, B2, n0, b);
  if (extrap) {
    double b2[L];
    splitk_load_b<L>(P2, B2, n0, b2);
#pragma unroll
    for (int q = 0; q < L; ++q) b[q] = 2.0 * b[q] - b2[q];
  }
  int row, col;
  const bool elem = threadIdx.x < 256;  // the tile's 256 elements (NW > 4: the other waves only sum)
  tile_elem(elem ? threadIdx.x : 0, row, col);
  const int gi = m0 + row, gj = n0 + col;
  const int64_t e = (int64_t)gi * B2 + gj;
  if (elem) st_wt(Y0 + e, extrap ? 2.0 * P1[e] - P2[e] : P1[e]);
#ifdef MIDAGMA_KSTAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (stamps: operands and the warm start arrived)
  KS_MARK(ks);
#endif
  dbl4 acc = {0.0, 0.0, 0.0, 0.0};
  splitk_mfma<L>(a, b, acc);
  const double sum = splitk_sum_w<NW>(acc, red);
  KS_MARK(ks);
  if (!elem) return;
  const double r = (gi == gj ? 1.0 : 0.0) - sum;
  st_wt(Q0 + e, r);
  store_row_partial(abs_or_inf(r), part0, m0, n0, nt);
  if (!FROM_W) KS_END(ks, KS_RESID);
}

// Pass p's tile wg (see nm_pass_kernel): rho = ||Q||_inf from the previous pass's row partials;
// converged -> P = Y + Y Q (done = p), else Y' = Y + Y Q, Q' = Q Q and the row partials of |Q'|.
// Far or diverging -> ST_NEED_GJ.  Uniform early returns only (every thread takes the same path).
template <int L, int NW = 4>
__device__ __forceinline__ void nm_pass_body(int wg, const double* __restrict__ Y, const double* __restrict__ Q,
                                             double* __restrict__ Yn, double* __restrict__ Qn, double* __restrict__ P,
                                             const double* __restrict__ part_prev, double* __restrict__ part_next,
                                             int* __restrict__ done, int pass, State* __restrict__ st, int xmap,
                                             double* red, float* red4) {
  constexpr int B2 = 4 * NW * L;
  const int nt = B2 / 16, tid = threadIdx.x;
  // an EARLIER pass converged (done holds its number; this pass's own workgroups may store
  // theirs meanwhile, which must not make a sibling skip its tile of P)
  const int dn = __hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (dn != 0 && dn < pass) return;
  KS_DECL(ks);
  int m0, n0;
  nm_tile(wg, nt, xmap, m0, n0);
  // operands first: their latency overlaps the rho reduction (Y, Q are complete: the
  // previous launch wrote them)
  double aY[L], aQ[L], bQ[L];
  splitk_load_a<L>(Y, B2, m0, aY);
  splitk_load_b<L>(Q, B2, n0, bQ);
  splitk_load_a<L>(Q, B2, m0, aQ);
  int row, col;
  const bool elem = tid < 256;  // the tile's 256 elements (NW > 4: the other waves only sum)
  tile_elem(elem ? tid : 0, row, col);
  const int gi = m0 + row, gj = n0 + col;
  const double yold = elem ? Y[(int64_t)gi * B2 + gj] : 0.0;
  const double rho = inf_norm<B2, 64 * NW>(part_prev, red4);
  KS_MARK(ks);
  if (!(rho <= 0.25)) {  // warm start too far, diverging, or not finite
    if (wg == 0 && tid == 0) st->status = ST_NEED_GJ;
    return;
  }
  dbl4 ay = {0.0, 0.0, 0.0, 0.0};
  if (rho <= 1e-8) {  // last factor: P = Y (I + Q)
    splitk_mfma<L>(aY, bQ, ay);
    const double yq = splitk_sum_w<NW>(ay, red);
    if (elem) st_wt(P + (int64_t)gi * B2 + gj, yold + yq);
    if (wg == 0 && tid == 0) __hip_atomic_store(done, pass, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  dbl4 aq = {0.0, 0.0, 0.0, 0.0};
  splitk_mfma<L>(aY, bQ, ay);
  splitk_mfma<L>(aQ, bQ, aq);
  const double yq = splitk_sum_w<NW>(ay, red);
  __syncthreads();  // red reused
  const double qq = splitk_sum_w<NW>(aq, red);
  KS_MARK(ks);
  if (!elem) return;
  st_wt(Yn + (int64_t)gi * B2 + gj, yold + yq);
  st_wt(Qn + (int64_t)gi * B2 + gj, qq);
  store_row_partial(abs_or_inf(qq), part_next, m0, n0, nt);
  KS_END(ks, KS_PASS);
}

}  // namespace midagma
