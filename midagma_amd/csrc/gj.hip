// Blocked Gauss-Jordan inverse + log-det of sI - W∘W on FP64 matrix cores.
//
// Replaces `sla.inv(s*I - W*W)` (LAPACK dgetrf+dgetri, linear.py:226, 240),
// `la.slogdet` (linear.py:114) and torch `slogdet` (nonlinear.py:85).
//
// In the M-matrix domain sI - W∘W is a nonsingular M-matrix, so elimination
// WITHOUT pivoting is stable and every pivot is > 0.
// The kernels run on A^T so the result is inv(A)^T = M^T, exactly the operand
// of the gradient 2 W∘M^T (linear.py:248), read coalesced by the fused update.
//
// Block Gauss-Jordan with NB = 32 (K = D/32 block steps), ONE launch per step.
// Step k reads three side panels published by step k-1 (double-buffered by
// parity): P = inv(A_kk), the column tiles C_i = A_ik and the row tiles
// R_j = A_kj, and updates every tile of A in place:
//     A_ij -= C_i (P R_j)      A_kj = P R_j      A_ik = -C_i P      A_kk = P
// Tiles landing in block column/row k+1 are also published as the next step's
// panels, and the workgroup owning tile (k+1, k+1) inverts it right away
// (unpivoted GJ in registers + LDS, pivots -> log|p|), so the only serial
// chain per step is one 32x32 inversion plus one kernel boundary.
#include "launch.h"
#include "tile32.h"

namespace midagma {


#ifdef MIDAGMA_STAMPS
// Diagnostic build only: s_memtime stamps of the diagonal-owner workgroup per block step.
__device__ unsigned long long g_stamps[256][16];
#define STAMP(k, slot)                                                                     \
  do {                                                                                     \
    if (threadIdx.x == 0) {                                                                \
      unsigned long long t_;                                                               \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");          \
      g_stamps[(k) & 255][slot] = t_;                                                      \
    }                                                                                      \
  } while (0)
#else
#define STAMP(k, slot) \
  do {                 \
  } while (0)
#endif
constexpr int EPT = NB * NB / NTHREADS;   // elements per thread in the tile inversion (4)
constexpr int TPR = NB / EPT;             // threads per tile row (8)

// A^T tile builder (build_at_tile, tile32.h): (D/32)^2 workgroups (1024 at D = 1024) keep
// enough loads in flight
template <bool SQUARE, int BT = 32>
__global__ __launch_bounds__(NTHREADS) void build_at_kernel(const double* __restrict__ X, int64_t ldx,
                                                            double* __restrict__ At, int64_t D, int64_t d,
                                                            double s_arg, const Params* __restrict__ pr,
                                                            const State* __restrict__ st, double* __restrict__ IW) {
  if (st && st->status != ST_RUNNING) return;
  // s comes from device Params when given: graph replays must see each call's s
  const double s = pr ? pr->s : s_arg;
  __shared__ double tile[BT][BT + 1];
  build_at_tile<SQUARE, BT>(blockIdx.y, blockIdx.x, X, ldx, At, D, d, s, IW, tile, pr && pr->w32);
}

// Reciprocal to ~1 ulp: hardware seed + two Newton steps (no IEEE division chain).
__device__ __forceinline__ double fast_rcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = __builtin_fma(-x, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-x, r, 1.0);
  return __builtin_fma(r, e, r);
}

// In-place unpivoted GJ inverse of the 32 x 32 tile held in `img` (row stride ST)
// by the whole workgroup; writes the inverse to Pout (ld NB) and log|pivot| to plog.
// `scratch` needs 4*NB doubles.  Ends with a barrier.
__device__ __forceinline__ void invert_tile32(double* __restrict__ img, double* __restrict__ Pout, double* __restrict__ plog,
                              double* __restrict__ scratch) {
  const int tid = threadIdx.x;
  const int r = tid / TPR, c0 = (tid % TPR) * EPT;
  double* rowbuf = scratch;           // [2][NB]
  double* colbuf = scratch + 2 * NB;  // [2][NB]
  double a[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) a[e] = img[r * ST + c0 + e];
  double pivs = 0.0;  // lane p of wave 0 keeps pivot p (p < 32)
  for (int pb = 0; pb < NB; pb += EPT) {
#pragma unroll
    for (int pp = 0; pp < EPT; ++pp) {
      const int p = pb + pp;
      const int par = p & 1;
      if (r == p) {
#pragma unroll
        for (int e = 0; e < EPT; ++e) rowbuf[par * NB + c0 + e] = a[e];
      }
      if (c0 == pb) colbuf[par * NB + r] = a[pp];
      __syncthreads();
      const double piv = rowbuf[par * NB + p];
      const double inv = fast_rcp(piv);
      const double arp = colbuf[par * NB + r];
      const double neg_arp_inv = -arp * inv;
      if (tid == p) pivs = piv;
#pragma unroll
      for (int e = 0; e < EPT; ++e) {
        const int c = c0 + e;
        const double rpc = rowbuf[par * NB + c] * inv;
        if (r == p)
          a[e] = (c == p) ? inv : rpc;
        else
          a[e] = (c == p) ? neg_arp_inv : __builtin_fma(-arp, rpc, a[e]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < EPT; ++e) Pout[r * NB + c0 + e] = a[e];
  if (plog && tid < NB) plog[tid] = log(fabs(pivs));
  __syncthreads();
}

// Warm-started inverse of the 32 x 32 tile S by a product-form Neumann series.
//   X0 = the same block's inverse one Adam step earlier (W moves by ~lr per step),
//   R = I - S X0 (small), and  S^-1 = X0 (I - R)^-1 = X0 (I + R)(I + R^2)(I + R^4)...
// Pass p holds Y = X0 (I + R)...(I + R^(2^(p-1))) and Q = R^(2^p) and computes the two
// independent products  Y <- Y + Y Q,  Q <- Q Q  in one pass (interleaved MFMA chains),
// one barrier per pass.  Q is the exact residual of the truncation (Y_p S = I - Q), so
// once rho = 32 max|Q_ij| (>= ||Q||_inf) <= 1e-8 the last factor lands at residual
// <= 1e-16 -- the same test as Newton-Schulz (whose residual after p steps is this Q),
// with one barrier per doubling instead of two.
// Returns false (caller falls back to Gauss-Jordan) if rho(R) > 0.25 or is not finite, or
// no convergence within 5 doublings.  On success the inverse is in `x` (accumulator layout).
// Precondition: Sl = S and Xa = X0 (= x) written and a barrier passed.  Sl, Xa, Rl, Xb
// are four LDS images; the pass images ping-pong between (Xa, Rl) and (Sl, Xb).
__device__ __forceinline__ float quad_absmax(const dbl4& q) {
  float m = 0.0f;
#pragma unroll
  for (int t = 0; t < 4; ++t) m = fmaxf(m, isfinite(q[t]) ? (float)fabs(q[t]) : INFINITY);
  return m;
}

__device__ __forceinline__ bool ns_invert_tile32(double* Sl, double* Xa, double* Xb, double* Rl, float* red,
                                                 dbl4& x, int sk = 0) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  STAMP(sk, 5);
  dbl4 q = {0.0, 0.0, 0.0, 0.0};
  mma32(Sl, Xa, q);
  acc_foreach(q, [&](int row, int col, double& v) {
    v = (row == col ? 1.0 : 0.0) - v;  // R = I - S X0
    Rl[row * ST + col] = v;
  });
  float amax = wave_max(quad_absmax(q));
  if (lane == 0) red[w] = amax;
  __syncthreads();  // R and red complete
  STAMP(sk, 6);
  double rho = 32.0 * (double)fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  if (!(rho <= 0.25)) return false;  // too far from the warm start (or not finite)
  double *Y = Xa, *Q = Rl, *Yn = Sl, *Qn = Xb;
  int p = 0;
  for (; rho > 1e-8; ++p) {
    if (p == 4) return false;
    q = dbl4{0.0, 0.0, 0.0, 0.0};
    mma32x2(Y, Q, x, Q, Q, q);  // x = Y + Y Q ; q = Q Q
    acc_foreach(x, [&](int row, int col, double& v) { Yn[row * ST + col] = v; });
    acc_foreach(q, [&](int row, int col, double& v) { Qn[row * ST + col] = v; });
    amax = wave_max(quad_absmax(q));
    if (lane == 0) red[4 * ((p + 1) & 1) + w] = amax;  // alternate slots: no read/write race
    __syncthreads();  // Y, Q of the next pass complete; this pass's reads done
    const float* rr = red + 4 * ((p + 1) & 1);
    rho = 32.0 * (double)fmaxf(fmaxf(rr[0], rr[1]), fmaxf(rr[2], rr[3]));
    double* t = Y;
    Y = Yn;
    Yn = t;
    t = Q;
    Q = Qn;
    Qn = t;
  }
#ifdef MIDAGMA_STAMPS
  if (threadIdx.x == 0) g_stamps[sk & 255][7] = p + 1;
#endif
  mma32(Y, Q, x);  // x = Y (I + Q)
  return true;
}

// Invert the 32 x 32 tile `acc` (accumulator layout) into Pn (+ Pstore): warm-started
// Newton-Schulz from x0 unless pivots are wanted (then, or on NS failure, Gauss-Jordan).
// Precondition: no wave still reads Simg or Xa (the caller's last MFMA chain used Xb / Rl
// at most).  Buffers: four 32 x ST images + scratch (4 * NB).
__device__ __forceinline__ void invert_diag_tile(dbl4 acc, dbl4 x0, double* __restrict__ Pn, double* __restrict__ Pstore,
                                 double* __restrict__ plog, bool want_gj, double* Simg, double* Xa, double* Xb,
                                 double* Rl, double* scratch, int sk = 0) {
  acc_foreach(acc, [&](int row, int col, double& v) { Simg[row * ST + col] = v; });
  if (!want_gj) acc_foreach(x0, [&](int row, int col, double& v) { Xa[row * ST + col] = v; });
  __syncthreads();
  if (!want_gj) {
    if (ns_invert_tile32(Simg, Xa, Xb, Rl, reinterpret_cast<float*>(scratch), x0, sk)) {
      acc_foreach(x0, [&](int row, int col, double& v) {
        st_wt(Pn + row * NB + col, v);
        st_wt(Pstore + row * NB + col, v);
      });
      return;
    }
    __syncthreads();
  }
  invert_tile32(Simg, Pn, plog, scratch);
  if (Pstore) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int it = 0; it < NB * NB / NTHREADS; ++it) {
      const int e = it * NTHREADS + tid;
      Pstore[e] = Pn[e];
    }
  }
}

__device__ __forceinline__ bool want_gauss_jordan(const double* Pstore, const State* st) {
  return st == nullptr || Pstore == nullptr || st->ckpt_pending || !st->warm_valid;
}

// Prologue tile t: publish step 0's panels (column tile t, row tile t) and, for t = 0, invert A_00.
// img: four 32 x ST LDS images, scratch: 4 * NB doubles.
__device__ __forceinline__ void gj_prologue_tile(int t, const double* __restrict__ A, int64_t lda, int64_t D,
                                                 double* __restrict__ Cside, double* __restrict__ Rside,
                                                 double* __restrict__ Pside, double* __restrict__ pivlog,
                                                 double* __restrict__ Pstore, const State* __restrict__ st,
                                                 double (*img)[NB * ST], double* scratch) {
  tile32_copy(Cside + (int64_t)t * NB * NB, NB, A + (int64_t)t * NB * lda, lda);  // column 0
  tile32_copy(Rside + (int64_t)t * NB, D, A + (int64_t)t * NB, lda);              // row 0
  if (t != 0) return;
  const bool want_gj = want_gauss_jordan(Pstore, st);
  dbl4 acc, x0 = {0.0, 0.0, 0.0, 0.0};
  acc_foreach(acc, [&](int row, int col, double& v) { v = A[(int64_t)row * lda + col]; });
  if (!want_gj) acc_foreach(x0, [&](int row, int col, double& v) { v = Pstore[row * NB + col]; });
  invert_diag_tile(acc, x0, Pside, Pstore, pivlog, want_gj, img[0], img[1], img[2], img[3], scratch);
}

// Prologue: publish step 0's panels and invert A_00.
__global__ __launch_bounds__(NTHREADS) void gj_prologue_kernel(const double* __restrict__ A, int64_t lda, int64_t D,
                                                               double* __restrict__ Cside,
                                                               double* __restrict__ Rside,
                                                               double* __restrict__ Pside,
                                                               double* __restrict__ pivlog,
                                                               double* __restrict__ Pstore,
                                                               const State* __restrict__ st) {
  if (st && st->status != ST_RUNNING) return;
  __shared__ __attribute__((aligned(16))) double img[4][NB * ST];
  __shared__ double scratch[4 * NB];
  gj_prologue_tile(blockIdx.x, A, lda, D, Cside, Rside, Pside, pivlog, Pstore, st, img, scratch);
}

// One block step of the elimination (see file header).
//   side buffers: Cside[2] (D x NB), Rside[2] (NB x D), Pside[2] (NB x NB), parity k & 1 read.
//   Every operand is requested from memory at kernel entry, so each step pays one
//   global-load latency before its MFMA chain.  The workgroup owning tile (k+1, k+1)
//   carries the step's serial chain: it takes linear block id 0 (dispatched first),
//   prefetches its warm start with the operands, inverts before any global store.
// Tile (bi, bj) of block step k.  L0, L1, R0, T0: 32 x ST LDS images; scratch 4 * NB doubles.
// PRIO: raise the diagonal owner's wave priority (the launch-per-step form, where co-resident
// tiles compete for its SIMD).
template <bool PRIO>
__device__ __forceinline__ void gj_step_tile(int bi, int bj, double* __restrict__ A, int64_t lda, int64_t D, int k,
                                             double* __restrict__ Cside0, double* __restrict__ Cside1,
                                             double* __restrict__ Rside0, double* __restrict__ Rside1,
                                             double* __restrict__ Pside0, double* __restrict__ Pside1,
                                             double* __restrict__ pivlog, double* __restrict__ Pstore,
                                             const State* __restrict__ st, double* L0, double* L1, double* R0,
                                             double* T0, double* scratch) {
  const int K = (int)(D / NB);
  const int k1 = k + 1;
  const bool odd = k & 1;
  const double* Cs = odd ? Cside1 : Cside0;
  const double* Rs = odd ? Rside1 : Rside0;
  const double* P = odd ? Pside1 : Pside0;
  double* Cn = odd ? Cside0 : Cside1;
  double* Rn = odd ? Rside0 : Rside1;
  double* Pn = odd ? Pside0 : Pside1;
  double* Aij = A + (int64_t)bi * NB * lda + (int64_t)bj * NB;
  const bool owner = k1 < K && bi == k1 && bj == k1;
  if (PRIO && owner) {
    __builtin_amdgcn_s_setprio(3);  // its waves win issue arbitration against co-resident tiles
    STAMP(k, 0);
  }

  dbl4 acc = {0.0, 0.0, 0.0, 0.0};
  if (bi == k && bj == k) {
    acc_foreach(acc, [&](int row, int col, double& v) { v = P[row * NB + col]; });  // A_kk = P
  } else if (bi == k) {
    tile32_to_lds(L0, P, NB, 1.0);  // A_kj = P R_j
    tile32_to_lds(R0, Rs + (int64_t)bj * NB, D, 1.0);
    __syncthreads();
    mma32(L0, R0, acc);
  } else if (bj == k) {
    tile32_to_lds(L1, Cs + (int64_t)bi * NB * NB, NB, -1.0);  // A_ik = -C_i P
    tile32_to_lds(R0, P, NB, 1.0);
    __syncthreads();
    mma32(L1, R0, acc);
  } else {
    // T = P R_j ; A_ij += (-C_i) T        (all operands requested up front)
    bool want_gj = true;
    dbl4 x0 = {0.0, 0.0, 0.0, 0.0};
    if (owner) {
      want_gj = want_gauss_jordan(Pstore, st);
      if (!want_gj) {
        const double* X0 = Pstore + (int64_t)k1 * NB * NB;
        acc_foreach(x0, [&](int row, int col, double& v) { v = X0[row * NB + col]; });
      }
    }
    tile32_to_lds(L0, P, NB, 1.0);
    tile32_to_lds(R0, Rs + (int64_t)bj * NB, D, 1.0);
    tile32_to_lds(L1, Cs + (int64_t)bi * NB * NB, NB, -1.0);
    dbl4 a_old;
    acc_foreach(a_old, [&](int row, int col, double& v) { v = Aij[(int64_t)row * lda + col]; });
    __syncthreads();
    if (owner) STAMP(k, 1);
    dbl4 tq = {0.0, 0.0, 0.0, 0.0};
    mma32(L0, R0, tq);
    acc_foreach(tq, [&](int row, int col, double& v) { T0[row * ST + col] = v; });
    __syncthreads();
    if (owner) STAMP(k, 2);
    acc = a_old;
    mma32(L1, T0, acc);
    if (owner) {
      // the only serial chain of the elimination: invert first, store afterwards.
      // L0 / R0 are free (last read before the barrier above); L1 / T0 after the next one.
      STAMP(k, 3);
#ifndef MIDAGMA_GJ_TIMING_NO_INV  // timing experiment only: results are wrong without it
      invert_diag_tile(acc, x0, Pn, Pstore ? Pstore + (int64_t)k1 * NB * NB : nullptr, pivlog ? pivlog + (int64_t)k1 * NB : nullptr, want_gj, L0, R0, L1,
                       T0, scratch, k);
#endif
      STAMP(k, 4);
    }
  }
  acc_foreach(acc, [&](int row, int col, double& v) { st_wt(Aij + (int64_t)row * lda + col, v); });
  if (k1 >= K) return;
  if (bj == k1) acc_foreach(acc, [&](int row, int col, double& v) { st_wt(Cn + ((int64_t)bi * NB + row) * NB + col, v); });
  if (bi == k1) acc_foreach(acc, [&](int row, int col, double& v) { st_wt(Rn + (int64_t)row * D + (int64_t)bj * NB + col, v); });
}

__global__ __launch_bounds__(NTHREADS) void gj_step_kernel(double* __restrict__ A, int64_t lda, int64_t D, int k,
                                                           double* __restrict__ Cside0, double* __restrict__ Cside1,
                                                           double* __restrict__ Rside0, double* __restrict__ Rside1,
                                                           double* __restrict__ Pside0, double* __restrict__ Pside1,
                                                           double* __restrict__ pivlog, double* __restrict__ Pstore,
                                                           const State* __restrict__ st) {
  if (st && st->status != ST_RUNNING) return;
  __shared__ __attribute__((aligned(16))) double L0[NB * ST];  // P            ([m][k])
  __shared__ __attribute__((aligned(16))) double L1[NB * ST];  // -C_i         ([m][k])
  __shared__ __attribute__((aligned(16))) double R0[NB * ST];  // R_j or P     ([k][n])
  __shared__ __attribute__((aligned(16))) double T0[NB * ST];  // P R_j        ([k][n])
  __shared__ double scratch[4 * NB];
  const int K = (int)(D / NB);
  const int k1 = k + 1;
  const int own = k1 < K ? k1 * K + k1 : 0;  // linear id of the diagonal owner
  int lin = blockIdx.y * K + blockIdx.x;
  lin = lin == 0 ? own : (lin == own ? 0 : lin);
  const int bi = lin / K, bj = lin - bi * K;
  gj_step_tile<true>(bi, bj, A, lda, D, k, Cside0, Cside1, Rside0, Rside1, Pside0, Pside1, pivlog, Pstore, st, L0, L1,
                     R0, T0, scratch);
}

// The whole Gauss-Jordan inverse of (sI - A)^T (build, prologue, the D/32 block steps) in ONE
// workgroup, gated on st: the fallback of a warm-started log-det step whose certificate failed
// (midagma_ldfast_*), where a closed gate must cost one launch, not the 2 + D/32 of the chain.
// The tiles run one after the other with the launch-per-step kernels' tile bodies in each phase,
// so the result is theirs bit for bit (a phase's tiles read only what earlier phases wrote).  Own
// stores are made visible to the workgroup's later loads by draining them, a barrier, and an
// agent-scope acquire (which invalidates this CU's L1) between phases.
__device__ __forceinline__ void gj_1wg_phase_end() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// ldfast_post's work (mlp.hip) for a fast step, in the workgroup that ran (or skipped) the
// gated chain: the same values and the same piv sum order.  One workgroup: every thread reads
// the step's slot before thread 0 counts it, after the reduction's barriers.
static __device__ void ldfast_end_1wg(const LdfastEnd& e, bool ran, const double* __restrict__ Wgj, int64_t Dgj) {
  const int64_t slot = e.st->slots + 1;
  if (ran) {
    double* dst = (slot & 1) ? e.ring1 : e.ring0;
    for (int64_t x = threadIdx.x; x < (int64_t)e.B * e.B; x += NTHREADS) {
      const int64_t i = x / e.B, j = x % e.B;
      dst[x] = (i < Dgj && j < Dgj) ? Wgj[i * Dgj + j] : (i == j ? 1.0 : 0.0);
    }
    for (int64_t x = threadIdx.x; x < e.d * e.d; x += NTHREADS) {
      const int64_t i = x / e.d, j = x % e.d;
      e.Mt[i * e.ldm + j] = Wgj[i * Dgj + j];
    }
  }
  __shared__ double red[NTHREADS];
  double acc = 0.0;
  if (ran)
    for (int64_t k = threadIdx.x; k < e.d; k += NTHREADS) acc += e.piv[k];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s2 = NTHREADS / 2; s2 > 0; s2 >>= 1) {
    if ((int)threadIdx.x < s2) red[threadIdx.x] += red[threadIdx.x + s2];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    State* st = e.st;
    const double hv = ran ? -red[0] + e.dls : e.hlast[0];
    e.h[0] = hv;
    if (ran) e.hlast[0] = hv;
    st->warm_run = st->warm_run < 2 ? st->warm_run + 1 : 2;
    st->ckpt_pending = 0;
    st->status = ST_RUNNING;
    st->iter += 1;
    if (ran) st->halvings += 1;
    st->slots = slot;
    if (e.counter) *e.counter += 1;  // (midagma_ldfast_set_counter: counter_advance's work)
  }
}

static __device__ void gj_inverse_1wg_body(const double* __restrict__ X, int64_t ldx, double* __restrict__ A,
                                           int64_t D, int64_t d, double s, const GJWork& w, const State* __restrict__ st) {
  __shared__ __attribute__((aligned(16))) double img[4][NB * ST];
  __shared__ double scratch[4 * NB];
  double(&tile)[32][33] = *reinterpret_cast<double(*)[32][33]>(&img[0][0]);  // build phase only
  const int K = (int)(D / NB);
  for (int bi = 0; bi < K; ++bi)
    for (int bj = 0; bj < K; ++bj) {
      build_at_tile<false, 32>(bi, bj, X, ldx, A, D, d, s, nullptr, tile);
      __syncthreads();
    }
  gj_1wg_phase_end();
  for (int t = 0; t < K; ++t) {
    gj_prologue_tile(t, A, D, D, w.C, w.R, w.P, w.pivlog, w.Pstore, st, img, scratch);
    __syncthreads();
  }
  gj_1wg_phase_end();
  for (int k = 0; k < K; ++k) {
    for (int bi = 0; bi < K; ++bi)
      for (int bj = 0; bj < K; ++bj) {
        gj_step_tile<false>(bi, bj, A, D, D, k, w.C, w.C + D * NB, w.R, w.R + NB * D, w.P, w.P + NB * NB, w.pivlog,
                            w.Pstore, st, img[0], img[1], img[2], img[3], scratch);
        __syncthreads();
      }
    gj_1wg_phase_end();
  }
}

__global__ __launch_bounds__(NTHREADS) void gj_inverse_1wg_kernel(const double* __restrict__ X, int64_t ldx,
                                                                  double* __restrict__ A, int64_t D, int64_t d,
                                                                  double s, GJWork w, const State* __restrict__ st,
                                                                  LdfastEnd end) {
  const bool ran = !st || st->status == ST_RUNNING;
  if (ran) gj_inverse_1wg_body(X, ldx, A, D, d, s, w, st);
  if (end.st) ldfast_end_1wg(end, ran, A, D);
}

void gj_setup_attributes() {}

#ifdef MIDAGMA_STAMPS
extern "C" int midagma_debug_stamps(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(g_stamps));
}
#endif

void launch_build_at(const double* X, int64_t ldx, bool square, double* At, int64_t D, int64_t d, double s,
                     const Params* pr, const State* st, hipStream_t stream, double* IW) {
  if (D % 32) throw std::invalid_argument("build_at: D must be a multiple of 32");
  const int K = (int)(D / 32);
  dim3 grid(K, K);
  if (square)
    hipLaunchKernelGGL(build_at_kernel<true>, grid, dim3(NTHREADS), 0, stream, X, ldx, At, D, d, s, pr, st, IW);
  else
    hipLaunchKernelGGL(build_at_kernel<false>, grid, dim3(NTHREADS), 0, stream, X, ldx, At, D, d, s, pr, st, IW);
  HIP_TRY(hipGetLastError());
}

void launch_gj_prologue(double* A, int64_t lda, int64_t D, const GJWork& w, const State* st, hipStream_t stream) {
  const int K = (int)(D / NB);
  hipLaunchKernelGGL(gj_prologue_kernel, dim3(K), dim3(NTHREADS), 0, stream, A, lda, D, w.C, w.R, w.P, w.pivlog,
                     w.Pstore, st);
  HIP_TRY(hipGetLastError());
}

void launch_gj_step(double* A, int64_t lda, int64_t D, const GJWork& w, const State* st, int k, hipStream_t stream) {
  const int K = (int)(D / NB);
  hipLaunchKernelGGL(gj_step_kernel, dim3(K, K), dim3(NTHREADS), 0, stream, A, lda, D, k, w.C, w.C + D * NB, w.R,
                     w.R + NB * D, w.P, w.P + NB * NB, w.pivlog, w.Pstore, st);
  HIP_TRY(hipGetLastError());
}

void launch_gj_inverse_1wg(const double* X, int64_t ldx, double* At, int64_t D, int64_t d, double s, const GJWork& w,
                           const State* st, hipStream_t stream, const LdfastEnd& end) {
  if (D % 32) throw std::invalid_argument("gj_inverse_1wg: D must be a multiple of 32");
  if (end.st && (end.d > D || end.d > end.B)) throw std::invalid_argument("gj_inverse_1wg: bad end arguments");
  hipLaunchKernelGGL(gj_inverse_1wg_kernel, dim3(1), dim3(NTHREADS), 0, stream, X, ldx, At, D, d, s, w, st, end);
  HIP_TRY(hipGetLastError());
}

void launch_gj_inverse(double* A, int64_t lda, int64_t D, const GJWork& w, const State* st, hipStream_t stream) {
  launch_gj_prologue(A, lda, D, w, st, stream);
  for (int k = 0; k < (int)(D / NB); ++k) launch_gj_step(A, lda, D, w, st, k, stream);
}

}  // namespace midagma
