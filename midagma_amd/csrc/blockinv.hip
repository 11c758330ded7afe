// Two-level blocked Gauss-Jordan inverse of sI - W∘W (transposed), the cov-mode slot's
// replacement for `sla.inv(s*I - W*W)` (linear.py:226, 240) when D = 128 or D >= 256 (D % 128 == 0).
//
// Outer block Gauss-Jordan over B2-wide pivot blocks (B2 = 256, or 128 when 256 does not
// divide D; one block, B2 = D, at D = 128, and at 512 as an experiment).  Outer step g sweeps pivot block
// G = [g B2, (g+1) B2):
//     P = S^-1 with S = A_GG (the Schur complement left by the steps before g)
//     A_Gj <- P A_Gj     A_iG <- -A_iG P     A_ij <- A_ij - A_iG (P A_Gj)     A_GG <- P
// -- the sweep gj.hip applies at 32 granularity; after every block is swept A holds A^-1.
// Each outer step reads one D x D buffer and writes the other (ping-pong), so the panel and
// trailing kernels never read what a workgroup of the same launch writes.
//
// S^-1 has two sources:
//   fast (this file)  S^-1 = X0 (I + R)(I + R^2)(I + R^4)...,  X0 = 2 P(k-1) - P(k-2), the
//         linear extrapolation of this block's P in the last two slots (W moves smoothly, by
//         ~lr per Adam step; P(k-1) alone right after a slow start), R = I - S X0.  One residual launch and up
//         to NM_PASSES pass launches of B2^3 products spread over (B2/16)^2 workgroups
//         with K split over the 4 waves -- no serial chain of 32 x 32 inversions.  Pass p
//         holds Y = X0 (I + R)...(I + R^(2^(p-1))) and Q = R^(2^p), the exact residual of
//         Y (Y S = I - Q); once rho = ||Q||_inf (max row sum of |Q|) is <= 1e-8 the last
//         factor Y (I + Q) lands at residual <= 1e-16 and the pass writes P instead.
//   slow  (gj.hip)    the 32-block Gauss-Jordan run in place on the B2 x B2 block: pivots
//         for the log-det on checkpoint slots, and every slot the fast path cannot take
//         (first slot of a minimize call, rho > 0.25, no convergence): the fast kernels
//         then set ST_NEED_GJ and the host re-runs the slot on the slow path.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "binv_tile.h"
#include "kstamps.h"
#include "launch.h"
#include "nm16.h"
#include "nm_series.h"

namespace midagma {

namespace {



// Look-ahead residual of the next outer block gn = g + 1 (fast path).  With X0 its warm start
// and S = A(gn,gn) - A(gn,G) P_g A(G,gn) the Schur complement the trailing update of step g
// leaves,  R = I - S X0 = I - (LW - A(gn,G) LPZ),  LW = A(gn,gn) X0,  LZ = A(G,gn) X0,
// LPZ = P_g LZ: LW and LZ are extra tiles of block g's first and second pass, LPZ of its panel launch and
// R of its trailing update, so block gn needs no residual launch of its own.
struct NmLA {  // extra tiles of a pass launch: out = A X0(gn) (A: a block of step g's input)
  const double* A;   // pass 1: A(gn, gn) -> LW; pass 2: A(G, gn) -> LZ
  int64_t lda;
  const double* Pe;  // block gn's warm-start stores
  const double* Po;
  double* out;
};
struct TrailLA {  // trailing-launch extra tiles
  const double* LW;
  const double* LPZ;
  const double* Pe;
  const double* Po;
  double* Y0;     // block gn's first iterate X0 and residual R, its row partials, its done word
  double* Q0;
  double* part0;
  int* done;
  int gn;
};

template <int L, int NW = 4>
__global__ __launch_bounds__(64 * NW) void nm_resid_kernel(const double* __restrict__ S, int64_t lds,
                                                           const double* __restrict__ Pe,
                                                           const double* __restrict__ Po, double* __restrict__ Y0,
                                                           double* __restrict__ Q0, double* __restrict__ part0,
                                                           int* __restrict__ done, State* __restrict__ st,
                                                           int xmap) {
  if (st->status != ST_RUNNING) return;
  __shared__ double red[NW * 256];
  nm_resid_body<L, NW, false>(blockIdx.x, S, lds, SFromW{}, Pe, Po, Y0, Q0, part0, done, st, xmap, red);
}

// The DagmaMLP log-det's fast step opened by its residual (no launch before it): the Gauss-Jordan
// gate reset to "skip", S = (sI - A)^T read from A by the tiles themselves, the warm start's
// parity that of the step the end (ldfast_end_1wg, gj.hip) will count, st->slots + 1
template <int L>
__global__ __launch_bounds__(NTHREADS) void ldfast_resid_kernel(const double* __restrict__ A, int64_t lda, int64_t d,
                                                                double s, const double* __restrict__ Pe,
                                                                const double* __restrict__ Po,
                                                                double* __restrict__ Y0, double* __restrict__ Q0,
                                                                double* __restrict__ part0, int* __restrict__ done,
                                                                State* __restrict__ st, State* __restrict__ gjst,
                                                                int xmap) {
  if (blockIdx.x == 0 && threadIdx.x == 0) gjst->status = ST_DONE;
  if (st->status != ST_RUNNING) return;
  __shared__ double red[4 * 256];
  SFromW sa{A, lda, d, nullptr, s};
  nm_resid_body<L, 4, false, true>(blockIdx.x, nullptr, 0, sa, Pe, Po, Y0, Q0, part0, done, st, xmap, red, 1);
}

#ifdef MIDAGMA_EXPERIMENTS
// build_at and outer block 0's residual in one launch (fast slots, B2 = 256): workgroups
// [0, (D/32)^2) build the At tiles, the next 256 the residual tiles with S read from W (the two
// read W only and write disjoint buffers), one dependent launch fewer per slot
__global__ __launch_bounds__(NTHREADS) void build_resid0_kernel(const double* __restrict__ W, int64_t ldw,
                                                                double* __restrict__ At, int64_t D, int64_t d,
                                                                const Params* __restrict__ pr,
                                                                const double* __restrict__ Pe,
                                                                const double* __restrict__ Po, double* __restrict__ Y0,
                                                                double* __restrict__ Q0, double* __restrict__ part0,
                                                                int* __restrict__ done, State* __restrict__ st,
                                                                int xmap) {
  if (st->status != ST_RUNNING) return;
  const int kb = (int)(D / 32), nbuild = kb * kb;
  if ((int)blockIdx.x < nbuild) {
    __shared__ double tile[32][33];
    build_at_tile<true, 32>((int)blockIdx.x / kb, (int)blockIdx.x % kb, W, ldw, At, D, d, pr->s, nullptr, tile,
                            pr->w32 != 0);
  } else {
    __shared__ double red[4 * 256];
    nm_resid_body<16, 4, true>((int)blockIdx.x - nbuild, nullptr, 0, SFromW{W, ldw, d, pr}, Pe, Po, Y0, Q0, part0,
                               done, st, xmap, red);
  }
}

#endif

// Pass p: rho = ||Q||_inf from the previous launch's row partials; converged -> P = Y + Y Q
// (done = p), else Y' = Y + Y Q, Q' = Q Q and the row partials of |Q'|.  Far or diverging
// -> ST_NEED_GJ.  (Tile body: nm_pass_body, nm_series.h.)
template <int L, int NW = 4>
__global__ __launch_bounds__(64 * NW) void nm_pass_kernel(const double* __restrict__ Y,
                                                          const double* __restrict__ Q, double* __restrict__ Yn,
                                                          double* __restrict__ Qn, double* __restrict__ P,
                                                          const double* __restrict__ part_prev,
                                                          double* __restrict__ part_next, int* __restrict__ done,
                                                          int pass, State* __restrict__ st, NmLA la, int xmap) {
  if (st->status != ST_RUNNING) return;
  constexpr int B2 = 4 * NW * L;
  __shared__ double red[NW * 256];
  __shared__ float red4[NW];
  const int nt = B2 / 16, tid = threadIdx.x;
  if ((int)blockIdx.x >= nt * nt) {  // look-ahead tiles of the next block (LW or LZ)
    const int t = (int)blockIdx.x - nt * nt;
    const int m0 = (t / nt) * 16, n0 = (t % nt) * 16;
    double a[L], b[L];
    splitk_load_a<L>(la.A, la.lda, m0, a);
    load_x0_b<L>(la.Pe, la.Po, st, n0, b);
    dbl4 acc = {0.0, 0.0, 0.0, 0.0};
    splitk_mfma<L>(a, b, acc);
    const double sum = splitk_sum_w<NW>(acc, red);
    if (tid >= 256) return;
    int row, col;
    tile_elem(tid, row, col);
    st_wt(la.out + (int64_t)(m0 + row) * B2 + n0 + col, sum);
    return;
  }
  nm_pass_body<L, NW>(blockIdx.x, Y, Q, Yn, Qn, P, part_prev, part_next, done, pass, st, xmap, red, red4);
}

#ifdef MIDAGMA_EXPERIMENTS
#include "../../experiments/blockinv_exp.inc"
#endif  // MIDAGMA_EXPERIMENTS

// the next block's series counters (launch_trail128_series), zeroed by the panel launch before
// the trailing update that runs that series: [0] diagonal tiles, [32 p] phase p (p <= NM_PASSES)
__device__ __forceinline__ void zero_sync(int* zsync) {
  if (zsync && blockIdx.x == 0 && threadIdx.x < 8) {  // the pass words, and the fused panel's (launch.h)
    const int w = threadIdx.x <= NM_PASSES ? 32 * threadIdx.x
                                           : (threadIdx.x == 5 ? TS_FIN : threadIdx.x == 6 ? TS_BAND : TS_JOB);
    __hip_atomic_store(zsync + w, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// prefetch depth of the panel / trailing tiles (experiment knob MIDAGMA_EXP_T32_PF: 1, 2, 3;
// d=1000 fast slot: 4160 steps/s at 1, 4340 at 3, two runs each)
static int t32_pf() {
  static const int pf = (int)knob("MIDAGMA_EXP_T32_PF", 3);
  return pf < 1 ? 1 : (pf > 3 ? 3 : pf);
}

// Panels of outer step g (one 32 x 32 tile per workgroup):
//   U  Aout[G, j] = P Ain[G, j]         (j outside G)
//   V  Aout[i, G] = -Ain[i, G] P        (i outside G)
//   P  Aout[G, G] = P, Pst = P          (next slot's warm start)
// With `done` (fast path) an unconverged block hands the slot to the host (ST_NEED_GJ).
// SBPF > 0: one LDS image per operand (17 KB instead of 34 KB; two barriers per chunk) at the
// fixed prefetch depth SBPF (fewer VGPRs than the runtime-depth kernel's 132), B2 = 256; the
// same arithmetic
template <int SBPF>
__global__ __launch_bounds__(NTHREADS) void binv_panel_kernel(const double* __restrict__ Ain,
                                                              double* __restrict__ Aout, int64_t D, int B2, int g,
                                                              const double* __restrict__ P, int64_t ldp,
                                                              double* __restrict__ Pe, double* __restrict__ Po,
                                                              const int* __restrict__ done, int check,
                                                              State* __restrict__ st, int pf,
                                                              const double* __restrict__ LZ,
                                                              double* __restrict__ LPZ, int* __restrict__ zsync) {
  if (st && st->status != ST_RUNNING) return;
  zero_sync(zsync);
  if (done && *done == 0) {
    if (blockIdx.x == 0 && threadIdx.x == 0) st->status = ST_NEED_GJ;
    return;
  }
  constexpr bool SB = SBPF > 0;
  __shared__ __attribute__((aligned(16))) double img[SB ? 2 : 4][NB * ST];
  binv_panel_job<SBPF>(xcd_spread(blockIdx.x, gridDim.x), Ain, Aout, D, B2, g, P, ldp, Pe, Po, check, st, pf, LZ, LPZ,
                       img[0], img[SB ? 0 : 1], img[SB ? 1 : 2], img[SB ? 1 : 3]);
}

using PanelKernel = void (*)(const double*, double*, int64_t, int, int, const double*, int64_t, double*, double*,
                             const int*, int, State*, int, const double*, double*, int*);
// the panel kernel at B2 = 256: single-buffered at prefetch depth MIDAGMA_EXP_PANEL_SB (1..3) from
// D >= MIDAGMA_EXP_PANEL_SB_MIN on (experiment knobs), else the double-buffered runtime-depth one
static PanelKernel panel_kernel_sb(int64_t D) {
  const long pf = knob("MIDAGMA_EXP_PANEL_SB", 0);  // (read per launch: tests switch it in one process)
  const long from = knob("MIDAGMA_EXP_PANEL_SB_MIN", 0);
  if (D < from || pf <= 0) return binv_panel_kernel<0>;
  return pf == 1 ? binv_panel_kernel<1> : pf == 2 ? binv_panel_kernel<2> : binv_panel_kernel<3>;
}

// ---- panels on 64 x 64 tiles (B2 = 256, large D) ------------------------------------------------
// The 32 x 32 panel tile reads a 32 x 256 and a 256 x 32 operand slab for 0.5 MFLOP (4 flop per
// byte, one 16 x 16 accumulator per wave): at D = 5120 its 2496 workgroups take 34 us for 1.27
// GFLOP (37 TF) against a 16 us MFMA floor.  The 64 x 64 tile gives each wave a 32 x 32 quadrant
// (2 x 2 accumulators: twice the flops per byte) in 624 workgroups, one round at three per CU.
constexpr int P64_AS = 34;  // A chunk image [64][32] (m-major; = 2 mod 32: conflict-free MFMA A reads)
constexpr int P64_BS = 80;  // B chunk image [32][64] (= 16 mod 32: the two kq halves on disjoint banks)
constexpr int P64_PF = 2;   // chunks in flight in registers ahead of the MFMAs

// acc[i][j] += A(64 x 32) B(32 x 64) on this wave's 32 x 32 quadrant.  CHAINS: mma32's order per
// accumulator (four k-chains per 32-deep chunk summed (c0 + c1) + (c2 + c3): bit-identical to
// the 32 x 32 panel), else one chain per accumulator, the four accumulators interleaved (fewer
// live registers)
template <bool CHAINS>
__device__ __forceinline__ void mma64x32(const double* __restrict__ As, const double* __restrict__ Bs,
                                         dbl4 (&acc)[2][2]) {
  const int lane = threadIdx.x & 63, r = lane & 15, kq = lane >> 4, w = threadIdx.x >> 6;
  const int m0 = (w >> 1) * 32, n0 = (w & 1) * 32;
  if constexpr (CHAINS) {
    const dbl4 z = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const double* La = As + (m0 + 16 * i + r) * P64_AS + kq;
        const double* Rb = Bs + kq * P64_BS + n0 + 16 * j + r;
        dbl4 c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(La[0], Rb[0], acc[i][j], 0, 0, 0);
        dbl4 c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(La[4], Rb[4 * P64_BS], z, 0, 0, 0);
        dbl4 c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(La[8], Rb[8 * P64_BS], z, 0, 0, 0);
        dbl4 c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(La[12], Rb[12 * P64_BS], z, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(La[16], Rb[16 * P64_BS], c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(La[20], Rb[20 * P64_BS], c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(La[24], Rb[24 * P64_BS], c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(La[28], Rb[28 * P64_BS], c3, 0, 0, 0);
        acc[i][j] = (c0 + c1) + (c2 + c3);
      }
  } else {
    const double* La = As + (m0 + r) * P64_AS + kq;
    const double* Rb = Bs + kq * P64_BS + n0 + r;
#pragma unroll
    for (int k = 0; k < 32; k += 4) {
      const double a0 = La[k], a1 = La[16 * P64_AS + k];
      const double b0 = Rb[k * P64_BS], b1 = Rb[k * P64_BS + 16];
      acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
    }
  }
}

// acc = A(64 x 256) B(256 x 64) (global, row-major): 32-deep chunks through one LDS image pair,
// the next P64_PF chunks in registers (the operands come from the previous launch: MALL trips)
template <bool CHAINS>
__device__ __forceinline__ void tile64_gemm_k256(const double* __restrict__ A, int64_t lda,
                                                 const double* __restrict__ B, int64_t ldb, dbl4 (&acc)[2][2],
                                                 double* As, double* Bs) {
  constexpr int NK = 8;
  const int tid = threadIdx.x;
  double2 ra[P64_PF][4], rb[P64_PF][4];
  auto load = [&](double2 (&a)[4], double2 (&b)[4], int kc) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int item = it * NTHREADS + tid;
      const int ar = item >> 4, ac = (item & 15) * 2;  // A chunk: 64 rows x 32
      const int br = item >> 5, bc = (item & 31) * 2;  // B chunk: 32 rows x 64
      a[it] = *reinterpret_cast<const double2*>(A + (int64_t)ar * lda + kc * 32 + ac);
      b[it] = *reinterpret_cast<const double2*>(B + (int64_t)(kc * 32 + br) * ldb + bc);
    }
  };
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int p = 0; p < P64_PF; ++p) load(ra[p], rb[p], p);
  for (int kc = 0; kc < NK; ++kc) {
    __syncthreads();  // the previous chunk's MFMAs are done with the images
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int item = it * NTHREADS + tid;
      *reinterpret_cast<double2*>(As + (item >> 4) * P64_AS + (item & 15) * 2) = ra[0][it];
      *reinterpret_cast<double2*>(Bs + (item >> 5) * P64_BS + (item & 31) * 2) = rb[0][it];
    }
#pragma unroll
    for (int p = 0; p + 1 < P64_PF; ++p)
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        ra[p][it] = ra[p + 1][it];
        rb[p][it] = rb[p + 1][it];
      }
    if (kc + P64_PF < NK) load(ra[P64_PF - 1], rb[P64_PF - 1], kc + P64_PF);
    __syncthreads();
    mma64x32<CHAINS>(As, Bs, acc);
  }
}

template <class F>
__device__ __forceinline__ void acc64_foreach(dbl4 (&acc)[2][2], F&& f) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int m0 = (w >> 1) * 32, n0 = (w & 1) * 32;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int t = 0; t < 4; ++t) f(m0 + 16 * i + acc_row(lane, t), n0 + 16 * j + acc_col(lane), acc[i][j][t]);
}

// binv_panel_kernel's U, V and P outputs at B2 = 256 on 64 x 64 tiles (jobs: U (cq, a) with the
// four row tiles of one column tile consecutive, V (iq, c), then the 16 P tiles); no look-ahead
// CHAINS (experiments: MIDAGMA_EXP_P64_CHAINS=1): mma32's summation order, bit-identical to
// binv_panel_kernel, at 2 workgroups per CU (its chains hold 186 VGPRs); the product runs one
// chain per accumulator at 3 per CU (160 VGPRs), which rounds differently in the last bits
template <bool CHAINS>
__global__ __launch_bounds__(NTHREADS, CHAINS ? 2 : 3) void binv_panel64_kernel(const double* __restrict__ Ain,
                                                                double* __restrict__ Aout, int64_t D, int g,
                                                                const double* __restrict__ P, int64_t ldp,
                                                                double* __restrict__ Pe, double* __restrict__ Po,
                                                                const int* __restrict__ done, int check,
                                                                State* __restrict__ st, int* __restrict__ zsync) {
  constexpr int B2 = 256, GB = B2 / 64;
  if (st && st->status != ST_RUNNING) return;
  zero_sync(zsync);
  if (done && *done == 0) {
    if (blockIdx.x == 0 && threadIdx.x == 0) st->status = ST_NEED_GJ;
    return;
  }
  __shared__ __attribute__((aligned(16))) double As[64 * P64_AS];
  __shared__ __attribute__((aligned(16))) double Bs[32 * P64_BS];
  const int nb = (int)(D / 64), g0 = g * GB, mb = nb - GB, nu = GB * mb;
  const int job = xcd_spread(blockIdx.x, gridDim.x);
  const int64_t G0 = (int64_t)g * B2;
  int flag = 0;
  if (job < 2 * nu) {
    const bool u = job < nu;
    const int j = u ? job : job - nu, q = j / GB, k = j % GB, t = q < g0 ? q : q + GB;
    // U: rows 64 k of G times column tile t; V: row tile t times columns 64 k of G
    const double* A = u ? P + (int64_t)k * 64 * ldp : Ain + (int64_t)t * 64 * D + G0;
    const double* B = u ? Ain + G0 * D + (int64_t)t * 64 : P + (int64_t)k * 64;
    double* out = u ? Aout + (G0 + (int64_t)k * 64) * D + (int64_t)t * 64 : Aout + (int64_t)t * 64 * D + G0 + k * 64;
    dbl4 acc[2][2];
    tile64_gemm_k256<CHAINS>(A, u ? ldp : D, B, u ? D : ldp, acc, As, Bs);
    acc64_foreach(acc, [&](int row, int col, double v) {
      const double o = u ? v : -v;
      st_wt(out + (int64_t)row * D + col, o);
      flag |= domain_flag(o);
    });
  } else if (job < 2 * nu + GB * GB) {
    const int j3 = job - 2 * nu, a = j3 / GB, c = j3 % GB;
    const double* src = P + (int64_t)a * 64 * ldp + c * 64;
    double* out = Aout + (G0 + (int64_t)a * 64) * D + G0 + c * 64;
    double* Pst = (st && (st->slots & 1)) ? Po : Pe;  // this slot's store (parity of k)
    double* ps = Pst + (int64_t)a * 64 * B2 + c * 64;
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int e = it * NTHREADS + threadIdx.x, row = e >> 6, col = e & 63;
      const double v = src[(int64_t)row * ldp + col];
      st_wt(out + (int64_t)row * D + col, v);
      st_wt(ps + (int64_t)row * B2 + col, v);
      flag |= domain_flag(v);
    }
  }
  if (check && flag) atomicOr(&st->flags, flag);
}

// Trailing update of outer step g, one 32 x 32 tile per workgroup (binv_trail_tile).
// With la.LW: the next block's residual tiles follow the mb x mb trailing tiles (TrailLA).
__global__ __launch_bounds__(NTHREADS) void binv_trail_kernel(const double* __restrict__ Ain,
                                                              double* __restrict__ Aout, int64_t D, int B2, int g,
                                                              int check, State* __restrict__ st, int pf, TrailLA la) {
  if (st && st->status != ST_RUNNING) return;
  __shared__ __attribute__((aligned(16))) double img[4][NB * ST];
  const int job = xcd_spread(blockIdx.x, gridDim.x);
  const int gb = B2 / NB, mb = (int)(D / NB) - gb;
  if (job < mb * mb) {
    KS_DECL(ks);
    binv_trail_tile(job, Ain, Aout, D, B2, g, check, st, pf, img[0], img[1], img[2], img[3]);
    KS_END(ks, KS_TRAIL);
    return;
  }
  // R = I - (LW - A(gn, G) LPZ) on the 32 x 32 tile (a, c) of block gn; X0 -> Y0, |R| row partials
  const int j = job - mb * mb, a = j / gb, c = j % gb;
  const int64_t GN0 = (int64_t)la.gn * B2, G0 = (int64_t)g * B2;
  dbl4 acc = {0.0, 0.0, 0.0, 0.0};
  tile32_gemm_any(pf, Ain + (GN0 + (int64_t)a * NB) * D + G0, D, la.LPZ + (int64_t)c * NB, B2, B2, acc, img[0],
                  img[1], img[2], img[3]);
  const bool odd = (st->slots & 1) != 0, extrap = st->warm_run >= 2;
  const double* P1 = odd ? la.Pe : la.Po;
  const double* P2 = odd ? la.Po : la.Pe;
  const int lane = threadIdx.x & 63, m0 = q_m0(), n0 = q_n0(), nt = B2 / 16;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int row = a * NB + m0 + acc_row(lane, t), col = c * NB + n0 + acc_col(lane);
    const int64_t e = (int64_t)row * B2 + col;
    const double r = (row == col ? 1.0 : 0.0) - (la.LW[e] - acc[t]);
    st_wt(la.Q0 + e, r);
    st_wt(la.Y0 + e, extrap ? 2.0 * P1[e] - P2[e] : P1[e]);
    const double rs = row_sum16(abs_or_inf(r));  // the 16 lanes of this row: one DPP row
    if (acc_col(lane) == 0) st_wt(la.part0 + (int64_t)row * nt + (c * NB + n0) / 16, rs);
  }
  if (j == 0 && threadIdx.x == 0) *la.done = 0;
}

}  // namespace

// (D - B2) from which the trailing update runs on the 128-tile GEMM: (D - B2)/128 >= 14
// gives >= 196 workgroups
static const int64_t TRAIL128_MIN = knob("MIDAGMA_EXP_TRAIL128", 1792);

// D from which the panels of B2 = 256 run on 64 x 64 tiles (binv_panel64_kernel; experiment knob
// MIDAGMA_EXP_PANEL64_MIN, e.g. 1000000 for the 32 x 32 panel everywhere)
static int64_t panel64_min() {
  static const int64_t m = knob("MIDAGMA_EXP_PANEL64_MIN", int64_t(1) << 40);  // off until measured
  return m;
}

// workgroups that run the next block's series inside a trailing update (launch_trail128_series):
// 64 where the update has >= 1024 tiles (D >= 4352: at least two rounds to hide the series
// behind; d = 5000 108.2 -> 110.7 steps/s, while at d = 2000 / 3000 the series outlasts the
// update's one round: 1100 -> 731, 393 -> 298; profiles/r04_probe_large3_ts*.log).  Experiment
// knob MIDAGMA_EXP_TRAIL_SERIES = workers (0: the series launches everywhere), read at each
// enqueue (graph capture).
static int trail_series_workers(int64_t D) {
  const int w = (int)knob("MIDAGMA_EXP_TRAIL_SERIES", -1);
  const int64_t tm = (D - 256) / 128;
  if (w < 0) return tm * tm >= 1024 ? 64 : 0;
  return w > 0 ? (w + 7) / 8 * 8 : 0;
}

// workgroups that claim the next block's panel jobs inside the trailing update
// (launch_trail128_panel; experiment knob MIDAGMA_EXP_TRAIL_PANEL, 0: the panel launches)
// (-1: the fused launch's tile order and band hand-offs without its panel workgroups; the
// panels stay launches: a diagnostic)
static int trail_panel_workers(int64_t) {
  const int w = (int)knob("MIDAGMA_EXP_TRAIL_PANEL", 0);
  return w > 0 || w == -1 ? w : 0;
}

int binv_block(int64_t D) {
  // D = 128 (64 < d <= 128): one outer block, so the fast slot's whole inverse is the warm-started
  // product form (3 launches instead of the Gauss-Jordan's prologue and 4 block steps)
  static const bool b128 = knob("MIDAGMA_EXP_BINV128", 1) != 0;
  if (D == 128) return b128 ? 128 : 0;
  // Experiment (MIDAGMA_EXP_BINV512=1): D = 512 as one 512-wide block, the fast slot's inverse
  // the product form alone (a residual and two pass launches instead of two outer steps of
  // five).  Correct (the GPU tier passes with it on) but slower: d=300/400/500 7.2k/6.9k/6.8k
  // vs 11.2k/10.7k/10.4k steps/s (the 512-wide pass kernel holds 256 VGPRs, one wave per SIMD,
  // and its 1024 workgroups run in four rounds).
  static const bool b512 = knob("MIDAGMA_EXP_BINV512", 0) == 1;
  if (D == 512 && b512) return 512;
  // Experiment (MIDAGMA_EXP_B2_512=1): 512-wide outer blocks where 512 divides D.  Correct (the
  // blocked parity tests at d = 1000, 2000 pass with it on) but slower: d=1000 4394 -> 3550,
  // d=2000 1089 -> 940 steps/s with the 32 x 32-tile series and panel, 4086 / 966 with the
  // 16 x 16 split-K series (4x the series flops of the 256 blocks at 20-30 TF)
  static const bool b2_512 = knob("MIDAGMA_EXP_B2_512", 0) == 1;
  if (b2_512 && D >= 1024 && D % 512 == 0) return 512;
  if (D < 256 || D % 128 != 0) return 0;  // fast path not available: plain GJ
  return D % 256 == 0 ? 256 : 128;
}

double* binv_build_target(double* Mt, int64_t D, const BInvWork& bw) {
  const int B2 = binv_block(D);
  if (B2 == 0) return Mt;
  return ((D / B2) & 1) ? bw.Aalt : Mt;  // K2 ping-pong flips land the inverse in Mt
}

#ifdef MIDAGMA_EXPERIMENTS
// the 512-block's series (nm5 kernels): residual and pass launches as launch_neumann
static void launch_neumann5(double* Ain, int64_t D, int64_t G0, const BInvWork& bw, int g, State* st, int passes,
                            hipStream_t stream) {
  const double* Pe = bw.Pst + (int64_t)g * N5 * N5;
  const double* Po = bw.Pst1 + (int64_t)g * N5 * N5;
  int* done = bw.done + g;
  double* part = bw.part + (int64_t)g * (NM_PASSES + 1) * PART_STRIDE;
  hipLaunchKernelGGL(nm5_resid_kernel, dim3(NT5 * NT5), dim3(NTHREADS), 0, stream, Ain + G0 * D + G0, D, Pe, Po,
                     bw.Y[0], bw.Q[0], part, done, st);
  for (int p = 1; p <= passes && p <= NM_PASSES; ++p)
    hipLaunchKernelGGL(nm5_pass_kernel, dim3(NT5 * NT5), dim3(NTHREADS), 0, stream, bw.Y[(p - 1) & 1],
                       bw.Q[(p - 1) & 1], bw.Y[p & 1], bw.Q[p & 1], bw.P, part + (p - 1) * PART_STRIDE,
                       part + p * PART_STRIDE, done, p, st);
}

#endif

// series tiles XCD-blocked (nm_tile; experiment knob MIDAGMA_EXP_NM_XCD=0: row-major)
static int nm_xmap() {
  static const int x = knob("MIDAGMA_EXP_NM_XCD", 1) != 0 ? 1 : 0;
  return x;
}

template <int L, int NW = 4>
static void launch_neumann(double* Ain, int64_t D, int64_t G0, const BInvWork& bw, int g, State* st, int passes,
                           bool resid, const NmLA* la, hipStream_t stream) {
  constexpr int B2 = 4 * NW * L;
  const int nwg = (B2 / 16) * (B2 / 16);
  const double* Pe = bw.Pst + (int64_t)g * B2 * B2;
  const double* Po = bw.Pst1 + (int64_t)g * B2 * B2;
  int* done = bw.done + g;
  double* part = bw.part + (int64_t)g * (NM_PASSES + 1) * PART_STRIDE;  // per block: kept for diagnostics
  if (resid)  // else the previous block's launches left X0, R and its row partials (look-ahead)
    hipLaunchKernelGGL((nm_resid_kernel<L, NW>), dim3(nwg), dim3(64 * NW), 0, stream, Ain + G0 * D + G0, D, Pe, Po,
                       bw.Y[0], bw.Q[0], part, done, st, nm_xmap());
  const NmLA none{};
  for (int p = 1; p <= passes && p <= NM_PASSES; ++p) {
    const double* Y = bw.Y[(p - 1) & 1];  // pass 1: X0 from nm_resid (or the look-ahead)
    // passes 1 and 2 carry the look-ahead products LW and LZ (one more tile grid each: the pass
    // kernel's registers admit two workgroups per CU, so both grids stay one round)
    const bool ext = la != nullptr && p <= 2;
    hipLaunchKernelGGL((nm_pass_kernel<L, NW>), dim3(ext ? 2 * nwg : nwg), dim3(64 * NW), 0, stream, Y,
                       bw.Q[(p - 1) & 1], bw.Y[p & 1], bw.Q[p & 1], bw.P, part + (p - 1) * PART_STRIDE,
                       part + p * PART_STRIDE, done, p, st, ext ? la[p - 1] : none, nm_xmap());
  }
}

// One B2 x B2 block's product-form series with explicit buffers (the DagmaMLP log-det's fast
// path, mlp.hip): the same kernels and arithmetic as an outer block of the fast blocked inverse.
template <class F>
static void with_series_l(int B2, F&& f) {
  if (B2 == 256)
    f(std::integral_constant<int, 16>{});
  else if (B2 == 128)
    f(std::integral_constant<int, 8>{});
  else
    throw std::invalid_argument("launch_series: B2 must be 128 or 256");
}

void launch_series_pass(int B2, const SeriesWork& w, State* st, int p, hipStream_t stream) {
  if (p < 1 || p > NM_PASSES) throw std::invalid_argument("launch_series_pass: pass out of range");
  const NmLA none{};
  with_series_l(B2, [&](auto Lc) {
    constexpr int L = decltype(Lc)::value;
    const int nwg = (B2 / 16) * (B2 / 16);
    hipLaunchKernelGGL(nm_pass_kernel<L>, dim3(nwg), dim3(NTHREADS), 0, stream, w.Y[(p - 1) & 1], w.Q[(p - 1) & 1],
                       w.Y[p & 1], w.Q[p & 1], w.P, w.part + (p - 1) * PART_STRIDE, w.part + p * PART_STRIDE, w.done,
                       p, st, none, nm_xmap());
  });
  HIP_TRY(hipGetLastError());
}

void launch_ldfast_resid(const double* A, int64_t lda, int64_t d, double s, int B2, const SeriesWork& w, State* st,
                         State* gjst, hipStream_t stream) {
  if (d > B2) throw std::invalid_argument("launch_ldfast_resid: d exceeds the series block");
  with_series_l(B2, [&](auto Lc) {
    constexpr int L = decltype(Lc)::value;
    const int nwg = (B2 / 16) * (B2 / 16);
    hipLaunchKernelGGL(ldfast_resid_kernel<L>, dim3(nwg), dim3(NTHREADS), 0, stream, A, lda, d, s, w.Pe, w.Po, w.Y[0],
                       w.Q[0], w.part, w.done, st, gjst, nm_xmap());
  });
  HIP_TRY(hipGetLastError());
}

void launch_series(const double* S, int64_t lds, int B2, const SeriesWork& w, State* st, int passes,
                   hipStream_t stream) {
  with_series_l(B2, [&](auto Lc) {
    constexpr int L = decltype(Lc)::value;
    const int nwg = (B2 / 16) * (B2 / 16);
    hipLaunchKernelGGL(nm_resid_kernel<L>, dim3(nwg), dim3(NTHREADS), 0, stream, S, lds, w.Pe, w.Po, w.Y[0], w.Q[0],
                       w.part, w.done, st, nm_xmap());
  });
  HIP_TRY(hipGetLastError());
  for (int p = 1; p <= passes; ++p) launch_series_pass(B2, w, st, p, stream);
}

// 512-wide blocks (experiments build): the 32 x 32-tile series and panel (nm5 / panel5 kernels;
// MIDAGMA_EXP_NM5=0: the 16 x 16 split-K series with 8 waves and the 32-tile panel)
#ifdef MIDAGMA_EXPERIMENTS
static bool nm5_on() {
  static const bool on = knob("MIDAGMA_EXP_NM5", 1) != 0;
  return on;
}
#endif

// Experiment knob MIDAGMA_EXP_RESID_LA=1: the look-ahead residual (read at each enqueue, i.e.
// when a slot graph is captured).  Correct (the blocked parity tests pass with it on) but not
// faster: the extra tiles lengthen the latency-bound pass, panel and trailing launches by more
// than the residual launch they remove (d=1000 4422 -> 4342, d=700 6709 -> 6414, d=1150 even,
// d=1400 1968 -> 2000 steps/s; with LW and LZ both in the first pass, whose grid then needs two
// rounds: d=1000 4285).
static bool resid_lookahead() {
  return knob("MIDAGMA_EXP_RESID_LA", 0) == 1;
}

// Fast slot at large D with the look-ahead: each outer step's trailing update in two launches,
// the tiles in block g + 1's row and column bands (its series and panel read only those) and the
// rest; the chain series(g+1) -> panel(g+1) -> band tiles(g+1) runs on the high-priority side
// stream while rest(g) runs on `stream`, so the serial series / panel phases hide behind the
// long trailing launches (classic LU look-ahead).  Dependencies: rest(g) after panel(g) and
// rest(g-1); band tiles(g) after panel(g) and rest(g-1) (which wrote its inputs, and whose
// inputs it overwrites); the last step's whole trailing update (with the fused score GEMM and the
// domain check) after rest(K2-2).  Every tile is computed by the same body as launch_trail128.
static bool blocked_inverse_lookahead(double* Mt, int64_t D, int B2, const BInvWork& bw, State* st,
                                      hipStream_t stream, int passes, const GemmSpec* fuse,
                                      const TrailLookAhead& la, double* ain0) {
  const int K2 = (int)(D / B2), gb = B2 / NB, mb = (int)(D / NB) - gb;
  double* bufs[2] = {binv_build_target(Mt, D, bw), nullptr};
  bufs[1] = bufs[0] == Mt ? bw.Aalt : Mt;
  hipEvent_t* ev = la.ev;  // [0] fork, [1 + 2g] panel(g), [2 + 2g] rest(g), [2 K2 + 1] join
  hipStream_t side = la.side;
  bool fused = false;
  HIP_TRY(hipEventRecord(ev[0], stream));
  HIP_TRY(hipStreamWaitEvent(side, ev[0], 0));
  for (int g = 0; g < K2; ++g) {
    double* Ain = g == 0 && ain0 ? ain0 : bufs[g & 1];
    double* Aout = bufs[(g + 1) & 1];
    const int64_t G0 = (int64_t)g * B2;
    double* Pe = bw.Pst + (int64_t)g * B2 * B2;
    double* Po = bw.Pst1 + (int64_t)g * B2 * B2;
    if (B2 == 256)
      launch_neumann<16>(Ain, D, G0, bw, g, st, passes, true, nullptr, side);
    else
      launch_neumann<8>(Ain, D, G0, bw, g, st, passes, true, nullptr, side);
    const int check = g == K2 - 1;
    hipLaunchKernelGGL(binv_panel_kernel<0>, dim3(2 * gb * mb + gb * gb), dim3(NTHREADS), 0, side, Ain, Aout, D, B2, g,
                       bw.P, (int64_t)B2, Pe, Po, bw.done + g, check, st, t32_pf(), nullptr, nullptr, nullptr);
    if (g < K2 - 1) {
      HIP_TRY(hipEventRecord(ev[1 + 2 * g], side));
      HIP_TRY(hipStreamWaitEvent(stream, ev[1 + 2 * g], 0));
      launch_trail128_split(Ain, Aout, D, B2, g, 1, st, stream);  // rest(g)
      HIP_TRY(hipEventRecord(ev[2 + 2 * g], stream));
      if (g >= 1) HIP_TRY(hipStreamWaitEvent(side, ev[2 * g], 0));  // rest(g - 1)
      launch_trail128_split(Ain, Aout, D, B2, g, 0, st, side);  // block g + 1's bands
    } else {
      if (g >= 1) HIP_TRY(hipStreamWaitEvent(side, ev[2 * g], 0));
      if (fuse && gemm_trail_supported(*fuse)) {
        launch_gemm_trail(*fuse, Ain, Aout, D, B2, g, true, st, t32_pf(), -1, side);
        fused = true;
      } else {
        launch_trail128(Ain, Aout, D, B2, g, true, st, side);
      }
    }
  }
  HIP_TRY(hipEventRecord(ev[2 * K2 + 1], side));
  HIP_TRY(hipStreamWaitEvent(stream, ev[2 * K2 + 1], 0));
  HIP_TRY(hipGetLastError());
  return fused;
}

#ifdef MIDAGMA_EXPERIMENTS
void launch_build_resid0(const double* W, int64_t ldw, double* At, int64_t D, int64_t d, const Params* pr,
                         const BInvWork& bw, State* st, hipStream_t stream) {
  if (binv_block(D) != 256 || D % 32) throw std::invalid_argument("launch_build_resid0: needs B2 = 256");
  const int kb = (int)(D / 32);
  hipLaunchKernelGGL(build_resid0_kernel, dim3((unsigned)(kb * kb + 256)), dim3(NTHREADS), 0, stream, W, ldw, At, D, d,
                     pr, bw.Pst, bw.Pst1, bw.Y[0], bw.Q[0], bw.part, bw.done, st, nm_xmap());
  HIP_TRY(hipGetLastError());
}
#endif

bool launch_blocked_inverse(double* Mt, int64_t D, const BInvWork& bw, bool fast, const GJWork& gw, State* st,
                            hipStream_t stream, int passes, const GemmSpec* fuse, const TrailLookAhead* tla,
                            bool resid0_done, double* ain0, int slow_from) {
  bool fused = false;
  const int B2 = binv_block(D);
  if (B2 == 0) throw std::invalid_argument("blocked inverse needs D >= 256, D % 128 == 0");
  const int K2 = (int)(D / B2), gb = B2 / NB, mb = (int)(D / NB) - gb;
  if (fast && tla && K2 >= 2 && D - B2 >= TRAIL128_MIN && (B2 == 256 || B2 == 128))
    return blocked_inverse_lookahead(Mt, D, B2, bw, st, stream, passes, fuse, *tla, ain0);
  double* bufs[2] = {binv_build_target(Mt, D, bw), nullptr};
  bufs[1] = bufs[0] == Mt ? bw.Aalt : Mt;
  // look-ahead residual (NmLA / TrailLA): fast path with 32 x 32 trailing updates
  const bool look = fast && bw.LW && K2 > 1 && D - B2 < TRAIL128_MIN && resid_lookahead();
  // blocks 1 .. K2 - 1's series inside the previous step's trailing update (128-tile updates)
  const bool tser = fast && bw.sync && B2 == 256 && K2 > 1 && D - B2 >= TRAIL128_MIN && trail_series_workers(D) > 0;
  // ... and their panels too (the default 32 x 32 panel only)
  const int tpan = tser && D < panel64_min() ? trail_panel_workers(D) : 0;  // (< 0: band order only)
  for (int g = 0; g < K2; ++g) {
    double* Ain = g == 0 && ain0 ? ain0 : bufs[g & 1];
    double* Aout = bufs[(g + 1) & 1];
    const int64_t G0 = (int64_t)g * B2;
    double* Pe = bw.Pst + (int64_t)g * B2 * B2;
    double* Po = bw.Pst1 + (int64_t)g * B2 * B2;
    const double* P;
    int64_t ldp;
    const int* done = nullptr;
    const bool ahead = look && g + 1 < K2;  // this block's launches prepare block g + 1's residual
    const int64_t GN0 = G0 + B2;
    NmLA la[2] = {};
    TrailLA tla{};
    if (ahead) {
      la[0] = NmLA{Ain + GN0 * D + GN0, D, bw.Pst + GN0 * B2, bw.Pst1 + GN0 * B2, bw.LW};
      la[1] = NmLA{Ain + G0 * D + GN0, D, bw.Pst + GN0 * B2, bw.Pst1 + GN0 * B2, bw.LZ};
      tla = TrailLA{bw.LW, bw.LPZ, bw.Pst + GN0 * B2, bw.Pst1 + GN0 * B2, bw.Y[0], bw.Q[0],
                    bw.part + (int64_t)(g + 1) * (NM_PASSES + 1) * PART_STRIDE, bw.done + g + 1, g + 1};
    }
    // (slow_from >= 0: the fast path's blocks from slow_from on take the pivoted Gauss-Jordan)
    const bool fast_g = fast && (slow_from < 0 || g < slow_from);
    if (fast_g) {
      const bool resid = (!look || g == 0) && !(g == 0 && resid0_done);  // (block 0: launch_build_resid0)
      const bool own = !(tser && g > 0);  // else the series ran in trailing update g - 1
#ifdef MIDAGMA_EXPERIMENTS
      if (B2 == 512 && !ahead && resid && nm5_on())
        launch_neumann5(Ain, D, G0, bw, g, st, passes, stream);
      else
#endif
      if (B2 == 512)
        launch_neumann<16, 8>(Ain, D, G0, bw, g, st, passes, resid, ahead ? la : nullptr, stream);
      else if (B2 == 256 && own)
        launch_neumann<16>(Ain, D, G0, bw, g, st, passes, resid, ahead ? la : nullptr, stream);
      else if (B2 == 256) {
      }
      else
        launch_neumann<8>(Ain, D, G0, bw, g, st, passes, resid, ahead ? la : nullptr, stream);
      P = bw.P;
      ldp = B2;
      done = bw.done + g;
    } else {
      GJWork w = gw;
      w.pivlog = gw.pivlog ? gw.pivlog + G0 : nullptr;
      w.Pstore = gw.Pstore ? gw.Pstore + G0 * NB : nullptr;
      launch_gj_inverse(Ain + G0 * D + G0, D, B2, w, st, stream);
      P = Ain + G0 * D + G0;
      ldp = D;
    }
    // the fast slot takes the domain flags from the last outer step's outputs (no reduce_check)
    const int check = fast_g && g == K2 - 1;
    const bool ser_next = tser && g + 1 < K2;  // trailing update g runs block g + 1's series
    int* zsync = ser_next ? bw.sync + (int64_t)(g + 1) * 256 : nullptr;
#ifdef MIDAGMA_EXPERIMENTS
    if (B2 == 512 && fast && !ahead && nm5_on()) {
      const int jobs = 2 * NT5 * (int)(D / 32 - NT5);
      hipLaunchKernelGGL(panel5_kernel, dim3((unsigned)std::max(NT5, jobs)), dim3(NTHREADS), 0, stream,
                         Ain, Aout, D, g, P, Pe, Po, done, check, st);
    } else
#endif
    if (tpan > 0 && g > 0) {
      // block g's panel ran inside trailing update g - 1
    } else if (B2 == 256 && !ahead && D >= panel64_min()) {
      const int m64 = (int)(D / 64) - 4;
      static const bool chains = knob("MIDAGMA_EXP_P64_CHAINS", 0) != 0;
      hipLaunchKernelGGL(chains ? binv_panel64_kernel<true> : binv_panel64_kernel<false>, dim3(2 * 4 * m64 + 16),
                         dim3(NTHREADS), 0, stream, Ain, Aout, D, g, P, ldp, Pe, Po, done, check, st, zsync);
    } else
    hipLaunchKernelGGL(B2 != 256 ? binv_panel_kernel<0> : panel_kernel_sb(D),
                       dim3(2 * gb * mb + gb * gb * (ahead ? 2 : 1)), dim3(NTHREADS), 0, stream,
                       Ain, Aout, D, B2, g, P, ldp, Pe, Po, done, check, st, t32_pf(), ahead ? bw.LZ : nullptr,
                       ahead ? bw.LPZ : nullptr, zsync);
    if (mb > 0) {
      // large D: 128 x 128 tiles (operand reuse; enough tiles to fill the chip), else 32 x 32
      if (D - B2 >= TRAIL128_MIN) {
        if (fuse && fast && g == K2 - 1 && gemm_trail_supported(*fuse)) {
          launch_gemm_trail(*fuse, Ain, Aout, D, B2, g, check, st, t32_pf(), -1, stream);
          fused = true;
        } else if (ser_next) {
          const int64_t gn = g + 1;
          TrailSeries ts{bw.Pst + gn * B2 * B2, bw.Pst1 + gn * B2 * B2, {bw.Y[0], bw.Y[1]}, {bw.Q[0], bw.Q[1]}, bw.P,
                         bw.part + gn * (NM_PASSES + 1) * PART_STRIDE, bw.done + gn, zsync,
                         std::min(passes, NM_PASSES), nm_xmap(), trail_series_workers(D)};
          if (tpan != 0) {
            TrailPanel tp{bw.Pst + gn * B2 * B2, bw.Pst1 + gn * B2 * B2,
                          tpan > 0 && gn + 1 < K2 ? bw.sync + (gn + 1) * 256 : nullptr, gn == K2 - 1 ? 1 : 0,
                          t32_pf(), tpan > 0 ? tpan : 0};
            launch_trail128_panel(Ain, Aout, D, g, check != 0, st, ts, tp, stream);
          } else {
            launch_trail128_series(Ain, Aout, D, g, check != 0, st, ts, stream);
          }
        } else {
          launch_trail128(Ain, Aout, D, B2, g, check, st, stream);
        }
      } else if (fuse && fast && g == K2 - 1 && gemm_trail_supported(*fuse)) {
        launch_gemm_trail(*fuse, Ain, Aout, D, B2, g, check, st, t32_pf(), mb * mb, stream);
        fused = true;
      } else {
        hipLaunchKernelGGL(binv_trail_kernel, dim3(mb * mb + (ahead ? gb * gb : 0)), dim3(NTHREADS), 0, stream, Ain,
                           Aout, D, B2, g, check, st, t32_pf(), tla);
      }
    }
  }
  HIP_TRY(hipGetLastError());
  return fused;
}

}  // namespace midagma

#ifdef MIDAGMA_KSTAMPS
// Diagnostics (kstamps build): the phase sums (KS_KINDS x (KS_POINTS + 2) u64), then zeroed.
extern "C" int midagma_debug_kstamps(unsigned long long* out) {
  using namespace midagma;
  const size_t bytes = sizeof(unsigned long long) * KS_KINDS * (KS_POINTS + 2);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_kstamps), bytes) != hipSuccess) return -1;
  static unsigned long long zero[KS_KINDS * (KS_POINTS + 2)] = {};
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_kstamps), zero, bytes) != hipSuccess) return -1;
  return 0;
}
#endif
