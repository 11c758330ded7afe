// TCC trek regularizer (notreks.py trek_cycle_coupling_value_gradW) for
// 2d <= 128 in ONE workgroup of 4 x 4 register blocks: the device body shared by tcc.hip's
// one-workgroup launch and the small-d persistent inner loop (small.hip), which runs it inside
// its slots.
#pragma once

#include <cmath>
#include <type_traits>

#include "launch.h"

namespace midagma {
namespace tccb {

struct Add {
  __device__ double operator()(double a, double b) const { return a + b; }
};
struct Min {
  __device__ double operator()(double a, double b) const { return fmin(a, b); }
};
struct Max {
  __device__ double operator()(double a, double b) const { return fmax(a, b); }
};

// ---- 2d <= 128: the whole TCC sequence in ONE workgroup of 4 x 4 register blocks --------------
// The launch-per-kernel sequence above is ~170 dependent launches per slot (24 gated Noda steps of
// shift, Gauss-Jordan prologue and steps, GEMV and update), almost all no-ops once Noda converged:
// at d = 20 that was 0.40 ms per Adam step.  Here every step of the same algorithm (the same
// Collatz-Wielandt start, Noda updates, stopping rules, breakdown handling, final sweeps, value and
// gradient, and the same scal / warm-start words) runs in one workgroup of NB x NB threads: thread
// (a, b) keeps rows 4a..4a+3 x columns 4b..4b+3 of A and of the shifted matrix / its inverse in
// registers.  The inverses are unpivoted Gauss-Jordan (sigma I - A is a nonsingular M-matrix on
// every Noda step) with ONE barrier per pivot: the owners of row and column p + 1 publish them to a
// double-buffered LDS pair as soon as pivot p's update is done.  GEMVs reduce a row block's 4 x 4
// partials over the NB lanes of the same a by butterfly (fixed order); the vector steps (Noda
// update, normalisation, value) run in wave 0 with wave reductions.  scal[6] counts the inverses of
// the call (diagnostic).
// BS: the register block edge (4; 5 for 2d <= 40 on one wave, NB = 8).  With BS = 5 a workgroup
// may have more threads than NB x NB (the small loop's): the others take block (0, 0)'s
// addresses, compute along, and write nothing (`act`); BS = 4 callers run exactly NB x NB.
template <int NB, int BS = 4>
struct TccBlk {
  static constexpr int NT = NB * NB;  // active threads
  static constexpr int NM = BS * NB;  // largest 2d
  static constexpr int VT = NM > 64 ? NM / 64 : 1;  // vector entries per wave-0 lane
};

// the body's LDS: pivot row / column pairs, transposed-GEMV partials, the vectors, scalars, A
template <int NB, int BS = 4>
struct TccLds {
  static constexpr int NM = BS * NB, LA = NM + 2;
  double rowb[2][NM], colb[2][NM], part[NB * NB / 64][NM];
  double xs[NM], ys[NM], us[NM], zs[NM], scs[16], pivb[2];
  double al[NM * LA];
};

// fixed-order butterfly over the 64 lanes of a wave (every lane ends with the result)
template <class Op>
__device__ __forceinline__ double wave_reduce(double v, Op op) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) v = op(v, __shfl_xor(v, off));
  return v;
}

// M (holding A's block) <- sig I - A on the logical block, identity padding
template <int BS>
__device__ __forceinline__ void blk_shift(double (&M)[BS][BS], int n, int a, int b, double sig) {
#pragma unroll
  for (int r = 0; r < BS; ++r)
#pragma unroll
    for (int c = 0; c < BS; ++c) {
      const int i = BS * a + r, j = BS * b + c;
      M[r][c] = (i < n && j < n) ? ((i == j ? sig : 0.0) - M[r][c]) : (i == j ? 1.0 : 0.0);
    }
}

// in-place unpivoted Gauss-Jordan inverse of the block-distributed matrix.  Pivot p's update is
// one rank-1 form for every entry, M'[i][j] = M~[i][j] - c[i] r[j], where the publishers of pivot p
// hand over r = row p with r[p] = 1, c = column p with c[p] = piv - 1, and replace column p of their
// blocks by e_p; with r scaled by 1 / piv this gives row p / piv, column p times -1 / piv and
// 1 / piv at the pivot (gj.hip's result, in a different rounding).  The pivot loop runs over 4-row
// blocks with the row inside the block unrolled, so every register index is static; the identity
// padding up to a multiple of 4 pivots on 1 and changes nothing.
template <int NB, int BS = 4>
__device__ __forceinline__ void blk_gj_inverse(double (&M)[BS][BS], int n, int a, int b, bool act,
                                               double (*rowb)[BS * NB], double (*colb)[BS * NB], double* pivb) {
  auto publish = [&](int q, auto Rc, int buf) {
    constexpr int R = decltype(Rc)::value;
    if (act && a == q) {
#pragma unroll
      for (int c = 0; c < BS; ++c) rowb[buf][BS * b + c] = (b == q && c == R) ? 1.0 : M[R][c];
    }
    if (b == q) {
#pragma unroll
      for (int r = 0; r < BS; ++r) {
        const bool piv = a == q && r == R;
        if (act) {
          colb[buf][BS * a + r] = piv ? M[r][R] - 1.0 : M[r][R];
          if (piv) pivb[buf] = M[r][R];
        }
        M[r][R] = piv ? 1.0 : 0.0;
      }
    }
  };
  // (the buffer parity is that of p = BS q + R: static for even BS)
  auto step = [&](int q, auto Rc, int nq) {
    constexpr int R = decltype(Rc)::value;
    const int buf = (BS & 1) ? ((BS * q + R) & 1) : (R & 1);
    __syncthreads();
    const double inv = 1.0 / pivb[buf];
    double rp[BS], cp[BS];
#pragma unroll
    for (int c = 0; c < BS; ++c) rp[c] = rowb[buf][BS * b + c] * inv;
#pragma unroll
    for (int r = 0; r < BS; ++r) cp[r] = colb[buf][BS * a + r];
#pragma unroll
    for (int r = 0; r < BS; ++r)
#pragma unroll
      for (int c = 0; c < BS; ++c) M[r][c] = M[r][c] - cp[r] * rp[c];
    if constexpr (R < BS - 1)
      publish(q, std::integral_constant<int, R + 1>(), buf ^ 1);
    else if (q + 1 < nq)
      publish(q + 1, std::integral_constant<int, 0>(), buf ^ 1);
  };
  const int nq = (n + BS - 1) / BS;
  publish(0, std::integral_constant<int, 0>(), 0);
  for (int q = 0; q < nq; ++q) {
    step(q, std::integral_constant<int, 0>(), nq);
    step(q, std::integral_constant<int, 1>(), nq);
    step(q, std::integral_constant<int, 2>(), nq);
    step(q, std::integral_constant<int, 3>(), nq);
    if constexpr (BS > 4) step(q, std::integral_constant<int, 4>(), nq);
  }
}

// y = M x (x, y in LDS, NM entries): each thread's 4 row partials over its 4 columns, summed over
// the NB threads of its row block (consecutive lanes) by butterfly
template <int NB, int BS = 4>
__device__ __forceinline__ void blk_gemv(const double (&M)[BS][BS], int a, int b, bool act, bool skip_tr, int d,
                                         const double* x, double* y) {
  double xv[BS], s[BS];
#pragma unroll
  for (int c = 0; c < BS; ++c) xv[c] = x[BS * b + c];
#pragma unroll
  for (int r = 0; r < BS; ++r) {
    double acc = 0.0;
#pragma unroll
    for (int c = 0; c < BS; ++c) {
      const bool zero = skip_tr && BS * a + r < d && BS * b + c >= d;  // B: top-right block 0
      acc += zero ? 0.0 : M[r][c] * xv[c];
    }
    s[r] = acc;
  }
#pragma unroll
  for (int off = 1; off < NB; off <<= 1)
#pragma unroll
    for (int r = 0; r < BS; ++r) s[r] += __shfl_xor(s[r], off);
  if (act && b == 0) {
#pragma unroll
    for (int r = 0; r < BS; ++r) y[BS * a + r] = s[r];
  }
  __syncthreads();
}

// y = M^T u: column partials per thread, summed over the row blocks of a wave by butterfly, then
// over the waves through LDS (fixed order)
template <int NB, int BS = 4>
__device__ __forceinline__ void blk_gemv_t(const double (&M)[BS][BS], int a, int b, bool act, const double* u,
                                           double (*part)[BS * NB], double* y) {
  constexpr int NW = NB * NB / 64;  // waves
  double uv[BS], t[BS];
#pragma unroll
  for (int r = 0; r < BS; ++r) uv[r] = u[BS * a + r];
#pragma unroll
  for (int c = 0; c < BS; ++c) {
    double acc = 0.0;
#pragma unroll
    for (int r = 0; r < BS; ++r) acc += M[r][c] * uv[r];
    t[c] = acc;
  }
#pragma unroll
  for (int off = NB; off < 64; off <<= 1)
#pragma unroll
    for (int c = 0; c < BS; ++c) t[c] += __shfl_xor(t[c], off);
  if (act && (threadIdx.x & 63) < NB) {
#pragma unroll
    for (int c = 0; c < BS; ++c) part[threadIdx.x >> 6][BS * b + c] = t[c];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < BS * NB; j += NB * NB) {
    double acc = 0.0;
    for (int w = 0; w < NW; ++w) acc += part[w][j];
    y[j] = acc;
  }
  __syncthreads();
}

// wave 0: warm start (tcc_init_kernel) into out: prev when the last solve converged and is inside
// the cone, else ones (0 on the padding)
template <int NB, int BS = 4>
__device__ __forceinline__ void w0_init(const double* __restrict__ prev, int n, bool conv, bool warm_ok,
                                        double* out) {
  const int lane = threadIdx.x;
  double pv[TccBlk<NB, BS>::VT], mn = INFINITY, mx = 0.0;
#pragma unroll
  for (int t = 0; t < TccBlk<NB, BS>::VT; ++t) {
    const int e = lane + 64 * t;
    pv[t] = e < n ? prev[e] : 0.0;
    if (e < n) {
      mn = fmin(mn, pv[t]);
      mx = fmax(mx, pv[t]);
    }
  }
  mn = wave_reduce(mn, Min());
  mx = wave_reduce(mx, Max());
  const bool warm = warm_ok && conv && mn > 1e-8 * mx && isfinite(mx);
#pragma unroll
  for (int t = 0; t < TccBlk<NB, BS>::VT; ++t) {
    const int e = lane + 64 * t;
    if (e < TccBlk<NB, BS>::NM) out[e] = e < n ? (warm ? pv[t] : 1.0) : 0.0;
  }
}

// wave 0: out = y / |y| with sum(out) > 0 (tcc_normalize_kernel), 0 on the padding
template <int NB, int BS = 4>
__device__ __forceinline__ void w0_normalize(const double* y, int n, double* out) {
  const int lane = threadIdx.x;
  double ss = 0.0, sm = 0.0;
#pragma unroll
  for (int t = 0; t < TccBlk<NB, BS>::VT; ++t) {
    const int e = lane + 64 * t;
    if (e < n) {
      ss += y[e] * y[e];
      sm += y[e];
    }
  }
  ss = wave_reduce(ss, Add());
  sm = wave_reduce(sm, Add());
  const double inv = (sm < 0.0 ? -1.0 : 1.0) / sqrt(ss);
#pragma unroll
  for (int t = 0; t < TccBlk<NB, BS>::VT; ++t) {
    const int e = lane + 64 * t;
    if (e < n) out[e] = y[e] * inv;
  }
}

// The whole TCC value (and, G non-null, gradient) of the current W by one workgroup of NB x NB
// threads; wget(i, j) / sget(i, j): W and the pair indicator S on the logical d x d block; scal,
// vprev, uprev: the regularizer's state words (global or LDS).  On return (all threads past a
// barrier) L.xs = v, L.us = u, L.scs[4] = u.v + eps, L.scs[5] = u.u + eps, from which a caller
// that passes G = nullptr forms the gradient itself (tcc_grad_elem).
template <int NB, int BS, class WGet, class SGet>
__device__ __forceinline__ void tcc_blk_body(WGet wget, SGet sget, double ws, int d, int mode, double eps, double m,
                                             double weight, double* __restrict__ scal, double* __restrict__ vprev,
                                             double* __restrict__ uprev, double* __restrict__ G, int64_t D,
                                             TccLds<NB, BS>& L, bool fix = true) {
  constexpr int NM = TccBlk<NB, BS>::NM, VT = TccBlk<NB, BS>::VT, LA = TccLds<NB, BS>::LA;
  auto& rowb = L.rowb;
  auto& colb = L.colb;
  auto& part = L.part;
  double* xs = L.xs;
  double* ys = L.ys;
  double* us = L.us;
  double* zs = L.zs;
  double* scs = L.scs;
  double* pivb = L.pivb;
  double* al = L.al;
  const int tid = threadIdx.x, lane = tid & 63;
  // (BS = 4: every caller runs NB x NB threads, and a run-time `act` there put M in scratch)
  const bool act = BS == 4 || tid < TccBlk<NB, BS>::NT;
  const int a = act ? tid / NB : 0, b = act ? tid % NB : 0;
  const bool w0 = tid < 64;
  const int n = 2 * d;
  // A (the logical 2d x 2d block, zero padding) in LDS; registers hold the working matrix only
  for (int e = tid; e < NM * NM; e += (int)blockDim.x) {  // tcc_build_kernel
    const int i = e / NM, j = e - i * NM;
    double v = 0.0;
    if (i < d) {
      if (j < d) {
        const double w = wget(i, j);
        v = w * w;
      } else if (j < n) {
        v = ws * sget(i, j - d);
      }
    } else if (i < n) {
      if (j < d) {
        v = (i - d == j) ? 1.0 : 0.0;
      } else if (j < n) {
        const double w = wget(j - d, i - d);
        v = w * w;
      }
    }
    al[i * LA + j] = v;
  }
  __syncthreads();
  double M[BS][BS];
  auto load_a = [&](double (&T)[BS][BS]) {
#pragma unroll
    for (int r = 0; r < BS; ++r)
#pragma unroll
      for (int c = 0; c < BS; ++c) T[r][c] = al[(BS * a + r) * LA + BS * b + c];
  };
  load_a(M);
  double sc[10];
#pragma unroll
  for (int t = 0; t < 10; ++t) sc[t] = scal[t];
  const bool conv_prev = sc[9] != 0.0;  // the last completed slot's solve converged
  if (w0) w0_init<NB, BS>(vprev, n, conv_prev, sc[8] != 0.0, xs);
  __syncthreads();
  blk_gemv<NB, BS>(M, a, b, act, false, d, xs, ys);
  if (w0) {  // tcc_sigma0_kernel
    double mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < VT; ++t) {
      const int e = lane + 64 * t;
      if (e < n) mx = fmax(mx, ys[e] / xs[e]);
    }
    mx = wave_reduce(mx, Max());
    if (lane == 0) scs[1] = mx;
  }
  __syncthreads();
  sc[1] = scs[1];
  sc[2] = 0.0;
  sc[7] = 0.0;
  sc[9] = 0.0;
  int ninv = 0;
  // the fixed-shift stage (tcc.hip tcc_fix_small_kernel: one inverse at sigma_0 (1 + 1e-14), then
  // inverse iteration for v and u with the same convergence rule); Noda and the final inverse only
  // when it does not converge in TCC_FIX_SWEEPS_SMALL sweeps or breaks down
  bool fixed = false;
  if (fix) {
    load_a(M);
    blk_shift<BS>(M, n, a, b, sc[1] * (1.0 + 1e-14));
    blk_gj_inverse<NB, BS>(M, n, a, b, act, rowb, colb, pivb);
    ++ninv;
    if (w0) w0_init<NB, BS>(uprev, n, conv_prev, sc[8] != 0.0, us);
    __syncthreads();
    const double sigs = sc[1] * (1.0 + 1e-14);
    double ub = sc[1];
    for (int k = 0; k < TCC_FIX_SWEEPS_SMALL; ++k) {
      blk_gemv<NB, BS>(M, a, b, act, false, d, xs, ys);
      blk_gemv_t<NB, BS>(M, a, b, act, us, part, zs);
      if (w0) {
        double vmin = INFINITY, vmax = -INFINITY, vss = 0.0, vs = 0.0;
        double umin = INFINITY, umax = -INFINITY, uss = 0.0, usm = 0.0, bad = 0.0;
#pragma unroll
        for (int t = 0; t < VT; ++t) {
          const int e = lane + 64 * t;
          if (e < n) {
            const double yi = ys[e], zi = zs[e];
            if (!(yi > 0.0) || !isfinite(yi) || !(zi > 0.0) || !isfinite(zi)) bad = 1.0;
            const double rv = xs[e] / yi, ru = us[e] / zi;
            vmin = fmin(vmin, rv);
            vmax = fmax(vmax, rv);
            vss += yi * yi;
            vs += yi;
            umin = fmin(umin, ru);
            umax = fmax(umax, ru);
            uss += zi * zi;
            usm += zi;
          }
        }
        vmin = wave_reduce(vmin, Min());
        vmax = wave_reduce(vmax, Max());
        vss = wave_reduce(vss, Add());
        vs = wave_reduce(vs, Add());
        umin = wave_reduce(umin, Min());
        umax = wave_reduce(umax, Max());
        uss = wave_reduce(uss, Add());
        usm = wave_reduce(usm, Add());
        bad = wave_reduce(bad, Max());
        double state = 2.0;  // 0 going on, 1 converged, 2 breakdown
        if (!(bad != 0.0 || !(vss > 0.0) || !(uss > 0.0) || !isfinite(vss) || !isfinite(uss))) {
          const double iv = (vs < 0.0 ? -1.0 : 1.0) / sqrt(vss), iu = (usm < 0.0 ? -1.0 : 1.0) / sqrt(uss);
#pragma unroll
          for (int t = 0; t < VT; ++t) {
            const int e = lane + 64 * t;
            if (e < n) {
              xs[e] = ys[e] * iv;
              us[e] = zs[e] * iu;
            }
          }
          ub = fmin(ub, sigs - vmin);
          state = (!(vmax - vmin > 1e-13 * vmin) && !(umax - umin > 1e-13 * umin)) ? 1.0 : 0.0;
        }
        if (lane == 0) {
          scs[11] = state;
          scs[12] = ub;
        }
      }
      __syncthreads();
      if (scs[11] != 0.0) break;
    }
    fixed = scs[11] == 1.0;
    if (fixed)
      sc[9] = 1.0;
    else if (scs[11] == 0.0)
      sc[1] = fmin(sc[1], scs[12]);  // Noda goes on from the stage's vector and bound
  }
  for (int k = 0; k < TCC_NODA_MAX && !fixed; ++k) {  // tcc_noda_kernel, until the stop rule
    ++ninv;
    load_a(M);
    blk_shift<BS>(M, n, a, b, sc[1]);
    blk_gj_inverse<NB, BS>(M, n, a, b, act, rowb, colb, pivb);
    blk_gemv<NB, BS>(M, a, b, act, false, d, xs, ys);
    if (w0) {
      double rmin = INFINITY, rmax = -INFINITY, ss = 0.0, bad = 0.0;
#pragma unroll
      for (int t = 0; t < VT; ++t) {
        const int e = lane + 64 * t;
        if (e < n) {
          const double yi = ys[e];
          if (!(yi > 0.0) || !isfinite(yi)) bad = 1.0;
          const double r = xs[e] / yi;
          rmin = fmin(rmin, r);
          rmax = fmax(rmax, r);
          ss += yi * yi;
        }
      }
      rmin = wave_reduce(rmin, Min());
      rmax = wave_reduce(rmax, Max());
      ss = wave_reduce(ss, Add());
      bad = wave_reduce(bad, Max());
      const double sig = sc[1];
      double up = sig, lo = sc[2], brk = 0.0, stop = 1.0;
      if (bad != 0.0 || !(ss > 0.0) || !isfinite(ss)) {  // keep x_k, sigma_k: the final inverse uses them
        brk = 1.0;
      } else {
        const double inv = 1.0 / sqrt(ss);
#pragma unroll
        for (int t = 0; t < VT; ++t) {
          const int e = lane + 64 * t;
          if (e < n) xs[e] = ys[e] * inv;
        }
        up = sig - rmin;
        lo = sig - rmax;
        // bounds met, or (reducible A: the lower bound need not tighten) the upper bound stalled
        stop = (!(up - lo > 1e-13 * fabs(up)) || !(sig - up > 1e-14 * fabs(up))) ? 1.0 : 0.0;
      }
      if (lane == 0) {
        scs[1] = up;
        scs[2] = lo;
        scs[7] = brk;
        scs[9] = (brk == 0.0 && stop != 0.0) ? 1.0 : 0.0;
        scs[10] = stop;
      }
    }
    __syncthreads();
    sc[1] = scs[1];
    sc[2] = scs[2];
    sc[7] = scs[7];
    sc[9] = scs[9];
    if (scs[10] != 0.0) break;
  }
  // the final inverse just above the root: two sweeps for v (x), two transposed for u
  if (!fixed) {
    load_a(M);
    blk_shift<BS>(M, n, a, b, sc[1] * (1.0 + 1e-14));
    blk_gj_inverse<NB, BS>(M, n, a, b, act, rowb, colb, pivb);
    ++ninv;
    for (int t = 0; t < 2; ++t) {
      blk_gemv<NB, BS>(M, a, b, act, false, d, xs, ys);
      if (w0) w0_normalize<NB, BS>(ys, n, xs);
      __syncthreads();
    }
    if (w0) w0_init<NB, BS>(uprev, n, sc[9] != 0.0, sc[8] != 0.0, us);
    __syncthreads();
    for (int t = 0; t < 2; ++t) {
      blk_gemv_t<NB, BS>(M, a, b, act, us, part, ys);
      if (w0) w0_normalize<NB, BS>(ys, n, us);
      __syncthreads();
    }
  }
  load_a(M);  // the inverse is no longer needed
  blk_gemv<NB, BS>(M, a, b, act, false, d, xs, ys);  // A v
  blk_gemv<NB, BS>(M, a, b, act, true, d, us, zs);   // B u
  if (w0) {  // tcc_value_kernel
    double uav = 0.0, uv = 0.0, uu = 0.0, ubu = 0.0;
#pragma unroll
    for (int t = 0; t < VT; ++t) {
      const int e = lane + 64 * t;
      if (e < n) {
        const double u = us[e], v = xs[e];
        uav += u * ys[e];
        uv += u * v;
        uu += u * u;
        ubu += u * zs[e];
        vprev[e] = v;
        uprev[e] = u;
      }
    }
    uav = wave_reduce(uav, Add());
    uv = wave_reduce(uv, Add());
    uu = wave_reduce(uu, Add());
    ubu = wave_reduce(ubu, Add());
    const double rho = uav / uv;
    const double val = (rho - ubu / (uu + eps)) / m;
    if (isfinite(val)) {
      sc[0] = val;
      sc[3] = rho;
      sc[4] = uv + eps;
      sc[5] = uu + eps;
      sc[8] = 1.0;
    } else {
      // no Perron gap (W o W and S nilpotent, e.g. W = 0): value 0, gradient 0 through the
      // infinite denominators, no warm start kept (tcc_value_kernel)
      sc[0] = 0.0;
      sc[3] = 0.0;
      sc[4] = INFINITY;
      sc[5] = INFINITY;
      sc[8] = 0.0;
    }
    sc[6] = (double)ninv;
    if (lane == 0) {
#pragma unroll
      for (int t = 0; t < 10; ++t) scal[t] = sc[t];
      scs[4] = sc[4];
      scs[5] = sc[5];
    }
  }
  __syncthreads();  // L.xs, L.us, L.scs[4..5] for every thread
  if (mode == 2 && G) {  // tcc_grad_kernel on the logical d x d block (the padding stays 0)
    const double denA = scs[4], denB = scs[5];
    for (int e = tid; e < d * d; e += (int)blockDim.x) {
      const int i = e / d, j = e - i * d;
      const double w = wget(i, j);
      double g = 0.0;
      if (w != 0.0) {
        const double gA = us[i] * xs[j] / denA + us[d + j] * xs[d + i] / denA;
        const double gB = (us[i] * us[j] + us[d + i] * us[d + j]) / denB;
        g = weight * (((2.0 * w) * gA - (2.0 * w) * gB) / m);
      }
      G[(int64_t)i * D + j] = g;
    }
  }
}


// weight * d value / d W[i][j] from the body's results (tcc_grad_kernel's arithmetic), for a
// caller that forms the gradient per element (w = W[i][j], zero gives zero)
template <int NB, int BS = 4>
__device__ __forceinline__ double tcc_grad_elem(const TccLds<NB, BS>& L, int d, int i, int j, double w, double m,
                                                double weight) {
  if (w == 0.0) return 0.0;
  const double denA = L.scs[4], denB = L.scs[5];
  const double gA = L.us[i] * L.xs[j] / denA + L.us[d + j] * L.xs[d + i] / denA;
  const double gB = (L.us[i] * L.us[j] + L.us[d + i] * L.us[d + j]) / denB;
  return weight * (((2.0 * w) * gA - (2.0 * w) * gB) / m);
}

}  // namespace tccb
}  // namespace midagma
