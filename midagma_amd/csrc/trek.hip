// PST trek regularizer on the GPU (fbleile/midagma src/notreks/notreks.py: pst / pst_mat /
// trek_value_grad, the "pst" branch), inside the slot like the reference's linear.py:251-258:
//
//     W2 = W o W,  F = f(W2),  H = F^T F,  value = agg(H[i_p, j_p]),  grad = d value / d W
//     f = expm (Taylor + scaling/squaring) | (I - W2 + eps I)^-1 | I + sum_{k<=K} W2^k / k |
//         (I + W2)^d (binary powering)
//
// The gradient is taken analytically, in the order autograd takes it:
//     C = d value / d H (c_p at (i_p, j_p)),  G_F = F (C + C^T),
//     G_W2 = L_f(W2^T, G_F)   (adjoint of the Frechet derivative of f),
//     grad = 2 W o G_W2
// using L_f(W2^T, G)^T = L_f(W2, G^T): one forward pass of f on W2 whose iterates are kept,
// then one directional pass (product rule through the same recurrence) in direction G_F^T.
// Every product is an FP64 MFMA GEMM (gemm.hip); every kernel obeys a gate word, so one
// captured sequence serves 'opt' (every slot) and 'log' (checkpoint slots only), and the
// exp path's data-dependent squaring count runs from a fixed number of launch slots.
#include <cmath>

#include "launch.h"

namespace midagma {

namespace {

constexpr int EB = NTHREADS;

__device__ __forceinline__ bool gate_on(const State* g) { return g->status == ST_RUNNING; }

__device__ __forceinline__ int64_t gstride() { return (int64_t)gridDim.x * EB; }
__device__ __forceinline__ int64_t gid() { return (int64_t)blockIdx.x * EB + threadIdx.x; }

// gates: [0] this slot runs the regularizer; [1 + t] squaring t runs; [1 + smax + t] it is skipped
__global__ void trek_gate_kernel(const State* __restrict__ st, int mode, State* __restrict__ gates, int smax) {
  if (threadIdx.x != 0) return;
  const bool on = st->status == ST_RUNNING && (mode == 2 || st->ckpt_pending);
  gates[0].status = on ? ST_RUNNING : ST_DONE;
  // squaring gates are set by trek_scale_kernel once the norm is known; default: all off
  for (int t = 0; t < 2 * smax; ++t) gates[1 + t].status = ST_DONE;
}

// X = W o W on the logical d x d block (0 padding); column partial sums of X per 64-row band
__global__ void trek_w2_kernel(const double* __restrict__ W, double* __restrict__ X, double* __restrict__ colpart,
                               int64_t d, int64_t D, const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  const int64_t j = (int64_t)blockIdx.x * EB + threadIdx.x;
  const int64_t band = blockIdx.y;
  if (j >= D) return;
  double cs = 0.0;
  for (int64_t i = band * 64; i < band * 64 + 64; ++i) {
    const double w = (i < d && j < d) ? W[i * D + j] : 0.0;
    const double x = w * w;
    X[i * D + j] = x;
    cs += x;
  }
  if (colpart) colpart[band * D + j] = cs;
}

// exp: s = max(0, ceil(log2(||W2||_1 / theta))) squarings, X *= 2^-s, gates for the slots
__global__ void trek_scale_kernel(const double* __restrict__ colpart, int64_t nbands, int64_t D, double theta,
                                  int smax, double* __restrict__ scal, State* __restrict__ gates) {
  if (!gate_on(gates)) return;
  __shared__ double red[EB];
  double m = 0.0;
  for (int64_t j = threadIdx.x; j < D; j += EB) {
    double c = 0.0;
    for (int64_t b = 0; b < nbands; ++b) c += colpart[b * D + j];
    m = fmax(m, c);
  }
  red[threadIdx.x] = m;
  __syncthreads();
  for (int s = EB / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  const double nrm = red[0];
  int s = 0;
  while (s < smax && nrm / ldexp(1.0, s) > theta) ++s;  // smax caps it (norm guard below)
  scal[1] = ldexp(1.0, -s);
  scal[2] = (double)s;
  scal[5] = nrm;
  for (int t = 0; t < smax; ++t) {
    gates[1 + t].status = t < s ? ST_RUNNING : ST_DONE;
    gates[1 + smax + t].status = t < s ? ST_DONE : ST_RUNNING;
  }
}

__global__ void trek_scale_by_kernel(double* __restrict__ X, int64_t n, const double* __restrict__ scal, int which,
                                     const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  const double a = scal[which];
  for (int64_t i = gid(); i < n; i += gstride()) X[i] *= a;
}

// Q = a I + b P  (D x D)
__global__ void trek_axpi_kernel(const double* __restrict__ P, double* __restrict__ Q, double a, double b, int64_t D,
                                 const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  for (int64_t e = gid(); e < D * D; e += gstride()) {
    const int64_t i = e / D, j = e - i * D;
    Q[e] = (i == j ? a : 0.0) + b * P[e];
  }
}

// out = b (P1 + P2)
__global__ void trek_sum2_kernel(const double* __restrict__ P1, const double* __restrict__ P2, double* __restrict__ out,
                                 double b, int64_t n, const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  for (int64_t i = gid(); i < n; i += gstride()) out[i] = b * (P1[i] + P2[i]);
}

__global__ void trek_copy_kernel(const double* __restrict__ src, double* __restrict__ dst, int64_t n,
                                 const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  for (int64_t i = gid(); i < n; i += gstride()) dst[i] = src[i];
}

__global__ void trek_identity_kernel(double* __restrict__ Q, int64_t D, const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  for (int64_t e = gid(); e < D * D; e += gstride()) Q[e] = (e / D == e % D) ? 1.0 : 0.0;
}

__global__ void trek_zero_kernel(double* __restrict__ Q, int64_t n, const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  for (int64_t i = gid(); i < n; i += gstride()) Q[i] = 0.0;
}

// B = a * A^T (64 x 64 tiles through LDS)
__global__ void trek_transpose_kernel(const double* __restrict__ A, double* __restrict__ B, int64_t D,
                                      const double* __restrict__ scal, int which, const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  __shared__ double t[64][65];
  const double a = scal ? scal[which] : 1.0;
  const int64_t bi = blockIdx.y, bj = blockIdx.x;
  for (int it = 0; it < 16; ++it) {
    const int e = it * EB + threadIdx.x, r = e >> 6, c = e & 63;
    t[r][c] = A[(bi * 64 + r) * D + bj * 64 + c];
  }
  __syncthreads();
  for (int it = 0; it < 16; ++it) {
    const int e = it * EB + threadIdx.x, r = e >> 6, c = e & 63;
    B[(bj * 64 + r) * D + bi * 64 + c] = a * t[c][r];
  }
}

// per-block partials of the pair values v_p = H[i_p, j_p]: sum, max
__global__ void trek_pairs_partial_kernel(const double* __restrict__ H, const int32_t* __restrict__ pairs, int64_t m,
                                          int64_t D, double* __restrict__ part, const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  __shared__ double rs[EB], rm[EB];
  double s = 0.0, mx = -INFINITY;
  for (int64_t p = gid(); p < m; p += gstride()) {
    const double v = H[(int64_t)pairs[2 * p] * D + pairs[2 * p + 1]];
    s += v;
    mx = fmax(mx, v);
  }
  rs[threadIdx.x] = s;
  rm[threadIdx.x] = mx;
  __syncthreads();
  for (int k = EB / 2; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) {
      rs[threadIdx.x] += rs[threadIdx.x + k];
      rm[threadIdx.x] = fmax(rm[threadIdx.x], rm[threadIdx.x + k]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = rs[0];
    part[2 * blockIdx.x + 1] = rm[0];
  }
}

// second pass for lse (sum exp(v - max)) and max (tie count)
__global__ void trek_pairs_partial2_kernel(const double* __restrict__ H, const int32_t* __restrict__ pairs, int64_t m,
                                           int64_t D, const double* __restrict__ scal, double* __restrict__ part2,
                                           const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  __shared__ double rs[EB], rc[EB];
  const double mx = scal[3];
  double s = 0.0, c = 0.0;
  for (int64_t p = gid(); p < m; p += gstride()) {
    const double v = H[(int64_t)pairs[2 * p] * D + pairs[2 * p + 1]];
    s += exp(v - mx);
    c += (v == mx) ? 1.0 : 0.0;
  }
  rs[threadIdx.x] = s;
  rc[threadIdx.x] = c;
  __syncthreads();
  for (int k = EB / 2; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) {
      rs[threadIdx.x] += rs[threadIdx.x + k];
      rc[threadIdx.x] += rc[threadIdx.x + k];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part2[2 * blockIdx.x] = rs[0];
    part2[2 * blockIdx.x + 1] = rc[0];
  }
}

// scal[3] = max over pairs (stage 1) ; scal[0] = value and scal[4] = coefficient base (stage 2)
__global__ void trek_pairs_final_kernel(const double* __restrict__ part, const double* __restrict__ part2, int nblk,
                                        int64_t m, int agg, int stage, double* __restrict__ scal,
                                        const State* __restrict__ gate) {
  if (!gate_on(gate) || threadIdx.x != 0) return;
  if (stage == 1) {
    double s = 0.0, mx = -INFINITY;
    for (int b = 0; b < nblk; ++b) {
      s += part[2 * b];
      mx = fmax(mx, part[2 * b + 1]);
    }
    scal[3] = mx;
    if (agg == 0) scal[0] = s / (double)m, scal[4] = 1.0 / (double)m;  // mean
    if (agg == 1) scal[0] = s, scal[4] = 1.0;                           // sum
    return;
  }
  double se = 0.0, ties = 0.0;
  for (int b = 0; b < nblk; ++b) {
    se += part2[2 * b];
    ties += part2[2 * b + 1];
  }
  if (agg == 2) scal[0] = scal[3], scal[4] = 1.0 / ties;           // max: ties share the gradient
  if (agg == 3) scal[0] = scal[3] + log(se), scal[4] = scal[3];    // lse: c_p = exp(v_p - lse)
}

// S = C + C^T with C = d value / d H (S zeroed before)
__global__ void trek_scatter_kernel(const double* __restrict__ H, const int32_t* __restrict__ pairs, int64_t m, int64_t D,
                                    int agg, const double* __restrict__ scal, double* __restrict__ S,
                                    const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  for (int64_t p = gid(); p < m; p += gstride()) {
    const int64_t i = pairs[2 * p], j = pairs[2 * p + 1];
    double c = scal[4];
    if (agg == 2) c = (H[i * D + j] == scal[3]) ? scal[4] : 0.0;
    if (agg == 3) c = exp(H[i * D + j] - scal[0]);
    if (c == 0.0) continue;
    atomicAdd(&S[i * D + j], c);
    atomicAdd(&S[j * D + i], c);
  }
}

// Gtrek[i][j] = weight * (2 W[i][j]) * L[j][i]  on the logical block (L = G_W2^T), 0 elsewhere
__global__ void trek_grad_kernel(const double* __restrict__ W, const double* __restrict__ L, double weight,
                                 double* __restrict__ G, int64_t d, int64_t D, const State* __restrict__ gate) {
  if (!gate_on(gate)) return;
  __shared__ double t[64][65];
  const int64_t bi = blockIdx.y, bj = blockIdx.x;
  for (int it = 0; it < 16; ++it) {
    const int e = it * EB + threadIdx.x, r = e >> 6, c = e & 63;
    t[r][c] = L[(bj * 64 + r) * D + bi * 64 + c];  // L rows bj-block, cols bi-block
  }
  __syncthreads();
  for (int it = 0; it < 16; ++it) {
    const int e = it * EB + threadIdx.x, r = e >> 6, c = e & 63;
    const int64_t i = bi * 64 + r, j = bj * 64 + c;
    double g = 0.0;
    if (i < d && j < d) g = weight * ((2.0 * W[i * D + j]) * t[c][r]);  // weight * grad, linear.py:258
    G[i * D + j] = g;
  }
}

int eb_grid(int64_t n) {
  int64_t b = (n + EB - 1) / EB;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

}  // namespace

// C = op(A) B on D x D operands (split-K slices summed in fixed order when the tile grid is small)
static void gemm_dd(int64_t D, const double* A, bool a_trans, const double* B, double* C, const TrekWork& w,
                    const State* gate, hipStream_t stream);

// log series by Horner (R_K = I/K, R_{k-1} = a_{k-1} I + X R_k) into w.F.  With `dres`, also the
// directional derivative in direction w.GT (dR_{k-1} = X dR_k + G R_k) into w.dQ[.], *dres set.
// Iterates ping-pong in Q[0], Q[1].
static void log_horner_forward(int K, const TrekWork& w, int64_t D, int gdd, const State* g0, hipStream_t stream,
                               double** dres) {
  const int64_t DD = D * D;
  double* R = w.Q[0];
  double* Rn = w.Q[1];
  hipLaunchKernelGGL(trek_identity_kernel, dim3(gdd), dim3(EB), 0, stream, R, D, g0);
  hipLaunchKernelGGL(trek_axpi_kernel, dim3(gdd), dim3(EB), 0, stream, R, R, 0.0, 1.0 / K, D, g0);
  double* dR = w.dQ[0];
  double* dRn = w.dQ[1];
  if (dres) hipLaunchKernelGGL(trek_zero_kernel, dim3(gdd), dim3(EB), 0, stream, dR, DD, g0);
  for (int k = K; k >= 1; --k) {
    if (dres) {  // uses R_k and dR_k before R advances
      gemm_dd(D, w.X, false, dR, w.tmp, w, g0, stream);
      gemm_dd(D, w.GT, false, R, w.tmp2, w, g0, stream);
      hipLaunchKernelGGL(trek_sum2_kernel, dim3(gdd), dim3(EB), 0, stream, w.tmp, w.tmp2, dRn, 1.0, DD, g0);
      double* t = dR;
      dR = dRn;
      dRn = t;
    }
    gemm_dd(D, w.X, false, R, w.tmp, w, g0, stream);
    double* out = k == 1 && !dres ? w.F : Rn;
    hipLaunchKernelGGL(trek_axpi_kernel, dim3(gdd), dim3(EB), 0, stream, w.tmp, out, k - 1 == 0 ? 1.0 : 1.0 / (k - 1),
                       1.0, D, g0);
    double* t = R;
    R = Rn;
    Rn = t;
  }
  if (dres) *dres = dR;
}

static void gemm_dd(int64_t D, const double* A, bool a_trans, const double* B, double* C, const TrekWork& w,
                    const State* gate, hipStream_t stream) {
  const int tiles = (int)((D / 128) * (D / 128));
  if (D % 128 == 0 && tiles < 256 && w.slices) {
    const int split = (int)std::min<int64_t>(4, D / 128);
    launch_gemm(D, D, D, A, D, a_trans, B, D, B_PLAIN, w.slices, D, EPI_STORE, split, D * D, nullptr, 0, 0, gate,
                stream);
    launch_sum_slices(w.slices, split, D * D, D * D, C, gate, stream);
  } else {
    launch_gemm(D, D, D, A, D, a_trans, B, D, B_PLAIN, C, D, EPI_STORE, 1, 0, nullptr, 0, 0, gate, stream);
  }
}

int trek_taylor_degree() { return TREK_TAYLOR_M; }

void launch_trek_pst(const double* W, int64_t d, int64_t D, const TrekCfg& cfg, const TrekWork& w,
                     const State* st, double* Gtrek, hipStream_t stream) {
  const int64_t DD = D * D;
  const int gdd = eb_grid(DD);
  State* g0 = w.gates;  // this slot runs the regularizer
  const dim3 tgrid((unsigned)(D / 64), (unsigned)(D / 64));
  hipLaunchKernelGGL(trek_gate_kernel, dim3(1), dim3(64), 0, stream, st, cfg.mode, w.gates, cfg.smax);
  const int64_t nbands = D / 64;

  // ---- forward pass: F = f(W2), iterates kept for the directional pass ---------------------
  const double* F = nullptr;
  if (cfg.seq == TREK_INV) {
    // F^T = ((1 + eps) I - W2)^-T by the log-det kernels' Gauss-Jordan (no pivots, no warm start)
    launch_build_at(W, D, true, w.L, D, d, 1.0 + cfg.eps_inv, nullptr, g0, stream);
    GJWork gw = w.gj;
    gw.pivlog = nullptr;
    gw.Pstore = nullptr;
    launch_gj_inverse(w.L, D, D, gw, g0, stream);
    hipLaunchKernelGGL(trek_transpose_kernel, tgrid, dim3(EB), 0, stream, w.L, w.F, D, nullptr, 0, g0);
    F = w.F;
  } else {
    hipLaunchKernelGGL(trek_w2_kernel, dim3((unsigned)((D + EB - 1) / EB), (unsigned)nbands), dim3(EB), 0, stream, W,
                       w.X, w.colpart, d, D, g0);
    if (cfg.seq == TREK_EXP) {
      hipLaunchKernelGGL(trek_scale_kernel, dim3(1), dim3(EB), 0, stream, w.colpart, nbands, D, 0.25, cfg.smax,
                         w.scal, w.gates);
      hipLaunchKernelGGL(trek_scale_by_kernel, dim3(gdd), dim3(EB), 0, stream, w.X, DD, w.scal, 1, g0);
      // Taylor by Horner: Q_m = I, Q_{k-1} = I + X Q_k / k; Q_0 = exp(X) to far below eps for ||X||_1 <= 0.25
      const int m = TREK_TAYLOR_M;
      hipLaunchKernelGGL(trek_identity_kernel, dim3(gdd), dim3(EB), 0, stream, w.Q[m], D, g0);
      for (int k = m; k >= 1; --k) {
        gemm_dd(D, w.X, false, w.Q[k], w.tmp, w, g0, stream);
        hipLaunchKernelGGL(trek_axpi_kernel, dim3(gdd), dim3(EB), 0, stream, w.tmp, w.Q[k - 1], 1.0, 1.0 / k, D, g0);
      }
      // squarings E_{t+1} = E_t^2 while t < s (E_0 = Q_0), copies beyond
      for (int t = 0; t < cfg.smax; ++t) {
        const double* Et = t == 0 ? w.Q[0] : w.E[t];
        gemm_dd(D, Et, false, Et, w.E[t + 1], w, &w.gates[1 + t], stream);
        hipLaunchKernelGGL(trek_copy_kernel, dim3(gdd), dim3(EB), 0, stream, Et, w.E[t + 1], DD,
                           &w.gates[1 + cfg.smax + t]);
      }
      F = w.E[cfg.smax];
    } else if (cfg.seq == TREK_LOG) {
      // F = I + sum_{k=1..K} X^k / k by Horner: R_K = I/K, R_{k-1} = a_{k-1} I + X R_k (a_0 = 1);
      // K can be 2d, so the iterates are not kept: the directional pass recomputes them
      log_horner_forward(cfg.K, w, D, gdd, g0, stream, nullptr);
      F = w.F;
    } else {  // TREK_BINOM: (I + X)^p by binary powering; Y_0 = I + X, Y_{t+1} = Y_t^2
      const int p = cfg.K;
      int nb = 0;
      while ((1 << (nb + 1)) <= p) ++nb;  // highest bit
      hipLaunchKernelGGL(trek_axpi_kernel, dim3(gdd), dim3(EB), 0, stream, w.X, w.E[0], 1.0, 1.0, D, g0);
      for (int t = 0; t < nb; ++t) gemm_dd(D, w.E[t], false, w.E[t], w.E[t + 1], w, g0, stream);
      // R over the set bits, low to high: R_0 = I; R <- R Y_t for bit t set (kept in Q[t+1])
      hipLaunchKernelGGL(trek_identity_kernel, dim3(gdd), dim3(EB), 0, stream, w.Q[0], D, g0);
      for (int t = 0; t <= nb; ++t) {
        if (p >> t & 1)
          gemm_dd(D, w.Q[t], false, w.E[t], w.Q[t + 1], w, g0, stream);
        else
          hipLaunchKernelGGL(trek_copy_kernel, dim3(gdd), dim3(EB), 0, stream, w.Q[t], w.Q[t + 1], DD, g0);
      }
      F = w.Q[nb + 1];
    }
  }

  // ---- value and dvalue/dH, G_F = F (C + C^T) ---------------------------------------------
  gemm_dd(D, F, true, F, w.H, w, g0, stream);  // H = F^T F
  const int pb = 256;
  hipLaunchKernelGGL(trek_pairs_partial_kernel, dim3(pb), dim3(EB), 0, stream, w.H, cfg.pairs, cfg.m, D, w.part, g0);
  hipLaunchKernelGGL(trek_pairs_final_kernel, dim3(1), dim3(64), 0, stream, w.part, w.part + 2 * pb, pb, cfg.m,
                     cfg.agg, 1, w.scal, g0);
  if (cfg.agg >= 2) {
    hipLaunchKernelGGL(trek_pairs_partial2_kernel, dim3(pb), dim3(EB), 0, stream, w.H, cfg.pairs, cfg.m, D, w.scal,
                       w.part + 2 * pb, g0);
    hipLaunchKernelGGL(trek_pairs_final_kernel, dim3(1), dim3(64), 0, stream, w.part, w.part + 2 * pb, pb, cfg.m,
                       cfg.agg, 2, w.scal, g0);
  }
  if (cfg.mode != 2) return;  // 'log': the value only (gradient is zero, linear.py:257)
  hipLaunchKernelGGL(trek_zero_kernel, dim3(gdd), dim3(EB), 0, stream, w.S, DD, g0);
  hipLaunchKernelGGL(trek_scatter_kernel, dim3(eb_grid(cfg.m)), dim3(EB), 0, stream, w.H, cfg.pairs, cfg.m, D, cfg.agg,
                     w.scal, w.S, g0);
  gemm_dd(D, F, false, w.S, w.tmp, w, g0, stream);  // G_F
  // directional input G = G_F^T (exp: scaled by 2^-s like X)
  hipLaunchKernelGGL(trek_transpose_kernel, tgrid, dim3(EB), 0, stream, w.tmp, w.GT, D,
                     cfg.seq == TREK_EXP ? w.scal : nullptr, 1, g0);

  // ---- directional pass: L = L_f(W2, G_F^T) = G_W2^T ----------------------------------------
  double* Lres = nullptr;
  if (cfg.seq == TREK_INV) {
    // L_inv(A, E) = F E F  (F = (sI - A)^-1)
    gemm_dd(D, F, false, w.GT, w.tmp, w, g0, stream);
    gemm_dd(D, w.tmp, false, F, w.L, w, g0, stream);
    Lres = w.L;
  } else if (cfg.seq == TREK_LOG) {
    // dR_K = 0; dR_{k-1} = X dR_k + G R_k, with R_k recomputed alongside
    log_horner_forward(cfg.K, w, D, gdd, g0, stream, &Lres);
  } else if (cfg.seq == TREK_EXP) {
    // Horner derivative: dQ_m = 0; dQ_{k-1} = (X dQ_k + G Q_k) / k
    const int top = TREK_TAYLOR_M;
    hipLaunchKernelGGL(trek_zero_kernel, dim3(gdd), dim3(EB), 0, stream, w.dQ[top & 1], DD, g0);
    for (int k = top; k >= 1; --k) {
      gemm_dd(D, w.X, false, w.dQ[k & 1], w.tmp, w, g0, stream);
      gemm_dd(D, w.GT, false, w.Q[k], w.tmp2, w, g0, stream);
      hipLaunchKernelGGL(trek_sum2_kernel, dim3(gdd), dim3(EB), 0, stream, w.tmp, w.tmp2, w.dQ[(k - 1) & 1],
                         1.0 / k, DD, g0);
    }
    Lres = w.dQ[0];
    {
      // squarings: L_{t+1} = E_t L_t + L_t E_t while t < s
      for (int t = 0; t < cfg.smax; ++t) {
        const double* Et = t == 0 ? w.Q[0] : w.E[t];
        double* Lt = w.dQ[t & 1];
        double* Ln = w.dQ[(t + 1) & 1];
        gemm_dd(D, Et, false, Lt, w.tmp, w, &w.gates[1 + t], stream);
        gemm_dd(D, Lt, false, Et, w.tmp2, w, &w.gates[1 + t], stream);
        hipLaunchKernelGGL(trek_sum2_kernel, dim3(gdd), dim3(EB), 0, stream, w.tmp, w.tmp2, Ln, 1.0, DD,
                           &w.gates[1 + t]);
        hipLaunchKernelGGL(trek_copy_kernel, dim3(gdd), dim3(EB), 0, stream, Lt, Ln, DD, &w.gates[1 + cfg.smax + t]);
      }
      Lres = w.dQ[cfg.smax & 1];
    }
  } else {  // binom: product rule through the powering; dY_0 = G, dY_{t+1} = Y_t dY_t + dY_t Y_t
    const int p = cfg.K;
    int nb = 0;
    while ((1 << (nb + 1)) <= p) ++nb;
    // dR_0 = 0; for set bits: dR <- dR Y_t + R dY_t ; dY_t advanced after use
    double* dY = w.GT;  // dY_0
    double* dYn = w.tmp3;
    double* dR = w.dQ[0];
    double* dRn = w.dQ[1];
    hipLaunchKernelGGL(trek_zero_kernel, dim3(gdd), dim3(EB), 0, stream, dR, DD, g0);
    for (int t = 0; t <= nb; ++t) {
      if (p >> t & 1) {
        gemm_dd(D, dR, false, w.E[t], w.tmp, w, g0, stream);
        gemm_dd(D, w.Q[t], false, dY, w.tmp2, w, g0, stream);
        hipLaunchKernelGGL(trek_sum2_kernel, dim3(gdd), dim3(EB), 0, stream, w.tmp, w.tmp2, dRn, 1.0, DD, g0);
        double* sw = dR;
        dR = dRn;
        dRn = sw;
      }
      if (t < nb) {
        gemm_dd(D, w.E[t], false, dY, w.tmp, w, g0, stream);
        gemm_dd(D, dY, false, w.E[t], w.tmp2, w, g0, stream);
        hipLaunchKernelGGL(trek_sum2_kernel, dim3(gdd), dim3(EB), 0, stream, w.tmp, w.tmp2, dYn, 1.0, DD, g0);
        double* sw = dY == w.GT ? w.tmp4 : dY;
        dY = dYn;
        dYn = sw;
      }
    }
    Lres = dR;
  }
  hipLaunchKernelGGL(trek_grad_kernel, tgrid, dim3(EB), 0, stream, W, Lres, cfg.weight, Gtrek, d, D, g0);
  HIP_TRY(hipGetLastError());
}

}  // namespace midagma
