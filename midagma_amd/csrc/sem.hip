// Linear-SEM sample generator on the GPU (reference
// /root/reference/src/dagma/utils.py:99-172, simulate_linear_sem).
//
// X (n x d, row-major) is produced slab by slab of rows:
//   1. one launch per topological level: every (node j of the level, row pair) evaluates
//      x_j = sum_{p in pa(j), ascending} W[p, j] x_p  (+ noise / link)  into a node-major
//      slab XT[j][r] -- coalesced over rows, the parents' columns were written by the
//      previous levels of the same slab (L2 / MALL resident for slabs of a few GB);
//   2. an LDS-tiled transpose XT -> X rows.
// Noise comes from Philox4x32-10 (key = seed, counter = (row pair, node, draw)): one block
// gives two uniforms, i.e. one Box-Muller pair, i.e. the noise of rows 2k and 2k+1 -- every
// row's values are independent of how rows are split into calls or shards.
// Algorithmic traffic: 8 B per element of X (the output); the slab adds 8 B (XT write)
// + 8 B x in-degree (parents) + 8 B (transpose read), mostly cache-resident.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "launch.h"

namespace midagma {
namespace {

constexpr uint32_t PH_M0 = 0xD2511F53u, PH_M1 = 0xCD9E8D57u;
constexpr uint32_t PH_W0 = 0x9E3779B9u, PH_W1 = 0xBB67AE85u;
constexpr uint32_t POISSON_DRAW0 = 1u << 30;

struct U4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += PH_W0;
      k1 += PH_W1;
    }
    const uint32_t hi0 = __umulhi(PH_M0, c.x), lo0 = PH_M0 * c.x;
    const uint32_t hi1 = __umulhi(PH_M1, c.z), lo1 = PH_M1 * c.z;
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
  }
  return c;
}

// (k + 1/2) 2^-52 with k the top 52 bits of hi:lo -- exact, in (0, 1)
__device__ __forceinline__ double u52(uint32_t hi, uint32_t lo) {
  const uint64_t k = ((static_cast<uint64_t>(hi) << 32) | lo) >> 12;
  return (static_cast<double>(k) + 0.5) * 0x1p-52;
}

struct Uniforms {
  double a, b;
};

__device__ __forceinline__ Uniforms block_uniforms(uint64_t pair, uint32_t node, uint32_t draw, uint32_t k0,
                                                   uint32_t k1) {
  const U4 x = philox4x32_10(U4{static_cast<uint32_t>(pair), static_cast<uint32_t>(pair >> 32), node, draw}, k0, k1);
  return Uniforms{u52(x.x, x.y), u52(x.z, x.w)};
}

// numpy's Poisson samplers (multiplication below 10, PTRS above) on this row's own blocks
__device__ __noinline__ double poisson_sample(double lam, uint64_t pair, uint32_t node, uint32_t odd, uint32_t k0, uint32_t k1) {
  if (!(lam > 0.0)) return 0.0;
  uint32_t draw = POISSON_DRAW0 + (odd << 29);
  double buf = 0.0;
  bool have = false;
  auto next = [&]() -> double {
    if (have) {
      have = false;
      return buf;
    }
    const Uniforms u = block_uniforms(pair, node, draw++, k0, k1);
    buf = u.b;
    have = true;
    return u.a;
  };
  if (lam < 10.0) {
    const double enlam = exp(-lam);
    double x = 0.0, prod = 1.0;
    for (int it = 0; it < 100000; ++it) {
      prod = prod * next();
      if (prod > enlam)
        x += 1.0;
      else
        return x;
    }
    return x;
  }
  const double slam = sqrt(lam), loglam = log(lam);
  const double b = 0.931 + 2.53 * slam;
  const double a = -0.059 + 0.02483 * b;
  const double invalpha = 1.1239 + 1.1328 / (b - 3.4);
  const double vr = 0.9277 - 3.6224 / (b - 2.0);
  double k = 0.0;
  for (int it = 0; it < 4096; ++it) {  // acceptance ~0.9 per try: the cap is never reached
    const double U = next() - 0.5;
    const double V = next();
    const double us = 0.5 - fabs(U);
    k = floor((2.0 * a / us + b) * U + lam + 0.43);
    if (us >= 0.07 && V <= vr) return k;
    if (k < 0.0 || (us < 0.013 && V > us)) continue;
    if ((log(V) + log(invalpha) - log(a / (us * us) + b)) <= (-lam + k * loglam - lgamma(k + 1.0))) return k;
  }
  return fmax(k, 0.0);
}

// One level: blockIdx.y = node of the level, each thread two consecutive rows (one Philox
// block).  XT is node-major with row stride ldt (even).  One instantiation per noise type
// keeps the Gaussian kernel free of the Poisson sampler's registers.
template <int SEM>
__global__ __launch_bounds__(256) void sem_level_kernel(const int32_t* __restrict__ nodes,
                                                        const int32_t* __restrict__ pptr,
                                                        const int32_t* __restrict__ pidx,
                                                        const double* __restrict__ pw,
                                                        const double* __restrict__ scale, uint32_t k0,
                                                        uint32_t k1, int64_t row0, int64_t rows, int64_t ldt,
                                                        double* __restrict__ XT) {
  const int j = nodes[blockIdx.y];
  const int64_t r = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) * 2;  // slab-local, even
  if (r >= rows) return;
  const bool two = r + 1 < rows;
  double acc0 = 0.0, acc1 = 0.0;
  const int e1 = pptr[j + 1];
  for (int e = pptr[j]; e < e1; ++e) {
    const double w = pw[e];
    const double2 x = *reinterpret_cast<const double2*>(XT + static_cast<int64_t>(pidx[e]) * ldt + r);
    acc0 = acc0 + w * x.x;
    acc1 = acc1 + w * x.y;
  }
  const int64_t g = row0 + r;  // global row (row0 even)
  const uint64_t pair = static_cast<uint64_t>(g) >> 1;
  const double s = scale[j];
  double x0, x1;
  if constexpr (SEM == 5) {
    x0 = poisson_sample(exp(acc0), pair, j, 0, k0, k1);
    x1 = two ? poisson_sample(exp(acc1), pair, j, 1, k0, k1) : 0.0;
  } else {
    const Uniforms u = block_uniforms(pair, static_cast<uint32_t>(j), 0u, k0, k1);
    switch (SEM) {
      case 0: {  // Box-Muller: both outputs of the pair
        const double rr = sqrt(-2.0 * log(u.a));
        const double t = 2.0 * M_PI * u.b;
        double sn, cs;
        sincos(t, &sn, &cs);
        x0 = acc0 + s * (rr * cs);
        x1 = acc1 + s * (rr * sn);
        break;
      }
      case 1:
        x0 = acc0 + (-s) * log(u.a);
        x1 = acc1 + (-s) * log(u.b);
        break;
      case 2:
        x0 = acc0 + (-s) * log(-log(u.a));
        x1 = acc1 + (-s) * log(-log(u.b));
        break;
      case 3:
        x0 = acc0 + (-s + (2.0 * s) * u.a);
        x1 = acc1 + (-s + (2.0 * s) * u.b);
        break;
      default:  // 4 logistic
        x0 = u.a < 1.0 / (1.0 + exp(-acc0)) ? 1.0 : 0.0;
        x1 = u.b < 1.0 / (1.0 + exp(-acc1)) ? 1.0 : 0.0;
        break;
    }
  }
  double* o = XT + static_cast<int64_t>(j) * ldt + r;
  if (two)
    *reinterpret_cast<double2*>(o) = double2{x0, x1};
  else
    o[0] = x0;
}

// X[(r) * ldx + j] = XT[j * ldt + r] for j < d, r < rows: 64 x 64 tiles through LDS.
__global__ __launch_bounds__(256) void sem_transpose_kernel(const double* __restrict__ XT, int64_t ldt,
                                                            int64_t d, int64_t rows, double* __restrict__ X,
                                                            int64_t ldx) {
  __shared__ double t[64][65];
  const int64_t j0 = static_cast<int64_t>(blockIdx.y) * 64, r0 = static_cast<int64_t>(blockIdx.x) * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int64_t j = j0 + i, r = r0 + tx;
    t[i][tx] = (j < d && r < rows) ? XT[j * ldt + r] : 0.0;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int64_t r = r0 + i, j = j0 + tx;
    if (r < rows && j < d) X[r * ldx + j] = t[tx][i];
  }
}

}  // namespace

bool sem_levels(const double* W, int64_t d, SemGraph& g) {
  g.pptr.assign(d + 1, 0);
  g.pidx.clear();
  g.pw.clear();
  std::vector<int32_t> indeg(d, 0);
  for (int64_t j = 0; j < d; ++j) {
    for (int64_t p = 0; p < d; ++p)
      if (W[p * d + j] != 0.0) {
        g.pidx.push_back(static_cast<int32_t>(p));
        g.pw.push_back(W[p * d + j]);
        ++indeg[j];
      }
    g.pptr[j + 1] = static_cast<int32_t>(g.pidx.size());
  }
  g.nodes.clear();
  g.level_off.assign(1, 0);
  std::vector<int32_t> level;
  for (int64_t j = 0; j < d; ++j)
    if (indeg[j] == 0) level.push_back(static_cast<int32_t>(j));
  while (!level.empty()) {
    g.nodes.insert(g.nodes.end(), level.begin(), level.end());
    g.level_off.push_back(static_cast<int32_t>(g.nodes.size()));
    std::vector<int32_t> next;
    for (int32_t j : level)
      for (int64_t c = 0; c < d; ++c)
        if (W[j * d + c] != 0.0 && --indeg[c] == 0) next.push_back(static_cast<int32_t>(c));
    std::sort(next.begin(), next.end());
    level.swap(next);
  }
  return static_cast<int64_t>(g.nodes.size()) == d;
}

void launch_sem_slab(const SemDev& g, const std::vector<int32_t>& level_off, int64_t d, int sem, uint64_t seed,
                     int64_t row0, int64_t rows, int64_t skip, double* XT, int64_t ldt, double* X, int64_t ldx,
                     hipStream_t stream) {
  const int64_t n_levels = static_cast<int64_t>(level_off.size()) - 1;
  const uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32);
  const unsigned gx = static_cast<unsigned>((rows + 511) / 512);
  for (int64_t l = 0; l < n_levels; ++l) {
    const int32_t off = level_off[l], cnt = level_off[l + 1] - level_off[l];
    auto kern = sem == 0 ? sem_level_kernel<0> : sem == 1 ? sem_level_kernel<1> : sem == 2 ? sem_level_kernel<2>
              : sem == 3 ? sem_level_kernel<3> : sem == 4 ? sem_level_kernel<4> : sem_level_kernel<5>;
    hipLaunchKernelGGL(kern, dim3(gx, cnt), dim3(256), 0, stream, g.nodes + off, g.pptr, g.pidx, g.pw, g.scale, k0,
                       k1, row0, rows, ldt, XT);
  }
  hipLaunchKernelGGL(sem_transpose_kernel, dim3(static_cast<unsigned>((rows - skip + 63) / 64),
                                                static_cast<unsigned>((d + 63) / 64)),
                     dim3(256), 0, stream, XT + skip, ldt, d, rows - skip, X, ldx);
}

}  // namespace midagma
