// The fast slot's blocked inverse as ONE launch: the two-level Gauss-Jordan of blockinv.hip
// (outer blocks of B2 = 256, diagonal blocks by the warm-started product form) cut into
// tile tasks that persistent workgroups run in a host-planned order, each task starting as
// soon as the tiles it reads are written -- the same arithmetic on the same tiles, so the
// result is bit-identical to the 4 x (residual, 2-3 passes, panel, trailing) launches it
// replaces (linear.py:226, the per-step `sla.inv(s*I - W*W)`).
//
// Why: at d = 1000 the launch-per-phase inverse is 20 dependent launches of 5-13 us whose
// work is a few us at the chip's rate; the chain of launch boundaries, grid fills and drains
// sets the slot time (profiles/r01_rocprof_cov_d1000_kernel_stats.csv).  Here the next outer
// block's diagonal block, its product-form series and its panels start while the current
// step's trailing update is still running (look-ahead), and no phase waits for a whole grid.
//
// Measured (MI355X, tools/probe_df.py): bit-identical, but SLOWER -- one
// launch 330 us (1 workgroup per CU) / 430 us (2 per CU) against 170 us for the 20 launches at
// d = 1000.  A task's own latency (poll, operand round trips that bypass L1, the 16-step
// series row-partial sum) is 4-15 us, no cheaper than a kernel boundary plus the same work,
// so the chain of 5 dependent hops per outer step costs what the 5 launches cost, and the
// look-ahead has nothing left to hide.  Kept as an experiment (MIDAGMA_EXP_DF=1) with its
// parity tests (tests/test_gpu_dfinv.py) and its plan checker (tests/test_df_plan.py).
//
// Tasks of outer step g (G = rows/cols [g B2, (g+1) B2), A^g the matrix after g steps,
// A^0 = (sI - W o W)^T from build_at, A^K2 = Mt = the inverse):
//   RESID(g, t)    16 x 16 tile t of R = I - S X0 (S = A^g_GG, X0 the extrapolated warm start)
//   PASS(g, p, t)  tile t of Y_p = Y_{p-1} + Y_{p-1} Q_{p-1}, Q_p = Q_{p-1}^2 (or P = ... once
//                  ||Q_{p-1}||_inf <= 1e-8)
//   U(g, a, j)     A^{g+1}[G_a, j] = P A^g[G, j]      (32 x 32 tiles, j outside G)
//   V(g, i, c)     A^{g+1}[i, G_c] = -A^g[i, G] P      (i outside G)
//   DIAG(g, a, c)  A^{g+1}[G_a, G_c] = P_ac, and the warm-start store
//   TRAIL(g, i, j) A^{g+1}[i, j] = A^g[i, j] - A^g[i, G] A^{g+1}[G, j]
// Every A^g is its own D x D buffer (written once per slot: no write-after-read hazards between
// steps that overlap), as are the series iterates of every (g, p).
//
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility, the measured row "one lane of each
// storing workgroup ... agent-scope atomic add / sc1 load poll"): producers store every
// handed-off byte write-through (sc1), every wave waits for its stores (vmcnt 0), then after a
// workgroup barrier one lane adds 1 to the task's completion counter; consumers poll the
// counters of their inputs with sc1 loads (one lane, then a workgroup barrier) and read every
// handed-off byte with sc1 buffer loads (they bypass the CU's L1, which no acquire refreshes).
// Counters of one purpose (a block of A^g, a series pass) each sit on their own 128-B line.
//
// Schedule: the host builds the task DAG, ranks every task by its longest path to the end and
// list-schedules it on the launch's workgroups (one per CU, forced by the LDS request) with a
// cost model; each workgroup runs its own list in start order.  Every dependency of a task
// starts earlier in that order, so with the whole grid resident (grid = CU count, one per CU)
// the lowest unfinished task always has its inputs: no deadlock for any timing.  Every wait
// is bounded (DF_TIMEOUT): a timeout aborts the slot to the host's slow path and is counted,
// and the solver raises on it -- a scheduling bug shows as an error, never as a hung GPU.
#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <utility>

#include "launch.h"
#include "nm16.h"

namespace midagma {

namespace {

constexpr int DF_B2 = 256, DF_L = DF_B2 / 16, DF_NT = DF_B2 / 16, DF_GB = DF_B2 / NB;
constexpr int CTR = 32;  // ints per control word / counter: one 128-B line each
enum CtlWord : int { DF_ABORT = 0, DF_EXIT = 1, DF_TIMEOUTS = 2, DF_DONE0 = 3 };
enum DfType : int { DF_RESID = 0, DF_PASS = 1, DF_U = 2, DF_V = 3, DF_DIAG = 4, DF_TRAIL = 5 };
constexpr int TASK_INTS = 12;  // type, g, p, a, b, sig, dep[3], tgt[3]
constexpr uint64_t DF_TIMEOUT = 20000000;  // device real-time ticks (100 MHz): 200 ms
// LDS: four 32 x 34 images, the 4 x 256 wave-sum buffer, the max scratch and the go word
constexpr int DF_LDS = 4 * NB * ST * 8 + 1024 * 8 + 64;

struct DfArgs {
  const int* tasks;
  const int* woff;
  int* ctl;
  int* ctr;
  double* A[DF_MAX_K2 + 1];
  double* Y;     // [g][p] B2 x B2
  double* Q;
  double* P;     // [g]
  double* part;  // [g][p] row partials (PART_STRIDE)
  double* Pe;    // warm-start stores of the even / odd slots (D x B2)
  double* Po;
  State* st;
  unsigned long long* stamps;  // nullable: per task (wait start, go, done) on the 100 MHz clock
  int D, K2, nctr;
};

// ---- sc1 (L1-bypassing) loads of data other workgroups of this launch wrote ----------------
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const double* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ double ld8(__amdgpu_buffer_rsrc_t r, int64_t elem) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)(elem * 8), 0, 16);
  double d;
  __builtin_memcpy(&d, &v, 8);
  return d;
}
__device__ __forceinline__ double2 ld16(__amdgpu_buffer_rsrc_t r, int64_t elem) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(elem * 8), 0, 16);
  double2 d;
  __builtin_memcpy(&d, &v, 16);
  return d;
}
__device__ __forceinline__ int ld_ctr(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_ctr(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// acc += A[ao.., 0:256] B[bo.., 0:32] for a 32 x 32 output tile, operands by sc1 loads
// (element offsets ao / bo of the tile origins in the buffers behind ra / rb), 32-deep
// chunks through double-buffered LDS images, loads 3 chunks ahead: tile32_gemm_pf's schedule
// and MFMA order (blockinv.hip), so the products are bit-identical.
__device__ __forceinline__ void t32_gemm_sc1(__amdgpu_buffer_rsrc_t ra, int64_t ao, int64_t lda,
                                             __amdgpu_buffer_rsrc_t rb, int64_t bo, int64_t ldb, dbl4& acc,
                                             double* As0, double* As1, double* Bs0, double* Bs1) {
  constexpr int PF = 3, nk = DF_B2 / NB;
  const int tid = threadIdx.x;
  const int r0 = tid >> 4, c0 = (tid & 15) * 2;
  double2 a0[PF], a1[PF], b0[PF], b1[PF];
#define DF_LOAD(slot, kc)                                               \
  do {                                                                  \
    const int64_t ap = ao + (int64_t)r0 * lda + (kc) * 32 + c0;         \
    const int64_t bp = bo + ((int64_t)(kc) * 32 + r0) * ldb + c0;       \
    a0[slot] = ld16(ra, ap);                                            \
    a1[slot] = ld16(ra, ap + 16 * lda);                                 \
    b0[slot] = ld16(rb, bp);                                            \
    b1[slot] = ld16(rb, bp + 16 * ldb);                                 \
  } while (0)
#pragma unroll
  for (int p = 0; p < PF; ++p) DF_LOAD(p, p);
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
    if (kc + PF < nk) DF_LOAD(PF - 1, kc + PF);
    mma32(As, Bs, acc);
  }
#undef DF_LOAD
}

// ---- waits and signals ----------------------------------------------------------------------
// 0: go; 1: abort (another task failed or timed out)
__device__ __forceinline__ bool df_wait(const DfArgs& a, const int* tk, int* sgo) {
  if (threadIdx.x == 0) {
    int ok = 1;
    uint64_t t0 = 0;
    for (;;) {
      bool ready = true;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int c = tk[6 + k];
        if (c >= 0 && ld_ctr(a.ctr + c * CTR) < tk[9 + k]) ready = false;
      }
      if (ready) break;
      if (ld_ctr(a.ctl + DF_ABORT * CTR) != 0) {
        ok = 0;
        break;
      }
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      if (t0 == 0) {
        t0 = now;
      } else if (now - t0 > DF_TIMEOUT) {
        st_ctr(a.ctl + DF_ABORT * CTR, 2);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    *sgo = ok;
  }
  __syncthreads();
  return *sgo != 0;
}

// the task's stores are done (every wave), then one lane counts the task
__device__ __forceinline__ void df_signal(const DfArgs& a, int sig) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && sig >= 0)
    __hip_atomic_fetch_add(a.ctr + sig * CTR, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// a failed task (warm start too far, no convergence): the slot goes back to the host's slow
// path; the last workgroup to leave moves the reason into the State
__device__ __forceinline__ void df_fail(const DfArgs& a) {
  if (threadIdx.x == 0) st_ctr(a.ctl + DF_ABORT * CTR, 1);
}

// ---- the tasks --------------------------------------------------------------------------------
__device__ void task_resid(const DfArgs& a, int g, int t, bool odd, bool extrap, double* red) {
  const int m0 = (t / DF_NT) * 16, n0 = (t % DF_NT) * 16;
  const int64_t G0 = (int64_t)g * DF_B2, D = a.D;
  const int r = threadIdx.x & 15, k0 = splitk_k0<DF_L>();
  const __amdgpu_buffer_rsrc_t rs = rsrc(a.A[g]);
  const double* P1 = (odd ? a.Pe : a.Po) + G0 * DF_B2;  // slot k-1 (previous launches: plain loads)
  const double* P2 = (odd ? a.Po : a.Pe) + G0 * DF_B2;  // slot k-2
  double av[DF_L], bv[DF_L];
  const int64_t so = (G0 + m0 + r) * D + G0 + k0;
#pragma unroll
  for (int q = 0; q < DF_L; ++q) av[q] = ld8(rs, so + q);
#pragma unroll
  for (int q = 0; q < DF_L; ++q) bv[q] = P1[(int64_t)(k0 + q) * DF_B2 + n0 + r];
  if (extrap) {
#pragma unroll
    for (int q = 0; q < DF_L; ++q) bv[q] = 2.0 * bv[q] - P2[(int64_t)(k0 + q) * DF_B2 + n0 + r];
  }
  int row, col;
  tile_elem(threadIdx.x, row, col);
  const int gi = m0 + row, gj = n0 + col;
  const int64_t e = (int64_t)gi * DF_B2 + gj;
  double* Y0 = a.Y + (int64_t)g * (NM_PASSES + 1) * DF_B2 * DF_B2;
  double* Q0 = a.Q + (int64_t)g * (NM_PASSES + 1) * DF_B2 * DF_B2;
  st_wt(Y0 + e, extrap ? 2.0 * P1[e] - P2[e] : P1[e]);
  dbl4 acc = {0.0, 0.0, 0.0, 0.0};
  splitk_mfma<DF_L>(av, bv, acc);
  const double sum = splitk_sum(acc, red);
  const double rv = (gi == gj ? 1.0 : 0.0) - sum;
  st_wt(Q0 + e, rv);
  const double rp = row_sum16(abs_or_inf(rv));
  if (col == 0) st_wt(a.part + (int64_t)g * (NM_PASSES + 1) * PART_STRIDE + (int64_t)gi * DF_NT + n0 / 16, rp);
}

// false: failed (the slot goes to the slow path)
__device__ bool task_pass(const DfArgs& a, int g, int p, int t, double* red, float* red4) {
  int* done = a.ctl + (DF_DONE0 + g) * CTR;
  // an EARLIER pass converged (done holds its number; sibling tasks of this pass may store
  // theirs meanwhile, which must not make this one skip its tile of P)
  const int dn = ld_ctr(done);
  if (dn != 0 && dn < p) return true;
  const int m0 = (t / DF_NT) * 16, n0 = (t % DF_NT) * 16;
  const int r = threadIdx.x & 15, k0 = splitk_k0<DF_L>();
  const int64_t BB = (int64_t)DF_B2 * DF_B2;
  const double* Yp = a.Y + ((int64_t)g * (NM_PASSES + 1) + p - 1) * BB;
  const double* Qp = a.Q + ((int64_t)g * (NM_PASSES + 1) + p - 1) * BB;
  const double* partp = a.part + ((int64_t)g * (NM_PASSES + 1) + p - 1) * PART_STRIDE;
  const __amdgpu_buffer_rsrc_t ry = rsrc(Yp), rq = rsrc(Qp), rp = rsrc(partp);
  double aY[DF_L], aQ[DF_L], bQ[DF_L];
#pragma unroll
  for (int q = 0; q < DF_L; ++q) aY[q] = ld8(ry, (int64_t)(m0 + r) * DF_B2 + k0 + q);
#pragma unroll
  for (int q = 0; q < DF_L; ++q) bQ[q] = ld8(rq, (int64_t)(k0 + q) * DF_B2 + n0 + r);
#pragma unroll
  for (int q = 0; q < DF_L; ++q) aQ[q] = ld8(rq, (int64_t)(m0 + r) * DF_B2 + k0 + q);
  int row, col;
  tile_elem(threadIdx.x, row, col);
  const int gi = m0 + row, gj = n0 + col;
  const double yold = ld8(ry, (int64_t)gi * DF_B2 + gj);
  const double rho = inf_norm_rows<DF_B2>([&](int i) { return ld8(rp, i); }, red4);
  if (!(rho <= 0.25)) return false;  // warm start too far, diverging, or not finite
  dbl4 ay = {0.0, 0.0, 0.0, 0.0};
  if (rho <= 1e-8) {  // last factor: P = Y (I + Q)
    splitk_mfma<DF_L>(aY, bQ, ay);
    const double yq = splitk_sum(ay, red);
    st_wt(a.P + (int64_t)g * BB + (int64_t)gi * DF_B2 + gj, yold + yq);
    if (threadIdx.x == 0) st_ctr(done, p);
    return true;
  }
  dbl4 aq = {0.0, 0.0, 0.0, 0.0};
  splitk_mfma<DF_L>(aY, bQ, ay);
  splitk_mfma<DF_L>(aQ, bQ, aq);
  const double yq = splitk_sum(ay, red);
  __syncthreads();  // red reused
  const double qq = splitk_sum(aq, red);
  st_wt(a.Y + ((int64_t)g * (NM_PASSES + 1) + p) * BB + (int64_t)gi * DF_B2 + gj, yold + yq);
  st_wt(a.Q + ((int64_t)g * (NM_PASSES + 1) + p) * BB + (int64_t)gi * DF_B2 + gj, qq);
  const double rs = row_sum16(abs_or_inf(qq));
  if (col == 0)
    st_wt(a.part + ((int64_t)g * (NM_PASSES + 1) + p) * PART_STRIDE + (int64_t)gi * DF_NT + n0 / 16, rs);
  return true;
}

__device__ __forceinline__ void or_flag(const DfArgs& a, int flag, bool check) {
  // (per-lane flags OR-ed into the State only on the last outer step: the fast slot's domain test)
  if (check && flag) atomicOr(&a.st->flags, flag);
}

// U, V, DIAG of step g; false: the series did not converge
__device__ bool task_panel(const DfArgs& a, int type, int g, int ti, int tj, bool odd, double* img) {
  if (ld_ctr(a.ctl + (DF_DONE0 + g) * CTR) == 0) return false;
  const int64_t D = a.D, G0 = (int64_t)g * DF_B2, BB = (int64_t)DF_B2 * DF_B2;
  const bool check = g == a.K2 - 1;
  double* out = a.A[g + 1];
  const double* P = a.P + (int64_t)g * BB;
  dbl4 acc = {0.0, 0.0, 0.0, 0.0};
  int flag = 0;
  if (type == DF_U) {  // A^{g+1}[G0 + 32 ti, 32 tj] = P[32 ti, :] A^g[G, 32 tj]
    t32_gemm_sc1(rsrc(P), (int64_t)ti * NB * DF_B2, DF_B2, rsrc(a.A[g]), G0 * D + (int64_t)tj * NB, D, acc, img,
                 img + NB * ST, img + 2 * NB * ST, img + 3 * NB * ST);
    double* o = out + (G0 + (int64_t)ti * NB) * D + (int64_t)tj * NB;
    acc_foreach(acc, [&](int row, int col, double& v) {
      st_wt(o + (int64_t)row * D + col, v);
      flag |= domain_flag(v);
    });
  } else if (type == DF_V) {  // A^{g+1}[32 ti, G0 + 32 tj] = -A^g[32 ti, G] P[:, 32 tj]
    t32_gemm_sc1(rsrc(a.A[g]), (int64_t)ti * NB * D + G0, D, rsrc(P), (int64_t)tj * NB, DF_B2, acc, img,
                 img + NB * ST, img + 2 * NB * ST, img + 3 * NB * ST);
    double* o = out + (int64_t)ti * NB * D + G0 + (int64_t)tj * NB;
    acc_foreach(acc, [&](int row, int col, double& v) {
      st_wt(o + (int64_t)row * D + col, -v);
      flag |= domain_flag(-v);
    });
  } else {  // DIAG: A^{g+1}[G_ti, G_tj] = P tile, and this slot's warm-start store
    const __amdgpu_buffer_rsrc_t rp = rsrc(P);
    double* o = out + (G0 + (int64_t)ti * NB) * D + G0 + (int64_t)tj * NB;
    double* ps = (odd ? a.Po : a.Pe) + G0 * DF_B2 + (int64_t)ti * NB * DF_B2 + (int64_t)tj * NB;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int e = it * NTHREADS + threadIdx.x, row = e >> 5, col = e & 31;
      const double v = ld8(rp, (int64_t)(ti * NB + row) * DF_B2 + tj * NB + col);
      st_wt(o + (int64_t)row * D + col, v);
      st_wt(ps + (int64_t)row * DF_B2 + col, v);
      flag |= domain_flag(v);
    }
  }
  or_flag(a, flag, check);
  return true;
}

__device__ void task_trail(const DfArgs& a, int g, int ti, int tj, double* img) {
  const int64_t D = a.D, G0 = (int64_t)g * DF_B2;
  const __amdgpu_buffer_rsrc_t ra = rsrc(a.A[g]), rn = rsrc(a.A[g + 1]);
  const int64_t ci = (int64_t)ti * NB * D + (int64_t)tj * NB;
  dbl4 c_old;
  acc_foreach(c_old, [&](int row, int col, double& v) { v = ld8(ra, ci + (int64_t)row * D + col); });
  dbl4 acc = {0.0, 0.0, 0.0, 0.0};
  t32_gemm_sc1(ra, (int64_t)ti * NB * D + G0, D, rn, G0 * D + (int64_t)tj * NB, D, acc, img, img + NB * ST,
               img + 2 * NB * ST, img + 3 * NB * ST);
  double* o = a.A[g + 1] + ci;
  const int lane = threadIdx.x & 63, m0 = q_m0(), n0 = q_n0();
  int flag = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int row = m0 + acc_row(lane, t), col = n0 + acc_col(lane);
    const double v = c_old[t] - acc[t];
    st_wt(o + (int64_t)row * D + col, v);
    flag |= domain_flag(v);
  }
  or_flag(a, flag, g == a.K2 - 1);
}

__global__ __launch_bounds__(NTHREADS, 2) void dfinv_kernel(DfArgs a) {
  State* st = a.st;
  if (st->status != ST_RUNNING) return;
  if (st->ckpt_pending) {  // a log-det is due: pivots come from the slow path only
    if (blockIdx.x == 0 && threadIdx.x == 0) st->status = ST_NEED_GJ;
    return;
  }
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* img = sm;                  // 4 x 32 x 34 images
  double* red = sm + 4 * NB * ST;    // 1024
  float* red4 = reinterpret_cast<float*>(red + 1024);
  int* sgo = reinterpret_cast<int*>(red4 + 4);
  const bool odd = (st->slots & 1) != 0;
  const bool extrap = st->warm_run >= 2;
  const int t_end = a.woff[blockIdx.x + 1];
  for (int t = a.woff[blockIdx.x]; t < t_end; ++t) {
    const int* tk = a.tasks + (int64_t)t * TASK_INTS;
    int tv[TASK_INTS];
#pragma unroll
    for (int k = 0; k < TASK_INTS; ++k) tv[k] = tk[k];
    const unsigned long long tw = a.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
    if (!df_wait(a, tv, sgo)) break;
    const unsigned long long tg = a.stamps ? __builtin_amdgcn_s_memrealtime() : 0;
    const int type = tv[0], g = tv[1];
    bool ok = true;
    if (type == DF_RESID)
      task_resid(a, g, tv[3], odd, extrap, red);
    else if (type == DF_PASS)
      ok = task_pass(a, g, tv[2], tv[3], red, red4);
    else if (type == DF_TRAIL)
      task_trail(a, g, tv[3], tv[4], img);
    else
      ok = task_panel(a, type, g, tv[3], tv[4], odd, img);
    if (!ok) {
      df_fail(a);
      break;
    }
    df_signal(a, tv[5]);
    if (a.stamps && threadIdx.x == 0) {
      a.stamps[3 * t] = tw;
      a.stamps[3 * t + 1] = tg;
      a.stamps[3 * t + 2] = __builtin_amdgcn_s_memrealtime();
    }
  }
  // leave: the last workgroup out resets the counters for the next slot's launch and hands a
  // failure to the host (the State is written only here, after every workgroup read it)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < 64) {
    int last = 0;
    if (threadIdx.x == 0)
      last = __hip_atomic_fetch_add(a.ctl + DF_EXIT * CTR, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             (int)gridDim.x - 1;
    last = __shfl(last, 0);
    if (last) {
      const int why = ld_ctr(a.ctl + DF_ABORT * CTR);
      for (int i = threadIdx.x; i < a.nctr; i += 64) st_ctr(a.ctr + i * CTR, 0);
      for (int g = threadIdx.x; g < a.K2; g += 64) st_ctr(a.ctl + (DF_DONE0 + g) * CTR, 0);
      if (threadIdx.x == 0) {
        if (why != 0) st->status = ST_NEED_GJ;
        if (why == 2) __hip_atomic_fetch_add(a.ctl + DF_TIMEOUTS * CTR, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        st_ctr(a.ctl + DF_ABORT * CTR, 0);
        st_ctr(a.ctl + DF_EXIT * CTR, 0);
      }
    }
  }
}

// ---- host: the task DAG and its list schedule -------------------------------------------------
struct Plan {
  std::vector<int> tasks, woff;
  int nctr = 0;
  double est_us = 0;
};

double cost_of(int type) {  // us, the list scheduler's model (measured per task type on MI355X)
  static const double c[6] = {4.2, 5.0, 7.0, 5.5, 2.5, 6.7};
  return c[type];
}

Plan make_plan(int64_t D, int passes, int nwg, double hop_us) {
  const int K2 = (int)(D / DF_B2), nb = (int)(D / NB);
  // counters: blk(g, bi, bj) for g = 1..K2 (of A^K2 = Mt only the U blocks, which the last
  // trailing update reads), then ser(g, p)
  auto blk = [&](int g, int bi, int bj) { return ((g - 1) * K2 + bi) * K2 + bj; };
  const int ser0 = K2 * K2 * K2;
  auto ser = [&](int g, int p) { return ser0 + g * (NM_PASSES + 1) + p; };
  Plan plan;
  plan.nctr = ser0 + K2 * (NM_PASSES + 1);
  struct T {
    int v[TASK_INTS];
  };
  std::vector<T> ts;
  auto add = [&](int type, int g, int p, int a, int b, int sig, std::initializer_list<std::pair<int, int>> deps) {
    T t;
    int* v = t.v;
    v[0] = type, v[1] = g, v[2] = p, v[3] = a, v[4] = b, v[5] = sig;
    int k = 0;
    for (auto& d : deps) {
      v[6 + k] = d.first;
      v[9 + k] = d.second;
      ++k;
    }
    for (; k < 3; ++k) v[6 + k] = -1, v[9 + k] = 0;
    ts.push_back(t);
  };
  const int nser = DF_NT * DF_NT, gg = DF_GB * DF_GB;
  for (int g = 0; g < K2; ++g) {
    const bool last = g == K2 - 1;
    for (int t = 0; t < nser; ++t) {
      if (g == 0)
        add(DF_RESID, g, 0, t, 0, ser(g, 0), {});
      else
        add(DF_RESID, g, 0, t, 0, ser(g, 0), {{blk(g, g, g), gg}});
    }
    for (int p = 1; p <= passes; ++p)
      for (int t = 0; t < nser; ++t) add(DF_PASS, g, p, t, 0, ser(g, p), {{ser(g, p - 1), nser}});
    const std::pair<int, int> pdone{ser(g, passes), nser};
    for (int a = 0; a < DF_GB; ++a)
      for (int j = 0; j < nb; ++j) {
        const int bj = j / DF_GB;
        if (bj == g) continue;
        const int sig = blk(g + 1, g, bj);
        if (g == 0)
          add(DF_U, g, 0, a, j, sig, {pdone});
        else
          add(DF_U, g, 0, a, j, sig, {pdone, {blk(g, g, bj), gg}});
      }
    for (int i = 0; i < nb; ++i) {
      const int bi = i / DF_GB;
      if (bi == g) continue;
      for (int c = 0; c < DF_GB; ++c) {
        const int sig = last ? -1 : blk(g + 1, bi, g);
        if (g == 0)
          add(DF_V, g, 0, i, c, sig, {pdone});
        else
          add(DF_V, g, 0, i, c, sig, {pdone, {blk(g, bi, g), gg}});
      }
    }
    for (int a = 0; a < DF_GB; ++a)
      for (int c = 0; c < DF_GB; ++c) add(DF_DIAG, g, 0, a, c, last ? -1 : blk(g + 1, g, g), {pdone});
    for (int i = 0; i < nb; ++i) {
      const int bi = i / DF_GB;
      if (bi == g) continue;
      for (int j = 0; j < nb; ++j) {
        const int bj = j / DF_GB;
        if (bj == g) continue;
        const int sig = last ? -1 : blk(g + 1, bi, bj);
        if (g == 0)
          add(DF_TRAIL, g, 0, i, j, sig, {{blk(g + 1, g, bj), gg}});
        else
          add(DF_TRAIL, g, 0, i, j, sig, {{blk(g + 1, g, bj), gg}, {blk(g, bi, bj), gg}, {blk(g, bi, g), gg}});
      }
    }
  }
  const int n = (int)ts.size();
  // signalers and waiters per counter; expected counts must match the targets
  std::vector<std::vector<int>> waiters(plan.nctr);
  std::vector<int> nsig(plan.nctr, 0);
  for (int i = 0; i < n; ++i) {
    if (ts[i].v[5] >= 0) ++nsig[ts[i].v[5]];
    for (int k = 0; k < 3; ++k)
      if (ts[i].v[6 + k] >= 0) waiters[ts[i].v[6 + k]].push_back(i);
  }
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k)
      if (ts[i].v[6 + k] >= 0 && nsig[ts[i].v[6 + k]] != ts[i].v[9 + k])
        throw std::logic_error("dfinv plan: counter target mismatch");
  // upward rank (tasks were generated in a topological order)
  std::vector<double> rank(n, 0.0), crank(plan.nctr, 0.0);
  for (int i = n - 1; i >= 0; --i) {
    const int s = ts[i].v[5];
    rank[i] = cost_of(ts[i].v[0]) + (s >= 0 ? hop_us + crank[s] : 0.0);
    for (int k = 0; k < 3; ++k) {
      const int c = ts[i].v[6 + k];
      if (c >= 0) crank[c] = std::max(crank[c], rank[i]);
    }
  }
  // list schedule on nwg identical workers
  std::vector<int> pend(n, 0), cleft(nsig);
  std::vector<double> cfin(plan.nctr, 0.0), ready(n, 0.0), start(n, 0.0);
  std::vector<int> avail;
  for (int i = 0; i < n; ++i) {
    for (int k = 0; k < 3; ++k)
      if (ts[i].v[6 + k] >= 0) ++pend[i];
    if (pend[i] == 0) avail.push_back(i);
  }
  std::vector<double> freeat(nwg, 0.0);
  std::vector<std::vector<int>> lists(nwg);
  double makespan = 0;
  for (int done = 0; done < n; ++done) {
    const int w = (int)(std::min_element(freeat.begin(), freeat.end()) - freeat.begin());
    const double T = freeat[w];
    int best = -1;
    for (int idx = 0; idx < (int)avail.size(); ++idx) {
      const int i = avail[idx];
      if (ready[i] <= T) {
        if (best < 0 || ready[avail[best]] > T || rank[i] > rank[avail[best]]) best = idx;
      } else if (best < 0 || (ready[avail[best]] > T && (ready[i] < ready[avail[best]] ||
                                                          (ready[i] == ready[avail[best]] &&
                                                           rank[i] > rank[avail[best]])))) {
        best = idx;
      }
    }
    if (best < 0) throw std::logic_error("dfinv plan: no task available (cycle)");
    const int i = avail[best];
    avail[best] = avail.back();
    avail.pop_back();
    start[i] = std::max(T, ready[i]);
    freeat[w] = start[i] + cost_of(ts[i].v[0]);
    makespan = std::max(makespan, freeat[w]);
    lists[w].push_back(i);
    const int s = ts[i].v[5];
    if (s >= 0) {
      cfin[s] = std::max(cfin[s], freeat[w]);
      if (--cleft[s] == 0)
        for (int j : waiters[s]) {
          ready[j] = std::max(ready[j], cfin[s] + hop_us);
          if (--pend[j] == 0) avail.push_back(j);
        }
    }
  }
  plan.woff.assign(nwg + 1, 0);
  for (int w = 0; w < nwg; ++w) {
    plan.woff[w + 1] = plan.woff[w] + (int)lists[w].size();
    for (int i : lists[w]) plan.tasks.insert(plan.tasks.end(), ts[i].v, ts[i].v + TASK_INTS);
  }
  plan.est_us = makespan;
  return plan;
}

}  // namespace

bool df_available(int64_t D) {
  if (D % DF_B2 != 0 || D < 2 * DF_B2 || D / DF_B2 > DF_MAX_K2 || binv_block(D) != DF_B2) return false;
  static const int64_t maxd = knob("MIDAGMA_EXP_DF_MAXD", 1536);
  return D <= maxd;
}

int64_t df_ctl_ints(int64_t D) {
  const int64_t K2 = D / DF_B2;
  const int64_t nctr = K2 * K2 * K2 + K2 * (NM_PASSES + 1);
  return (int64_t)CTR * (DF_DONE0 + K2 + nctr);
}

DfPlanHost df_plan(int64_t D, int passes, int nwg) {
  static std::mutex mu;
  static std::map<std::pair<int64_t, int>, std::pair<int, Plan>> cache;  // (D, passes) -> (nwg, plan)
  static const double hop = knob_f("MIDAGMA_EXP_DF_HOP", 1.0);
  std::lock_guard<std::mutex> lk(mu);
  auto key = std::make_pair(D, passes);
  auto it = cache.find(key);
  if (it == cache.end() || it->second.first != nwg)
    it = cache.insert_or_assign(key, std::make_pair(nwg, make_plan(D, passes, nwg, hop))).first;
  const Plan& p = it->second.second;
  return DfPlanHost{&p.tasks, &p.woff, p.nctr, p.est_us};
}

void launch_df_inverse(double* Mt, int64_t D, const DfWork& w, const BInvWork& bw, int passes, State* st,
                       hipStream_t stream) {
  if (!df_available(D)) throw std::invalid_argument("dfinv: D not supported");
  static bool attr = false;
  if (!attr) {
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(dfinv_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, DF_LDS));
    attr = true;
  }
  const int K2 = (int)(D / DF_B2);
  DfArgs a{};
  a.tasks = w.tasks[passes == 2 ? 0 : 1];
  a.woff = w.woff[passes == 2 ? 0 : 1];
  a.ctl = w.ctl;
  a.ctr = w.ctl + CTR * (DF_DONE0 + K2);
  for (int g = 0; g < K2; ++g) a.A[g] = w.A[g];
  a.A[K2] = Mt;
  a.Y = w.Y;
  a.Q = w.Q;
  a.P = w.P;
  a.part = bw.part;
  a.Pe = bw.Pst;
  a.Po = bw.Pst1;
  a.st = st;
  a.stamps = w.stamps;
  a.D = (int)D;
  a.K2 = K2;
  a.nctr = (int)(K2 * K2 * K2 + K2 * (NM_PASSES + 1));
  hipLaunchKernelGGL(dfinv_kernel, dim3(w.nwg), dim3(NTHREADS), DF_LDS, stream, a);
  HIP_TRY(hipGetLastError());
}

}  // namespace midagma
