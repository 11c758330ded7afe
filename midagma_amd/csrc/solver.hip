// Host orchestration + C ABI (include/midagma_hip.h).  The solver object and its drivers:
// solver_impl.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/midagma_hip.h"
#include "solver_impl.h"

namespace {
thread_local std::string g_global_error;

// scipy's check_finite (linear.py:226 -> sla.inv(..., check_finite=True)): a non-finite input
// is a ValueError, not a singular matrix
bool all_finite(const double* p, int64_t rows, int64_t cols, int64_t ld) {
  for (int64_t i = 0; i < rows; ++i)
    for (int64_t j = 0; j < cols; ++j)
      if (!std::isfinite(p[i * ld + j])) return false;
  return true;
}
constexpr const char* kNonFinite = "array must not contain infs or NaNs";
}  // namespace

namespace {

__global__ void div_kernel(const double* __restrict__ x, double n, double* __restrict__ y, int64_t count) {
  for (int64_t i = (int64_t)blockIdx.x * NTHREADS + threadIdx.x; i < count; i += (int64_t)gridDim.x * NTHREADS)
    y[i] = x[i] / n;
}

int fail(midagma_solver* s, int code, const std::string& msg) {
  if (s)
    s->err = msg;
  else
    g_global_error = msg;
  return code;
}

template <class F>
int guarded(midagma_solver* s, F&& f) {
  try {
    if (s) HIP_TRY(hipSetDevice(s->device));
    return f();
  } catch (const HipError& e) {
    return fail(s, MIDAGMA_E_HIP, e.what());
  } catch (const std::invalid_argument& e) {
    return fail(s, MIDAGMA_E_ARG, e.what());
  } catch (const std::exception& e) {
    return fail(s, MIDAGMA_E_STATE, e.what());
  }
}

std::once_flag g_attr_once;
void setup_attributes_once() {
  std::call_once(g_attr_once, [] {
    gj_setup_attributes();
    gemm_setup_attributes();
  });
}

// A minimize that ended ST_SINGULAR: the reference's sla.inv raised at that step.  scipy
// raises ValueError when sI - W*W has a non-finite entry (check_finite: W itself went
// non-finite, e.g. from non-finite data) and LinAlgError when the finite matrix is singular.
int singular_or_nonfinite(midagma_solver* s, int rc, const midagma_result* res, const double* W) {
  if (rc != MIDAGMA_OK || !res || res->status != MIDAGMA_ST_SINGULAR) return rc;
  if (!all_finite(W, s->d, s->d, s->d)) return fail(s, MIDAGMA_E_ARG, std::string("minimize: ") + kNonFinite);
  return fail(s, MIDAGMA_E_SINGULAR, "singular matrix: inverse of sI - W*W is not finite");
}

}  // namespace

extern "C" {

int midagma_abi_version(void) { return MIDAGMA_ABI_VERSION; }

int midagma_device_count(int* n) {
  return guarded(nullptr, [&] {
    HIP_TRY(hipGetDeviceCount(n));
    return MIDAGMA_OK;
  });
}

const char* midagma_last_error(const midagma_solver* s) { return s ? s->err.c_str() : g_global_error.c_str(); }

int midagma_create(midagma_solver** out, int loss, int mode, int64_t d, int device, void* stream) {
  if (!out || d < 1 || (loss != 0 && loss != 1) || (mode != 0 && mode != 1) ||
      (loss == MIDAGMA_LOSS_LOGISTIC && mode == MIDAGMA_MODE_COV))
    return fail(nullptr, MIDAGMA_E_ARG, "midagma_create: bad arguments (logistic needs data mode)");
  midagma_solver* s = new midagma_solver();
  s->loss = loss;
  s->mode = mode;
  s->d = d;
  // 128-multiples feed the 128x128 GEMM tiles.  Cov mode pads 129 <= d <= 192 to 256 as well: the
  // blocked inverse then has one 256-wide outer block, and its warm-started product form beats
  // the flat Gauss-Jordan's 6 block steps on 192 (data mode keeps 192: X's columns are GEMM work)
  const bool pad256 = mode == MIDAGMA_MODE_COV && knob("MIDAGMA_EXP_COV_PAD256", 1) != 0;
  s->D = d > 192 || (pad256 && d > 128) ? (d + 127) / 128 * 128 : round_up64(d);
  // Cov mode, 256 < d <= 640: D to a multiple of 256, so the blocked inverse runs B2 = 256 outer
  // blocks (2 instead of 3 at D = 384 -> 512, 3 instead of 5 at 640 -> 768: d=300 11.1k -> 11.3k,
  // d=600 6.4k -> 7.0k steps/s).  Larger D keep B2 = 128 (d=1150 even, d=1400 -3.5%, d=1700
  // even: the padded GEMM work outweighs the saved outer steps).  Knob MIDAGMA_EXP_COV_PAD_B2:
  // 0 off, 1 at every d > 256.
  const int pad_b2 = (int)knob("MIDAGMA_EXP_COV_PAD_B2", -1);
  if (mode == MIDAGMA_MODE_COV && d > 256 && (pad_b2 == 1 || (pad_b2 < 0 && d <= 640)))
    s->D = (d + 255) / 256 * 256;
  s->device = device;
  int rc = guarded(s, [&] {
    setup_attributes_once();
    if (stream) {
      s->stream = reinterpret_cast<hipStream_t>(stream);
    } else {
      HIP_TRY(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
      s->own_stream = true;
    }
    s->alloc_core();
    HIP_TRY(hipStreamSynchronize(s->stream));
    return MIDAGMA_OK;
  });
  if (rc != MIDAGMA_OK) {
    g_global_error = s->err;
    delete s;
    return rc;
  }
  *out = s;
  return MIDAGMA_OK;
}

void midagma_destroy(midagma_solver* s) {
  if (!s) return;
  (void)hipSetDevice(s->device);
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  delete s;
}

void* midagma_stream(midagma_solver* s) { return s ? reinterpret_cast<void*>(s->stream) : nullptr; }
int64_t midagma_padded_dim(const midagma_solver* s) { return s ? s->D : 0; }

int midagma_set_cov(midagma_solver* s, const double* cov, int64_t ld) {
  if (!s || !cov || ld < s->d) return fail(s, MIDAGMA_E_ARG, "set_cov: bad arguments");
  if (!all_finite(cov, s->d, s->d, ld)) return fail(s, MIDAGMA_E_ARG, std::string("set_cov: ") + kNonFinite);
  return guarded(s, [&] {
    s->upload_matrix(s->cov, cov, ld);
    HIP_TRY(hipStreamSynchronize(s->stream));
    s->has_cov = true;
    return MIDAGMA_OK;
  });
}

int midagma_set_masks(midagma_solver* s, const double* mask_inc, const double* mask_exc) {
  if (!s) return fail(s, MIDAGMA_E_ARG, "set_masks: null solver");
  return guarded(s, [&] {
    const size_t DD = (size_t)s->D * s->D;
    const bool inc = mask_inc != nullptr, exc = mask_exc != nullptr;
    if (inc) {
      s->minc.alloc(DD);
      HIP_TRY(hipMemsetAsync(s->minc.p, 0, DD * sizeof(double), s->stream));
      s->upload_matrix(s->minc, mask_inc, s->d);
    }
    if (exc) {
      s->mexc.alloc(DD);
      HIP_TRY(hipMemsetAsync(s->mexc.p, 0, DD * sizeof(double), s->stream));
      s->upload_matrix(s->mexc, mask_exc, s->d);
    }
    HIP_TRY(hipStreamSynchronize(s->stream));
    const double* pi = inc ? s->minc.p : nullptr;
    const double* pe = exc ? s->mexc.p : nullptr;
    if (pi != s->cap_minc || pe != s->cap_mexc) s->graphs_valid = false;  // captured pointers changed
    s->cap_minc = pi;
    s->cap_mexc = pe;
    s->has_inc = inc;
    s->has_exc = exc;
    return MIDAGMA_OK;
  });
}

int midagma_set_data(midagma_solver* s, const double* X, int64_t n_local, int64_t n_global, int on_device) {
  if (!s || !X || n_local < 1 || n_global < n_local || s->mode != MIDAGMA_MODE_DATA)
    return fail(s, MIDAGMA_E_ARG, "set_data: bad arguments (data mode only)");
  if (!on_device && !all_finite(X, n_local, s->d, s->d))
    return fail(s, MIDAGMA_E_ARG, std::string("set_data: ") + kNonFinite);
  return guarded(s, [&] {
    const int64_t D = s->D;
    s->n_local = n_local;
    s->n_global = n_global;
    s->n_pad = (n_local + 127) / 128 * 128;
    const size_t nx = (size_t)s->n_pad * D;
    // experiments build: MIDAGMA_EXP_PREPAD_MB of device memory allocated (and kept) before X, to
    // move X, X^T and Y elsewhere (the X^T Y GEMM's fetched bytes against placement)
    if (const long pad = knob("MIDAGMA_EXP_PREPAD_MB", 0); pad > 0 && !s->prepad.p)
      s->prepad.alloc((size_t)pad << 17);
    s->X.alloc(nx);
    // logistic with few 128-tiles: the sigmoid GEMM in two serial K halves when its last round of
    // tiles would be at most half full (n = 1e4, d = 1000: 632 tiles for 512 resident slots)
    const int64_t sig_tiles = (s->n_pad / 128) * (D / 128);
    const int sig_rule = (int)knob("MIDAGMA_EXP_SIG_SPLIT", 1);
    const bool sig_ok = s->loss == MIDAGMA_LOSS_LOGISTIC && D % 128 == 0 && sig_tiles % 8 == 0;
    s->sig_split = sig_ok && sig_rule > 0 && sig_tiles < 2048 && sig_tiles % 512 != 0 && sig_tiles % 512 <= 256 ? 2 : 1;
    if (s->sig_split_force == 1) s->sig_split = 1;  // midagma_debug_sig_split (tests)
    if (s->sig_split_force == 2 && sig_ok) s->sig_split = 2;
    if (s->sig_split == 2) {  // the output, the first halves' partial, then one flag word per tile
      s->Y.alloc(2 * nx + (size_t)(sig_tiles + 1) / 2);
      HIP_TRY(hipMemsetAsync(s->Y.p + 2 * nx, 0, (size_t)(sig_tiles + 1) / 2 * sizeof(double), s->stream));
    } else {
      // experiments build: Y placed MIDAGMA_EXP_Y_OFFSET bytes into its allocation (L2 set
      // aliasing between X and Y in the X^T Y GEMM)
      s->Y.alloc_shifted(nx, (size_t)knob("MIDAGMA_EXP_Y_OFFSET", 0) / sizeof(double));
    }
    HIP_TRY(hipMemsetAsync(s->X.p, 0, nx * sizeof(double), s->stream));
    HIP_TRY(hipMemcpy2DAsync(s->X.p, D * sizeof(double), X, s->d * sizeof(double), s->d * sizeof(double), n_local,
                             on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s->stream));
    if (on_device) {  // the host path checked before the copy
      int* flag = reinterpret_cast<int*>(s->partials.p);
      launch_any_nonfinite(s->X.p, (int64_t)nx, flag, s->stream);
      int bad = 0;
      HIP_TRY(hipMemcpyAsync(&bad, flag, sizeof(int), hipMemcpyDeviceToHost, s->stream));
      HIP_TRY(hipStreamSynchronize(s->stream));
      if (bad) throw std::invalid_argument(std::string("set_data: ") + kNonFinite);
    }
    size_t mem_free = 0, mem_total = 0;
    HIP_TRY(hipMemGetInfo(&mem_free, &mem_total));
    // (the 128-tile GEMM only: D % 128 == 0; smaller problems are not worth the copy)
    s->use_xt = getenv("MIDAGMA_NO_XT") == nullptr && D % 128 == 0 &&
                mem_free > nx * sizeof(double) + (size_t(2) << 30);
    if (s->use_xt) {
      s->XT.alloc(nx);
      launch_transpose(s->X.p, D, s->n_pad, D, s->XT.p, s->n_pad, s->stream);
    } else {
      s->XT.release();
    }
    if (s->loss == MIDAGMA_LOSS_L2 && (D % 128 == 0 || s->w32))  // (float32 W: I - W from build_at)
      s->IW.alloc((size_t)D * D);
    else
      s->IW.release();
    // split-K over the rows so the X^T Y GEMM fills the chip: (D/64)^2 tiles x split >= ~1024 workgroups
    const int64_t tiles = (D % 128 == 0) ? (D / 128) * (D / 128) : (D / 64) * (D / 64);
    const int64_t ktiles = s->n_pad / 64;
    int split = (int)std::max<int64_t>(1, std::min<int64_t>(ktiles / 8, (1024 + tiles - 1) / tiles));
    s->split = std::min(split, 32);
    if (knob_set("MIDAGMA_EXP_DATA_SPLIT")) s->split = (int)knob("MIDAGMA_EXP_DATA_SPLIT", s->split);
    if (s->split > 1) s->Zparts.alloc((size_t)s->split * D * D);
    s->loss_part_count = (s->n_pad / 64) * (D / 64);
    // small shards run the cov-mode slot structure: the warm-started fast blocked inverse in
    // sequence with the GEMMs (hand-backs and checkpoint slots on the pivoted path).  Forked beside
    // GEMMs that fill the chip, the pivoted inverse's 20-odd dependent launches wait for CU slots
    // and end after the GEMMs (logistic d=1000, n=1e4: 1.01 ms per slot for 0.70 ms of GEMMs);
    // large shards keep the fork, which hides it (MIDAGMA_EXP_DATA_FAST_ROWS: the row bound)
    static const int64_t fast_rows = knob("MIDAGMA_EXP_DATA_FAST_ROWS", 16384);
    const int b2 = binv_block(D);
    const int B2_new = (b2 > 0 && s->n_pad <= fast_rows && s->Malt.p) ? b2 : 0;
    if (B2_new != s->B2) s->graphs_valid = false;
    s->B2 = B2_new;
    if (s->loss == MIDAGMA_LOSS_LOGISTIC) {
      s->loss_part.alloc(s->loss_part_count);
      HIP_TRY(hipMemsetAsync(s->loss_part.p, 0, s->loss_part_count * sizeof(double), s->stream));
    }
    HIP_TRY(hipStreamSynchronize(s->stream));
    s->has_data = true;
    s->graphs_valid = false;
    return MIDAGMA_OK;
  });
}

int midagma_data_gram(midagma_solver* s) {
  if (!s || !s->has_data) return fail(s, MIDAGMA_E_STATE, "data_gram: set_data first");
  return guarded(s, [&] {
    const int64_t D = s->D;
    if (s->split == 1)
      launch_gemm(D, D, s->n_pad, s->X.p, D, true, s->X.p, D, B_PLAIN, s->zbuf, D, EPI_STORE, 1, 0, nullptr, 0, 0,
                  nullptr, s->stream);
    else {
      launch_gemm(D, D, s->n_pad, s->X.p, D, true, s->X.p, D, B_PLAIN, s->Zparts.p, D, EPI_STORE, s->split, D * D,
                  nullptr, 0, 0, nullptr, s->stream);
      launch_sum_slices(s->Zparts.p, s->split, D * D, D * D, s->zbuf, nullptr, s->stream);
    }
    HIP_TRY(hipStreamSynchronize(s->stream));
    return MIDAGMA_OK;
  });
}

int midagma_cov_from_zbuf(midagma_solver* s, double n) {
  if (!s || !(n > 0)) return fail(s, MIDAGMA_E_ARG, "cov_from_zbuf: n must be > 0");
  return guarded(s, [&] {
    // cov = (X^T X) / float(n), a division as in linear.py:428
    const int64_t DD = s->D * s->D;
    hipLaunchKernelGGL(div_kernel, dim3(4096), dim3(NTHREADS), 0, s->stream, s->zbuf, n, s->cov.p, DD);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(s->stream));
    s->has_cov = true;
    return MIDAGMA_OK;
  });
}

int midagma_get_cov(midagma_solver* s, double* out, int64_t ld) {
  if (!s || !out || ld < s->d) return fail(s, MIDAGMA_E_ARG, "get_cov: bad arguments");
  if (!s->has_cov) return fail(s, MIDAGMA_E_STATE, "get_cov: no cov (set_cov or cov_from_zbuf first)");
  return guarded(s, [&] {
    HIP_TRY(hipMemcpy2DAsync(out, ld * sizeof(double), s->cov.p, s->D * sizeof(double), s->d * sizeof(double), s->d,
                             hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return MIDAGMA_OK;
  });
}

// ABI 7: fit()'s data preparation on device memory (linear.py:406-428), csrc/gram.hip.
int midagma_colsum_dev(const double* X, int64_t n, int64_t d, int64_t ldx, double* out_dev, void* stream) {
  if (n < 0 || d < 1 || ldx < d || !out_dev || (n > 0 && !X))
    return fail(nullptr, MIDAGMA_E_ARG, "colsum_dev: bad arguments");
  return guarded(nullptr, [&] {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    DevBuf part;
    part.alloc((size_t)colsum_parts(n) * d);
    launch_colsum(X, n, d, ldx, part.p, out_dev, st);
    HIP_TRY(hipStreamSynchronize(st));  // the partials are freed on return
    return MIDAGMA_OK;
  });
}

int midagma_center_dev(double* X, int64_t n, int64_t d, int64_t ldx, const double* colsum_dev, double nrows,
                       void* stream) {
  if (n < 0 || d < 1 || ldx < d || !colsum_dev || (n > 0 && !X) || !(nrows > 0))
    return fail(nullptr, MIDAGMA_E_ARG, "center_dev: bad arguments");
  return guarded(nullptr, [&] {
    launch_center(X, n, d, ldx, colsum_dev, nrows, reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

int midagma_gram(const double* X, int64_t n, int64_t d, int64_t ldx, int on_device, double* G_dev, int64_t ldg,
                 void* stream) {
  if (n < 0 || d < 1 || ldx < d || !G_dev || ldg < d || (n > 0 && !X))
    return fail(nullptr, MIDAGMA_E_ARG, "gram: bad arguments");
  return guarded(nullptr, [&] {
    setup_attributes_once();
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    static const int64_t chunk_rows = [] {
      const char* e = getenv("MIDAGMA_GRAM_CHUNK_ROWS");
      return e ? std::max<int64_t>(256, atoll(e)) : int64_t(262144);
    }();
    const GramPlan p = gram_plan(n, d, chunk_rows);
    const int64_t D = p.D, DD = D * D;
    DevBuf S, Z, fl;
    S.alloc((size_t)p.chunk * D);
    Z.alloc((size_t)(p.split + 2) * DD);  // [0] the running sum, [1..split] a chunk's slices, [split+1] the new sum
    fl.alloc(1);
    int* flag = reinterpret_cast<int*>(fl.p);
    HIP_TRY(hipMemsetAsync(flag, 0, sizeof(int), st));
    HIP_TRY(hipMemsetAsync(Z.p, 0, DD * sizeof(double), st));
    if (!on_device) HIP_TRY(hipMemsetAsync(S.p, 0, (size_t)p.chunk * D * sizeof(double), st));
    for (int64_t c = 0; c < p.nchunks; ++c) {
      const int64_t r0 = c * p.chunk, rows = std::min(p.chunk, n - r0);
      const int64_t rpad = (rows + 255) / 256 * 256;
      if (on_device) {
        launch_stage_rows(X + r0 * ldx, ldx, rows, d, S.p, D, rpad, flag, st);
      } else {
        if (rows < rpad) HIP_TRY(hipMemsetAsync(S.p + rows * D, 0, (rpad - rows) * D * sizeof(double), st));
        HIP_TRY(hipMemcpy2DAsync(S.p, D * sizeof(double), X + r0 * ldx, ldx * sizeof(double), d * sizeof(double),
                                 rows, hipMemcpyHostToDevice, st));
        launch_nonfinite_or(S.p, rows, d, D, flag, st);
      }
      launch_gemm(D, D, rpad, S.p, D, true, S.p, D, B_PLAIN, Z.p + DD, D, EPI_STORE, p.split, DD, nullptr, 0, 0,
                  nullptr, st);
      launch_sum_slices(Z.p, p.split + 1, DD, DD, Z.p + (p.split + 1) * DD, nullptr, st);
      HIP_TRY(hipMemcpyAsync(Z.p, Z.p + (p.split + 1) * DD, DD * sizeof(double), hipMemcpyDeviceToDevice, st));
    }
    HIP_TRY(hipMemcpy2DAsync(G_dev, ldg * sizeof(double), Z.p, D * sizeof(double), d * sizeof(double), d,
                             hipMemcpyDeviceToDevice, st));
    int bad = 0;
    HIP_TRY(hipMemcpyAsync(&bad, flag, sizeof(int), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (bad) throw std::invalid_argument(std::string("gram: ") + kNonFinite);
    return MIDAGMA_OK;
  });
}

int midagma_set_cov_dev(midagma_solver* s, const double* G_dev, int64_t ldg, double divisor) {
  if (!s || !G_dev || ldg < s->d || !(divisor > 0)) return fail(s, MIDAGMA_E_ARG, "set_cov_dev: bad arguments");
  return guarded(s, [&] {
    // cov = (X^T X) / float(n), a division as in linear.py:428 (the caller all-reduced the Gram)
    int* flag = reinterpret_cast<int*>(s->partials.p);
    HIP_TRY(hipMemsetAsync(flag, 0, sizeof(int), s->stream));
    launch_div_block(G_dev, ldg, divisor, s->d, s->cov.p, s->D, flag, s->stream);
    int bad = 0;
    HIP_TRY(hipMemcpyAsync(&bad, flag, sizeof(int), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (bad) throw std::invalid_argument(std::string("set_cov_dev: ") + kNonFinite);
    s->has_cov = true;
    return MIDAGMA_OK;
  });
}

int midagma_comm_unique_id(void* out, int64_t cap) {
  if (!out || cap < 128) return fail(nullptr, MIDAGMA_E_ARG, "comm_unique_id: needs a 128-byte buffer");
  return guarded(nullptr, [&] { return comm_unique_id(out); });
}

int midagma_comm_init(midagma_solver* s, const void* id, int64_t id_len, int nranks, int rank) {
  if (!s || !id || id_len != 128 || nranks < 1 || rank < 0 || rank >= nranks || s->mode != MIDAGMA_MODE_DATA)
    return fail(s, MIDAGMA_E_ARG, "comm_init: bad arguments (data mode, a 128-byte unique id, 0 <= rank < nranks)");
  return guarded(s, [&] {
    HIP_TRY(hipStreamSynchronize(s->stream));
    comm_destroy(s->comm);
    s->comm = nullptr;
    s->comm = comm_create(id, nranks, rank);
    s->comm_ranks = nranks;
    s->agree.alloc(8);
    if (!s->h_agree) HIP_TRY(hipHostMalloc(&s->h_agree, 8 * sizeof(double), hipHostMallocDefault));
    s->graphs_valid = false;  // the slot graphs now carry the all-reduce
    return MIDAGMA_OK;
  });
}

int midagma_comm_ranks(const midagma_solver* s) { return s ? (s->comm ? s->comm_ranks : 0) : 0; }

int midagma_comm_allreduce_zbuf(midagma_solver* s) {
  if (!s || !s->comm) return fail(s, MIDAGMA_E_STATE, "comm_allreduce_zbuf: comm_init first");
  return guarded(s, [&] {
    comm_allreduce(s->comm, s->zbuf, (size_t)(s->D * s->D + 64), false, s->stream);
    return MIDAGMA_OK;
  });
}

int64_t midagma_zbuf_len(const midagma_solver* s) { return s ? s->D * s->D + 64 : 0; }

int midagma_bind_zbuf(midagma_solver* s, void* dev_ptr, int64_t len) {
  if (!s || len < s->D * s->D + 64) return fail(s, MIDAGMA_E_ARG, "bind_zbuf: buffer too small");
  return guarded(s, [&] {
    s->zbuf = dev_ptr ? static_cast<double*>(dev_ptr) : s->zown.p;
    s->graphs_valid = false;
    return MIDAGMA_OK;
  });
}

int midagma_minimize(midagma_solver* s, double* W, double mu, int64_t max_iter, double s_dom, double lr, double tol,
                     double beta1, double beta2, double lambda1, int64_t checkpoint, midagma_result* res) {
  if (!s || !W) return fail(s, MIDAGMA_E_ARG, "minimize: null argument");
  if (!all_finite(W, s->d, s->d, s->d)) return fail(s, MIDAGMA_E_ARG, std::string("minimize: ") + kNonFinite);
  int rc = guarded(s, [&] {
    s->begin(W, mu, max_iter, s_dom, lr, tol, beta1, beta2, lambda1, checkpoint);
    s->run_loop(max_iter, checkpoint);
    s->finish(W, res);
    return MIDAGMA_OK;
  });
  return singular_or_nonfinite(s, rc, res, W);
}

int midagma_begin(midagma_solver* s, const double* W, double mu, int64_t max_iter, double s_dom, double lr,
                  double tol, double beta1, double beta2, double lambda1, int64_t checkpoint) {
  if (!s || !W) return fail(s, MIDAGMA_E_ARG, "begin: null argument");
  if (!all_finite(W, s->d, s->d, s->d)) return fail(s, MIDAGMA_E_ARG, std::string("begin: ") + kNonFinite);
  return guarded(s, [&] {
    s->begin(W, mu, max_iter, s_dom, lr, tol, beta1, beta2, lambda1, checkpoint);
    s->ensure_graphs();
    return MIDAGMA_OK;
  });
}

int midagma_run_slots(midagma_solver* s, int64_t n) {
  if (!s || !s->begun || n < 0) return fail(s, MIDAGMA_E_STATE, "run_slots: call begin first");
  return guarded(s, [&] {
    if (s->blocked()) {
      s->drive_blocked(n);
      return MIDAGMA_OK;
    }
    if (s->small_on()) {
      s->drive_small(n);
      return MIDAGMA_OK;
    }
    for (int64_t i = 0; i < n; ++i) HIP_TRY(hipGraphLaunch(s->g_full, s->stream));
    return MIDAGMA_OK;
  });
}

int midagma_sync(midagma_solver* s) {
  if (!s) return fail(s, MIDAGMA_E_ARG, "null solver");
  return guarded(s, [&] {
    HIP_TRY(hipStreamSynchronize(s->stream));
    return MIDAGMA_OK;
  });
}

int midagma_profile_parts(midagma_solver* s, int reps, double* ms_out) {
  if (!s || !s->begun || reps < 1 || !ms_out) return fail(s, MIDAGMA_E_STATE, "profile_parts: call begin first");
  return guarded(s, [&] {
    hipEvent_t a, b;
    HIP_TRY(hipEventCreate(&a));
    HIP_TRY(hipEventCreate(&b));
    auto timed = [&](auto&& body) {
      HIP_TRY(hipEventRecord(a, s->stream));
      for (int r = 0; r < reps; ++r) body();
      HIP_TRY(hipEventRecord(b, s->stream));
      HIP_TRY(hipEventSynchronize(b));
      float ms = 0.f;
      HIP_TRY(hipEventElapsedTime(&ms, a, b));
      return (double)ms / reps;
    };
    const int64_t D = s->D;
    // [0] build (sI - W o W)^T   [1] GJ inverse   [2] score GEMM(s)   [3] whole slot (graph)
    // data mode: [4] Y = X (I - W) GEMM   [5] Z = X^T Y GEMM (+ slice sum)
    ms_out[0] = timed([&] { launch_build_at(s->W.p, D, true, s->Mt.p, D, s->d, 0.0, s->d_params, s->d_state,
                                            s->stream, s->IW.p); });
    ms_out[1] = timed([&] { launch_gj_inverse(s->Mt.p, D, D, s->gj(), s->d_state, s->stream); });
    if (s->mode == MIDAGMA_MODE_COV) {
      ms_out[2] = timed([&] { s->enqueue_score_cov(s->zbuf, s->d_state, true); });
      ms_out[4] = ms_out[5] = 0.0;
    } else {
      ms_out[2] = timed([&] { s->enqueue_data_partial(s->W.p, s->d_state, s->IW.p); });
      ms_out[4] = timed([&] {
        if (s->loss == MIDAGMA_LOSS_L2)
          launch_gemm(s->n_pad, D, s->Kd(), s->xw_a(), s->xw_lda(), s->use_xt, s->IW.p ? s->IW.p : s->W.p, D,
                      s->IW.p ? B_PLAIN : B_IMINUS, s->Y.p, D, EPI_STORE, 1, 0, nullptr, 0, 0, s->d_state, s->stream);
        else
          launch_gemm(s->n_pad, D, s->Kd(), s->xw_a(), s->xw_lda(), s->use_xt, s->W.p, D, B_PLAIN, s->Y.p, D, EPI_SIGMOID,
                      s->sig_split, s->sig_split > 1 ? s->n_pad * D : 0, s->loss_part.p, s->n_local, s->d,
                      s->d_state, s->stream);
      });
      ms_out[5] = timed([&] {
        if (s->split == 1)
          launch_gemm(D, D, s->n_pad, s->X.p, D, true, s->Y.p, D, B_PLAIN, s->zbuf, D, EPI_STORE, 1, 0, nullptr, 0, 0,
                      s->d_state, s->stream);
        else {
          launch_gemm(D, D, s->n_pad, s->X.p, D, true, s->Y.p, D, B_PLAIN, s->Zparts.p, D, EPI_STORE, s->split,
                      D * D, nullptr, 0, 0, s->d_state, s->stream);
          launch_sum_slices(s->Zparts.p, s->split, D * D, D * D, s->zbuf, s->d_state, s->stream);
        }
      });
    }
    ms_out[3] = timed([&] { HIP_TRY(hipGraphLaunch(s->g_full, s->stream)); });
    ms_out[6] = ms_out[7] = 0.0;
    if (s->blocked()) {
      // [6] build + fast blocked inverse, less [0]   [7] whole fast slot (graph).  Both need a
      // warm start and no pending checkpoint: one slow slot first.
      HIP_TRY(hipGraphLaunch(s->g_full, s->stream));
      ms_out[6] = timed([&] { s->enqueue_build_inverse(/*fast=*/true, 2); }) - ms_out[0];
      ms_out[7] = timed([&] { HIP_TRY(hipGraphLaunch(s->g_fast, s->stream)); });
      State st{};
      HIP_TRY(hipMemcpy(&st, s->d_state, sizeof(State), hipMemcpyDeviceToHost));
      if (st.status == ST_NEED_GJ) {  // the fast path did not run: report it, leave a clean state
        ms_out[6] = ms_out[7] = -1.0;
        static const int32_t running = ST_RUNNING;
        HIP_TRY(hipMemcpy(&s->d_state->status, &running, sizeof(int32_t), hipMemcpyHostToDevice));
        s->fast_ready = false;
      }
    }
    HIP_TRY(hipEventDestroy(a));
    HIP_TRY(hipEventDestroy(b));
    return MIDAGMA_OK;
  });
}

int midagma_step_partial(midagma_solver* s) {
  if (!s || !s->begun) return fail(s, MIDAGMA_E_STATE, "step_partial: call begin first");
  return guarded(s, [&] {
    HIP_TRY(hipGraphLaunch(s->g_part1, s->stream));
    return MIDAGMA_OK;
  });
}

int midagma_step_finish(midagma_solver* s) {
  if (!s || !s->begun) return fail(s, MIDAGMA_E_STATE, "step_finish: call begin first");
  return guarded(s, [&] {
    HIP_TRY(hipGraphLaunch(s->g_part2, s->stream));
    return MIDAGMA_OK;
  });
}

int midagma_poll(midagma_solver* s, midagma_result* res) {
  if (!s) return fail(s, MIDAGMA_E_ARG, "null solver");
  return guarded(s, [&] {
    HIP_TRY(hipMemcpyAsync(&s->h_state[1], s->d_state, sizeof(State), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    s->check_handoff(s->h_state[1]);
    midagma_solver::fill_result(s->h_state[1], res);
    return MIDAGMA_OK;
  });
}

int midagma_end(midagma_solver* s, double* W, midagma_result* res) {
  if (!s || !W || !s->begun) return fail(s, MIDAGMA_E_STATE, "end: call begin first");
  int rc = guarded(s, [&] {
    s->finish(W, res);
    return MIDAGMA_OK;
  });
  return singular_or_nonfinite(s, rc, res, W);
}

int midagma_set_w_float32(midagma_solver* s, int float32) {
  if (!s) return fail(s, MIDAGMA_E_ARG, "null solver");
  return guarded(s, [&] {
    const bool on = float32 != 0;
    if (on != s->w32) s->graphs_valid = false;  // the float32 slots carry numpy's L1 sum
    if (on && !s->l1w.p) s->l1w.alloc((size_t)(1 + (np_l1_chunks(s->d) + 1) / 2));
    if (on && (s->mode == MIDAGMA_MODE_COV || s->loss == MIDAGMA_LOSS_L2) && !s->IW.p) {
      // the score GEMM's I - W (float32 diagonal) comes from build_at, not the GEMM's staging
      s->IW.alloc((size_t)s->D * s->D);
      HIP_TRY(hipMemsetAsync(s->IW.p, 0, (size_t)s->D * s->D * sizeof(double), s->stream));
      s->graphs_valid = false;
    }
    s->w32 = on;
    return MIDAGMA_OK;
  });
}

// Test hook (not in the public header): choose the logistic sigmoid GEMM's form for the next
// set_data (0: the size rule, 1: the one-pass kernel, 2: the serial K split wherever the shape
// allows it; -1: no change).  Returns the form the current data uses (1 or 2).
extern "C" int midagma_debug_sig_split(midagma_solver* s, int mode) {
  if (!s || mode < -1 || mode > 2) return -1;
  if (mode >= 0) s->sig_split_force = mode;
  return s->sig_split;
}

// Test hooks (not in the public header) for the hand-back path of the blocked inverse:
// spoil_warm zeroes the stored diagonal-block inverses of the last two slots, so the next fast
// slot's warm start is 0, its residual I, and its first product-form pass hands the slot back
// (ST_NEED_GJ) while the rest of the slot (in data mode: the score GEMMs beside the forked
// inverse) is running; handbacks counts the hand-backs the scheduler has re-run.
extern "C" int midagma_debug_spoil_warm(midagma_solver* s) {
  if (!s || !s->blocked()) return -1;
  return guarded(s, [&] {
    for (DevBuf* b : {&s->Pst2, &s->Pst2b})
      if (b->p) HIP_TRY(hipMemsetAsync(b->p, 0, b->n * sizeof(double), s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return MIDAGMA_OK;
  });
}
extern "C" int64_t midagma_debug_handbacks(const midagma_solver* s) { return s ? s->handback_count : -1; }
// Test hook (not in the public header): the Noda steps a fast cov slot's TCC chain enqueues before
// it hands back (0: the whole gated chain on every slot; < 0: no change).  Returns the old value.
extern "C" int midagma_debug_tcc_fast_steps(midagma_solver* s, int steps) {
  if (!s) return -1;
  const int old = s->tcc_fast_steps;
  if (steps >= 0 && steps != old) {
    s->tcc_fast_steps = steps;
    s->graphs_valid = false;
  }
  return old;
}

// Test hook (not in the public header): the TCC fixed-shift stage on (1) or off (0); < 0 leaves
// it.  Returns the old setting.
extern "C" int midagma_debug_tcc_fix(midagma_solver* s, int on) {
  if (!s) return -1;
  const int old = s->tcc_fix != 0 ? 1 : 0;
  if (on >= 0 && (on != 0 ? 1 : 0) != old) {
    s->tcc_fix = on != 0 ? 1 : 0;
    s->cw.fix = s->tcc_fix;
    s->graphs_valid = false;
  }
  return old;
}

// Test hook (not in the public header): the TCC fixed-stage inverse's fast blocks (D2 >= 2048) on (1)
// or off (0) for the next set_trek_tcc; < 0 leaves it.  Returns the old setting.
extern "C" int midagma_debug_tcc_fastblk(midagma_solver* s, int on) {
  if (!s) return -1;
  const int old = s->tcc_fastblk ? 1 : 0;
  if (on >= 0) s->tcc_fastblk = on != 0;
  return old;
}

// Test hook (not in the public header): build_at folded into the previous slot's update
// (at_fold, MIDAGMA_EXP_AT_FOLD) on (1) or off (0); < 0 leaves it.  Returns the old setting, or -1
// (no handle / the fold cannot apply: not a blocked cov solver).
extern "C" int midagma_debug_at_fold(midagma_solver* s, int on) {
  if (!s || s->begun) return -1;
  const int old = s->at_fold ? 1 : 0;
  if (on < 0 || (on != 0) == s->at_fold) return old;
  if (on && !(s->mode == MIDAGMA_MODE_COV && s->blocked())) return -1;
  return guarded(s, [&] {
    if (on && !s->A0.p) s->A0.alloc(s->D * s->D);
    s->at_fold = on != 0;
    s->graphs_valid = false;
    return old;
  });
}

// Diagnostics of the fast blocked inverse (not in the public header): per outer block g,
// out[g*(NM_PASSES+2) + 0] = done word, out[... + 1 + p] = ||Q_p||_inf of pass p (stale for
// passes that did not run in the last slot).
extern "C" int midagma_debug_blocked(midagma_solver* s, double* out, int64_t cap) {
  if (!s || !s->blocked()) return 0;
  const int64_t K2 = s->D / s->B2, per = NM_PASSES + 2;
  if (cap < K2 * per) return -1;
  std::vector<double> part((size_t)K2 * (NM_PASSES + 1) * PART_STRIDE);
  std::vector<int> done(K2);
  if (hipMemcpy(part.data(), s->nmPart.p, part.size() * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (hipMemcpy(done.data(), s->nmDone.p, K2 * sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  const int B2 = s->B2, NT = B2 / 16;
  for (int64_t g = 0; g < K2; ++g) {
    out[g * per] = done[g];
    for (int p = 0; p <= NM_PASSES; ++p) {
      const double* rp = part.data() + ((size_t)g * (NM_PASSES + 1) + p) * PART_STRIDE;
      double m = 0.0;
      for (int r = 0; r < B2; ++r) {
        double acc = 0.0;
        for (int t = 0; t < NT; ++t) acc += rp[r * NT + t];
        m = std::max(m, acc);
      }
      out[g * per + 1 + p] = m;
    }
  }
  return (int)K2;
}

int64_t midagma_checkpoints(midagma_solver* s, midagma_ckpt* out, int64_t cap) {
  if (!s || !s->d_ckpt) return 0;
  int64_t n = 0;
  int rc = guarded(s, [&] {
    State st{};
    HIP_TRY(hipMemcpy(&st, s->d_state, sizeof(State), hipMemcpyDeviceToHost));
    n = std::min<int64_t>(std::min<int64_t>(st.n_ckpt, s->ckpt_cap), cap);
    static_assert(sizeof(midagma_ckpt) == sizeof(CkptRec), "ckpt layout");
    if (n > 0 && out) HIP_TRY(hipMemcpy(out, s->d_ckpt, n * sizeof(CkptRec), hipMemcpyDeviceToHost));
    return MIDAGMA_OK;
  });
  return rc == MIDAGMA_OK ? n : rc;
}

int midagma_set_trek(midagma_solver* s, int seq, int agg, int mode, double weight, double eps_inv, int64_t K,
                     const int64_t* pairs, int64_t m) {
  if (!s || (m > 0 && !pairs) || m < 0) return fail(s, MIDAGMA_E_ARG, "set_trek: bad arguments");
  return guarded(s, [&] {
    s->set_trek(seq, agg, mode, weight, eps_inv, K, pairs, m);
    HIP_TRY(hipStreamSynchronize(s->stream));
    return MIDAGMA_OK;
  });
}

int midagma_set_trek_tcc(midagma_solver* s, int mode, double weight, double w, double eps, const int64_t* pairs,
                         int64_t m) {
  if (!s || (m > 0 && !pairs) || m < 0) return fail(s, MIDAGMA_E_ARG, "set_trek_tcc: bad arguments");
  return guarded(s, [&] {
    s->set_trek_tcc(mode, weight, w, eps, pairs, m);
    HIP_TRY(hipStreamSynchronize(s->stream));
    return MIDAGMA_OK;
  });
}

int midagma_trek(midagma_solver* s, const double* W, double* value, double* G) {
  if (!s || !W || !value) return fail(s, MIDAGMA_E_ARG, "trek: null argument");
  return guarded(s, [&] {
    const int64_t D = s->D, d = s->d, DD = D * D;
    if (!s->trek_on) {  // trek_value_grad: (0, zeros) when disabled (notreks.py)
      *value = 0.0;
      if (G) std::fill(G, G + d * d, 0.0);
      return MIDAGMA_OK;
    }
    s->scratch.alloc(DD);
    HIP_TRY(hipMemsetAsync(s->scratch.p, 0, DD * sizeof(double), s->stream));
    s->upload_matrix(s->scratch, W, d);
    const double* scal;
    if (s->trek_tcc) {
      TccCfg c = s->ccfg;
      c.weight = 1.0;  // the bare gradient, as trek_value_grad returns it
      launch_trek_tcc(s->scratch.p, d, D, c, s->cw, s->d_state_probe, s->Gtrek.p, s->stream);
      scal = s->cw.scal;
    } else {
      TrekCfg c = s->tcfg;
      c.weight = 1.0;
      launch_trek_pst(s->scratch.p, d, D, c, s->tw, s->d_state_probe, s->Gtrek.p, s->stream);
      scal = s->tw.scal;
    }
    HIP_TRY(hipMemcpyAsync(value, scal, sizeof(double), hipMemcpyDeviceToHost, s->stream));
    if (G) {
      if (s->tcfg.mode == 2) {
        HIP_TRY(hipMemcpy2DAsync(G, d * sizeof(double), s->Gtrek.p, D * sizeof(double), d * sizeof(double), d,
                                 hipMemcpyDeviceToHost, s->stream));
      } else {
        std::fill(G, G + d * d, 0.0);
      }
    }
    HIP_TRY(hipStreamSynchronize(s->stream));
    return MIDAGMA_OK;
  });
}

int midagma_h(midagma_solver* s, const double* W, double s_dom, double* h, double* G) {
  if (!s || !W || !h) return fail(s, MIDAGMA_E_ARG, "h: null argument");
  if (!all_finite(W, s->d, s->d, s->d)) return fail(s, MIDAGMA_E_ARG, std::string("h: ") + kNonFinite);
  return guarded(s, [&] {
    const int64_t D = s->D, d = s->d, DD = D * D;
    s->scratch.alloc(DD);
    HIP_TRY(hipMemsetAsync(s->scratch.p, 0, DD * sizeof(double), s->stream));
    s->upload_matrix(s->scratch, W, d);
    DevBuf work;
    work.alloc(DD);
    launch_build_at(s->scratch.p, D, true, work.p, D, d, s_dom, nullptr, nullptr, s->stream);
    GJWork gw = s->gj();
    gw.Pstore = nullptr;
    launch_gj_inverse(work.p, D, D, gw, nullptr, s->stream);
    std::vector<double> pl(D);
    HIP_TRY(hipMemcpyAsync(pl.data(), s->pivlog.p, D * sizeof(double), hipMemcpyDeviceToHost, s->stream));
    if (G) {
      s->Gtmp.alloc((size_t)d * d);
      launch_h_grad(s->scratch.p, work.p, s->Gtmp.p, d, D, s->stream);
      HIP_TRY(hipMemcpyAsync(G, s->Gtmp.p, (size_t)d * d * sizeof(double), hipMemcpyDeviceToHost, s->stream));
    }
    HIP_TRY(hipStreamSynchronize(s->stream));
    work.release();
    double ld = 0.0;
    for (int64_t i = 0; i < d; ++i) ld += pl[i];
    *h = -ld + (double)d * std::log(s_dom);
    return MIDAGMA_OK;
  });
}

static void host_trace_l1(midagma_solver* s, const double* Wd, const double* Z, double* sd, double* l1) {
  launch_trace_l1(Wd, Z, s->partials.p, s->d, s->D, s->stream);
  std::vector<double> part(2 * NRED);
  HIP_TRY(hipMemcpyAsync(part.data(), s->partials.p, part.size() * sizeof(double), hipMemcpyDeviceToHost,
                         s->stream));
  HIP_TRY(hipStreamSynchronize(s->stream));
  double a = 0.0, b = 0.0;
  for (int i = 0; i < NRED; ++i) {
    a += part[2 * i];
    b += part[2 * i + 1];
  }
  *sd = a;
  if (l1) *l1 = b;
}

int midagma_score(midagma_solver* s, const double* W, double* loss, double* G) {
  if (!s || !W || !loss) return fail(s, MIDAGMA_E_ARG, "score: null argument");
  if (s->mode != MIDAGMA_MODE_COV || !s->has_cov) return fail(s, MIDAGMA_E_STATE, "score: cov mode with set_cov");
  return guarded(s, [&] {
    const int64_t D = s->D, d = s->d, DD = D * D;
    s->scratch.alloc(DD);
    HIP_TRY(hipMemsetAsync(s->scratch.p, 0, DD * sizeof(double), s->stream));
    s->upload_matrix(s->scratch, W, d);
    DevBuf rhs;
    rhs.alloc(DD);
    s->enqueue_cov_gemm(s->cov.p, s->scratch.p, rhs.p, nullptr);  // rhs = cov @ (I - W)   (linear.py:85-86)
    double sd = 0;
    host_trace_l1(s, s->scratch.p, rhs.p, &sd, nullptr);
    *loss = 0.5 * sd;
    if (G) {
      s->Gtmp.alloc((size_t)d * d);
      launch_scale(rhs.p, -1.0, rhs.p, DD, s->stream);  // G_loss = -rhs
      s->download_matrix(G, rhs.p);
    }
    HIP_TRY(hipStreamSynchronize(s->stream));
    rhs.release();
    return MIDAGMA_OK;
  });
}

int midagma_score_partial(midagma_solver* s, const double* W) {
  if (!s || !W || s->mode != MIDAGMA_MODE_DATA || !s->has_data)
    return fail(s, MIDAGMA_E_STATE, "score_partial: data mode with set_data");
  return guarded(s, [&] {
    const int64_t DD = s->D * s->D;
    s->scratch.alloc(DD);
    HIP_TRY(hipMemsetAsync(s->scratch.p, 0, DD * sizeof(double), s->stream));
    s->upload_matrix(s->scratch, W, s->d);
    HIP_TRY(hipMemsetAsync(s->zbuf + DD, 0, 64 * sizeof(double), s->stream));
    // Force loss partials: pass no state (st == nullptr computes them unconditionally).
    s->enqueue_data_partial(s->scratch.p, nullptr);
    HIP_TRY(hipStreamSynchronize(s->stream));
    return MIDAGMA_OK;
  });
}

int midagma_score_finish(midagma_solver* s, double* loss, double* G) {
  if (!s || !loss || s->mode != MIDAGMA_MODE_DATA) return fail(s, MIDAGMA_E_STATE, "score_finish: data mode");
  return guarded(s, [&] {
    const int64_t D = s->D, d = s->d, DD = D * D;
    const double n = (double)s->n_global;
    if (s->loss == MIDAGMA_LOSS_L2) {
      // loss = 0.5 tr((I-W)^T cov (I-W)) with cov (I-W) = Z / n ; G = -Z / n
      double sd = 0;
      host_trace_l1(s, s->scratch.p, s->zbuf, &sd, nullptr);
      *loss = 0.5 * (sd / n);
      if (G) {
        std::vector<double> z((size_t)d * d);
        s->download_matrix(z.data(), s->zbuf);
        HIP_TRY(hipStreamSynchronize(s->stream));
        for (size_t i = 0; i < z.size(); ++i) G[i] = -(z[i] / n);
      }
    } else {
      double tail = 0;
      HIP_TRY(hipMemcpyAsync(&tail, s->zbuf + DD, sizeof(double), hipMemcpyDeviceToHost, s->stream));
      HIP_TRY(hipStreamSynchronize(s->stream));
      *loss = 1.0 / n * tail;
      if (G) {
        std::vector<double> z((size_t)d * d), c((size_t)d * d);
        s->download_matrix(z.data(), s->zbuf);
        s->download_matrix(c.data(), s->cov.p);
        HIP_TRY(hipStreamSynchronize(s->stream));
        for (size_t i = 0; i < z.size(); ++i) G[i] = (1.0 / n) * z[i] - c[i];
      }
    }
    return MIDAGMA_OK;
  });
}

}  // extern "C"

// ---- device-pointer log-det / inverse for torch (DagmaMLP.h_func) ------------
namespace {
struct LogdetWorkspace {
  int device = -1;
  int64_t D = 0;
  DevBuf A, P, R, C, piv;
};
std::mutex g_ws_mu;
std::vector<LogdetWorkspace*> g_ws;
}  // namespace

// the 32-padded workspace of the h log-det for this device (created on first use)
static LogdetWorkspace* logdet_h_ws(int64_t d) {
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  const int64_t D = (d + 31) / 32 * 32;  // the 32-block Gauss-Jordan's own granularity
  std::lock_guard<std::mutex> lock(g_ws_mu);
  for (auto* w : g_ws)
    if (w->device == dev && w->D == D) return w;
  LogdetWorkspace* ws = new LogdetWorkspace();
  ws->device = dev;
  ws->D = D;
  ws->A.alloc((size_t)D * D);
  ws->P.alloc(64 * 64);
  ws->R.alloc((size_t)64 * D);
  ws->C.alloc((size_t)D * 64);
  ws->piv.alloc(D);
  g_ws.push_back(ws);
  return ws;
}

// part 0: build + the Gauss-Jordan prologue; parts 1 .. D/32: its block steps; part D/32 + 1: the
// epilogue (h and (sI - A)^-T).  part < 0: all of them.
static void logdet_h_enqueue(const double* A, int64_t d, int64_t lda, double s, double* h_dev, double* Mt_dev,
                             int64_t ldm, hipStream_t st, int part) {
  setup_attributes_once();
  LogdetWorkspace* ws = logdet_h_ws(d);
  const int64_t D = ws->D;
  const int K = (int)(D / 32);
  const GJWork w{ws->P.p, ws->R.p, ws->C.p, ws->piv.p};
  if (part < 0 || part == 0) {
    launch_build_at(A, lda, false, ws->A.p, D, d, s, nullptr, nullptr, st);
    launch_gj_prologue(ws->A.p, D, D, w, nullptr, st);
  }
  for (int k = 0; k < K; ++k)
    if (part < 0 || part == k + 1) launch_gj_step(ws->A.p, D, D, w, nullptr, k, st);
  if (part < 0 || part == K + 1)
    launch_logdet_post(ws->piv.p, d, (double)d * std::log(s), h_dev, ws->A.p, D, Mt_dev, ldm, st);
}

extern "C" int midagma_logdet_h_dev(const double* A, int64_t d, int64_t lda, double s, double* h_dev, double* Mt_dev,
                                    int64_t ldm, void* stream) {
  if (!A || !h_dev || d < 1 || lda < d || !(s > 0.0) || (Mt_dev && ldm < d))
    return fail(nullptr, MIDAGMA_E_ARG, "logdet_h_dev: bad arguments");
  return guarded(nullptr, [&] {
    logdet_h_enqueue(A, d, lda, s, h_dev, Mt_dev, ldm, reinterpret_cast<hipStream_t>(stream), -1);
    return MIDAGMA_OK;
  });
}

extern "C" int64_t midagma_logdet_h_parts(int64_t d) { return d < 1 ? 0 : (d + 31) / 32 + 2; }

// ---- the h log-det's warm-started fast path (ABI 6; mlp.hip) -------------------------------------
struct midagma_ldfast {
  int device = 0;
  int64_t d = 0, Dgj = 0;  // Gauss-Jordan workspace: 32-padded, as midagma_logdet_h_dev
  int B = 0;               // series block: 128 or 256 (0: d > 256, every step exact)
  DevBuf ring0, ring1, Y0, Y1, Q0, Q1, P, part, done, hlast;
  DevBuf A, Pgj, Rgj, Cgj, piv;
  State* st = nullptr;    // the ring's state (slots: step index; warm_run; status of the series)
  State* gjst = nullptr;  // the Gauss-Jordan gate of a fast step (ST_RUNNING: run the chain)
  int64_t* counter = nullptr;  // advanced by a fast step's end (midagma_ldfast_set_counter)
  std::string err;
  ~midagma_ldfast() {
    for (DevBuf* b : {&ring0, &ring1, &Y0, &Y1, &Q0, &Q1, &P, &part, &done, &hlast, &A, &Pgj, &Rgj, &Cgj, &piv})
      b->release();
    if (st) (void)hipFree(st);
    if (gjst) (void)hipFree(gjst);
  }
  GJWork gjw() const { return GJWork{Pgj.p, Rgj.p, Cgj.p, piv.p}; }
  SeriesWork sw() const {
    return SeriesWork{ring0.p, ring1.p, {Y0.p, Y1.p}, {Q0.p, Q1.p}, P.p, part.p, reinterpret_cast<int*>(done.p)};
  }
};

extern "C" int midagma_ldfast_create(midagma_ldfast** out, int64_t d) {
  if (!out || d < 1) return fail(nullptr, MIDAGMA_E_ARG, "ldfast_create: bad arguments");
  auto* h = new midagma_ldfast();
  int rc = guarded(nullptr, [&] {
    setup_attributes_once();
    HIP_TRY(hipGetDevice(&h->device));
    h->d = d;
    h->Dgj = (d + 31) / 32 * 32;
    h->B = d <= 128 ? 128 : (d <= 256 ? 256 : 0);
    const size_t DD = (size_t)h->Dgj * h->Dgj;
    h->A.alloc(DD);
    h->Pgj.alloc(64 * 64);
    h->Rgj.alloc((size_t)64 * h->Dgj);
    h->Cgj.alloc((size_t)h->Dgj * 64);
    h->piv.alloc(h->Dgj);
    h->hlast.alloc(1);
    if (h->B) {
      const size_t BB = (size_t)h->B * h->B;
      for (DevBuf* b : {&h->ring0, &h->ring1, &h->Y0, &h->Y1, &h->Q0, &h->Q1, &h->P}) b->alloc(BB);
      h->part.alloc((size_t)(NM_PASSES + 1) * PART_STRIDE);
      h->done.alloc(1);
    }
    HIP_TRY(hipMalloc(&h->st, sizeof(State)));
    HIP_TRY(hipMalloc(&h->gjst, sizeof(State)));
    return midagma_ldfast_reset(h);
  });
  if (rc != MIDAGMA_OK) {
    delete h;
    return rc;
  }
  *out = h;
  return MIDAGMA_OK;
}

extern "C" void midagma_ldfast_destroy(midagma_ldfast* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  (void)hipDeviceSynchronize();
  delete h;
}

extern "C" int midagma_ldfast_reset(midagma_ldfast* h) {
  if (!h) return fail(nullptr, MIDAGMA_E_ARG, "ldfast_reset: null handle");
  return guarded(nullptr, [&] {
    HIP_TRY(hipSetDevice(h->device));
    State st{};
    st.status = ST_RUNNING;
    st.slots = -1;        // step 0: opened by ldfast_begin (exact) or counted by the fast step's end
    st.ckpt_pending = 1;  // no warm start: the first step runs the Gauss-Jordan chain
    State gj{};
    gj.status = ST_DONE;
    HIP_TRY(hipMemcpy(h->st, &st, sizeof(State), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(h->gjst, &gj, sizeof(State), hipMemcpyHostToDevice));
    HIP_TRY(hipMemset(h->hlast.p, 0, sizeof(double)));
    if (h->done.p) HIP_TRY(hipMemset(h->done.p, 0, sizeof(double)));
    return MIDAGMA_OK;
  });
}

// fast: 0 the series residual (opening the step), 1 .. 3 the passes, 4 certificate + the gated
// chain with the step's end; exact: 0 begin + build + prologue, 1 .. Dgj/32 the block steps, last
// the end
static constexpr int kLdfastPasses = 3;
extern "C" int64_t midagma_ldfast_parts(const midagma_ldfast* h, int exact) {
  if (!h) return 0;
  return (exact || !h->B) ? h->Dgj / 32 + 2 : kLdfastPasses + 2;
}

extern "C" int midagma_ldfast_enqueue(midagma_ldfast* h, const double* A, int64_t d_in, int64_t lda, double s,
                                      double* h_dev, double* Mt_dev, int64_t ldm, void* stream, int exact, int64_t part) {
  if (!h || d_in != h->d)  // the handle's buffers and warm-start ring are sized for its d
    return fail(nullptr, MIDAGMA_E_ARG, "ldfast_enqueue: A's d differs from the handle's");
  if (!A || !h_dev || !Mt_dev || lda < h->d || ldm < h->d || !(s > 0.0) || part >= midagma_ldfast_parts(h, exact))
    return fail(nullptr, MIDAGMA_E_ARG, "ldfast_enqueue: bad arguments");
  return guarded(nullptr, [&] {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t d = h->d, D = h->Dgj;
    const int K = (int)(D / 32);
    const double dls = (double)d * std::log(s);
    const bool ex = exact || !h->B;
    auto want = [&](int64_t p) { return part < 0 || part == p; };
    if (ex) {  // the Gauss-Jordan chain, ungated
      if (want(0)) {
        launch_ldfast_begin(h->st, h->gjst, st);
        launch_build_at(A, lda, false, h->A.p, D, d, s, nullptr, nullptr, st);
        launch_gj_prologue(h->A.p, D, D, h->gjw(), nullptr, st);
      }
      for (int k = 0; k < K; ++k)
        if (want(k + 1)) launch_gj_step(h->A.p, D, D, h->gjw(), nullptr, k, st);
      if (want(K + 1))
        launch_ldfast_post(h->piv.p, d, dls, h_dev, h->A.p, D, Mt_dev, ldm, h->P.p, h->B, h->ring0.p, h->ring1.p,
                           h->st, h->gjst, h->hlast.p, true, st);
      return MIDAGMA_OK;
    }
    const SeriesWork w = h->sw();
    if (want(0)) launch_ldfast_resid(A, lda, d, s, h->B, w, h->st, h->gjst, st);
    // the passes one by one (each its own part: the caller interleaves them)
    for (int p = 1; p <= kLdfastPasses; ++p)
      if (want(p)) launch_series_pass(h->B, w, h->st, p, st);
    if (want(kLdfastPasses + 1)) {
      launch_ldfast_certify(h->P.p, h->B, d, Mt_dev, ldm, h->st, reinterpret_cast<const int*>(h->done.p), h->gjst,
                            h->ring0.p, h->ring1.p, st);
      // gated: opened by the certificate.  One launch, the whole Gauss-Jordan chain in one
      // workgroup (bit-identical; slow when open, which the bench window never is): a closed gate
      // costs one launch instead of the chain's 2 + D/32, and that launch also ends the step
      // (ldfast_post's fast-step work in the same workgroup: one dependent launch fewer)
      const LdfastEnd end{h->piv.p, d, dls, h_dev, Mt_dev, ldm, h->B, h->ring0.p, h->ring1.p, h->st, h->hlast.p,
                          h->counter};
      launch_gj_inverse_1wg(A, lda, h->A.p, D, d, s, h->gjw(), h->gjst, st, end);
    }
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_ldfast_set_counter(midagma_ldfast* h, int64_t* counter) {
  if (!h) return fail(nullptr, MIDAGMA_E_ARG, "ldfast_set_counter: null handle");
  // a handle without the fast path (d > 256: every step runs the Gauss-Jordan chain, which never
  // advances the counter) cannot honour the contract: refuse instead of stalling the caller's table
  if (counter && !h->B) return fail(nullptr, MIDAGMA_E_ARG, "ldfast_set_counter: the handle has no fast path (d > 256)");
  h->counter = counter;
  return MIDAGMA_OK;
}

extern "C" int midagma_ldfast_stats(midagma_ldfast* h, int64_t* steps, int64_t* exact_steps) {
  if (!h) return fail(nullptr, MIDAGMA_E_ARG, "ldfast_stats: null handle");
  return guarded(nullptr, [&] {
    HIP_TRY(hipSetDevice(h->device));
    HIP_TRY(hipDeviceSynchronize());
    State st{};
    HIP_TRY(hipMemcpy(&st, h->st, sizeof(State), hipMemcpyDeviceToHost));
    if (steps) *steps = st.iter;
    if (exact_steps) *exact_steps = st.halvings;
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_logdet_h_dev_part(const double* A, int64_t d, int64_t lda, double s, double* h_dev,
                                         double* Mt_dev, int64_t ldm, void* stream, int64_t part) {
  if (!A || !h_dev || d < 1 || lda < d || !(s > 0.0) || (Mt_dev && ldm < d) || part < 0 ||
      part >= midagma_logdet_h_parts(d))
    return fail(nullptr, MIDAGMA_E_ARG, "logdet_h_dev_part: bad arguments");
  return guarded(nullptr, [&] {
    logdet_h_enqueue(A, d, lda, s, h_dev, Mt_dev, ldm, reinterpret_cast<hipStream_t>(stream), (int)part);
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_logdet_inv_dev(const double* A, int64_t d, int64_t lda, double s_dom, double* logdet_dev,
                                      double* Mt_dev, int64_t ldm, void* stream) {
  if (!A || d < 1 || lda < d || (Mt_dev && ldm < d))
    return fail(nullptr, MIDAGMA_E_ARG, "logdet_inv_dev: bad arguments");
  return guarded(nullptr, [&] {
    setup_attributes_once();
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    const int64_t D = round_up64(d);
    std::lock_guard<std::mutex> lock(g_ws_mu);
    LogdetWorkspace* ws = nullptr;
    for (auto* w : g_ws)
      if (w->device == dev && w->D == D) ws = w;
    if (!ws) {
      ws = new LogdetWorkspace();
      ws->device = dev;
      ws->D = D;
      ws->A.alloc((size_t)D * D);
      ws->P.alloc(64 * 64);
      ws->R.alloc((size_t)64 * D);
      ws->C.alloc((size_t)D * 64);
      ws->piv.alloc(D);
      g_ws.push_back(ws);
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    launch_build_at(A, lda, false, ws->A.p, D, d, s_dom, nullptr, nullptr, st);
    launch_gj_inverse(ws->A.p, D, D, GJWork{ws->P.p, ws->R.p, ws->C.p, ws->piv.p}, nullptr, st);
    if (logdet_dev) launch_sum_vector(ws->piv.p, d, logdet_dev, nullptr, st);
    if (Mt_dev)
      HIP_TRY(hipMemcpy2DAsync(Mt_dev, ldm * sizeof(double), ws->A.p, D * sizeof(double), d * sizeof(double), d,
                               hipMemcpyDeviceToDevice, st));
    return MIDAGMA_OK;
  });
}

// ---------------------------------------------------------------------------
// Linear-SEM generator (sem.hip; utils.py:99-172)
extern "C" int midagma_sem_linear(const double* W, int64_t d, int64_t row0, int64_t n_rows, int sem_type,
                                  const double* noise_scale, uint64_t seed, double* X_dev, int64_t ldx,
                                  void* stream) {
  if (!W || d < 1 || d > (1 << 30)) return fail(nullptr, MIDAGMA_E_ARG, "sem_linear: bad W / d");
  SemGraph g;
  if (!sem_levels(W, d, g)) return fail(nullptr, MIDAGMA_E_ARG, "sem_linear: W must be a DAG");
  if (row0 < 0 || n_rows < 0 || ldx < d || sem_type < 0 || sem_type > 5 || (n_rows > 0 && !X_dev))
    return fail(nullptr, MIDAGMA_E_ARG, "sem_linear: bad arguments");
  if (n_rows == 0) return MIDAGMA_OK;
  return guarded(nullptr, [&] {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    std::vector<double> scale(d, 1.0);
    if (noise_scale) std::copy(noise_scale, noise_scale + d, scale.begin());
    // slab: rows of the node-major scratch, even, ~MIDAGMA_SEM_SLAB_MB (default 2048) MB
    int64_t budget = 2048;
    if (const char* e = getenv("MIDAGMA_SEM_SLAB_MB")) budget = std::max<int64_t>(1, atoll(e));
    const int64_t first = row0 & ~int64_t(1), end = row0 + n_rows;
    int64_t S = std::max<int64_t>(1024, (budget << 20) / (8 * d));
    S = std::min<int64_t>(S, (end - first + 1) & ~int64_t(1));
    S = (S + 1) & ~int64_t(1);
    const size_t nnz = g.pidx.size();
    struct Raw {
      void* p = nullptr;
      ~Raw() {
        if (p) (void)hipFree(p);
      }
    } ints, dbls, xt;
    const size_t n_int = g.nodes.size() + g.pptr.size() + std::max<size_t>(nnz, 1);
    HIP_TRY(hipMalloc(&ints.p, n_int * sizeof(int32_t)));
    HIP_TRY(hipMalloc(&dbls.p, (std::max<size_t>(nnz, 1) + d) * sizeof(double)));
    HIP_TRY(hipMalloc(&xt.p, static_cast<size_t>(S) * d * sizeof(double)));
    int32_t* ip = static_cast<int32_t*>(ints.p);
    double* dp = static_cast<double*>(dbls.p);
    SemDev dev{ip, ip + g.nodes.size(), ip + g.nodes.size() + g.pptr.size(), dp, dp + std::max<size_t>(nnz, 1)};
    HIP_TRY(hipMemcpyAsync(ip, g.nodes.data(), g.nodes.size() * sizeof(int32_t), hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(ip + g.nodes.size(), g.pptr.data(), g.pptr.size() * sizeof(int32_t),
                           hipMemcpyHostToDevice, st));
    if (nnz) {
      HIP_TRY(hipMemcpyAsync(const_cast<int32_t*>(dev.pidx), g.pidx.data(), nnz * sizeof(int32_t),
                             hipMemcpyHostToDevice, st));
      HIP_TRY(hipMemcpyAsync(dp, g.pw.data(), nnz * sizeof(double), hipMemcpyHostToDevice, st));
    }
    HIP_TRY(hipMemcpyAsync(const_cast<double*>(dev.scale), scale.data(), d * sizeof(double), hipMemcpyHostToDevice,
                           st));
    for (int64_t a = first; a < end; a += S) {
      const int64_t rows = std::min<int64_t>(S, end - a);
      const int64_t skip = a < row0 ? row0 - a : 0;
      launch_sem_slab(dev, g.level_off, d, sem_type, seed, a, rows, skip, static_cast<double*>(xt.p), S,
                      X_dev + (a + skip - row0) * ldx, ldx, st);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(st));  // the scratch is freed on return
    return MIDAGMA_OK;
  });
}

// ---------------------------------------------------------------------------
// Gated Adam step (adam.hip) for DagmaNonlinear on torch tensors
extern "C" int64_t midagma_mlp_tail_scratch(int64_t n, int64_t d, int64_t m1) {
  if (n < 1 || d < 1 || m1 < 1) return 0;
  return mlp_tail_scratch(n, d, m1);
}

extern "C" int midagma_mlp_tail_fwd(const double* Z, const double* b1, const double* w2, const double* b2,
                                    const double* X, int64_t n, int64_t d, int64_t m1, double* R, double* scratch,
                                    double* ssq, void* stream) {
  if (!Z || !w2 || !b2 || !X || !R || !scratch || !ssq || n < 1 || d < 1 || m1 < 1 || d * m1 > MLP_TAIL_MAX_DM)
    return fail(nullptr, MIDAGMA_E_ARG, "mlp_tail_fwd: bad arguments");
  return guarded(nullptr, [&] {
    launch_mlp_tail_fwd(Z, b1, w2, b2, X, n, d, (int)m1, R, scratch, ssq, reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_mlp_tail_bwd(const double* Z, const double* b1, const double* w2, const double* R,
                                    const double* g, int64_t n, int64_t d, int64_t m1, double* dZ, double* dw2,
                                    double* db2, double* db1, double* scratch, void* stream) {
  if (!Z || !w2 || !R || !g || !dZ || !dw2 || !db2 || !scratch || n < 1 || d < 1 || m1 < 1 ||
      d * m1 > MLP_TAIL_MAX_DM)
    return fail(nullptr, MIDAGMA_E_ARG, "mlp_tail_bwd: bad arguments");
  return guarded(nullptr, [&] {
    launch_mlp_tail_bwd(Z, b1, w2, R, g, n, d, (int)m1, dZ, dw2, db2, db1, scratch,
                        reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

extern "C" int64_t midagma_fc1_terms_parts(int64_t d) { return d < 1 ? 0 : fc1_terms_parts(d); }

extern "C" int midagma_fc1_terms(const double* W1, int64_t d, int64_t m1, double* A, double* l1part, void* stream) {
  if (!W1 || !A || !l1part || d < 1 || m1 < 1) return fail(nullptr, MIDAGMA_E_ARG, "fc1_terms: bad arguments");
  return guarded(nullptr, [&] {
    launch_fc1_terms(W1, d, (int)m1, A, l1part, reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_fc1_terms_bwd(const double* W1, int64_t d, int64_t m1, const double* gA, const double* gscale,
                                     const double* gl1part, const double* lin, int64_t nlin, double* dW1,
                                     void* stream) {
  if (!W1 || !gA || !gl1part || !dW1 || d < 1 || m1 < 1 || nlin < 0 || (nlin > 0 && !lin))
    return fail(nullptr, MIDAGMA_E_ARG, "fc1_terms_bwd: bad arguments");
  return guarded(nullptr, [&] {
    launch_fc1_terms_bwd(W1, d, (int)m1, gA, gscale, gl1part, lin, (int)nlin, dW1,
                         reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_mlp_objective(const double* ssq, const double* l1part, int64_t np, const double* h, double mu,
                                     double lambda1, double half_d, double inv_n, double* obj, void* stream) {
  if (!ssq || !l1part || !h || !obj || np < 1) return fail(nullptr, MIDAGMA_E_ARG, "mlp_objective: bad arguments");
  return guarded(nullptr, [&] {
    launch_mlp_objective(ssq, l1part, np, h, mu, lambda1, half_d, inv_n, obj, reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_mlp_objective_bwd(const double* g, const double* ssq, int64_t np, double mu, double lambda1,
                                         double half_d, double inv_n, double* gssq, double* gl1part, double* gh,
                                         void* stream) {
  if (!g || (!ssq) != (!gssq) || !gl1part || !gh || np < 1)
    return fail(nullptr, MIDAGMA_E_ARG, "mlp_objective_bwd: bad arguments");
  return guarded(nullptr, [&] {
    launch_mlp_objective_bwd(g, ssq, np, mu, lambda1, half_d, inv_n, gssq, gl1part, gh,
                             reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

// ABI 6: the [d, m1, 1] objective's step with the scalar objective's backward folded into its
// consumers (no mlp_sum / mlp_objective_bwd launches): the tail forward leaves its n row partials,
// the objective sums them (and advances the Adam table counter), the tail backward and the fc1
// terms' backward derive d obj / d ssq, d h and d l1 from gobj themselves.  Bit-identical to the
// ABI-5 sequence (the same sums in the same order, the same scalar arithmetic).
extern "C" int midagma_mlp_tail_fwd_part(const double* Z, const double* b1, const double* w2, const double* b2,
                                         const double* X, int64_t n, int64_t d, int64_t m1, double* R, double* part,
                                         void* stream) {
  if (!Z || !w2 || !b2 || !X || !R || !part || n < 1 || d < 1 || m1 < 1 || d * m1 > MLP_TAIL_MAX_DM)
    return fail(nullptr, MIDAGMA_E_ARG, "mlp_tail_fwd_part: bad arguments");
  return guarded(nullptr, [&] {
    launch_mlp_tail_fwd(Z, b1, w2, b2, X, n, d, (int)m1, R, part, nullptr, reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_mlp_tail_bwd_obj(const double* Z, const double* b1, const double* w2, const double* R,
                                        const double* part, const double* gobj, double mu, double half_d,
                                        double inv_n, int64_t n, int64_t d, int64_t m1, double* dZ, double* dw2,
                                        double* db2, double* db1, double* scratch, void* stream) {
  // (ABI 9: dw2 = db2 = db1 = NULL leaves the chunk partials in scratch for midagma_mlp_step)
  const bool sums = dw2 || db2 || db1;
  if (!Z || !w2 || !R || !part || !gobj || !dZ || (sums && (!dw2 || !db2)) || !scratch || n < 1 || d < 1 ||
      m1 < 1 || d * m1 > MLP_TAIL_MAX_DM)
    return fail(nullptr, MIDAGMA_E_ARG, "mlp_tail_bwd_obj: bad arguments");
  return guarded(nullptr, [&] {
    launch_mlp_tail_bwd(Z, b1, w2, R, nullptr, n, d, (int)m1, dZ, dw2, db2, db1, scratch,
                        reinterpret_cast<hipStream_t>(stream), part, gobj, mu, half_d, inv_n, sums);
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_mlp_step(double* const* params, double* const* exp_avg, double* const* exp_avg_sq, int64_t n,
                                int64_t d, int64_t m1, const double* gA, const double* gobj, double mu,
                                double lambda1, const double* lin, int64_t nlin, const double* scratch,
                                const double* table, const int64_t* counter, double w1, double beta2, double c2,
                                double eps, double wd, const double* gate, double* A, double* l1part, void* stream) {
  if (!params || !exp_avg || !exp_avg_sq || !gA || !gobj || !scratch || !table || !counter || !A || !l1part ||
      n < 1 || d < 1 || m1 < 1 || d * m1 > MLP_TAIL_MAX_DM || nlin < 0 || (nlin > 0 && !lin))
    return fail(nullptr, MIDAGMA_E_ARG, "mlp_step: bad arguments");
  for (int q = 0; q < 4; ++q)
    if (!params[q] || !exp_avg[q] || !exp_avg_sq[q]) return fail(nullptr, MIDAGMA_E_ARG, "mlp_step: bad tensor");
  const MlpStepPtrs p{params[0], params[1], params[2], params[3], exp_avg[0], exp_avg_sq[0], exp_avg[1],
                      exp_avg_sq[1], exp_avg[2], exp_avg_sq[2], exp_avg[3], exp_avg_sq[3]};
  return guarded(nullptr, [&] {
    launch_mlp_step(p, n, d, (int)m1, gA, gobj, mu, lambda1, lin, (int)nlin, scratch, table, counter, w1, beta2, c2,
                    eps, wd, gate, A, l1part, reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

#ifdef MIDAGMA_EXPERIMENTS
// fc1 and the tail fused on the MFMA (mlp.hip; measured slower at config 5):
// not in the public header, bound by nonlinear.py when the loaded library has them
extern "C" int64_t midagma_mlp_fused_parts(int64_t n, int64_t d, int64_t m1) { return mlp_fused_parts(n, d, m1); }

extern "C" int64_t midagma_mlp_fused_splits(int64_t n) { return n < 1 ? 0 : mlp_fused_splits(n); }

extern "C" int midagma_mlp_fc1_tail_fwd(const double* X, const double* W1, const double* b1, const double* w2,
                                        const double* b2, int64_t n, int64_t d, int64_t m1, double* S, double* R,
                                        double* part, void* stream) {
  if (!X || !W1 || !w2 || !b2 || !S || !R || !part || mlp_fused_parts(n, d, m1) < 1)
    return fail(nullptr, MIDAGMA_E_ARG, "mlp_fc1_tail_fwd: bad arguments");
  return guarded(nullptr, [&] {
    launch_mlp_fc1_tail_fwd(X, W1, b1, w2, b2, n, d, (int)m1, S, R, part, reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_mlp_tail_bwd_lin(const double* S, const double* w2, const double* R, const double* X,
                                        const double* part, int64_t npart, const double* gobj, double mu,
                                        double half_d, double inv_n, int64_t n, int64_t d, int64_t m1, double* lin,
                                        double* dw2, double* db2, double* db1, double* scratch, void* stream) {
  if (!S || !w2 || !R || !X || !part || npart < 1 || !gobj || !lin || !dw2 || !db2 || !scratch ||
      mlp_fused_parts(n, d, m1) < 1)
    return fail(nullptr, MIDAGMA_E_ARG, "mlp_tail_bwd_lin: bad arguments");
  return guarded(nullptr, [&] {
    launch_mlp_tail_bwd_lin(S, w2, R, X, part, npart, gobj, mu, half_d, inv_n, n, d, (int)m1, lin, dw2, db2, db1,
                            scratch, reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}
#endif

extern "C" int midagma_fc1_terms_bwd_obj(const double* W1, int64_t d, int64_t m1, const double* gA, const double* gobj,
                                         double mu, double lambda1, const double* lin, int64_t nlin, double* dW1,
                                         void* stream) {
  if (!W1 || !gA || !gobj || !dW1 || d < 1 || m1 < 1 || nlin < 0 || (nlin > 0 && !lin))
    return fail(nullptr, MIDAGMA_E_ARG, "fc1_terms_bwd_obj: bad arguments");
  return guarded(nullptr, [&] {
    launch_fc1_terms_bwd(W1, d, (int)m1, gA, nullptr, nullptr, lin, (int)nlin, dW1,
                         reinterpret_cast<hipStream_t>(stream), gobj, mu, lambda1);
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_mlp_objective_part(const double* part, int64_t npart, const double* l1part, int64_t np,
                                          const double* h, double mu, double lambda1, double half_d, double inv_n,
                                          double* obj, int64_t* counter, void* stream) {
  if (!part || npart < 1 || !l1part || !h || !obj || np < 1)
    return fail(nullptr, MIDAGMA_E_ARG, "mlp_objective_part: bad arguments");
  return guarded(nullptr, [&] {
    launch_mlp_objective(nullptr, l1part, np, h, mu, lambda1, half_d, inv_n, obj,
                         reinterpret_cast<hipStream_t>(stream), part, npart, counter);
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_adam_step(double* p, const double* g, double* m, double* v, int64_t n, double step_size,
                                 double w1, double beta2, double c2, double bc2_sqrt, double eps, double wd,
                                 const double* gate, void* stream) {
  if (!p || !g || !m || !v || n < 0) return fail(nullptr, MIDAGMA_E_ARG, "adam_step: bad arguments");
  if (n == 0) return MIDAGMA_OK;
  return guarded(nullptr, [&] {
    launch_adam_gated(p, g, m, v, n, AdamCoef{step_size, w1, beta2, c2, bc2_sqrt, eps, wd}, gate,
                      reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_adam_step_table(double* p, const double* g, double* m, double* v, int64_t n,
                                       const double* table, const int64_t* counter, double w1, double beta2,
                                       double c2, double eps, double wd, const double* gate, void* stream) {
  if (!p || !g || !m || !v || !table || !counter || n < 0) return fail(nullptr, MIDAGMA_E_ARG, "adam_step_table: bad arguments");
  if (n == 0) return MIDAGMA_OK;
  return guarded(nullptr, [&] {
    launch_adam_gated_table(p, g, m, v, n, AdamCoef{0.0, w1, beta2, c2, 1.0, eps, wd}, table, counter, gate,
                            reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_adam_step_table_multi(int64_t k, double* const* p, const double* const* g, double* const* m,
                                             double* const* v, const int64_t* n, const double* table,
                                             const int64_t* counter, double w1, double beta2, double c2, double eps,
                                             double wd, const double* gate, void* stream) {
  if (k < 1 || k > ADAM_MULTI || !p || !g || !m || !v || !n || !table || !counter)
    return fail(nullptr, MIDAGMA_E_ARG, "adam_step_table_multi: bad arguments");
  AdamSet set{};
  set.k = (int)k;
  set.off[0] = 0;
  for (int64_t q = 0; q < k; ++q) {
    if (!p[q] || !g[q] || !m[q] || !v[q] || n[q] < 0)
      return fail(nullptr, MIDAGMA_E_ARG, "adam_step_table_multi: bad tensor");
    set.p[q] = p[q];
    set.g[q] = g[q];
    set.m[q] = m[q];
    set.v[q] = v[q];
    set.off[q + 1] = set.off[q] + n[q];
  }
  if (set.off[k] == 0) return MIDAGMA_OK;
  return guarded(nullptr, [&] {
    launch_adam_gated_table_multi(set, AdamCoef{0.0, w1, beta2, c2, 1.0, eps, wd}, table, counter, gate,
                                  reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

extern "C" int midagma_counter_advance(int64_t* counter, void* stream) {
  if (!counter) return fail(nullptr, MIDAGMA_E_ARG, "counter_advance: null counter");
  return guarded(nullptr, [&] {
    launch_counter_advance(counter, reinterpret_cast<hipStream_t>(stream));
    return MIDAGMA_OK;
  });
}

#ifdef MIDAGMA_EXPERIMENTS
// Diagnostics (not part of the ABI header): the one-launch inverse's task plan for D, passes
// and nwg workgroups, as planned on the host (no GPU needed).  tasks (12 ints per task, grouped
// by workgroup) and woff (nwg + 1) may be null to query the sizes.  Returns 0, or -1.
extern "C" int midagma_debug_df_plan(int64_t D, int passes, int nwg, double* est_us, int64_t* ntasks, int* tasks,
                                     int* woff, int* nctr) {
  try {
    if (!df_available(D) || (passes != 2 && passes != 3) || nwg < 1) return -1;
    const DfPlanHost p = df_plan(D, passes, nwg);
    if (est_us) *est_us = p.est_us;
    if (ntasks) *ntasks = (int64_t)(p.tasks->size() / 12);
    if (nctr) *nctr = p.nctr;
    if (tasks) std::memcpy(tasks, p.tasks->data(), p.tasks->size() * sizeof(int));
    if (woff) std::memcpy(woff, p.woff->data(), p.woff->size() * sizeof(int));
    return 0;
  } catch (const std::exception& e) {
    fprintf(stderr, "midagma_debug_df_plan: %s\n", e.what());
    return -1;
  }
}

// Diagnostics: the one-launch inverse's per-task timestamps of the last launch (3 per task in
// plan order: wait start, go, done; 100 MHz ticks), with MIDAGMA_DF_STAMPS set at create.
// Returns the number of values copied, or -1.
extern "C" int64_t midagma_debug_df_stamps(midagma_solver* s, unsigned long long* out, int64_t cap) {
  if (!s || !s->dfw.stamps) return -1;
  const int64_t n = std::min<int64_t>(cap, (int64_t)s->dfStamps.n);
  if (hipStreamSynchronize(s->stream) != hipSuccess) return -1;
  if (hipMemcpy(out, s->dfStamps.p, n * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return n;
}
#endif  // MIDAGMA_EXPERIMENTS
