// ABI 11: data mode on several devices from one process (include/midagma_hip.h, midagma_group_*).
//
// The reference fits from one process (DagmaLinear.fit, linear.py:335-351) and its per-step score
// gradient (linear.py:244-246) is a sum over the rows of X.  A group keeps one data-mode solver per
// device, each holding a row shard, and sums their score partials inside every slot (SURVEY 5 and
// 8(b): one host process drives all devices; the Python side stays single-process):
//
//   * distinct devices: ncclCommInitAll gives member k its rank-k communicator, so each member's
//     captured slot graphs carry the all-reduce exactly as a torchrun rank's do (midagma_comm_init);
//     the library runs one host thread per member to replay them (a thread blocks in its own
//     stream's syncs, so one thread per device keeps every device fed).  The members finish their
//     setup (begin, graph capture) and meet at a host barrier before any of them issues a
//     collective, so a member that fails there fails the call everywhere instead of leaving the
//     others waiting in an all-reduce.
//   * MIDAGMA_GROUP_EMULATE (all members on one device): no RCCL.  Member 0's slot
//     graphs are captured over every member's stream at once -- every member's part 1, then the
//     partials summed in a fixed order (member 0 + member 1 + ...) and copied back to each member,
//     then every member's part 2 -- and the calling thread replays them with member 0's drivers.
//     The members decide identically (same W, same sum), so member 0's state stands for all.
#include <hip/hip_runtime.h>

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/midagma_hip.h"
#include "solver_impl.h"

namespace {

constexpr int kMaxEmulated = 16;

// diagnostics (MIDAGMA_GROUP_DEBUG=1): stage marks on stderr and a native backtrace on SIGSEGV
bool gdebug() {
  static const bool on = std::getenv("MIDAGMA_GROUP_DEBUG") != nullptr;
  return on;
}
void segv_trace(int sig) {
  void* fr[64];
  const int n = backtrace(fr, 64);
  fprintf(stderr, "midagma group: signal %d, native backtrace:\n", sig);
  backtrace_symbols_fd(fr, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}
void gmark(const char* what, int k = -1) {
  if (!gdebug()) return;
  static bool installed = false;
  if (!installed) {
    installed = true;
    signal(SIGSEGV, segv_trace);
  }
  fprintf(stderr, "midagma group: %s %d\n", what, k);
  fflush(stderr);
}

struct GroupParts {
  double* p[kMaxEmulated];
  int n;
};

// parts.p[0][i] <- ((p0 + p1) + p2) + ... : the emulated all-reduce's sum, in place in member 0's
// buffer (each element read and written by one thread, so in place is safe)
__global__ void group_sum_kernel(GroupParts parts, int64_t len) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < len; i += (int64_t)gridDim.x * blockDim.x) {
    double acc = parts.p[0][i];
    for (int k = 1; k < parts.n; ++k) acc += parts.p[k][i];
    parts.p[0][i] = acc;
  }
}

bool all_finite_w(const double* p, int64_t n) {
  for (int64_t i = 0; i < n; ++i)
    if (!std::isfinite(p[i])) return false;
  return true;
}

// an exception from a member's work as a C ABI code (solver.hip's `guarded` mapping)
int classify(std::exception_ptr e, std::string& msg) {
  try {
    std::rethrow_exception(e);
  } catch (const HipError& x) {
    msg = x.what();
    return MIDAGMA_E_HIP;
  } catch (const std::invalid_argument& x) {
    msg = x.what();
    return MIDAGMA_E_ARG;
  } catch (const std::exception& x) {
    msg = x.what();
    return MIDAGMA_E_STATE;
  } catch (...) {
    msg = "unknown error";
    return MIDAGMA_E_STATE;
  }
}

// the members' meeting point before any collective: every member arrives with whether its setup
// succeeded; all leave with the conjunction
class SetupBarrier {
 public:
  explicit SetupBarrier(int n) : left_(n) {}
  bool arrive(bool ok) {
    std::unique_lock<std::mutex> lk(mu_);
    all_ok_ = all_ok_ && ok;
    if (--left_ == 0) {
      cv_.notify_all();
    } else {
      cv_.wait(lk, [&] { return left_ == 0; });
    }
    return all_ok_;
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  int left_;
  bool all_ok_ = true;
};

}  // namespace

struct midagma_group {
  std::vector<midagma_solver*> m;
  std::vector<int> devices;
  bool emulated = false;
  int loss = 0;
  int64_t d = 0;
  std::string err;
  ~midagma_group() {
    for (midagma_solver* s : m) midagma_destroy(s);  // (each destroys its communicator)
  }

  hipStream_t s0() const { return m[0]->stream; }
  int64_t zlen() const { return m[0]->D * m[0]->D + 64; }

  // emulated all-reduce of the members' score buffers, on member 0's stream: the fixed-order sum
  // into member 0's buffer, then copies to the others
  void enqueue_emulated_allreduce() {
    GroupParts parts{};
    parts.n = (int)m.size();
    for (size_t k = 0; k < m.size(); ++k) parts.p[k] = m[k]->zbuf;
    hipLaunchKernelGGL(group_sum_kernel, dim3(1024), dim3(NTHREADS), 0, s0(), parts, zlen());
    HIP_TRY(hipGetLastError());
    for (size_t k = 1; k < m.size(); ++k)
      HIP_TRY(hipMemcpyAsync(m[k]->zbuf, m[0]->zbuf, (size_t)zlen() * sizeof(double), hipMemcpyDeviceToDevice, s0()));
  }

  // every member's work enqueued on member 0's stream (the emulated group's capture; each member's
  // own side stream still forks from it and joins back, as in a one-solver slot)
  struct OnStream0 {
    midagma_group* g;
    std::vector<hipStream_t> saved;
    explicit OnStream0(midagma_group* g_) : g(g_) {
      for (midagma_solver* s : g->m) {
        saved.push_back(s->stream);
        s->stream = g->s0();
      }
    }
    ~OnStream0() {
      for (size_t k = 0; k < g->m.size(); ++k) g->m[k]->stream = saved[k];
    }
  };

  // runs f(k) for every member on a thread of its own (device k current), joined; the first
  // failure's code (and message, prefixed with the member) is returned
  template <class F>
  int parallel(F&& f) {
    const int N = (int)m.size();
    std::vector<int> rc((size_t)N, MIDAGMA_OK);
    std::vector<std::string> msg((size_t)N);
    auto run = [&](int k) {
      try {
        HIP_TRY(hipSetDevice(m[k]->device));
        f(k);
      } catch (...) {
        rc[k] = classify(std::current_exception(), msg[k]);
      }
    };
    if (N == 1) {
      run(0);
    } else {
      std::vector<std::thread> th;
      for (int k = 0; k < N; ++k) th.emplace_back(run, k);
      for (auto& t : th) t.join();
    }
    for (int k = 0; k < N; ++k)
      if (rc[k] != MIDAGMA_OK) {
        err = "member " + std::to_string(k) + " (device " + std::to_string(devices[k]) + "): " + msg[k];
        return rc[k];
      }
    return MIDAGMA_OK;
  }
};

namespace midagma {

hipGraphExec_t group_capture(midagma_group* g, const midagma_solver* caller, int which, int reps, int passes) {
  if (caller != g->m[0])
    throw std::logic_error("emulated device group: its slots are driven through the group (midagma_group_minimize)");
  const bool fast = (which & 4) != 0;
  hipGraph_t graph = nullptr;
  gmark("capture begin", which);
  // one capturing stream: the members' work in sequence on member 0's stream (a capture that
  // forked member streams from it and joined them back crashed hipStreamEndCapture on the box,
  // ROCm 7.2; the emulated group checks arithmetic, not overlap)
  // (on member 0's capture stream, not its launch stream: midagma_solver::capture)
  midagma_solver::StreamSwap on_cap(g->m[0], g->m[0]->capture_stream());
  midagma_group::OnStream0 on(g);
  HIP_TRY(hipStreamBeginCapture(g->s0(), hipStreamCaptureModeThreadLocal));
  try {
    for (int r = 0; r < reps; ++r) {
      if (which & 1)
        for (midagma_solver* s : g->m) s->enqueue_part1(fast, passes);
      if ((which & 3) == 3) g->enqueue_emulated_allreduce();
      if (which & 2)
        for (midagma_solver* s : g->m) s->enqueue_part2(fast);
    }
  } catch (...) {
    (void)hipStreamEndCapture(g->s0(), &graph);
    if (graph) (void)hipGraphDestroy(graph);
    throw;
  }
  HIP_TRY(hipStreamEndCapture(g->s0(), &graph));
  gmark("capture ended", which);
  hipGraphExec_t exec = nullptr;
  HIP_TRY(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
  HIP_TRY(hipGraphDestroy(graph));
  gmark("instantiated", which);
  return exec;
}

void group_clear_handback(midagma_group* g) {
  static const int32_t running = ST_RUNNING;
  for (midagma_solver* s : g->m)
    HIP_TRY(hipMemcpyAsync(&s->d_state->status, &running, sizeof(int32_t), hipMemcpyHostToDevice, g->s0()));
}

}  // namespace midagma

namespace {
thread_local std::string g_group_error;

int gfail(midagma_group* g, int code, const std::string& msg) {
  (g ? g->err : g_group_error) = msg;
  return code;
}

template <class F>
int gguard(midagma_group* g, F&& f) {
  try {
    HIP_TRY(hipSetDevice(g->devices[0]));
    return f();
  } catch (...) {
    std::string msg;
    const int rc = classify(std::current_exception(), msg);
    return gfail(g, rc, msg);
  }
}

bool same_result(const midagma_result& a, const midagma_result& b) {
  return a.iters == b.iters && a.status == b.status && a.halvings == b.halvings && a.slots == b.slots &&
         a.n_checkpoints == b.n_checkpoints && a.early_stop == b.early_stop;
}
}  // namespace

extern "C" {

int midagma_group_create(midagma_group** out, int loss, int64_t d, const int* devices, int ndev, int flags) {
  if (!out || !devices || ndev < 1 || d < 1 || (loss != MIDAGMA_LOSS_L2 && loss != MIDAGMA_LOSS_LOGISTIC) ||
      (flags & ~MIDAGMA_GROUP_EMULATE))
    return gfail(nullptr, MIDAGMA_E_ARG, "group_create: bad arguments");
  const bool emulate = (flags & MIDAGMA_GROUP_EMULATE) != 0;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess) return gfail(nullptr, MIDAGMA_E_HIP, "group_create: no HIP device");
  for (int k = 0; k < ndev; ++k) {
    if (devices[k] < 0 || devices[k] >= count)
      return gfail(nullptr, MIDAGMA_E_ARG, "group_create: device " + std::to_string(devices[k]) + " out of range");
    for (int j = 0; j < k; ++j) {
      if (!emulate && devices[j] == devices[k])
        return gfail(nullptr, MIDAGMA_E_ARG,
                     "group_create: a device appears twice (one RCCL rank per device; MIDAGMA_GROUP_EMULATE "
                     "puts every member on one device)");
    }
    if (emulate && devices[k] != devices[0])
      return gfail(nullptr, MIDAGMA_E_ARG, "group_create: an emulated group keeps every member on one device");
  }
  if (emulate && ndev > kMaxEmulated)
    return gfail(nullptr, MIDAGMA_E_ARG, "group_create: an emulated group holds at most 16 members");
  midagma_group* g = new midagma_group();
  g->emulated = emulate;
  g->loss = loss;
  g->d = d;
  g->devices.assign(devices, devices + ndev);
  for (int k = 0; k < ndev; ++k) {
    midagma_solver* s = nullptr;
    const int rc = midagma_create(&s, loss, MIDAGMA_MODE_DATA, d, devices[k], nullptr);
    if (rc != MIDAGMA_OK) {
      const std::string why = std::string("group_create: member ") + std::to_string(k) + ": " + midagma_last_error(nullptr);
      delete g;
      return gfail(nullptr, rc, why);
    }
    g->m.push_back(s);
  }
  const int rc = gguard(g, [&] {
    if (emulate) {
      for (midagma_solver* s : g->m) s->group = g;
    } else {
      std::vector<void*> comms((size_t)ndev, nullptr);
      comm_create_all(ndev, devices, comms.data());
      for (int k = 0; k < ndev; ++k) {
        midagma_solver* s = g->m[(size_t)k];
        HIP_TRY(hipSetDevice(s->device));
        s->comm = comms[(size_t)k];
        s->comm_ranks = ndev;
        s->agree.alloc(8);
        if (!s->h_agree) HIP_TRY(hipHostMalloc(&s->h_agree, 8 * sizeof(double), hipHostMallocDefault));
        s->graphs_valid = false;  // its slot graphs now carry the all-reduce
      }
    }
    return MIDAGMA_OK;
  });
  if (rc != MIDAGMA_OK) {
    const std::string why = g->err;
    delete g;
    return gfail(nullptr, rc, why);
  }
  *out = g;
  return MIDAGMA_OK;
}

void midagma_group_destroy(midagma_group* g) { delete g; }

const char* midagma_group_last_error(const midagma_group* g) { return g ? g->err.c_str() : g_group_error.c_str(); }

int midagma_group_size(const midagma_group* g) { return g ? (int)g->m.size() : 0; }

int midagma_group_emulated(const midagma_group* g) { return g && g->emulated ? 1 : 0; }

midagma_solver* midagma_group_member(midagma_group* g, int k) {
  return (g && k >= 0 && k < (int)g->m.size()) ? g->m[(size_t)k] : nullptr;
}

int midagma_group_set_data(midagma_group* g, const double* X, int64_t n) {
  if (!g || !X) return gfail(g, MIDAGMA_E_ARG, "group_set_data: null argument");
  const int64_t N = (int64_t)g->m.size();
  if (n < N) return gfail(g, MIDAGMA_E_ARG, "group_set_data: fewer rows than members");
  const int64_t base = n / N, extra = n % N;
  for (int64_t k = 0; k < N; ++k) {
    const int64_t lo = k * base + std::min(k, extra), rows = base + (k < extra ? 1 : 0);
    const int rc = midagma_set_data(g->m[(size_t)k], X + lo * g->d, rows, n, 0);
    if (rc != MIDAGMA_OK)
      return gfail(g, rc, "group_set_data: member " + std::to_string(k) + ": " + midagma_last_error(g->m[(size_t)k]));
  }
  return MIDAGMA_OK;
}

int midagma_group_allreduce_zbuf(midagma_group* g) {
  if (!g) return gfail(g, MIDAGMA_E_ARG, "group_allreduce_zbuf: null group");
  if (g->emulated) {
    return gguard(g, [&] {
      for (midagma_solver* s : g->m) HIP_TRY(hipStreamSynchronize(s->stream));
      g->enqueue_emulated_allreduce();
      HIP_TRY(hipStreamSynchronize(g->s0()));
      return MIDAGMA_OK;
    });
  }
  return g->parallel([&](int k) {
    midagma_solver* s = g->m[(size_t)k];
    comm_allreduce(s->comm, s->zbuf, (size_t)g->zlen(), false, s->stream);
    HIP_TRY(hipStreamSynchronize(s->stream));
  });
}

int midagma_group_minimize(midagma_group* g, double* W, double mu, int64_t max_iter, double s_dom, double lr,
                           double tol, double beta1, double beta2, double lambda1, int64_t checkpoint,
                           midagma_result* res) {
  if (!g || !W) return gfail(g, MIDAGMA_E_ARG, "group_minimize: null argument");
  const int64_t d = g->d, N = (int64_t)g->m.size();
  if (!all_finite_w(W, d * d)) return gfail(g, MIDAGMA_E_ARG, "group_minimize: array must not contain infs or NaNs");
  std::vector<std::vector<double>> Wk((size_t)N, std::vector<double>((size_t)(d * d)));
  std::vector<midagma_result> rk((size_t)N);
  for (auto& w : Wk) std::memcpy(w.data(), W, (size_t)(d * d) * sizeof(double));
  int rc;
  if (g->emulated) {
    rc = gguard(g, [&] {
      for (midagma_solver* s : g->m) s->begin(W, mu, max_iter, s_dom, lr, tol, beta1, beta2, lambda1, checkpoint);
      gmark("begun");
      // the combined graphs bake every member's buffers and settings in: captured afresh per call
      g->m[0]->destroy_graphs();
      g->m[0]->run_loop(max_iter, checkpoint);
      gmark("loop done");
      for (int64_t k = 0; k < N; ++k) g->m[(size_t)k]->finish(Wk[(size_t)k].data(), &rk[(size_t)k]);
      gmark("finished");
      return MIDAGMA_OK;
    });
  } else {
    std::atomic<bool> stop{false};
    SetupBarrier meet((int)N);
    rc = g->parallel([&](int k) {
      midagma_solver* s = g->m[(size_t)k];
      bool ok = true;
      std::exception_ptr e;
      try {
        s->begin(W, mu, max_iter, s_dom, lr, tol, beta1, beta2, lambda1, checkpoint);
        s->ensure_graphs();  // (the capture issues no collective that runs)
      } catch (...) {
        ok = false;
        e = std::current_exception();
      }
      if (!meet.arrive(ok)) {
        if (e) std::rethrow_exception(e);
        throw std::runtime_error("device group: another member failed its setup; no step was run");
      }
      s->group_stop = &stop;
      try {
        s->run_loop(max_iter, checkpoint);
        s->finish(Wk[(size_t)k].data(), &rk[(size_t)k]);
      } catch (...) {
        stop = true;
        s->group_stop = nullptr;
        throw;
      }
      s->group_stop = nullptr;
    });
  }
  if (rc != MIDAGMA_OK) return rc;
  for (int64_t k = 1; k < N; ++k) {
    if (std::memcmp(Wk[(size_t)k].data(), Wk[0].data(), (size_t)(d * d) * sizeof(double)) != 0 ||
        !same_result(rk[(size_t)k], rk[0]))
      return gfail(g, MIDAGMA_E_STATE,
                   "device group: member " + std::to_string(k) + " ended with a different W or state than member 0 "
                   "(replicas diverged)");
  }
  std::memcpy(W, Wk[0].data(), (size_t)(d * d) * sizeof(double));
  if (res) *res = rk[0];
  if (rk[0].status == MIDAGMA_ST_SINGULAR) {
    if (!all_finite_w(W, d * d)) return gfail(g, MIDAGMA_E_ARG, "group_minimize: array must not contain infs or NaNs");
    return gfail(g, MIDAGMA_E_SINGULAR, "singular matrix: inverse of sI - W*W is not finite");
  }
  return MIDAGMA_OK;
}

}  // extern "C"
