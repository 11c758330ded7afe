// The data-mode score all-reduce inside the library (linear.py:244-246 summed over
// the ranks' row shards): an RCCL communicator owned by the solver, so the sum of the score
// partial Z_k = X_k^T(...) is captured into the replayed slot graph between the GEMMs and the
// update, and a multi-rank minimize runs from the device like a single-process one (the host
// polls once per batch, with a small agreement all-reduce of every rank's (status, iters)).
//
// RCCL is resolved at run time (dlopen): the copy the process already loaded (PyTorch's) when
// there is one, else MIDAGMA_RCCL_LIB or the ROCm install's; the product library has no link-time
// RCCL dependency and solvers without a communicator never touch it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "launch.h"

namespace midagma {

namespace {

struct RcclApi {
  void* lib = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommInitAll) init_all = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  std::string why;
};

RcclApi& api() {
  static RcclApi a;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* env = std::getenv("MIDAGMA_RCCL_LIB");
    // already in the process (torch's librccl.so) first: one RCCL for all communicators
    for (const char* name : {"librccl.so", "librccl.so.1"}) {
      if (env) break;
      a.lib = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
      if (a.lib) break;
    }
    for (const char* name : {env, "librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
      if (a.lib || !name) continue;
      a.lib = dlopen(name, RTLD_NOW | RTLD_LOCAL);
    }
    if (!a.lib) {
      const char* e = dlerror();
      a.why = std::string("RCCL not loadable: ") + (e ? e : "unknown");
      return;
    }
    a.get_unique_id = reinterpret_cast<decltype(a.get_unique_id)>(dlsym(a.lib, "ncclGetUniqueId"));
    a.init_rank = reinterpret_cast<decltype(a.init_rank)>(dlsym(a.lib, "ncclCommInitRank"));
    a.init_all = reinterpret_cast<decltype(a.init_all)>(dlsym(a.lib, "ncclCommInitAll"));
    a.all_reduce = reinterpret_cast<decltype(a.all_reduce)>(dlsym(a.lib, "ncclAllReduce"));
    a.destroy = reinterpret_cast<decltype(a.destroy)>(dlsym(a.lib, "ncclCommDestroy"));
    a.error_string = reinterpret_cast<decltype(a.error_string)>(dlsym(a.lib, "ncclGetErrorString"));
    if (!a.get_unique_id || !a.init_rank || !a.init_all || !a.all_reduce || !a.destroy || !a.error_string)
      a.why = "RCCL: a symbol is missing";
  });
  if (!a.why.empty()) throw std::runtime_error(a.why);
  return a;
}

void check_nccl(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + api().error_string(r));
}

// the agreement vector of one poll: every rank's (status, iters) and their negations, so one
// max all-reduce yields max and min over the ranks
__global__ void agree_pack_kernel(const State* __restrict__ st, double* __restrict__ out) {
  if (threadIdx.x == 0) {
    const double s = (double)st->status, it = (double)st->iter;
    out[0] = s;
    out[1] = it;
    out[2] = -s;
    out[3] = -it;
  }
}

}  // namespace

int comm_unique_id(void* out) {
  ncclUniqueId id;
  check_nccl(api().get_unique_id(&id), "ncclGetUniqueId");
  std::memcpy(out, &id, sizeof(id));
  return (int)sizeof(id);
}

void* comm_create(const void* id, int nranks, int rank) {
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  check_nccl(api().init_rank(&c, nranks, u, rank), "ncclCommInitRank");
  return c;
}

// ABI 11: the communicators of a single-process device group, one per device of devlist (RCCL's
// own group initialisation: ncclCommInitAll); comms[k] is rank k
void comm_create_all(int ndev, const int* devlist, void** comms) {
  std::vector<ncclComm_t> c((size_t)ndev, nullptr);
  check_nccl(api().init_all(c.data(), ndev, devlist), "ncclCommInitAll");
  for (int k = 0; k < ndev; ++k) comms[k] = c[(size_t)k];
}

void comm_destroy(void* comm) {
  if (comm) (void)api().destroy(static_cast<ncclComm_t>(comm));
}

void comm_allreduce(void* comm, double* buf, size_t n, bool max, hipStream_t stream) {
  check_nccl(api().all_reduce(buf, buf, n, ncclFloat64, max ? ncclMax : ncclSum, static_cast<ncclComm_t>(comm),
                              stream),
             "ncclAllReduce");
}

void launch_agree_pack(const State* st, double* out, hipStream_t stream) {
  hipLaunchKernelGGL(agree_pack_kernel, dim3(1), dim3(64), 0, stream, st, out);
  HIP_TRY(hipGetLastError());
}

}  // namespace midagma
