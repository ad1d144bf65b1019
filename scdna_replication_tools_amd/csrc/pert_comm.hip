// pert_comm.hip -- the cross-rank sum of a sharded fit's shared-gradient block, issued by the
// library itself: an RCCL communicator over the fit's ranks (one process per GPU, xGMI), so a
// sharded SVI loop runs as GIL-free C calls (pert_svi_run_sharded) with the all-reduce queued
// on the fit's stream between the reductions and Adam, like the single-rank loop.
//
// Reference: pert_model.py:800-816 runs svi_s.step() on one CPU process; the shard/all-reduce
// decomposition is SURVEY.md section 8e.  RCCL is not linked: pert_comm_load() dlopens the copy
// the process already has (torch's, which libtorch_hip links), so the communicator and torch's
// process group use one RCCL.  Only the types of rccl.h are used here.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <mutex>

#include "pert_hip.h"

struct pert_comm {
  ncclComm_t comm;
  int32_t world, rank;
};

namespace {

struct Rccl {
  void* handle = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
};

Rccl g_rccl;
std::mutex g_mu;

int comm_status(ncclResult_t r) { return r == ncclSuccess ? PERT_OK : PERT_E_COMM_BASE + (int)r; }

}  // namespace

extern "C" {

int pert_comm_load(const char* rccl_path) {
  std::lock_guard<std::mutex> lock(g_mu);
  if (g_rccl.handle) return PERT_OK;
  if (!rccl_path) return PERT_E_ARG;
  void* h = dlopen(rccl_path, RTLD_NOW | RTLD_LOCAL);
  if (!h) return PERT_E_COMM_UNAVAILABLE;
  Rccl r;
  r.handle = h;
  r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
  r.init_rank = reinterpret_cast<decltype(r.init_rank)>(dlsym(h, "ncclCommInitRank"));
  r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(h, "ncclAllReduce"));
  r.destroy = reinterpret_cast<decltype(r.destroy)>(dlsym(h, "ncclCommDestroy"));
  if (!r.get_unique_id || !r.init_rank || !r.all_reduce || !r.destroy) {
    dlclose(h);
    return PERT_E_COMM_UNAVAILABLE;
  }
  g_rccl = r;
  return PERT_OK;
}

int pert_comm_unique_id(uint8_t* id, int32_t n) {
  if (!id || n != (int32_t)sizeof(ncclUniqueId)) return PERT_E_ARG;
  if (!g_rccl.handle) return PERT_E_COMM_UNAVAILABLE;
  ncclUniqueId u;
  const int rc = comm_status(g_rccl.get_unique_id(&u));
  if (rc == PERT_OK) __builtin_memcpy(id, u.internal, sizeof(u.internal));
  return rc;
}

int pert_comm_init(const uint8_t* id, int32_t n, int32_t world, int32_t rank, pert_comm** out) {
  if (!id || n != (int32_t)sizeof(ncclUniqueId) || !out || world < 1 || rank < 0 || rank >= world)
    return PERT_E_ARG;
  if (!g_rccl.handle) return PERT_E_COMM_UNAVAILABLE;
  *out = nullptr;
  ncclUniqueId u;
  __builtin_memcpy(u.internal, id, sizeof(u.internal));
  pert_comm* c = new pert_comm{nullptr, world, rank};
  const int rc = comm_status(g_rccl.init_rank(&c->comm, world, u, rank));   // collective: blocks for every rank
  if (rc != PERT_OK) {
    delete c;
    return rc;
  }
  *out = c;
  return PERT_OK;
}

int pert_comm_destroy(pert_comm* c) {
  if (!c) return PERT_OK;
  const int rc = g_rccl.handle ? comm_status(g_rccl.destroy(c->comm)) : PERT_E_COMM_UNAVAILABLE;
  delete c;
  return rc;
}

int pert_comm_allreduce_sum_f64(pert_comm* c, const double* send, double* recv, int64_t n, hipStream_t stream) {
  if (!c || !send || !recv || n < 0) return PERT_E_ARG;
  if (!g_rccl.handle) return PERT_E_COMM_UNAVAILABLE;
  if (n == 0) return PERT_OK;
  return comm_status(g_rccl.all_reduce(send, recv, (size_t)n, ncclFloat64, ncclSum, c->comm, stream));
}

}  // extern "C"
