// pert_comm.hip -- the cross-rank sum of a sharded fit's shared-gradient block, issued by the
// library itself, so a sharded SVI loop runs as GIL-free C calls (pert_svi_run_sharded) with the
// all-reduce queued on the fit's stream between the reductions and Adam, like the single-rank loop.
//
// Two backends behind one pert_comm handle:
//   * RCCL (the product path): an RCCL communicator over the fit's ranks (one process per GPU,
//     xGMI).  RCCL is not linked: pert_comm_load() dlopens the copy the process already has
//     (torch's, which libtorch_hip links), so the communicator and torch's process group use one
//     RCCL.  Only the types of rccl.h are used here.
//   * host-staged (pert_comm_init_host; tests, and ranks that share a GPU, which RCCL refuses):
//     the block is copied to pinned host memory, a host function queued on the stream adds the
//     ranks' blocks through a POSIX shared-memory segment in fixed rank order, and the sum is
//     copied back -- the same place in the stream as the RCCL call, so the loop is unchanged.
//
// Failure is bounded on both: every comm has an abort word shared by the ranks of the node
// (the host backend's segment, or one attached by pert_comm_set_watchdog), a rank whose loop
// fails raises it (pert_comm_abort), and a rank waiting on its stream polls it, RCCL's async
// error and a deadline instead of blocking (pert_comm_wait_event), aborting its RCCL
// communicator so its queued collectives return.
//
// Reference: pert_model.py:800-816 runs svi_s.step() on one CPU process; the shard/all-reduce
// decomposition is SURVEY.md section 8e.
#include <dlfcn.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstring>
#include <mutex>

#include "pert_hip.h"

namespace {

constexpr int kKindRccl = 0, kKindHost = 1;
constexpr double kDefaultTimeoutS = 600.0;

// a node-local segment shared by the ranks: the header (one cache line each for the attach
// count, the abort word and every rank's arrival generation), then for the host backend two
// generations of every rank's block
struct alignas(64) Line {
  std::atomic<int64_t> v;
  char pad[64 - sizeof(std::atomic<int64_t>)];
};
static_assert(sizeof(Line) == 64, "one counter per cache line");
static_assert(std::atomic<int64_t>::is_always_lock_free, "cross-process atomics must be lock-free");

struct Segment {
  void* base = nullptr;
  size_t bytes = 0;
  int32_t world = 0;
  int64_t max_n = 0;
  Line* lines() const { return static_cast<Line*>(base); }
  std::atomic<int64_t>& attached() const { return lines()[0].v; }
  std::atomic<int64_t>& abort_word() const { return lines()[1].v; }
  std::atomic<int64_t>& arrive(int r) const { return lines()[2 + r].v; }
  double* block(int64_t gen, int r) const {
    double* d = reinterpret_cast<double*>(lines() + 2 + world);
    return d + ((gen & 1) * world + r) * max_n;
  }
  static size_t size_for(int32_t world, int64_t max_n) {
    return sizeof(Line) * (2 + (size_t)world) + sizeof(double) * 2 * (size_t)world * (size_t)max_n;
  }
};

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

// spin briefly, then yield, then sleep: the wait between two ranks' arrivals is microseconds
// in a fit, but a rank may wait seconds for a peer still setting up
void backoff(int64_t k) {
  if (k < 256) return;
  if (k < 4096) {
    sched_yield();
    return;
  }
  timespec ts{0, 50000};
  nanosleep(&ts, nullptr);
}

// Map the segment `name` (every rank calls; created by whichever comes first, zero-filled),
// then wait until all `world` ranks have mapped it and unlink the name (rank 0), so nothing is
// left in /dev/shm however the fit ends.
int attach_segment(const char* name, int32_t world, int32_t rank, int64_t max_n, double timeout_s, Segment* out) {
  if (!name || name[0] != '/' || std::strlen(name) > 200) return PERT_E_ARG;
  const size_t bytes = Segment::size_for(world, max_n);
  const int fd = shm_open(name, O_CREAT | O_RDWR, 0600);
  if (fd < 0) return PERT_E_COMM_UNAVAILABLE;
  struct stat sb;
  if (fstat(fd, &sb) != 0 || ((size_t)sb.st_size != bytes && ftruncate(fd, (off_t)bytes) != 0)) {
    close(fd);
    return PERT_E_COMM_UNAVAILABLE;
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return PERT_E_COMM_UNAVAILABLE;
  Segment s;
  s.base = p;
  s.bytes = bytes;
  s.world = world;
  s.max_n = max_n;
  s.attached().fetch_add(1, std::memory_order_acq_rel);
  const double t0 = now_s();
  for (int64_t k = 0; s.attached().load(std::memory_order_acquire) < world; ++k) {
    if (now_s() - t0 > timeout_s) {
      munmap(p, bytes);
      shm_unlink(name);                       // (every rank: a late one may have re-created it)
      return PERT_E_COMM_TIMEOUT;
    }
    backoff(k);
  }
  if (rank == 0) shm_unlink(name);
  *out = s;
  return PERT_OK;
}

struct Rccl {
  void* handle = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclCommAbort) abort = nullptr;
  decltype(&ncclCommGetAsyncError) async_error = nullptr;
};

Rccl g_rccl;
std::mutex g_mu;

int comm_status(ncclResult_t r) { return r == ncclSuccess ? PERT_OK : PERT_E_COMM_BASE + (int)r; }

}  // namespace

struct pert_comm {
  int32_t kind;
  int32_t world, rank;
  ncclComm_t nccl = nullptr;            // RCCL backend (nullptr once aborted)
  Segment seg;                          // host backend's segment, or the watchdog's abort word
  bool own_abort_word = false;          // seg mapped (host backend, or a watchdog segment)
  std::atomic<int64_t> local_abort{0};  // the abort word when no segment is attached
  std::atomic<int32_t> failed{0};       // this rank's first failure (PERT_OK = none)
  double timeout_s = kDefaultTimeoutS;
  int64_t fault_at = -1;                // test hook: the all-reduce call of this index fails
  int64_t n_calls = 0;                  // all-reduce calls queued
  // the split step's overlap (pert_comm_allreduce_async / pert_comm_join): a side stream and
  // two events, made on first use on the current device.  Off by default: on ROCm 7.2 each
  // cross-stream hop costs ~14 us (tools/xstream_probe.py) and RCCL on the side stream made the
  // 1,250-cell step 0.42 -> 0.69 ms, more than the per-cell work it hides
  int32_t overlap = 0;
  int64_t delay_ticks = 0;              // stand-in latency (pert_comm_set_options), 100 MHz ticks
  hipStream_t side = nullptr;
  hipEvent_t ev_sums = nullptr, ev_done = nullptr;
  // host backend
  double* pin_send = nullptr;
  double* pin_recv = nullptr;
  int64_t gen = 0;                      // host functions run (stream order)

  std::atomic<int64_t>& abort_word() { return seg.base ? seg.abort_word() : local_abort; }
};

namespace {

// first failure wins; raising the shared word stops the peers' waits too
void fail(pert_comm* c, int code) {
  int32_t expect = 0;
  c->failed.compare_exchange_strong(expect, code);
  int64_t z = 0;
  c->abort_word().compare_exchange_strong(z, (int64_t)code);
}

int poll_failure(pert_comm* c) {
  const int f = c->failed.load(std::memory_order_acquire);
  if (f) return f;
  const int64_t a = c->abort_word().load(std::memory_order_acquire);
  if (a) {
    fail(c, PERT_E_COMM_ABORTED);
    return PERT_E_COMM_ABORTED;
  }
  if (c->kind == kKindRccl && c->nccl && g_rccl.async_error) {
    ncclResult_t r = ncclSuccess;
    if (g_rccl.async_error(c->nccl, &r) == ncclSuccess && r != ncclSuccess && r != ncclInProgress) {
      fail(c, comm_status(r));
      return comm_status(r);
    }
  }
  return PERT_OK;
}

// the stand-in for a ring's latency (pert_comm_set_options): one wave spinning on the
// device's constant 100 MHz clock
__global__ void delay_kernel(int64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) __builtin_amdgcn_s_sleep(1);
}

int hip_rc(hipError_t e) { return e == hipSuccess ? PERT_OK : PERT_E_HIP_BASE + (int)e; }

struct HostCall {
  pert_comm* c;
  int64_t n;
};

// The host backend's sum, run by the HIP runtime in stream order after the block's copy to
// c->pin_send: publish it for generation g, wait for every rank's, add them in rank order (the
// same bits on every rank), leave the sum in c->pin_recv for the copy back.  A failure or a peer's
// abort leaves the stream running (the copies and kernels behind it see a stale sum) with the
// comm failed; the waiting host loop then returns the failure.
void host_sum(void* arg) {
  const HostCall call = *static_cast<HostCall*>(arg);
  delete static_cast<HostCall*>(arg);
  pert_comm* c = call.c;
  if (c->failed.load(std::memory_order_acquire)) return;
  const int64_t g = ++c->gen;
  const Segment& s = c->seg;
  std::memcpy(s.block(g, c->rank), c->pin_send, sizeof(double) * call.n);
  s.arrive(c->rank).store(g, std::memory_order_release);
  const double t0 = now_s();
  for (int r = 0; r < s.world; ++r) {
    for (int64_t k = 0; s.arrive(r).load(std::memory_order_acquire) < g; ++k) {
      if (s.abort_word().load(std::memory_order_acquire)) {
        fail(c, PERT_E_COMM_ABORTED);
        return;
      }
      if ((k & 255) == 255 && now_s() - t0 > c->timeout_s) {
        fail(c, PERT_E_COMM_TIMEOUT);
        return;
      }
      backoff(k);
    }
  }
  double* out = c->pin_recv;
  std::memcpy(out, s.block(g, 0), sizeof(double) * call.n);
  for (int r = 1; r < s.world; ++r) {
    const double* b = s.block(g, r);
    for (int64_t i = 0; i < call.n; ++i) out[i] += b[i];
  }
}

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
  r.abort = reinterpret_cast<decltype(r.abort)>(dlsym(h, "ncclCommAbort"));
  r.async_error = reinterpret_cast<decltype(r.async_error)>(dlsym(h, "ncclCommGetAsyncError"));
  if (!r.get_unique_id || !r.init_rank || !r.all_reduce || !r.destroy || !r.abort || !r.async_error) {
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
  pert_comm* c = new pert_comm;
  c->kind = kKindRccl;
  c->world = world;
  c->rank = rank;
  const int rc = comm_status(g_rccl.init_rank(&c->nccl, world, u, rank));   // collective: blocks for every rank
  if (rc != PERT_OK) {
    delete c;
    return rc;
  }
  *out = c;
  return PERT_OK;
}

int pert_comm_init_host(const char* name, int32_t world, int32_t rank, int64_t max_n, double timeout_s,
                        pert_comm** out) {
  if (!out || world < 1 || world > 64 || rank < 0 || rank >= world || max_n < 1 || !(timeout_s > 0.0))
    return PERT_E_ARG;
  *out = nullptr;
  pert_comm* c = new pert_comm;
  c->kind = kKindHost;
  c->world = world;
  c->rank = rank;
  c->timeout_s = timeout_s;
  int rc = attach_segment(name, world, rank, max_n, timeout_s, &c->seg);
  if (rc != PERT_OK) {
    delete c;
    return rc;
  }
  c->own_abort_word = true;
  *out = c;                                   // (the pinned buffers come with the first all-reduce)
  return PERT_OK;
}

int pert_comm_set_watchdog(pert_comm* c, const char* abort_name, double timeout_s) {
  if (!c || !(timeout_s > 0.0)) return PERT_E_ARG;
  c->timeout_s = timeout_s;
  if (!abort_name || c->own_abort_word) return PERT_OK;   // the host backend's segment has one
  Segment s;
  const int rc = attach_segment(abort_name, c->world, c->rank, 1, timeout_s, &s);
  if (rc != PERT_OK) return rc;
  c->seg = s;
  c->own_abort_word = true;
  return PERT_OK;
}

int pert_comm_inject_fault(pert_comm* c, int64_t at_call) {
  if (!c) return PERT_E_ARG;
  c->fault_at = at_call;
  return PERT_OK;
}

int pert_comm_status(pert_comm* c) {
  if (!c) return PERT_E_ARG;
  return poll_failure(c);
}

int pert_comm_abort(pert_comm* c, int32_t code) {
  if (!c) return PERT_E_ARG;
  fail(c, code != PERT_OK ? code : PERT_E_COMM_ABORTED);
  if (c->kind == kKindRccl && c->nccl && g_rccl.abort) {
    (void)g_rccl.abort(c->nccl);            // its queued collectives return; the comm is gone
    c->nccl = nullptr;
  }
  return PERT_OK;
}

int pert_comm_wait_event(pert_comm* c, hipEvent_t ev, int32_t eager) {
  if (!ev) return PERT_E_ARG;
  if (!c && !eager) {
    const hipError_t e = hipEventSynchronize(ev);
    return e == hipSuccess ? PERT_OK : PERT_E_HIP_BASE + (int)e;
  }
  const double t0 = now_s();
  for (int64_t k = 0;; ++k) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return c ? poll_failure(c) : PERT_OK;
    if (q != hipErrorNotReady) return PERT_E_HIP_BASE + (int)q;
    if (!c) {                                   // eager, no comm: poll, yielding the core
      if (k >= 256) sched_yield();
      continue;
    }
    int rc = poll_failure(c);
    if (rc == PERT_OK && (k & 63) == 63 && now_s() - t0 > c->timeout_s) {
      fail(c, PERT_E_COMM_TIMEOUT);
      rc = PERT_E_COMM_TIMEOUT;
    }
    if (rc != PERT_OK) {
      // stop this rank's collectives so its stream drains (the host backend's queued sums
      // return at once on a failed comm); the caller then synchronises the stream
      (void)pert_comm_abort(c, rc);
      return rc;
    }
    if (eager && k >= 256) sched_yield();
    else backoff(k);
  }
}

int pert_comm_set_options(pert_comm* c, int32_t overlap, double delay_us) {
  if (!c || delay_us < 0.0) return PERT_E_ARG;
  c->overlap = overlap ? 1 : 0;
  c->delay_ticks = (int64_t)(delay_us * 100.0 + 0.5);
  return PERT_OK;
}

int pert_comm_overlap(const pert_comm* c) { return c && c->overlap ? 1 : 0; }

int pert_comm_allreduce_async(pert_comm* c, const double* send, double* recv, int64_t n, hipStream_t stream) {
  if (!c) return PERT_E_ARG;
  if (!c->overlap) return pert_comm_allreduce_sum_f64(c, send, recv, n, stream);
  if (!c->side) {
    int lo = 0, hi = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&lo, &hi);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, hi);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_sums, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming);
    if (e != hipSuccess) return hip_rc(e);
  }
  int rc = hip_rc(hipEventRecord(c->ev_sums, stream));
  if (rc == PERT_OK) rc = hip_rc(hipStreamWaitEvent(c->side, c->ev_sums, 0));
  if (rc == PERT_OK) rc = pert_comm_allreduce_sum_f64(c, send, recv, n, c->side);
  if (rc == PERT_OK) rc = hip_rc(hipEventRecord(c->ev_done, c->side));
  return rc;
}

int pert_comm_join(pert_comm* c, hipStream_t stream) {
  if (!c) return PERT_E_ARG;
  if (!c->overlap || !c->side) return PERT_OK;
  return hip_rc(hipStreamWaitEvent(stream, c->ev_done, 0));
}

int pert_comm_destroy(pert_comm* c) {
  if (!c) return PERT_OK;
  int rc = PERT_OK;
  if (c->side) {
    (void)hipStreamSynchronize(c->side);
    (void)hipStreamDestroy(c->side);
    (void)hipEventDestroy(c->ev_sums);
    (void)hipEventDestroy(c->ev_done);
  }
  if (c->kind == kKindRccl && c->nccl)
    rc = g_rccl.handle ? comm_status(g_rccl.destroy(c->nccl)) : PERT_E_COMM_UNAVAILABLE;
  if (c->pin_send) (void)hipHostFree(c->pin_send);
  if (c->pin_recv) (void)hipHostFree(c->pin_recv);
  if (c->own_abort_word) munmap(c->seg.base, c->seg.bytes);
  delete c;
  return rc;
}

int pert_comm_allreduce_sum_f64(pert_comm* c, const double* send, double* recv, int64_t n, hipStream_t stream) {
  if (!c || !send || !recv || n < 0) return PERT_E_ARG;
  if (n == 0) return PERT_OK;
  const int64_t call = c->n_calls++;
  if (call == c->fault_at) return PERT_E_COMM_FAULT;          // test hook (pert_comm_inject_fault)
  const int f = c->failed.load(std::memory_order_acquire);
  if (f) return f;
  if (c->delay_ticks > 0) {
    hipLaunchKernelGGL(delay_kernel, dim3(1), dim3(64), 0, stream, c->delay_ticks);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_rc(e);
  }
  if (c->kind == kKindHost) {
    if (n > c->seg.max_n) return PERT_E_ARG;
    if (!c->pin_send) {
      hipError_t e = hipHostMalloc(&c->pin_send, sizeof(double) * c->seg.max_n, hipHostMallocDefault);
      if (e == hipSuccess) e = hipHostMalloc(&c->pin_recv, sizeof(double) * c->seg.max_n, hipHostMallocDefault);
      if (e != hipSuccess) {
        if (c->pin_send) (void)hipHostFree(c->pin_send);
        c->pin_send = c->pin_recv = nullptr;
        return hip_rc(e);
      }
    }
    hipError_t e = hipMemcpyAsync(c->pin_send, send, sizeof(double) * n, hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipLaunchHostFunc(stream, host_sum, new HostCall{c, n});
    if (e == hipSuccess) e = hipMemcpyAsync(recv, c->pin_recv, sizeof(double) * n, hipMemcpyHostToDevice, stream);
    return e == hipSuccess ? PERT_OK : PERT_E_HIP_BASE + (int)e;
  }
  if (!g_rccl.handle) return PERT_E_COMM_UNAVAILABLE;
  if (!c->nccl) return PERT_E_COMM_ABORTED;
  return comm_status(g_rccl.all_reduce(send, recv, (size_t)n, ncclFloat64, ncclSum, c->nccl, stream));
}

}  // extern "C"
