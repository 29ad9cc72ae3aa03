// Native RCCL communicator (SURVEY.md §2.4 "Process group", §5.8): a thin C ABI over the
// RCCL collectives the engines use -- all-reduce, reduce-scatter, all-gather, broadcast,
// grouped send/recv -- issued on the caller's HIP stream, so a communicator built here
// rides the same xGMI rings as torch's "nccl" process group but without the c10d work
// objects, watchdog thread or per-call tensor checks on the hot path.
//
// RCCL is not linked: the library torch already loaded (torch/lib/librccl.so) is found with
// dlopen(RTLD_NOLOAD) -- or loaded from the path the caller passes -- and the entry points
// are resolved with dlsym, so the process keeps exactly one RCCL and one HIP runtime.
// The ncclUniqueId travels through torch.distributed's TCPStore rendezvous (Python side,
// parallel/native_comm.py), replacing the reference's implicit init_process_group("nccl")
// (main-ddp.py:26, main-fsdp.py:30).
#include <dlfcn.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#define DPC_API extern "C" __attribute__((visibility("default")))

namespace {

typedef int ncclResult_t;  // ncclSuccess = 0
typedef void* ncclComm_t;
typedef void* hipStream_t;
struct ncclUniqueId {
  char internal[128];
};

typedef ncclResult_t (*get_unique_id_t)(ncclUniqueId*);
typedef ncclResult_t (*comm_init_rank_t)(ncclComm_t*, int, ncclUniqueId, int);
typedef ncclResult_t (*comm_destroy_t)(ncclComm_t);
typedef ncclResult_t (*comm_abort_t)(ncclComm_t);
typedef ncclResult_t (*comm_split_t)(ncclComm_t, int, int, ncclComm_t*, void*);
typedef ncclResult_t (*comm_async_error_t)(ncclComm_t, ncclResult_t*);
typedef const char* (*error_string_t)(ncclResult_t);
typedef ncclResult_t (*all_reduce_t)(const void*, void*, size_t, int, int, ncclComm_t, hipStream_t);
typedef ncclResult_t (*reduce_scatter_t)(const void*, void*, size_t, int, int, ncclComm_t, hipStream_t);
typedef ncclResult_t (*all_gather_t)(const void*, void*, size_t, int, ncclComm_t, hipStream_t);
typedef ncclResult_t (*broadcast_t)(const void*, void*, size_t, int, int, ncclComm_t, hipStream_t);
typedef ncclResult_t (*send_t)(const void*, size_t, int, int, ncclComm_t, hipStream_t);
typedef ncclResult_t (*recv_t)(void*, size_t, int, int, ncclComm_t, hipStream_t);
typedef ncclResult_t (*group_t)();

struct Rccl {
  void* handle = nullptr;
  get_unique_id_t get_unique_id = nullptr;
  comm_init_rank_t comm_init_rank = nullptr;
  comm_destroy_t comm_destroy = nullptr;
  comm_abort_t comm_abort = nullptr;
  comm_split_t comm_split = nullptr;
  comm_async_error_t comm_async_error = nullptr;
  error_string_t error_string = nullptr;
  all_reduce_t all_reduce = nullptr;
  reduce_scatter_t reduce_scatter = nullptr;
  all_gather_t all_gather = nullptr;
  broadcast_t broadcast = nullptr;
  send_t send = nullptr;
  recv_t recv = nullptr;
  group_t group_start = nullptr;
  group_t group_end = nullptr;
};

Rccl g;
char g_err[512];
constexpr ncclResult_t kInProgress = 7;  // ncclInProgress: a non-blocking call still running

template <typename F>
bool sym(F& f, const char* name) {
  f = reinterpret_cast<F>(dlsym(g.handle, name));
  if (!f) snprintf(g_err, sizeof(g_err), "RCCL symbol %s not found", name);
  return f != nullptr;
}

}  // namespace

// Resolve RCCL: prefer the copy already mapped into the process (torch's), else dlopen(path).
// force != 0: dlopen(path) only (the CPU tests' fake library).  Returns 0 on success;
// dpc_rccl_error() explains a failure.
DPC_API int dpc_rccl_load(const char* path, int force) {
  if (g.handle) return 0;
  void* h = force ? nullptr : dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
  if (!h && path && *path) h = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
  if (!h) {
    snprintf(g_err, sizeof(g_err), "cannot load RCCL (%s): %s", path ? path : "", dlerror());
    return 1;
  }
  g.handle = h;
  bool ok = sym(g.get_unique_id, "ncclGetUniqueId") && sym(g.comm_init_rank, "ncclCommInitRank") &&
            sym(g.comm_destroy, "ncclCommDestroy") && sym(g.comm_abort, "ncclCommAbort") &&
            sym(g.comm_async_error, "ncclCommGetAsyncError") &&
            sym(g.error_string, "ncclGetErrorString") && sym(g.all_reduce, "ncclAllReduce") &&
            sym(g.reduce_scatter, "ncclReduceScatter") && sym(g.all_gather, "ncclAllGather") &&
            sym(g.broadcast, "ncclBroadcast") && sym(g.send, "ncclSend") && sym(g.recv, "ncclRecv") &&
            sym(g.group_start, "ncclGroupStart") && sym(g.group_end, "ncclGroupEnd");
  g.comm_split = reinterpret_cast<comm_split_t>(dlsym(h, "ncclCommSplit"));  // optional
  if (!ok) {
    g.handle = nullptr;
    return 2;
  }
  return 0;
}

DPC_API const char* dpc_rccl_error() { return g_err; }

static int check(ncclResult_t r, const char* what) {
  if (r != 0) snprintf(g_err, sizeof(g_err), "%s: %s", what, g.error_string ? g.error_string(r) : "RCCL error");
  return r;
}

DPC_API int dpc_rccl_unique_id(char* out128) {
  if (!g.handle) return -1;
  ncclUniqueId id;
  const int r = check(g.get_unique_id(&id), "ncclGetUniqueId");
  if (r == 0) memcpy(out128, id.internal, 128);
  return r;
}

// The caller has made the target device current (torch.cuda.set_device).
DPC_API int dpc_rccl_init(const char* id128, int nranks, int rank, void** comm) {
  if (!g.handle) return -1;
  ncclUniqueId id;
  memcpy(id.internal, id128, 128);
  ncclComm_t c = nullptr;
  const int r = check(g.comm_init_rank(&c, nranks, id, rank), "ncclCommInitRank");
  *comm = c;
  return r;
}

DPC_API int dpc_rccl_split(void* comm, int color, int key, void** out) {
  if (!g.handle || !g.comm_split) return -1;
  ncclComm_t c = nullptr;
  const int r = check(g.comm_split(comm, color, key, &c, nullptr), "ncclCommSplit");
  *out = c;
  return r;
}

int wd_destroy_locked(void* comm);  // below: unregisters from the watchdog, then destroys

DPC_API int dpc_rccl_destroy(void* comm) { return g.handle ? wd_destroy_locked(comm) : -1; }

DPC_API int dpc_rccl_abort(void* comm) { return g.handle ? check(g.comm_abort(comm), "ncclCommAbort") : -1; }

DPC_API int dpc_rccl_async_error(void* comm) {
  if (!g.handle) return -1;
  ncclResult_t e = 0;
  const int r = g.comm_async_error(comm, &e);
  return r ? r : (e == kInProgress ? 0 : check(e, "async"));
}

DPC_API int dpc_rccl_all_reduce(void* comm, const void* send, void* recv, size_t count, int dtype, int op,
                                void* stream) {
  return check(g.all_reduce(send, recv, count, dtype, op, comm, stream), "ncclAllReduce");
}

DPC_API int dpc_rccl_reduce_scatter(void* comm, const void* send, void* recv, size_t recvcount, int dtype,
                                    int op, void* stream) {
  return check(g.reduce_scatter(send, recv, recvcount, dtype, op, comm, stream), "ncclReduceScatter");
}

DPC_API int dpc_rccl_all_gather(void* comm, const void* send, void* recv, size_t sendcount, int dtype,
                                void* stream) {
  return check(g.all_gather(send, recv, sendcount, dtype, comm, stream), "ncclAllGather");
}

DPC_API int dpc_rccl_broadcast(void* comm, const void* send, void* recv, size_t count, int dtype, int root,
                               void* stream) {
  return check(g.broadcast(send, recv, count, dtype, root, comm, stream), "ncclBroadcast");
}

DPC_API int dpc_rccl_send(void* comm, const void* buf, size_t count, int dtype, int peer, void* stream) {
  return check(g.send(buf, count, dtype, peer, comm, stream), "ncclSend");
}

DPC_API int dpc_rccl_recv(void* comm, void* buf, size_t count, int dtype, int peer, void* stream) {
  return check(g.recv(buf, count, dtype, peer, comm, stream), "ncclRecv");
}

DPC_API int dpc_rccl_group_start() { return g.handle ? check(g.group_start(), "ncclGroupStart") : -1; }
DPC_API int dpc_rccl_group_end() { return g.handle ? check(g.group_end(), "ncclGroupEnd") : -1; }

// ---------------------------------------------------------------- collective watchdog
// the reference gets a c10d watchdog and destroy_process_group
// (/root/reference/main-ddp.py:26,34-35).  The engines' collectives bypass c10d, so this
// thread is their watchdog: every collective the transport enqueues is followed by an event
// on the comm stream (dpc_wd_track); the thread polls those events (hipEventQuery) and every
// registered communicator's asynchronous error (ncclCommGetAsyncError).  A collective still
// pending after the deadline, or an RCCL error, aborts every registered communicator
// (ncclCommAbort, which also releases kernels spinning on a dead peer) and ends the process
// with a non-zero status, so torchrun tears the job down instead of hanging forever.  It never
// restarts anything itself.  HIP is resolved like RCCL (the runtime torch already mapped), so
// this library still links neither.
namespace {

typedef int hipError_t;
typedef void* hipEvent_t;
typedef hipError_t (*ev_create_t)(hipEvent_t*, unsigned);
typedef hipError_t (*ev_record_t)(hipEvent_t, hipStream_t);
typedef hipError_t (*ev_query_t)(hipEvent_t);
typedef hipError_t (*ev_destroy_t)(hipEvent_t);

struct Hip {
  void* handle = nullptr;
  ev_create_t create = nullptr;
  ev_record_t record = nullptr;
  ev_query_t query = nullptr;
  ev_destroy_t destroy = nullptr;
};
Hip gh;
constexpr hipError_t kHipNotReady = 600;
constexpr unsigned kEventDisableTiming = 2;

struct Pending {
  hipEvent_t ev;
  std::chrono::steady_clock::time_point t0;
  std::string desc;
};

struct Watchdog {
  std::mutex mu;
  // held across "unregister + ncclCommDestroy" by the owner and across "copy + ncclCommAbort"
  // by wd_fire: the watchdog never aborts a communicator that is being (or has been) destroyed
  std::timed_mutex life;
  std::deque<Pending> q;
  std::vector<hipEvent_t> pool;  // completed events, re-recorded instead of re-created
  std::vector<ncclComm_t> comms;
  // set (under mu) by wd_fire when it aborts its copy of `comms`: a destroy that starts after it
  // parks instead of freeing a communicator that copy may still be aborting (wd_destroy_locked)
  bool aborting = false;
  std::thread th;
  std::atomic<bool> running{false};
  std::atomic<int> paused{0};
  double timeout_s = 1800.0;
  int poll_ms = 100;
  int exit_code = 17;
  int rank = 0;
};
// Never destroyed: the thread may outlive static destruction.  An atexit hook registered at
// start (so it runs BEFORE the HIP runtime's own teardown, registered earlier) joins it.
Watchdog& wd = *new Watchdog;

[[noreturn]] void wd_fire(const std::string& why) {
  fprintf(stderr, "[dpc watchdog] rank %d: %s; aborting %zu RCCL communicator(s) and exiting with status %d\n",
          wd.rank, why.c_str(), wd.comms.size(), wd.exit_code);
  fflush(stderr);
  // ncclCommAbort can itself wait on a wedged device: give it a bounded time, then leave anyway.
  // A destroy in progress on the main thread holds `life` (so no communicator is aborted while
  // it is being freed).  If that destroy does not finish within 2 s -- e.g. ncclCommDestroy
  // waiting on the very collective that hung -- every OTHER registered communicator is still
  // aborted: the one being destroyed was unregistered under `mu` before its destroy began (and
  // the owner destroys one communicator at a time), so the copy below never holds it.
  std::vector<ncclComm_t> comms;
  const bool owned = wd.life.try_lock_for(std::chrono::seconds(2));
  {
    std::lock_guard<std::mutex> lk(wd.mu);
    comms = wd.comms;
    wd.aborting = true;  // (no later destroy touches a communicator of this copy)
  }  // (`life`, when taken, stays held: this thread ends the process)
  if (!owned) {
    fprintf(stderr, "[dpc watchdog] rank %d: a communicator destroy is stuck; aborting the other %zu\n", wd.rank,
            comms.size());
    fflush(stderr);
  }
  std::atomic<bool> done{false};
  std::thread ab([&comms, &done] {
    for (ncclComm_t c : comms)
      if (g.comm_abort) g.comm_abort(c);
    done = true;
  });
  ab.detach();
  for (int i = 0; i < 100 && !done; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(100));
  fprintf(stderr, "[dpc watchdog] rank %d: communicators %s\n", wd.rank, done ? "aborted" : "abort timed out");
  fflush(stderr);
  _exit(wd.exit_code);
}

void wd_loop() {
  while (wd.running) {
    std::this_thread::sleep_for(std::chrono::milliseconds(wd.poll_ms));
    if (wd.paused) continue;  // a HIP-graph capture is running: no HIP calls from this thread
    std::string why;
    {
      std::lock_guard<std::mutex> lk(wd.mu);
      const auto now = std::chrono::steady_clock::now();
      for (auto it = wd.q.begin(); it != wd.q.end();) {
        const hipError_t r = gh.query(it->ev);
        if (r == 0) {
          wd.pool.push_back(it->ev);
          it = wd.q.erase(it);
          continue;
        }
        const double age = std::chrono::duration<double>(now - it->t0).count();
        if (r != kHipNotReady) {
          why = "HIP error " + std::to_string(r) + " waiting for " + it->desc;
          break;
        }
        if (age > wd.timeout_s) {
          char b[96];
          snprintf(b, sizeof(b), " still pending after %.1f s (timeout %.1f s)", age, wd.timeout_s);
          why = "collective " + it->desc + b;
          break;
        }
        ++it;
      }
      if (why.empty() && g.comm_async_error) {
        for (ncclComm_t c : wd.comms) {
          ncclResult_t e = 0;
          if (g.comm_async_error(c, &e) == 0 && e != 0 && e != kInProgress) {
            why = std::string("RCCL asynchronous error: ") + (g.error_string ? g.error_string(e) : "?");
            break;
          }
        }
      }
    }
    if (!why.empty()) wd_fire(why);
  }
}

}  // namespace

// Resolve the HIP event entry points (the runtime already in the process unless force).
DPC_API int dpc_hip_load(const char* path, int force) {
  if (gh.handle) return 0;
  void* h = force ? nullptr : dlopen("libamdhip64.so", RTLD_NOW | RTLD_NOLOAD);
  if (!h && path && *path) h = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
  if (!h) {
    snprintf(g_err, sizeof(g_err), "cannot load HIP (%s): %s", path ? path : "", dlerror());
    return 1;
  }
  gh.handle = h;
  gh.create = reinterpret_cast<ev_create_t>(dlsym(h, "hipEventCreateWithFlags"));
  gh.record = reinterpret_cast<ev_record_t>(dlsym(h, "hipEventRecord"));
  gh.query = reinterpret_cast<ev_query_t>(dlsym(h, "hipEventQuery"));
  gh.destroy = reinterpret_cast<ev_destroy_t>(dlsym(h, "hipEventDestroy"));
  if (!gh.create || !gh.record || !gh.query || !gh.destroy) {
    snprintf(g_err, sizeof(g_err), "HIP event entry points not found");
    gh = Hip();
    return 2;
  }
  return 0;
}

static void dpc_wd_stop_at_exit() {
  if (!wd.running) return;
  wd.running = false;
  if (wd.th.joinable()) wd.th.join();
}

// Start the watchdog thread (idempotent; the first call's settings hold).
DPC_API int dpc_wd_start(double timeout_s, int poll_ms, int rank, int exit_code) {
  if (!gh.handle) return -1;
  std::lock_guard<std::mutex> lk(wd.mu);
  if (wd.running) return 0;
  wd.timeout_s = timeout_s;
  wd.poll_ms = poll_ms > 0 ? poll_ms : 100;
  wd.rank = rank;
  wd.exit_code = exit_code;
  wd.running = true;
  wd.th = std::thread(wd_loop);
  static bool hooked = false;
  if (!hooked) {
    hooked = true;
    atexit(dpc_wd_stop_at_exit);
  }
  return 0;
}

DPC_API int dpc_wd_running() { return wd.running ? 1 : 0; }

DPC_API void dpc_wd_register(void* comm) {
  std::lock_guard<std::mutex> lk(wd.mu);
  wd.comms.push_back(comm);
}

DPC_API void dpc_wd_unregister(void* comm) {
  std::lock_guard<std::mutex> lk(wd.mu);
  for (auto it = wd.comms.begin(); it != wd.comms.end(); ++it)
    if (*it == comm) {
      wd.comms.erase(it);
      break;
    }
}

int wd_destroy_locked(void* comm) {
  std::lock_guard<std::timed_mutex> life(wd.life);
  bool aborting;
  {
    std::lock_guard<std::mutex> lk(wd.mu);
    aborting = wd.aborting;
  }
  // the watchdog took its copy while an earlier destroy was stuck (it could not take `life`) and
  // may be aborting this very communicator now: never destroy it concurrently -- park until the
  // watchdog's _exit (at most ~10 s away)
  while (aborting) std::this_thread::sleep_for(std::chrono::seconds(1));
  dpc_wd_unregister(comm);
  return check(g.comm_destroy(static_cast<ncclComm_t>(comm)), "ncclCommDestroy");
}

// Record an event behind the work just enqueued on `stream` and watch it.  Not during a
// stream capture (the caller checks): the event would become a graph node.
DPC_API int dpc_wd_track(void* stream, const char* desc) {
  if (!wd.running) return -1;
  std::lock_guard<std::mutex> lk(wd.mu);
  hipEvent_t ev = nullptr;
  if (!wd.pool.empty()) {
    ev = wd.pool.back();
    wd.pool.pop_back();
  } else if (gh.create(&ev, kEventDisableTiming) != 0) {
    return -2;
  }
  if (gh.record(ev, stream) != 0) {
    gh.destroy(ev);
    return -3;
  }
  wd.q.push_back(Pending{ev, std::chrono::steady_clock::now(), desc ? desc : "collective"});
  return 0;
}

DPC_API int dpc_wd_pending() {
  std::lock_guard<std::mutex> lk(wd.mu);
  return (int)wd.q.size();
}

// pause != 0 while a HIP graph is being captured (no HIP call from the watchdog thread then)
DPC_API void dpc_wd_pause(int pause) { wd.paused = pause; }

DPC_API void dpc_wd_stop() {
  if (!wd.running) return;
  wd.running = false;
  if (wd.th.joinable()) wd.th.join();
  std::lock_guard<std::mutex> lk(wd.mu);
  for (auto& p : wd.q) gh.destroy(p.ev);
  for (hipEvent_t e : wd.pool) gh.destroy(e);
  wd.q.clear();
  wd.pool.clear();
  wd.comms.clear();
}
