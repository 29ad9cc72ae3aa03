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
#include <string.h>

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

template <typename F>
bool sym(F& f, const char* name) {
  f = reinterpret_cast<F>(dlsym(g.handle, name));
  if (!f) snprintf(g_err, sizeof(g_err), "RCCL symbol %s not found", name);
  return f != nullptr;
}

}  // namespace

// Resolve RCCL: prefer the copy already mapped into the process (torch's), else dlopen(path).
// Returns 0 on success; dpc_rccl_error() explains a failure.
DPC_API int dpc_rccl_load(const char* path) {
  if (g.handle) return 0;
  void* h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
  if (!h && path && *path) h = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
  if (!h) {
    snprintf(g_err, sizeof(g_err), "cannot load RCCL (%s): %s", path ? path : "", dlerror());
    return 1;
  }
  g.handle = h;
  bool ok = sym(g.get_unique_id, "ncclGetUniqueId") && sym(g.comm_init_rank, "ncclCommInitRank") &&
            sym(g.comm_destroy, "ncclCommDestroy") && sym(g.comm_async_error, "ncclCommGetAsyncError") &&
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

DPC_API int dpc_rccl_destroy(void* comm) { return g.handle ? check(g.comm_destroy(comm), "ncclCommDestroy") : -1; }

DPC_API int dpc_rccl_async_error(void* comm) {
  if (!g.handle) return -1;
  ncclResult_t e = 0;
  const int r = g.comm_async_error(comm, &e);
  return r ? r : check(e, "async");
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
