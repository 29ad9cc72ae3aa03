// Host-only stand-in for librccl + the HIP event API, for the CPU tests of the native
// communicator's bring-up agreement, collective fingerprints and watchdog
// (runtime/csrc/rccl_comm.cpp).  Built by the tests with g++; never loaded on a GPU box.
// Behaviour is chosen per process with environment variables:
//   FAKE_UID_FAIL=1      ncclGetUniqueId fails
//   FAKE_INIT_FAIL=1     ncclCommInitRank fails
//   FAKE_EVENT_STALL=1   hipEventQuery never reports completion (a hung collective)
//   FAKE_ASYNC_ERR=<n>   ncclCommGetAsyncError reports error n
//   FAKE_ABORT_MARK=path ncclCommAbort appends "abort" to that file
//   FAKE_LOG=path        every collective appends its name to that file
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

extern "C" {

typedef int ncclResult_t;
struct ncclUniqueId {
  char internal[128];
};

static int env_on(const char* n) {
  const char* v = getenv(n);
  return v && *v && strcmp(v, "0") != 0;
}

static void log_op(const char* what) {
  const char* p = getenv("FAKE_LOG");
  if (!p) return;
  FILE* f = fopen(p, "a");
  if (!f) return;
  fprintf(f, "%s\n", what);
  fclose(f);
}

static int g_comms[64];
static int g_next = 0;

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  if (env_on("FAKE_UID_FAIL")) return 3;
  memset(id->internal, 7, sizeof(id->internal));
  return 0;
}
ncclResult_t ncclCommInitRank(void** comm, int, ncclUniqueId, int) {
  if (env_on("FAKE_INIT_FAIL")) return 2;
  *comm = &g_comms[g_next++ % 64];
  return 0;
}
ncclResult_t ncclCommSplit(void*, int, int, void** out, void*) {
  *out = &g_comms[g_next++ % 64];
  return 0;
}
ncclResult_t ncclCommDestroy(void*) {
  log_op("destroy");
  return 0;
}
ncclResult_t ncclCommAbort(void*) {
  const char* p = getenv("FAKE_ABORT_MARK");
  if (p) {
    FILE* f = fopen(p, "a");
    if (f) {
      fprintf(f, "abort\n");
      fclose(f);
    }
  }
  return 0;
}
ncclResult_t ncclCommGetAsyncError(void*, ncclResult_t* e) {
  const char* v = getenv("FAKE_ASYNC_ERR");
  *e = v ? atoi(v) : 0;
  return 0;
}
const char* ncclGetErrorString(ncclResult_t) { return "fake RCCL error"; }
ncclResult_t ncclAllReduce(const void*, void*, size_t, int, int, void*, void*) {
  log_op("all_reduce");
  return 0;
}
ncclResult_t ncclReduceScatter(const void*, void*, size_t, int, int, void*, void*) {
  log_op("reduce_scatter");
  return 0;
}
ncclResult_t ncclAllGather(const void*, void*, size_t, int, void*, void*) {
  log_op("all_gather");
  return 0;
}
ncclResult_t ncclBroadcast(const void*, void*, size_t, int, int, void*, void*) {
  log_op("broadcast");
  return 0;
}
ncclResult_t ncclSend(const void*, size_t, int, int, void*, void*) {
  log_op("send");
  return 0;
}
ncclResult_t ncclRecv(void*, size_t, int, int, void*, void*) {
  log_op("recv");
  return 0;
}
ncclResult_t ncclGroupStart() { return 0; }
ncclResult_t ncclGroupEnd() { return 0; }

// ---- HIP events
static int g_events[4096];
static int g_ev = 0;
int hipEventCreateWithFlags(void** ev, unsigned) {
  *ev = &g_events[g_ev++ % 4096];
  return 0;
}
int hipEventRecord(void*, void*) { return 0; }
int hipEventQuery(void*) { return env_on("FAKE_EVENT_STALL") ? 600 : 0; }
int hipEventDestroy(void*) { return 0; }

}  // extern "C"
