// Host-only stand-in for librccl + the HIP event API, for the CPU tests of the native
// communicator (runtime/csrc/rccl_comm.cpp, parallel/native_comm.py, parallel/transport.py).
// Built by the tests with g++; never loaded on a GPU box.  The "device" buffers of a CPU test
// are host tensors, so this library can move their bytes itself.
//
// Two modes, chosen per process:
//   FAKE_DIR unset   collectives succeed without touching buffers (bring-up, fingerprint,
//                    watchdog tests: a rank may post collectives its peers never match)
//   FAKE_DIR=<dir>   collectives MOVE DATA between the processes of a communicator through
//                    files in <dir> (one directory per test): the collective of sequence
//                    number s on communicator K is a rendezvous on the files K_s_<rank>, each
//                    holding a header (op, count, dtype, root) and the rank's send buffer;
//                    every rank reads all of them and computes its own output (reductions in
//                    rank order, f32 accumulation for bf16 / f16, rounded once).  A header
//                    that differs between ranks (op, count, dtype or root) fails the call:
//                    the fake doubles as a collective-matching checker.  Send / recv post into
//                    per-pair mailboxes K_p_<src>_<dst>_<n> (the n-th message from src to dst);
//                    a receive blocks until its message is there, consumes it and leaves an
//                    acknowledgement (<message>.ack).  A send COMPLETES only when that
//                    acknowledgement is there -- RCCL's rule: ncclSend blocks the stream until the
//                    peer's matching ncclRecv runs, and a group ends only when every operation of
//                    it has completed -- so an ungrouped send waits for its ack at the call, and
//                    inside ncclGroupStart / ncclGroupEnd every send is posted first, then the rest
//                    run in issue order (RCCL's fused group progresses them concurrently), then
//                    the group waits for the acks of all its sends.  An exchange whose order would
//                    deadlock on xGMI (each rank's send waiting for a receive the peer posts only
//                    after its own send completes) times out here instead of passing.  ncclCommSplit is a
//                    rendezvous on the parent that exchanges (color, key) and derives the
//                    child's key, rank (by key, then parent rank) and size.
// Other switches:
//   FAKE_UID_FAIL=1      ncclGetUniqueId fails
//   FAKE_INIT_FAIL=1     ncclCommInitRank fails
//   FAKE_EVENT_STALL=1   hipEventQuery never reports completion (a hung collective)
//   FAKE_ASYNC_ERR=<n>   ncclCommGetAsyncError reports error n
//   FAKE_ABORT_MARK=path ncclCommAbort appends "abort" to that file
//   FAKE_LOG=path        every collective appends its name to that file
//   FAKE_TIMEOUT_S=<s>   a rendezvous waits at most this long (default 120), then fails
//   FAKE_DESTROY_SLEEP=<s> ncclCommDestroy blocks this long (a destroy stuck on a hung peer)
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

extern "C" {

typedef int ncclResult_t;
struct ncclUniqueId {
  char internal[128];
};

}  // extern "C"

namespace {

int env_on(const char* n) {
  const char* v = getenv(n);
  return v && *v && strcmp(v, "0") != 0;
}

void log_op(const char* what) {
  const char* p = getenv("FAKE_LOG");
  if (!p) return;
  FILE* f = fopen(p, "a");
  if (!f) return;
  fprintf(f, "%s\n", what);
  fclose(f);
}

const char* data_dir() {
  const char* d = getenv("FAKE_DIR");
  return (d && *d) ? d : nullptr;
}

struct Comm {
  uint64_t key = 0;
  int nranks = 1, rank = 0;
  uint64_t seq = 0;     // collectives issued on this communicator
  uint64_t splits = 0;  // children split off it
  std::vector<uint64_t> sent, recvd;  // per peer: messages sent to / received from it
};

constexpr ncclResult_t kSystemError = 2, kInvalidUsage = 5;

struct Header {
  uint32_t magic, op;
  uint64_t count;
  int32_t dtype, root, rank, pad;
};
constexpr uint32_t kMagic = 0x46524343u;  // "FRCC"

size_t dsize(int dt) {
  switch (dt) {
    case 0: case 1: return 1;
    case 6: case 9: return 2;
    case 2: case 3: case 7: return 4;
    case 4: case 5: case 8: return 8;
    default: return 0;
  }
}

float bf16_to_f(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
uint16_t f_to_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // NaN stays NaN
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
float f16_to_f(uint16_t h) {
  const uint32_t s = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1f, m = h & 0x3ff;
  uint32_t u;
  if (e == 0) {
    if (m == 0) {
      u = s;
    } else {  // subnormal
      int ee = -1;
      uint32_t mm = m;
      do { ++ee; mm <<= 1; } while (!(mm & 0x400));
      u = s | ((uint32_t)(127 - 15 - ee) << 23) | ((mm & 0x3ff) << 13);
    }
  } else if (e == 31) {
    u = s | 0x7f800000u | (m << 13);
  } else {
    u = s | ((e + 112) << 23) | (m << 13);
  }
  float f;
  memcpy(&f, &u, 4);
  return f;
}
uint16_t f_to_f16(float f) {  // round to nearest even
  uint32_t u;
  memcpy(&u, &f, 4);
  const uint32_t s = (u >> 16) & 0x8000u;
  const int e = (int)((u >> 23) & 0xff) - 127 + 15;
  uint32_t m = u & 0x7fffffu;
  if (((u >> 23) & 0xff) == 0xff) return (uint16_t)(s | 0x7c00u | (m ? 0x200u : 0u));
  if (e >= 31) return (uint16_t)(s | 0x7c00u);
  if (e <= 0) {
    if (e < -10) return (uint16_t)s;
    m |= 0x800000u;
    const int sh = 14 - e;
    uint32_t r = m >> sh;
    const uint32_t rem = m & ((1u << sh) - 1), half = 1u << (sh - 1);
    if (rem > half || (rem == half && (r & 1))) ++r;
    return (uint16_t)(s | r);
  }
  uint32_t r = ((uint32_t)e << 10) | (m >> 13);
  const uint32_t rem = m & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (r & 1))) ++r;
  return (uint16_t)(s | r);
}

template <typename T, typename A>
void reduce_typed(void* out, const std::vector<const void*>& ins, size_t n, int op, A (*load)(T), T (*store)(A)) {
  T* o = static_cast<T*>(out);
  for (size_t i = 0; i < n; ++i) {
    A acc = load(static_cast<const T*>(ins[0])[i]);
    for (size_t r = 1; r < ins.size(); ++r) {
      const A v = load(static_cast<const T*>(ins[r])[i]);
      switch (op) {
        case 1: acc = acc * v; break;
        case 2: acc = v > acc ? v : acc; break;
        case 3: acc = v < acc ? v : acc; break;
        default: acc = acc + v; break;
      }
    }
    if (op == 4) acc = acc / (A)ins.size();
    o[i] = store(acc);
  }
}

template <typename T>
T ident(T v) { return v; }

bool reduce(void* out, const std::vector<const void*>& ins, size_t n, int dt, int op) {
  switch (dt) {
    case 0: reduce_typed<int8_t, int64_t>(out, ins, n, op, [](int8_t v) { return (int64_t)v; }, [](int64_t v) { return (int8_t)v; }); return true;
    case 1: reduce_typed<uint8_t, int64_t>(out, ins, n, op, [](uint8_t v) { return (int64_t)v; }, [](int64_t v) { return (uint8_t)v; }); return true;
    case 2: reduce_typed<int32_t, int64_t>(out, ins, n, op, [](int32_t v) { return (int64_t)v; }, [](int64_t v) { return (int32_t)v; }); return true;
    case 4: reduce_typed<int64_t, int64_t>(out, ins, n, op, ident<int64_t>, ident<int64_t>); return true;
    case 6: reduce_typed<uint16_t, float>(out, ins, n, op, f16_to_f, f_to_f16); return true;
    case 7: reduce_typed<float, float>(out, ins, n, op, ident<float>, ident<float>); return true;
    case 8: reduce_typed<double, double>(out, ins, n, op, ident<double>, ident<double>); return true;
    case 9: reduce_typed<uint16_t, float>(out, ins, n, op, bf16_to_f, f_to_bf16); return true;
    default: return false;
  }
}

double timeout_s() {
  const char* v = getenv("FAKE_TIMEOUT_S");
  return v ? atof(v) : 120.0;
}

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

std::string path_of(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
std::string path_of(const char* fmt, ...) {
  char b[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(b, sizeof(b), fmt, ap);
  va_end(ap);
  return std::string(data_dir()) + "/" + b;
}

bool post(const std::string& path, const Header& h, const void* data, size_t bytes) {
  const std::string tmp = path + ".tmp";
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) return false;
  bool ok = fwrite(&h, sizeof(h), 1, f) == 1 && (bytes == 0 || fwrite(data, 1, bytes, f) == bytes);
  ok = (fclose(f) == 0) && ok;
  return ok && rename(tmp.c_str(), path.c_str()) == 0;
}

// wait for `path`, then read header + payload
bool fetch(const std::string& path, Header& h, std::vector<char>& data) {
  const double t0 = now_s(), lim = timeout_s();
  struct stat st;
  int spin = 0;
  while (stat(path.c_str(), &st) != 0) {
    if (now_s() - t0 > lim) {
      fprintf(stderr, "[fake rccl] timed out after %.0f s waiting for %s\n", lim, path.c_str());
      return false;
    }
    usleep(spin++ < 100 ? 50 : 1000);
  }
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  bool ok = fread(&h, sizeof(h), 1, f) == 1 && h.magic == kMagic;
  const size_t bytes = ok ? (size_t)st.st_size - sizeof(h) : 0;
  data.resize(bytes);
  ok = ok && (bytes == 0 || fread(data.data(), 1, bytes, f) == bytes);
  fclose(f);
  return ok;
}

// One collective rendezvous on comm c: post this rank's header + payload, gather everyone's.
// Returns 0, or an error with a message on stderr.
ncclResult_t rendezvous(Comm* c, const Header& mine, const void* data, size_t bytes, std::vector<std::vector<char>>& all,
                        const char* what) {
  const uint64_t s = c->seq++;
  if (!post(path_of("%016llx_%llu_%d", (unsigned long long)c->key, (unsigned long long)s, c->rank), mine, data, bytes))
    return kSystemError;
  all.assign(c->nranks, {});
  for (int r = 0; r < c->nranks; ++r) {
    Header h;
    if (!fetch(path_of("%016llx_%llu_%d", (unsigned long long)c->key, (unsigned long long)s, r), h, all[r]))
      return kSystemError;
    if (h.op != mine.op || h.count != mine.count || h.dtype != mine.dtype || h.root != mine.root) {
      fprintf(stderr,
              "[fake rccl] %s #%llu mismatch: rank %d posted (op %u, count %llu, dtype %d, root %d), rank %d "
              "(op %u, count %llu, dtype %d, root %d)\n",
              what, (unsigned long long)s, c->rank, mine.op, (unsigned long long)mine.count, mine.dtype, mine.root, r,
              h.op, (unsigned long long)h.count, h.dtype, h.root);
      return kInvalidUsage;
    }
  }
  // every rank has posted collective s, so every rank has finished reading collective s - 1:
  // this rank's file of s - 2 is read by nobody any more
  if (s >= 2)
    unlink(path_of("%016llx_%llu_%d", (unsigned long long)c->key, (unsigned long long)(s - 2), c->rank).c_str());
  return 0;
}

enum Op : uint32_t { OP_AR = 1, OP_RS, OP_AG, OP_BC, OP_SPLIT };

int g_group = 0;
std::vector<std::function<ncclResult_t()>> g_sends, g_rest;
std::vector<std::pair<std::string, int>> g_acks;  // (message path, peer) of the open group's sends

// a send completes when its receiver has consumed the message (the .ack the receive leaves)
ncclResult_t wait_ack(const std::string& msg, int peer) {
  const std::string ack = msg + ".ack";
  const double t0 = now_s(), lim = timeout_s();
  struct stat st;
  int spin = 0;
  while (stat(ack.c_str(), &st) != 0) {
    if (now_s() - t0 > lim) {
      fprintf(stderr,
              "[fake rccl] send to rank %d never completed: no matching receive consumed %s within %.0f s "
              "(an unmatched send, or an exchange ordered so that it deadlocks under RCCL's blocking sends)\n",
              peer, msg.c_str(), lim);
      return kSystemError;
    }
    usleep(spin++ < 100 ? 50 : 1000);
  }
  unlink(ack.c_str());
  return 0;
}

ncclResult_t run_or_queue(bool is_send, std::function<ncclResult_t()> fn) {
  if (g_group > 0) {
    (is_send ? g_sends : g_rest).push_back(std::move(fn));
    return 0;
  }
  return fn();
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  if (env_on("FAKE_UID_FAIL")) return 3;
  memset(id->internal, 7, sizeof(id->internal));
  uint64_t k = ((uint64_t)getpid() << 32) ^ (uint64_t)(now_s() * 1e9);
  FILE* f = fopen("/dev/urandom", "rb");
  if (f) {
    if (fread(&k, sizeof(k), 1, f) != 1) k ^= 0x9e3779b97f4a7c15ull;
    fclose(f);
  }
  memcpy(id->internal, &k, sizeof(k));
  return 0;
}
ncclResult_t ncclCommInitRank(void** comm, int nranks, ncclUniqueId id, int rank) {
  if (env_on("FAKE_INIT_FAIL")) return 2;
  Comm* c = new Comm;
  memcpy(&c->key, id.internal, sizeof(c->key));
  c->nranks = nranks;
  c->rank = rank;
  c->sent.assign(nranks, 0);
  c->recvd.assign(nranks, 0);
  *comm = c;
  return 0;
}
ncclResult_t ncclCommSplit(void* comm, int color, int key, void** out, void*) {
  Comm* p = static_cast<Comm*>(comm);
  Comm* c = new Comm;
  const uint64_t nth = p->splits++;
  c->key = (p->key ^ (0x9e3779b97f4a7c15ull * (nth + 1))) * 0xff51afd7ed558ccdull + (uint64_t)(uint32_t)color;
  if (!data_dir()) {
    *out = c;
    return 0;
  }
  int32_t mine[2] = {color, key};
  Header h{kMagic, OP_SPLIT, 2, 2, 0, p->rank, 0};
  std::vector<std::vector<char>> all;
  const ncclResult_t r = rendezvous(p, h, mine, sizeof(mine), all, "ncclCommSplit");
  if (r != 0) {
    delete c;
    return r;
  }
  // members of my colour ordered by (key, parent rank)
  std::vector<std::pair<long long, int>> members;
  for (int q = 0; q < p->nranks; ++q) {
    int32_t v[2];
    memcpy(v, all[q].data(), sizeof(v));
    if (v[0] == color) members.push_back({(long long)v[1] * 65536 + q, q});
  }
  std::sort(members.begin(), members.end());
  c->nranks = (int)members.size();
  for (int i = 0; i < c->nranks; ++i)
    if (members[i].second == p->rank) c->rank = i;
  c->sent.assign(c->nranks, 0);
  c->recvd.assign(c->nranks, 0);
  *out = c;
  return 0;
}
ncclResult_t ncclCommDestroy(void* comm) {
  log_op("destroy");
  if (const char* v = getenv("FAKE_DESTROY_SLEEP")) sleep((unsigned)atoi(v));  // a hung destroy
  delete static_cast<Comm*>(comm);
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

ncclResult_t ncclAllReduce(const void* send, void* recv, size_t count, int dt, int op, void* comm, void*) {
  log_op("all_reduce");
  if (!data_dir()) return 0;
  Comm* c = static_cast<Comm*>(comm);
  return run_or_queue(false, [=]() -> ncclResult_t {
    const size_t bytes = count * dsize(dt);
    Header h{kMagic, OP_AR, count, dt, op, c->rank, 0};
    std::vector<std::vector<char>> all;
    const ncclResult_t r = rendezvous(c, h, send, bytes, all, "ncclAllReduce");
    if (r) return r;
    std::vector<const void*> ins;
    for (auto& v : all) ins.push_back(v.data());
    return reduce(recv, ins, count, dt, op) ? 0 : kInvalidUsage;
  });
}
ncclResult_t ncclReduceScatter(const void* send, void* recv, size_t recvcount, int dt, int op, void* comm, void*) {
  log_op("reduce_scatter");
  if (!data_dir()) return 0;
  Comm* c = static_cast<Comm*>(comm);
  return run_or_queue(false, [=]() -> ncclResult_t {
    const size_t es = dsize(dt), bytes = recvcount * es * c->nranks;
    Header h{kMagic, OP_RS, recvcount, dt, op, c->rank, 0};
    std::vector<std::vector<char>> all;
    const ncclResult_t r = rendezvous(c, h, send, bytes, all, "ncclReduceScatter");
    if (r) return r;
    std::vector<const void*> ins;
    for (auto& v : all) ins.push_back(v.data() + (size_t)c->rank * recvcount * es);
    return reduce(recv, ins, recvcount, dt, op) ? 0 : kInvalidUsage;
  });
}
ncclResult_t ncclAllGather(const void* send, void* recv, size_t sendcount, int dt, void* comm, void*) {
  log_op("all_gather");
  if (!data_dir()) return 0;
  Comm* c = static_cast<Comm*>(comm);
  return run_or_queue(false, [=]() -> ncclResult_t {
    const size_t bytes = sendcount * dsize(dt);
    Header h{kMagic, OP_AG, sendcount, dt, 0, c->rank, 0};
    std::vector<std::vector<char>> all;
    const ncclResult_t r = rendezvous(c, h, send, bytes, all, "ncclAllGather");
    if (r) return r;
    for (int q = 0; q < c->nranks; ++q) memcpy(static_cast<char*>(recv) + q * bytes, all[q].data(), bytes);
    return 0;
  });
}
ncclResult_t ncclBroadcast(const void* send, void* recv, size_t count, int dt, int root, void* comm, void*) {
  log_op("broadcast");
  if (!data_dir()) return 0;
  Comm* c = static_cast<Comm*>(comm);
  return run_or_queue(false, [=]() -> ncclResult_t {
    const size_t bytes = count * dsize(dt);
    Header h{kMagic, OP_BC, count, dt, root, c->rank, 0};
    std::vector<std::vector<char>> all;
    // (only the root's payload is used; the others post a header)
    const ncclResult_t r = rendezvous(c, h, send, c->rank == root ? bytes : 0, all, "ncclBroadcast");
    if (r) return r;
    if (root < 0 || root >= c->nranks || all[root].size() != bytes) return kInvalidUsage;
    memcpy(recv, all[root].data(), bytes);
    return 0;
  });
}
ncclResult_t ncclSend(const void* buf, size_t count, int dt, int peer, void* comm, void*) {
  log_op("send");
  if (!data_dir()) return 0;
  Comm* c = static_cast<Comm*>(comm);
  if (peer < 0 || peer >= c->nranks) return kInvalidUsage;
  // (the bytes are taken at the call, as the fake runs the group's sends first at its end:
  // callers keep send buffers alive and unchanged until the group completes, as RCCL needs)
  const bool grouped = g_group > 0;
  return run_or_queue(true, [=]() -> ncclResult_t {
    const uint64_t n = c->sent[peer]++;
    Header h{kMagic, 100, count, dt, 0, c->rank, 0};
    const std::string msg =
        path_of("%016llx_p_%d_%d_%llu", (unsigned long long)c->key, c->rank, peer, (unsigned long long)n);
    if (!post(msg, h, buf, count * dsize(dt))) return kSystemError;
    if (grouped) {  // completed at ncclGroupEnd, with the rest of the group
      g_acks.push_back({msg, peer});
      return 0;
    }
    return wait_ack(msg, peer);
  });
}
ncclResult_t ncclRecv(void* buf, size_t count, int dt, int peer, void* comm, void*) {
  log_op("recv");
  if (!data_dir()) return 0;
  Comm* c = static_cast<Comm*>(comm);
  if (peer < 0 || peer >= c->nranks) return kInvalidUsage;
  return run_or_queue(false, [=]() -> ncclResult_t {
    const uint64_t n = c->recvd[peer]++;
    const std::string p =
        path_of("%016llx_p_%d_%d_%llu", (unsigned long long)c->key, peer, c->rank, (unsigned long long)n);
    Header h;
    std::vector<char> data;
    if (!fetch(p, h, data)) return kSystemError;
    unlink(p.c_str());
    {  // the acknowledgement the sender's completion waits for
      FILE* f = fopen((p + ".ack").c_str(), "wb");
      if (!f) return kSystemError;
      fclose(f);
    }
    if (h.count != count || h.dtype != dt) {
      fprintf(stderr, "[fake rccl] recv #%llu from %d: expected (count %zu, dtype %d), the send carried (%llu, %d)\n",
              (unsigned long long)n, peer, count, dt, (unsigned long long)h.count, h.dtype);
      return kInvalidUsage;
    }
    memcpy(buf, data.data(), data.size());
    return 0;
  });
}
ncclResult_t ncclGroupStart() {
  ++g_group;
  return 0;
}
ncclResult_t ncclGroupEnd() {
  if (g_group <= 0) return kInvalidUsage;
  if (--g_group > 0) return 0;
  ncclResult_t err = 0;
  for (auto& f : g_sends)
    if (!err) err = f();
  for (auto& f : g_rest)
    if (!err) err = f();
  for (auto& a : g_acks)  // the group ends when every send of it has been received
    if (!err) err = wait_ack(a.first, a.second);
  g_sends.clear();
  g_rest.clear();
  g_acks.clear();
  return err;
}

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
