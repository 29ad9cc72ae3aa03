// Host-side native runtime of the cookbook (C ABI, loaded with ctypes).
//
//   * Token-file batch loader: a pre-tokenised corpus (flat uint16 / uint32 token ids, the
//     common ".bin" layout) is memory-mapped; worker threads cut [B, S+1] windows at
//     deterministic pseudo-random offsets (disjoint streams per data-parallel rank) into a
//     ring of host buffers ahead of the training loop.  Replaces the reference's
//     HF-datasets tokenize + DataLoader worker processes (reference data.py:23-36,
//     main-single.py:62-75) for large-scale runs: no Python in the hot path, no pickling,
//     no per-sample collation.
//   * Synthetic Markov-chain token generator (the structured synthetic corpus of
//     utils/data.py, ~100x faster than the Python loop).
//   * Host AdamW (OpenMP) for FSDP --cpu_offload (reference main-fsdp.py:68 CPUOffload):
//     one fused pass over the f32 master shard, moments, gradient and the bf16 copy.
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <fcntl.h>
#include <mutex>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

#define API extern "C" __attribute__((visibility("default")))

namespace {

inline uint64_t splitmix64(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

struct TokFile {
  int fd = -1;
  const uint8_t* base = nullptr;
  size_t bytes = 0;
  int width = 2;  // bytes per token
  size_t ntok = 0;
  int64_t get(size_t i) const {
    if (width == 2) return reinterpret_cast<const uint16_t*>(base)[i];
    return reinterpret_cast<const uint32_t*>(base)[i];
  }
};

struct Loader {
  const TokFile* tf = nullptr;
  int B = 0, S = 0;  // windows of S+1 tokens
  uint64_t seed = 0;
  int rank = 0, world = 1;
  int depth = 4;
  std::vector<std::thread> workers;
  std::mutex mu;
  std::condition_variable cv_full, cv_space;
  std::deque<std::pair<uint64_t, std::vector<int64_t>>> ready;  // (batch index, data)
  uint64_t next_to_make = 0, next_to_take = 0;
  uint64_t gen = 0;  // bumped by every seek: a batch made under an older generation is dropped
  std::atomic<bool> stop{false};

  void fill(uint64_t bi, int64_t* out) const {
    const size_t win = (size_t)S + 1;
    const size_t span = tf->ntok > win ? tf->ntok - win : 0;
    for (int b = 0; b < B; ++b) {
      uint64_t st = seed ^ (0x51ED270B27ULL * (bi * (uint64_t)world + rank)) ^ (0x9E37ULL * b);
      const size_t off = span ? (size_t)(splitmix64(st) % (span + 1)) : 0;
      for (size_t s = 0; s < win; ++s) out[(size_t)b * win + s] = off + s < tf->ntok ? tf->get(off + s) : 0;
    }
  }

  void work() {
    for (;;) {
      uint64_t bi, my_gen;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv_space.wait(lk, [&] { return stop.load() || next_to_make < next_to_take + depth; });
        if (stop) return;
        bi = next_to_make++;
        my_gen = gen;
      }
      std::vector<int64_t> buf((size_t)B * (S + 1));
      fill(bi, buf.data());
      {
        std::lock_guard<std::mutex> lk(mu);
        // made before a seek (backward seeks included: the val loader's seek(0) every epoch):
        // dropped, so `ready` never holds an index that next() will not take
        if (my_gen == gen && bi >= next_to_take) ready.emplace_back(bi, std::move(buf));
      }
      cv_full.notify_all();
    }
  }
};

}  // namespace

// ------------------------------------------------------------------ token files
API void* dpc_tokfile_open(const char* path, int width) {
  if (width != 2 && width != 4) return nullptr;
  int fd = ::open(path, O_RDONLY);
  if (fd < 0) return nullptr;
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size < width) {
    ::close(fd);
    return nullptr;
  }
  void* p = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) {
    ::close(fd);
    return nullptr;
  }
  madvise(p, (size_t)st.st_size, MADV_RANDOM);
  auto* tf = new TokFile;
  tf->fd = fd;
  tf->base = static_cast<const uint8_t*>(p);
  tf->bytes = (size_t)st.st_size;
  tf->width = width;
  tf->ntok = tf->bytes / width;
  return tf;
}

API int64_t dpc_tokfile_len(void* h) { return h ? (int64_t) static_cast<TokFile*>(h)->ntok : -1; }

API void dpc_tokfile_close(void* h) {
  if (!h) return;
  auto* tf = static_cast<TokFile*>(h);
  munmap((void*)tf->base, tf->bytes);
  ::close(tf->fd);
  delete tf;
}

// ------------------------------------------------------------------ batch loader
API void* dpc_loader_create(void* tokfile, int B, int S, uint64_t seed, int rank, int world, int nthreads,
                            int depth) {
  if (!tokfile || B <= 0 || S <= 0 || nthreads <= 0 || depth <= 0) return nullptr;
  auto* L = new Loader;
  L->tf = static_cast<TokFile*>(tokfile);
  L->B = B;
  L->S = S;
  L->seed = seed;
  L->rank = rank;
  L->world = world;
  L->depth = depth;
  for (int i = 0; i < nthreads; ++i) L->workers.emplace_back([L] { L->work(); });
  return L;
}

// Copy the next batch (in order) into out[B * (S+1)] (e.g. a pinned tensor); returns the batch index.
API int64_t dpc_loader_next(void* h, int64_t* out) {
  auto* L = static_cast<Loader*>(h);
  std::vector<int64_t> data;
  uint64_t want;
  {
    std::unique_lock<std::mutex> lk(L->mu);
    want = L->next_to_take;
    L->cv_full.wait(lk, [&] {
      for (auto& e : L->ready)
        if (e.first == want) return true;
      return false;
    });
    for (auto it = L->ready.begin(); it != L->ready.end(); ++it)
      if (it->first == want) {
        data = std::move(it->second);
        L->ready.erase(it);
        break;
      }
    L->next_to_take++;
  }
  L->cv_space.notify_all();
  std::memcpy(out, data.data(), data.size() * sizeof(int64_t));
  return (int64_t)want;
}

// Position the stream at batch `bi` (batch contents are a pure function of their index, so a
// resumed run reads exactly the batches an uninterrupted one would, without loading the
// skipped ones).
API void dpc_loader_seek(void* h, int64_t bi) {
  auto* L = static_cast<Loader*>(h);
  {
    std::lock_guard<std::mutex> lk(L->mu);
    L->ready.clear();
    L->gen++;
    L->next_to_make = L->next_to_take = (uint64_t)(bi < 0 ? 0 : bi);
  }
  L->cv_space.notify_all();
}

API void dpc_loader_destroy(void* h) {
  if (!h) return;
  auto* L = static_cast<Loader*>(h);
  L->stop = true;
  L->cv_space.notify_all();
  L->cv_full.notify_all();
  for (auto& t : L->workers) t.join();
  delete L;
}

// ------------------------------------------------------------------ synthetic Markov tokens
// Same chain as utils/data.py (successor table of `branching` candidates per token, 10%
// uniform noise), drawn from a counter-based generator so any row is reproducible alone.
API void dpc_synth_markov(int64_t* out, int64_t rows, int S, int vocab, uint64_t seed, int branching,
                          int64_t row0) {
  static std::mutex table_mu;
  static std::vector<int32_t> table;
  static int t_vocab = -1, t_branch = -1;
  {
    std::lock_guard<std::mutex> lk(table_mu);
    if (t_vocab != vocab || t_branch != branching) {
      table.assign((size_t)vocab * branching, 0);
      uint64_t ts = 1234567;
      for (auto& v : table) v = (int32_t)(splitmix64(ts) % (uint64_t)vocab);
      t_vocab = vocab;
      t_branch = branching;
    }
  }
  const std::vector<int32_t>& succ = table;
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < rows; ++r) {
    uint64_t st = seed * 1000003ULL + (uint64_t)(row0 + r) * 0x9E3779B97F4A7C15ULL;
    int64_t t = (int64_t)(splitmix64(st) % (uint64_t)vocab);
    int64_t* o = out + r * S;
    for (int s = 0; s < S; ++s) {
      o[s] = t;
      const uint64_t x = splitmix64(st);
      if ((x & 1023) < 102) t = (int64_t)((x >> 10) % (uint64_t)vocab);
      else t = succ[(size_t)t * branching + (size_t)((x >> 10) % (uint64_t)branching)];
    }
  }
}

// ------------------------------------------------------------------ host AdamW (torch.optim.AdamW math)
static inline uint16_t f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // NaN stays NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

API void dpc_adamw_host(float* p, const float* g, float* m, float* v, int64_t n, float lr, float b1, float b2,
                        float eps, float wd, float bc1, float bc2s, float grad_scale, uint16_t* shadow) {
  const float step = lr / bc1, decay = 1.f - lr * wd;
#pragma omp parallel for simd schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    const float gi = g[i] * grad_scale;
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float pi = p[i] * decay - step * mi / (std::sqrt(vi) / bc2s + eps);
    p[i] = pi;
    if (shadow) shadow[i] = f2bf(pi);
  }
}

API int dpc_runtime_version() { return 1; }
