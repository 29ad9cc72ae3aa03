// HBM roofline lab: what a read + write stream reaches on MI355X, by access form (the memory-bound
// kernels of the step -- LayerNorm, cross-entropy, AdamW, bias/act backward -- measure against it).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 bench/copylab.hip -o bench/copylab
//   bench/copylab [MiB] [rounds]
//
// Variants (same bytes, interleaved in rounds, median): grid-stride float4 copy with U loads in
// flight per thread before the stores, plain / non-temporal loads and stores, separate buffers or
// in place (y = x * 1.0001f, as the cross-entropy writes its gradient over the logits).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));             \
      exit(2);                                                                              \
    }                                                                                       \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copy_k(const f4* __restrict__ x, f4* __restrict__ y, long long n) {
  const long long stride = (long long)gridDim.x * 256 * U;
  for (long long i0 = (long long)blockIdx.x * 256 * U + threadIdx.x; i0 < n; i0 += stride) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + (long long)u * 256;
      if (i < n) v[u] = NTL ? __builtin_nontemporal_load(x + i) : x[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + (long long)u * 256;
      if (i < n) {
        const f4 w = v[u] * 1.0001f;
        if (NTS) __builtin_nontemporal_store(w, y + i);
        else y[i] = w;
      }
    }
  }
}

struct Var {
  std::string name;
  std::function<void()> run;
  std::vector<double> ms;
};

int main(int argc, char** argv) {
  const long long mib = argc > 1 ? atoll(argv[1]) : 1024;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5;
  const long long n = mib * (1 << 20) / 16;
  f4 *x, *y;
  CK(hipMalloc(&x, n * 16));
  CK(hipMalloc(&y, n * 16));
  CK(hipMemset(x, 0, n * 16));
  CK(hipMemset(y, 0, n * 16));
  int cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount;
  std::vector<Var> vs;
  auto add = [&](const char* nm, auto kern, int U, int blocks_per_cu, bool inplace) {
    const long long maxg = (n + 256LL * U - 1) / (256LL * U);
    const unsigned g = (unsigned)std::min<long long>(maxg, (long long)cus * blocks_per_cu);
    f4* dst = inplace ? x : y;
    vs.push_back({std::string(nm) + (inplace ? "_inplace" : "") + "_g" + std::to_string(blocks_per_cu),
                  [=] { hipLaunchKernelGGL(kern, dim3(g), dim3(256), 0, 0, x, dst, n); }, {}});
  };
  for (bool ip : {false, true}) {
    add("u1", copy_k<1, false, false>, 1, 8, ip);
    add("u4", copy_k<4, false, false>, 4, 8, ip);
    add("u4", copy_k<4, false, false>, 4, 32, ip);
    add("u8", copy_k<8, false, false>, 8, 8, ip);
    add("u4_nts", copy_k<4, false, true>, 4, 8, ip);
    add("u4_ntl_nts", copy_k<4, true, true>, 4, 8, ip);
    add("u8_nts", copy_k<8, false, true>, 8, 8, ip);
    add("u4_nts", copy_k<4, false, true>, 4, 32, ip);
  }
  for (auto& v : vs) v.run();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 5;
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vs) {
      CK(hipEventRecord(e0, 0));
      for (int k = 0; k < reps; ++k) v.run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms / reps);
    }
  for (auto& v : vs) {
    auto m = v.ms;
    std::sort(m.begin(), m.end());
    const double med = m[m.size() / 2];
    printf("{\"variant\": \"%s\", \"MiB\": %lld, \"us\": %.1f, \"TBps\": %.3f}\n", v.name.c_str(), mib, med * 1e3,
           2.0 * n * 16 / (med * 1e-3) / 1e12);
  }
  return 0;
}
