// Standalone A/B + ablation driver for the persistent GEMM kernels (gemm7_kern.h), no torch:
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=fast bench/g7lab.hip -o bench/g7lab
//   bench/g7lab M N K [nt|nn|tn] [rounds] [reps] [sched|abl]
//
// Every variant runs on the same random bf16 operands (uniform [-1, 1): DVFS reads high on
// zeros), interleaved in rounds inside one process (median per variant).  The ABL variants
// are main-loop ablations (gemm7_kern.h): their outputs are garbage by design; the base
// variant is checked against a host double-precision product at sampled points.  Variants
// built with ABL 128 also report the in-kernel clock (s_memtime / s_memrealtime, median over
// workgroups).
#include "../distributed_pytorch_cookbook_amd/ops/csrc/gemm9_kern.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

using namespace dpc;

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));               \
      exit(2);                                                                                \
    }                                                                                         \
  } while (0)

__global__ void lab_fill(bf16_t* p, long long n, unsigned seed) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += gridDim.x * 256LL) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    p[i] = f2bf((float)(x & 0xffffff) / 8388608.f - 1.f);
  }
}

static float h_bf(unsigned short v) {
  unsigned u = (unsigned)v << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

struct Variant {
  std::string name;
  std::function<void()> run;
  bool clock;
  std::vector<double> ms;
};

template <int ABL, bool AK, bool BK, int SCHED = 3>
static void launch(const GemmArgs& a, G7Plan pl, unsigned long long ab, unsigned long long bb) {
  hipLaunchKernelGGL((gemm7_kernel<0, SCHED, AK, BK, 128, ABL>), dim3(pl.grid), dim3(256), 0, 0, a, ab, bb, pl);
}
template <int ABL, bool AK, bool BK, int ER = 0>
static void launch9(const GemmArgs& a, G7Plan pl, unsigned long long ab, unsigned long long bb) {
  pl.nk = a.K / 64;  // (v9: 64-deep stages)
  hipLaunchKernelGGL((gemm9_kernel<0, AK, BK, ABL, ER>), dim3(pl.grid), dim3(256), 0, 0, a, ab, bb, pl);
}

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s M N K [nt|nn|tn] [rounds] [reps] [sched|abl]\n", argv[0]);
    return 1;
  }
  const int M = atoi(argv[1]), N = atoi(argv[2]), K = atoi(argv[3]);
  const std::string lay = argc > 4 ? argv[4] : "nt";
  const bool nn = lay == "nn", tn = lay == "tn";
  const int rounds = argc > 5 ? atoi(argv[5]) : 5;
  const int reps = argc > 6 ? atoi(argv[6]) : 10;
  if (M % 256 || N % 256 || K % 64) {
    fprintf(stderr, "lab shapes: M, N multiples of 256, K of 64\n");
    return 1;
  }
  bf16_t *A, *B, *C;
  CK(hipMalloc(&A, (size_t)M * K * 2));
  CK(hipMalloc(&B, (size_t)N * K * 2));
  CK(hipMalloc(&C, (size_t)M * N * 2));
  hipLaunchKernelGGL(lab_fill, dim3(4096), dim3(256), 0, 0, A, (long long)M * K, 0x1234u);
  hipLaunchKernelGGL(lab_fill, dim3(4096), dim3(256), 0, 0, B, (long long)N * K, 0x9876u);
  CK(hipDeviceSynchronize());

  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.A = A;
  a.B = B;
  a.C = C;
  a.M = M;
  a.N = N;
  a.K = K;
  a.alpha = 1.f;
  a.a_kmaj = tn ? 0 : 1;
  a.b_kmaj = (nn || tn) ? 0 : 1;
  a.lda = tn ? M : K;
  a.ldb = (nn || tn) ? N : K;
  a.ldc = N;
  a.a_r = tn ? K : M;
  a.a_c = tn ? M : K;
  a.b_r = (nn || tn) ? K : N;
  a.b_c = (nn || tn) ? N : K;
  const unsigned long long ab = (unsigned long long)M * K * 2, bb = (unsigned long long)N * K * 2;

  G7Plan pl{};
  memset(&pl, 0, sizeof(pl));
  pl.tile_n = 256;
  pl.tiles_m = M / 256;
  pl.tiles_n = N / 256;
  pl.nk_all = K / 32;
  pl.splits = 1;
  pl.nk = 2 * ((pl.nk_all + 1) / 2);
  pl.units = pl.tiles_m * pl.tiles_n;
  pl.grid = std::min(pl.units, 256);
  pl.store_cnt = 32;
  G7Plan noepi = pl;
  noepi.debug = 1;

  std::vector<Variant> vs;
  const std::string set = argc > 7 ? argv[7] : "sched";
#define LAB_SET(AK_, BK_)                                                                                 \
  if (set == "abl") {                                                                                     \
    vs.push_back({"base", [&] { launch<0, AK_, BK_>(a, pl, ab, bb); }, false, {}});                       \
    vs.push_back({"clk", [&] { launch<128, AK_, BK_>(a, pl, ab, bb); }, true, {}});                       \
    vs.push_back({"no_epilogue", [&] { launch<128, AK_, BK_>(a, noepi, ab, bb); }, true, {}});            \
    vs.push_back({"no_dma", [&] { launch<128 | 2, AK_, BK_>(a, pl, ab, bb); }, true, {}});                \
    vs.push_back({"no_barrier", [&] { launch<128 | 16, AK_, BK_>(a, pl, ab, bb); }, true, {}});           \
    vs.push_back({"no_read", [&] { launch<128 | 32, AK_, BK_>(a, pl, ab, bb); }, true, {}});              \
    vs.push_back({"no_read_no_dma", [&] { launch<128 | 32 | 2, AK_, BK_>(a, pl, ab, bb); }, true, {}});   \
    vs.push_back({"mfma_only", [&] { launch<128 | 32 | 16 | 2, AK_, BK_>(a, pl, ab, bb); }, true, {}});   \
  } else if (set == "er") {                                                                              \
    vs.push_back({"v9", [&] { launch9<1024, AK_, BK_>(a, pl, ab, bb); }, false, {}});                     \
    vs.push_back({"v9_er2", [&] { launch9<1024, AK_, BK_, 2>(a, pl, ab, bb); }, false, {}});              \
    vs.push_back({"v9_er4", [&] { launch9<1024, AK_, BK_, 4>(a, pl, ab, bb); }, false, {}});              \
    vs.push_back({"v9_clk", [&] { launch9<128 | 1024, AK_, BK_>(a, pl, ab, bb); }, true, {}});            \
    vs.push_back({"v9_er2_clk", [&] { launch9<128 | 1024, AK_, BK_, 2>(a, pl, ab, bb); }, true, {}});     \
    vs.push_back({"v9_er4_clk", [&] { launch9<128 | 1024, AK_, BK_, 4>(a, pl, ab, bb); }, true, {}});     \
    vs.push_back({"v9_er2_noepi", [&] { launch9<128, AK_, BK_, 2>(a, noepi, ab, bb); }, true, {}});       \
    vs.push_back({"v9_noepi", [&] { launch9<128, AK_, BK_>(a, noepi, ab, bb); }, true, {}});              \
  } else if (set == "epi") {                                                                             \
    vs.push_back({"v9", [&] { launch9<0, AK_, BK_>(a, pl, ab, bb); }, false, {}});                        \
    vs.push_back({"v9_nt", [&] { launch9<1024, AK_, BK_>(a, pl, ab, bb); }, false, {}});                  \
    vs.push_back({"v9_clk", [&] { launch9<128, AK_, BK_>(a, pl, ab, bb); }, true, {}});                   \
    vs.push_back({"v9_nt_clk", [&] { launch9<128 | 1024, AK_, BK_>(a, pl, ab, bb); }, true, {}});         \
    vs.push_back({"v9_no_epilogue", [&] { launch9<128, AK_, BK_>(a, noepi, ab, bb); }, true, {}});        \
    vs.push_back({"v9_no_stores", [&] { launch9<128 | 512, AK_, BK_>(a, pl, ab, bb); }, true, {}});       \
    vs.push_back({"v9_no_credit", [&] { launch9<128 | 2048, AK_, BK_>(a, pl, ab, bb); }, true, {}});      \
    vs.push_back({"v9_no_dma", [&] { launch9<128 | 2, AK_, BK_>(a, pl, ab, bb); }, true, {}});            \
    vs.push_back({"s6", [&] { launch<0, AK_, BK_, 6>(a, pl, ab, bb); }, false, {}});                      \
  } else {                                                                                                \
    vs.push_back({"s3", [&] { launch<0, AK_, BK_>(a, pl, ab, bb); }, false, {}});                         \
    vs.push_back({"s3_old", [&] { launch<256, AK_, BK_>(a, pl, ab, bb); }, false, {}});                   \
    vs.push_back({"s6", [&] { launch<0, AK_, BK_, 6>(a, pl, ab, bb); }, false, {}});                      \
    vs.push_back({"s3_clk", [&] { launch<128, AK_, BK_>(a, pl, ab, bb); }, true, {}});                    \
    vs.push_back({"s6_clk", [&] { launch<128, AK_, BK_, 6>(a, pl, ab, bb); }, true, {}});                 \
    vs.push_back({"s6_no_dma", [&] { launch<128 | 2, AK_, BK_, 6>(a, pl, ab, bb); }, true, {}});          \
    vs.push_back({"v9", [&] { launch9<0, AK_, BK_>(a, pl, ab, bb); }, false, {}});                        \
    vs.push_back({"v9_clk", [&] { launch9<128, AK_, BK_>(a, pl, ab, bb); }, true, {}});                   \
    vs.push_back({"v9_no_dma", [&] { launch9<128 | 2, AK_, BK_>(a, pl, ab, bb); }, true, {}});            \
  }
  if (tn) { LAB_SET(false, false) }
  else if (nn) { LAB_SET(true, false) }
  else { LAB_SET(true, true) }

  // correctness of every non-ablation variant at sampled points
  std::vector<unsigned short> hA((size_t)M * K), hB((size_t)N * K), hC((size_t)M * N);
  CK(hipMemcpy(hA.data(), A, hA.size() * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hB.data(), B, hB.size() * 2, hipMemcpyDeviceToHost));
  for (auto& v : vs) {
    if (v.clock) continue;  // (clock variants of a checked schedule, or ablations)
    CK(hipMemset(C, 0, (size_t)M * N * 2));
    v.run();
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hC.data(), C, hC.size() * 2, hipMemcpyDeviceToHost));
    double maxerr = 0, maxref = 0;
    unsigned s = 12345;
    for (int t = 0; t < 1024; ++t) {
      s = s * 1103515245u + 12345u;
      const int m = (int)((s >> 8) % (unsigned)M);
      s = s * 1103515245u + 12345u;
      const int n = (int)((s >> 8) % (unsigned)N);
      double ref = 0;
      for (int k = 0; k < K; ++k) {
        const float bv = (nn || tn) ? h_bf(hB[(size_t)k * N + n]) : h_bf(hB[(size_t)n * K + k]);
        const float av = tn ? h_bf(hA[(size_t)k * M + m]) : h_bf(hA[(size_t)m * K + k]);
        ref += (double)av * bv;
      }
      maxerr = std::max(maxerr, std::fabs(ref - (double)h_bf(hC[(size_t)m * N + n])));
      maxref = std::max(maxref, std::fabs(ref));
    }
    printf("{\"check\": \"%s\", \"max_abs_err\": %.4g, \"max_abs_ref\": %.4g, \"rel\": %.3g, \"ok\": %s}\n",
           v.name.c_str(), maxerr, maxref, maxerr / maxref, maxerr / maxref < 0.01 ? "true" : "false");
  }
  for (auto& v : vs) v.run();  // warm every variant
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<double> ghz(vs.size(), 0.0);
  for (int r = 0; r < rounds; ++r) {
    for (size_t i = 0; i < vs.size(); ++i) {
      CK(hipEventRecord(e0, 0));
      for (int k = 0; k < reps; ++k) vs[i].run();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      vs[i].ms.push_back(ms / reps);
      if (vs[i].clock && r == rounds - 1) {
        std::vector<unsigned long long> clk(2 * 2048);
        CK(hipMemcpyFromSymbol(clk.data(), HIP_SYMBOL(g7_clk), clk.size() * 8));
        std::vector<double> f;
        for (int b = 0; b < pl.grid; ++b)
          if (clk[2 * b + 1] > 0) f.push_back((double)clk[2 * b] / (double)clk[2 * b + 1] * 0.1);
        std::sort(f.begin(), f.end());
        ghz[i] = f.empty() ? 0.0 : f[f.size() / 2];
      }
    }
  }
  const double flop = 2.0 * M * N * K;
  for (size_t i = 0; i < vs.size(); ++i) {
    auto m = vs[i].ms;
    std::sort(m.begin(), m.end());
    const double med = m[m.size() / 2];
    printf("{\"M\": %d, \"N\": %d, \"K\": %d, \"layout\": \"%s\", \"variant\": \"%s\", \"ms\": %.4f, \"min_ms\": %.4f, "
           "\"tflops\": %.1f, \"clock_ghz\": %.3f}\n",
           M, N, K, lay.c_str(), vs[i].name.c_str(), med, m[0], flop / med / 1e9, ghz[i]);
  }
  CK(hipFree(A));
  CK(hipFree(B));
  CK(hipFree(C));
  return 0;
}
