// f32 GEMM on the f32 matrix cores (v_mfma_f32_32x32x2_f32, exact f32 products and sums) for
// the --disable_amp path (reference: /root/reference/main-single.py:88-90 runs the model in
// f32 when AMP is off).  Same operand conventions and fused epilogue as the bf16 kernels
// (gemm.h GemmArgs: k-major / mn-major A and B, bias, act, act', pre-activation aux_out, f32
// residual, bias-gradient column sums, alpha (x device scalar), accumulate), with f32
// operands; aux_in / aux_out are f32 or bf16 (GemmArgs::aux_f32).
//
// Tile: 128 x 128 per 256-thread workgroup, 4 waves of 64 x 64 (2 x 2 MFMA tiles of 32 x 32),
// k-slices of 16 staged through LDS as [k][m] / [k][n] images (row pad 4 floats: the
// k-major transposing stores and the per-k-step operand reads are conflict free), double
// buffered with the next slice held in registers during the MFMAs.
#include "gemm.h"

namespace dpc {

constexpr int F_BM = 128, F_BK = 16, F_LD = F_BM + 4;

// one k-slice of an operand: rows r0 .. r0+127 of the logical [R][K] matrix (k-major: R x K
// stored row-major; mn-major: K x R), k0 .. k0+15.  Two float4 per thread.
template <bool KMAJ>
__device__ __forceinline__ void f32_load(float4 (&v)[2], const float* X, long long ld, int r0, int k0, int R, int K,
                                         int xr, int xc, bool vec) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    float e[4] = {0.f, 0.f, 0.f, 0.f};
    if (KMAJ) {
      const int r = r0 + (t >> 2) + 64 * i, k = k0 + 4 * (t & 3);
      if (r < min(R, xr)) {
        const float* p = X + (long long)r * ld + k;
        if (vec && k + 3 < min(K, xc)) {
          const float4 q = *reinterpret_cast<const float4*>(p);
          e[0] = q.x; e[1] = q.y; e[2] = q.z; e[3] = q.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) e[j] = (k + j < min(K, xc)) ? p[j] : 0.f;
        }
      }
    } else {
      const int k = k0 + (t >> 5) + 8 * i, r = r0 + 4 * (t & 31);
      if (k < min(K, xr)) {
        const float* p = X + (long long)k * ld + r;
        if (vec && r + 3 < min(R, xc)) {
          const float4 q = *reinterpret_cast<const float4*>(p);
          e[0] = q.x; e[1] = q.y; e[2] = q.z; e[3] = q.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) e[j] = (r + j < min(R, xc)) ? p[j] : 0.f;
        }
      }
    }
    v[i] = make_float4(e[0], e[1], e[2], e[3]);
  }
}

template <bool KMAJ>
__device__ __forceinline__ void f32_store(const float4 (&v)[2], float* s) {  // s: [F_BK][F_LD]
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if (KMAJ) {
      const int r = (t >> 2) + 64 * i, k = 4 * (t & 3);
      s[(k + 0) * F_LD + r] = v[i].x;
      s[(k + 1) * F_LD + r] = v[i].y;
      s[(k + 2) * F_LD + r] = v[i].z;
      s[(k + 3) * F_LD + r] = v[i].w;
    } else {
      const int k = (t >> 5) + 8 * i, r = 4 * (t & 31);
      *reinterpret_cast<float4*>(s + k * F_LD + r) = v[i];
    }
  }
}

__device__ __forceinline__ float f32_aux(const void* p, long long idx, bool is_f32) {
  return is_f32 ? static_cast<const float*>(p)[idx] : bf2f(static_cast<const bf16_t*>(p)[idx]);
}

template <bool AK, bool BK>
__global__ __launch_bounds__(256, 2) void gemm_f32_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) float sa[2][F_BK * F_LD];
  __shared__ __attribute__((aligned(16))) float sb[2][F_BK * F_LD];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int m0 = blockIdx.y * F_BM, n0 = blockIdx.x * F_BM;
  const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64;
  const float* A = static_cast<const float*>(p.A);
  const float* B = static_cast<const float*>(p.B);
  const bool va = (p.lda % 4 == 0) && (((uintptr_t)A & 15) == 0);
  const bool vb = (p.ldb % 4 == 0) && (((uintptr_t)B & 15) == 0);

  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = (p.K + F_BK - 1) / F_BK;
  float4 ra[2], rb[2];
  f32_load<AK>(ra, A, p.lda, m0, 0, p.M, p.K, p.a_r, p.a_c, va);
  f32_load<BK>(rb, B, p.ldb, n0, 0, p.N, p.K, p.b_r, p.b_c, vb);
  f32_store<AK>(ra, sa[0]);
  f32_store<BK>(rb, sb[0]);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      f32_load<AK>(ra, A, p.lda, m0, (kt + 1) * F_BK, p.M, p.K, p.a_r, p.a_c, va);
      f32_load<BK>(rb, B, p.ldb, n0, (kt + 1) * F_BK, p.N, p.K, p.b_r, p.b_c, vb);
    }
    const float* a_s = sa[cur];
    const float* b_s = sb[cur];
#pragma unroll
    for (int s = 0; s < F_BK / 2; ++s) {
      const int kr = (2 * s + (lane >> 5)) * F_LD;
      float af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = a_s[kr + wm + 32 * i + (lane & 31)];
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = b_s[kr + wn + 32 * j + (lane & 31)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      f32_store<AK>(ra, sa[cur ^ 1]);
      f32_store<BK>(rb, sb[cur ^ 1]);
    }
    __syncthreads();
  }

  // ---- epilogue: lane l, accumulator (i, j), register r holds
  // C[m0 + wm + 32 i + (r & 3) + 8 (r >> 2) + 4 (l >> 5)][n0 + wn + 32 j + (l & 31)]
  float alpha = p.alpha;
  if (p.alpha_ptr) alpha *= *p.alpha_ptr;
  float* C = static_cast<float*>(p.C);
  const bool aux_f32 = p.aux_f32 != 0;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn + 32 * j + (lane & 31);
    const bool nok = n < p.N;
    const float bias = (p.bias && nok) ? p.bias[n] : 0.f;
    float cs = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (!nok || m >= p.M) continue;
        float v = acc[i][j][r] * alpha + bias;
        if (p.act_bwd) v *= act_grad(f32_aux(p.aux_in, (long long)m * p.ld_aux_in + n, aux_f32), p.act_bwd);
        cs += v;
        if (p.aux_out) {
          const long long ai = (long long)m * p.ld_aux_out + n;
          const float av = p.aux_deriv ? act_grad(v, p.act) : v;  // (act'(v): aux_deriv)
          if (aux_f32) static_cast<float*>(p.aux_out)[ai] = av;
          else static_cast<bf16_t*>(p.aux_out)[ai] = f2bf(av);
        }
        v = act_fwd(v, p.act);
        if (p.residual) v += p.residual[(long long)m * p.ldr + n];
        float* c = C + (long long)m * p.ldc + n;
        if (p.accumulate) v += *c;
        *c = v;
      }
    if (p.colsum) {
      cs += __shfl_xor(cs, 32, 64);
      if (lane < 32 && nok) atomicAdd(p.colsum + n, cs);
    }
  }
}

}  // namespace dpc

using namespace dpc;

// f32 A, B, C (out_f32 must be set); returns the hipError_t of the launch, or -1 for an
// argument this kernel does not take.
DPC_API int dpc_gemm_f32(const GemmArgs* a, hipStream_t stream) {
  if (a->M <= 0 || a->N <= 0) return 0;
  if (!a->out_f32 || a->K <= 0) return -1;
  dim3 grid((unsigned)((a->N + F_BM - 1) / F_BM), (unsigned)((a->M + F_BM - 1) / F_BM)), block(256);
  if (a->a_kmaj && a->b_kmaj) hipLaunchKernelGGL((gemm_f32_kernel<true, true>), grid, block, 0, stream, *a);
  else if (a->a_kmaj) hipLaunchKernelGGL((gemm_f32_kernel<true, false>), grid, block, 0, stream, *a);
  else if (a->b_kmaj) hipLaunchKernelGGL((gemm_f32_kernel<false, true>), grid, block, 0, stream, *a);
  else hipLaunchKernelGGL((gemm_f32_kernel<false, false>), grid, block, 0, stream, *a);
  return (int)hipGetLastError();
}
