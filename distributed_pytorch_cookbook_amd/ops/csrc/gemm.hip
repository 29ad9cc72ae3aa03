// bf16 MFMA GEMM for gfx950 with fused epilogues.
//
//   C[m, n] = epilogue( alpha * sum_k A[m, k] * B[n, k] )
//
// Operand storage (template flags):
//   A_KMAJ = true : A stored [M][lda] (k contiguous)   -- activations in forward / dgrad
//   A_KMAJ = false: A stored [K][lda] (m contiguous)   -- dY^T in wgrad
//   B_KMAJ = true : B stored [N][ldb] (k contiguous)   -- nn.Linear weight [out, in] in forward
//   B_KMAJ = false: B stored [K][ldb] (n contiguous)   -- weight in dgrad, X in wgrad
// so one kernel family covers the three products of a Linear layer without any explicit
// transpose pass (reference: every nn.Linear of models/gpt.py).
//
// Tiling (CDNA4): 128x128 output tile per 256-thread workgroup (4 waves in 2x2), each
// wave owns 64x64 = 4x4 tiles of v_mfma_f32_16x16x32_bf16.  BK = 64, two LDS stages
// (64 KiB -> 2 workgroups per CU), register-staged global->LDS copies issued one k-tile
// ahead (async-STAGE split: loads before the MFMA block, LDS writes after it).
//   * k-major tiles live in LDS as [row][64] bf16 (128-B rows) with a 16-B chunk XOR
//     swizzle  chunk ^ ((row >> 1) & 7)  -> fragment reads (ds_read_b128) are conflict free.
//   * mn-major tiles live as [k][128] bf16 (256-B rows) with a 32-B block XOR swizzle
//     blk ^ ((k & 3) | ((k >> 3) & 1) << 2) and are read with ds_read_b64_tr_b16, the
//     CDNA4 transposing LDS read, which yields the k-run per lane that MFMA wants.
//   * workgroup ids are remapped so consecutive tiles share an XCD (private L2), then
//     walked in GROUP_M-row supertiles for operand reuse.
#include "common.h"

namespace dpc {

struct GemmArgs {
  const void* A;
  const void* B;
  void* C;
  const float* bias;      // [N] f32, optional
  const float* residual;  // [M][ldr] f32, optional (may alias C)
  const void* aux_in;     // [M][ld_aux_in] bf16, optional: multiply by act'(aux_in)
  void* aux_out;          // [M][ld_aux_out] bf16, optional: store pre-activation
  const float* alpha_ptr; // device scalar multiplier, optional
  float* colsum;          // [N] f32, optional: colsum[n] += sum_m v (v after act_bwd, before act)
  long long lda, ldb, ldc, ldr, ld_aux_in, ld_aux_out;
  int M, N, K;
  float alpha;
  int act;         // activation applied after bias (Act)
  int act_bwd;     // multiply by act'(aux_in) (Act)
  int out_f32;     // C is f32 (else bf16)
  int accumulate;  // C += result (f32 output only)
  int a_kmaj, b_kmaj;
};

constexpr int BM = 128, BN = 128, BKT = 64, NT = 256;
constexpr int TILE_ELEMS = BM * BKT;  // 8192 bf16 = 16 KiB per operand per stage
constexpr int GROUP_M = 8;

// ---- LDS addressing (element offsets inside one operand tile) ----
__device__ __forceinline__ int kmaj_off(int row, int chunk) {  // chunk = 8 k-elements
  return row * 64 + ((chunk ^ ((row >> 1) & 7)) << 3);
}
__device__ __forceinline__ int mn_swz(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }
__device__ __forceinline__ int mnmaj_off(int k, int col) {      // col multiple of 4
  const int blk = col >> 4, within = col & 15;
  return k * 128 + (((blk ^ mn_swz(k)) << 4) | within);
}

// Load this thread's 4 x 16 B of a 128x64 (k-major) or 64x128 (mn-major) tile.
template <bool KMAJ>
__device__ __forceinline__ void g_load(uint4 (&r)[4], const bf16_t* __restrict__ P, long long ld,
                                       int mn0, int k0, int MN, int K) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = t + i * NT;
    int row, col, rlim, clim;
    if (KMAJ) { row = c >> 3; col = (c & 7) * 8; rlim = MN - mn0; clim = K - k0; }
    else      { row = c >> 4; col = (c & 15) * 8; rlim = K - k0; clim = MN - mn0; }
    uint4 v = make_uint4(0, 0, 0, 0);
    if (row < rlim && col < clim) {
      const bf16_t* src = KMAJ ? P + (long long)(mn0 + row) * ld + (k0 + col)
                               : P + (long long)(k0 + row) * ld + (mn0 + col);
      v = *reinterpret_cast<const uint4*>(src);
      if (KMAJ && clim - col < 8) {  // K tail inside a chunk (K % 8 != 0): zero the rest
        const int keep = clim - col;
        unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (e >= keep) w[e >> 1] &= (e & 1) ? 0x0000ffffu : 0xffff0000u;
        v = make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
    r[i] = v;
  }
}

template <bool KMAJ>
__device__ __forceinline__ void s_store(const uint4 (&r)[4], bf16_t* lds) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = t + i * NT;
    int off;
    if (KMAJ) off = kmaj_off(c >> 3, c & 7);
    else      off = mnmaj_off(c >> 4, (c & 15) * 8);
    *reinterpret_cast<uint4*>(lds + off) = r[i];
  }
}

// Fragment for v_mfma_f32_16x16x32_bf16: lane l holds X[r = l & 15][k = 8 (l >> 4) + j].
template <bool KMAJ>
__device__ __forceinline__ bf16x8 frag(const bf16_t* lds, int r0, int kstep, int lane) {
  if (KMAJ) {
    const int row = r0 + (lane & 15);
    const int chunk = kstep * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(lds + kmaj_off(row, chunk));
  } else {
    const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pp = i16 & 3;
    const int k = kstep * 32 + 8 * g + q;
    const int col = r0 + 4 * pp;
    typedef short4_t __attribute__((address_space(3))) * lptr;
    short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lptr)(lds + mnmaj_off(k, col)));
    short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lptr)(lds + mnmaj_off(k + 4, col)));
    typedef short short8_t __attribute__((ext_vector_type(8)));
    short8_t s = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, s);
  }
}

template <bool AK, bool BK>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * TILE_ELEMS];  // [stage][A|B]
  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  // XCD-aware bijective remap: blocks b, b+8, ... share an XCD; give each XCD a
  // contiguous run of logical tile ids.
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  // grouped ordering for L2 reuse
  const int group = GROUP_M * tiles_n;
  const int gid = bid / group, first_m = gid * GROUP_M;
  const int gsz = min(tiles_m - first_m, GROUP_M);
  const int tm = first_m + (bid % group) % gsz;
  const int tn = (bid % group) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const bf16_t* A = static_cast<const bf16_t*>(p.A);
  const bf16_t* B = static_cast<const bf16_t*>(p.B);

  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BKT - 1) / BKT;
  uint4 ra[4], rb[4];
  g_load<AK>(ra, A, p.lda, m0, 0, p.M, p.K);
  g_load<BK>(rb, B, p.ldb, n0, 0, p.N, p.K);
  s_store<AK>(ra, smem);
  s_store<BK>(rb, smem + TILE_ELEMS);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      g_load<AK>(ra, A, p.lda, m0, (kt + 1) * BKT, p.M, p.K);
      g_load<BK>(rb, B, p.ldb, n0, (kt + 1) * BKT, p.N, p.K);
    }
    const bf16_t* la = smem + cur * 2 * TILE_ELEMS;
    const bf16_t* lb = la + TILE_ELEMS;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag<AK>(la, wr * 64 + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag<BK>(lb, wc * 64 + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      bf16_t* nxt = smem + (cur ^ 1) * 2 * TILE_ELEMS;
      s_store<AK>(ra, nxt);
      s_store<BK>(rb, nxt + TILE_ELEMS);
    }
    __syncthreads();
  }

  // ---- epilogue: C/D map of 16x16x32: col = lane & 15, row = 4 (lane >> 4) + r ----
  float alpha = p.alpha;
  if (p.alpha_ptr) alpha *= *p.alpha_ptr;
  const bf16_t* aux_in = static_cast<const bf16_t*>(p.aux_in);
  bf16_t* aux_out = static_cast<bf16_t*>(p.aux_out);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wc * 64 + j * 16 + (lane & 15);
    const bool nok = n < p.N;
    const float bn = (p.bias && nok) ? p.bias[n] : 0.f;
    float csum = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * 64 + i * 16 + (lane >> 4) * 4 + r;
        if (m >= p.M || !nok) continue;
        float v = acc[i][j][r] * alpha + bn;
        if (p.act_bwd) v *= act_grad(bf2f(aux_in[(long long)m * p.ld_aux_in + n]), p.act_bwd);
        csum += v;
        if (aux_out) aux_out[(long long)m * p.ld_aux_out + n] = f2bf(v);
        v = act_fwd(v, p.act);
        if (p.residual) v += p.residual[(long long)m * p.ldr + n];
        const long long ci = (long long)m * p.ldc + n;
        if (p.out_f32) {
          float* C = static_cast<float*>(p.C);
          if (p.accumulate) v += C[ci];
          C[ci] = v;
        } else {
          static_cast<bf16_t*>(p.C)[ci] = f2bf(v);
        }
      }
    }
    if (p.colsum) {  // reduce over the 4 row-groups of lanes sharing this column
      csum += __shfl_xor(csum, 16, 64);
      csum += __shfl_xor(csum, 32, 64);
      if ((lane >> 4) == 0 && nok) atomicAdd(p.colsum + n, csum);
    }
  }
}

}  // namespace dpc

using namespace dpc;

DPC_API int dpc_gemm(const GemmArgs* a, hipStream_t stream) {
  if (a->M <= 0 || a->N <= 0) return 0;
  const int tiles = ((a->M + BM - 1) / BM) * ((a->N + BN - 1) / BN);
  dim3 grid(tiles), block(NT);
  if (a->a_kmaj && a->b_kmaj) hipLaunchKernelGGL((gemm_kernel<true, true>), grid, block, 0, stream, *a);
  else if (a->a_kmaj && !a->b_kmaj) hipLaunchKernelGGL((gemm_kernel<true, false>), grid, block, 0, stream, *a);
  else if (!a->a_kmaj && !a->b_kmaj) hipLaunchKernelGGL((gemm_kernel<false, false>), grid, block, 0, stream, *a);
  else hipLaunchKernelGGL((gemm_kernel<false, true>), grid, block, 0, stream, *a);
  return (int)hipGetLastError();
}
