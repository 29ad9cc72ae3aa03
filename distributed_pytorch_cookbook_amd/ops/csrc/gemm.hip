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
#include "gemm.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace dpc {


// Which output tile and k-range a workgroup computes.  The grid is 1-D, ntiles x splits
// workgroups (splits = |ksplit|, set by the dispatcher; 0 = 1), and block b runs on XCD b % 8.
//  * default (ksplit >= 0): a bijective remap gives every XCD a contiguous run of work ids,
//    split-major (id = split * ntiles + tile), walked in GROUP_M supertiles: the workgroups
//    that share an XCD's L2 compute the SAME k-range of neighbouring tiles, so each k-slice of
//    both operands is fetched into that L2 once and read by all of them.  (A 2-D grid with the
//    split on blockIdx.y put block (x, y) on XCD (x + ntiles * y) % 8 -- every XCD mixed all
//    k-ranges, and the weight gradients streamed their operands from beyond L2.)
//  * ksplit < 0: split = b % splits pins each k-range to its own XCD(s) (sweeps only).
struct TileSlot {
  int bid, split, splits;
};
__device__ __forceinline__ TileSlot tile_slot(const GemmArgs& p, int ntiles) {
  TileSlot t;
  if (p.ksplit < -1) {
    t.splits = -p.ksplit;
    t.split = blockIdx.x % t.splits;
    t.bid = blockIdx.x / t.splits;
    return t;
  }
  t.splits = p.ksplit > 1 ? p.ksplit : 1;
  const int nwg = ntiles * t.splits;
  const int b = blockIdx.x, xcd = b & 7, q = nwg >> 3, r = nwg & 7;
  const int w = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  t.split = w / ntiles;
  t.bid = w - t.split * ntiles;
  return t;
}

// Split-K partial sums: the f32 tile rows staged in LDS (32 x 64 per wave, columns XOR-swizzled
// by ((row >> 2) & 3) << 4) are added with one float atomic per lane, lanes along the row, so
// every wave-instruction covers 256 contiguous bytes -- the full memory-side atomic rate.  (A
// lane-owns-4-columns pattern touches each 64-B segment four times and ran ~4x slower.)
__device__ __forceinline__ void split_rows_atomic(const float* ct, float* C, long long ldc, int mbase,
                                                  int ncol0, int M, int N, int lane) {
  const int n = ncol0 + lane;
  if (n >= N) return;
  const int rows = min(32, M - mbase);
  float* c = C + (long long)mbase * ldc + n;
#pragma unroll 8
  for (int row = 0; row < rows; ++row)
    atomicAdd(c + (long long)row * ldc, ct[row * 64 + (lane ^ (((row >> 2) & 3) << 4))]);
}

// Bias-gradient column sums of a wave's 64 columns [nb, nb + 64): lane l & 15 holds columns
// nb + 4 (l & 15) + e in cs[e], summed over its row group l >> 4.  Reduce over the four row
// groups, then hand column nb + l to lane l so ONE atomic instruction covers 256 contiguous
// bytes (four lane-owns-4-columns instructions hit every 64-B segment four times; with every
// M-tile adding to the same N columns the serialised atomics cost ~20 % of a dgrad GEMM).
__device__ __forceinline__ void colsum_flush(float (&cs)[4], float* colsum, int nb, int N, int lane) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    cs[e] += __shfl_xor(cs[e], 16, 64);
    cs[e] += __shfl_xor(cs[e], 32, 64);
  }
  const int src = lane >> 2, e = lane & 3;
  const float v0 = __shfl(cs[0], src, 64), v1 = __shfl(cs[1], src, 64);
  const float v2 = __shfl(cs[2], src, 64), v3 = __shfl(cs[3], src, 64);
  const float v = e == 0 ? v0 : (e == 1 ? v1 : (e == 2 ? v2 : v3));
  if (nb + lane < N) atomicAdd(colsum + nb + lane, v);
}

// ---- Shared epilogue of the LDS-DMA kernels (v2, v3).  A wave owns FM x 4 fragments of
// 16x16 (FM/2 passes of 32 rows x 64 columns).  Each pass stages its f32 rows through LDS
// ([32][64] per wave, columns XOR-swizzled by ((row >> 2) & 3) << 4) so that bias /
// residual / aux / C move 16 B (f32) or 8 B (bf16) per lane along rows.  Every global READ
// of a pass (aux_in for act', the f32 residual or the accumulated C) is issued as one batch
// one pass AHEAD, into a double buffer: one HBM round trip per pass overlapped with the
// previous pass, instead of one exposed round trip per 4 rows (the v12 epilogue waited on
// each row group's aux load before issuing the next: act' dgrad ran at ~65 % of the plain
// product's rate).  DB = false (kernels that need their registers: several workgroups per CU,
// or 128-row wave tiles) issues a pass's reads right after staging it instead, overlapping
// only the barrier and LDS re-read.
struct EpiIn {
  // per row group t: the f32 residual (or accumulated C) when there is one, else the act'
  // operand (bf16 x 4 in .x/.y) -- one 16-B slot, so the prefetch costs 32 VGPRs not 48
  // (no caller combines act' with a residual; if one did, its aux is read late)
  uint4 v[8];
};

__device__ __forceinline__ const float* epi_fsrc(const GemmArgs& p) {
  return p.residual ? p.residual : (p.out_f32 && p.accumulate ? static_cast<const float*>(p.C) : nullptr);
}

__device__ __forceinline__ void epi_load(const GemmArgs& p, EpiIn& e, int mb, int n, bool nok, int lane) {
  const bf16_t* aux_in = static_cast<const bf16_t*>(p.aux_in);
  const float* fsrc = epi_fsrc(p);
  const long long ldf = p.residual ? p.ldr : p.ldc;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int m = mb + (lane >> 4) + 4 * t;
    const bool ok = nok && m < p.M;
    e.v[t] = make_uint4(0u, 0u, 0u, 0u);
    if (ok && fsrc) {
      e.v[t] = *reinterpret_cast<const uint4*>(fsrc + (long long)m * ldf + n);
    } else if (ok && p.act_bwd) {
      const uint2 z = *reinterpret_cast<const uint2*>(aux_in + (long long)m * p.ld_aux_in + n);
      e.v[t].x = z.x;
      e.v[t].y = z.y;
    }
  }
}

template <int FM, bool DB>
__device__ __forceinline__ void epi_tile(const GemmArgs& p, floatx4 (&acc)[FM][4], float* ct, int splits,
                                         int mw, int nw, int lane) {
  constexpr int NP = FM / 2;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float alpha = p.alpha;
  if (p.alpha_ptr) alpha *= *p.alpha_ptr;
  const int c4 = lane & 15;
  const int n = nw + c4 * 4;
  const bool nok = n < p.N;  // N % 4 == 0 is required by the host for v2+
  float4 bias4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (p.bias && nok) bias4 = *reinterpret_cast<const float4*>(p.bias + n);
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  bf16_t* aux_out = static_cast<bf16_t*>(p.aux_out);
  const float* fsrc = epi_fsrc(p);
  EpiIn e[DB ? 2 : 1];
  if (DB && splits <= 1) epi_load(p, e[0], mw, n, nok, lane);
#pragma unroll
  for (int h = 0; h < NP; ++h) {
    __syncthreads();  // the ring (h = 0) / previous pass (h > 0) fully consumed
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = ii * 16 + (lane >> 4) * 4 + r;
          const int col = (j * 16 + (lane & 15)) ^ (((row >> 2) & 3) << 4);
          ct[row * 64 + col] = acc[2 * h + ii][j][r] * alpha;
        }
    // (after the staging writes, so this pass's accumulators are dead before the loads land)
    if (!DB && splits <= 1) epi_load(p, e[0], mw + h * 32, n, nok, lane);
    __syncthreads();
    if (splits > 1) {  // f32 partial sums: atomics (no epilogue operands)
      split_rows_atomic(ct, static_cast<float*>(p.C), p.ldc, mw + h * 32, nw, p.M, p.N, lane);
      continue;
    }
    if (DB && h + 1 < NP) epi_load(p, e[(h + 1) & 1], mw + (h + 1) * 32, n, nok, lane);
    const EpiIn& cur = e[DB ? (h & 1) : 0];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int row = (lane >> 4) + 4 * t;
      const int m = mw + h * 32 + row;
      const int col = (c4 * 4) ^ (((row >> 2) & 3) << 4);
      const float4 v4 = *reinterpret_cast<const float4*>(ct + row * 64 + col);
      if (m >= p.M || !nok) continue;
      float v[4] = {v4.x + bias4.x, v4.y + bias4.y, v4.z + bias4.z, v4.w + bias4.w};
      if (p.act_bwd) {
        const uint2 z = fsrc ? *reinterpret_cast<const uint2*>(static_cast<const bf16_t*>(p.aux_in) +
                                                              (long long)m * p.ld_aux_in + n)
                             : make_uint2(cur.v[t].x, cur.v[t].y);
        v[0] *= act_grad(__uint_as_float(z.x << 16), p.act_bwd);
        v[1] *= act_grad(__uint_as_float(z.x & 0xffff0000u), p.act_bwd);
        v[2] *= act_grad(__uint_as_float(z.y << 16), p.act_bwd);
        v[3] *= act_grad(__uint_as_float(z.y & 0xffff0000u), p.act_bwd);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) cs[q] += v[q];
      if (aux_out) {  // the pre-activation, or act'(v) (aux_deriv)
        uint2 w;
        if (p.aux_deriv) {
          w.x = pack2bf(act_grad(v[0], p.act), act_grad(v[1], p.act));
          w.y = pack2bf(act_grad(v[2], p.act), act_grad(v[3], p.act));
        } else {
          w.x = pack2bf(v[0], v[1]);
          w.y = pack2bf(v[2], v[3]);
        }
        st8(aux_out + (long long)m * p.ld_aux_out + n, w, p.nt_store & 1);
      }
      if (p.act == ACT_GELU) {  // packed-f32 math (common.h:gelu_tanh2)
        const dpc_f2_t g01 = gelu_tanh2(dpc_f2_t{v[0], v[1]}), g23 = gelu_tanh2(dpc_f2_t{v[2], v[3]});
        v[0] = g01.x; v[1] = g01.y; v[2] = g23.x; v[3] = g23.y;
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = act_fwd(v[q], p.act);
      }
      const long long ci = (long long)m * p.ldc + n;
      if (fsrc) {
        v[0] += __uint_as_float(cur.v[t].x); v[1] += __uint_as_float(cur.v[t].y);
        v[2] += __uint_as_float(cur.v[t].z); v[3] += __uint_as_float(cur.v[t].w);
      }
      if (p.out_f32) {
        float4* C = reinterpret_cast<float4*>(static_cast<float*>(p.C) + ci);
        if (p.accumulate && p.residual) {  // (no caller does both; C read late)
          const float4 o = *C;
          v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
        }
        st16(C, make_float4(v[0], v[1], v[2], v[3]), p.nt_store & 2);
      } else {
        uint2 w;
        w.x = pack2bf(v[0], v[1]);
        w.y = pack2bf(v[2], v[3]);
        st8(static_cast<bf16_t*>(p.C) + ci, w, p.nt_store & 1);
      }
    }
  }
  if (p.colsum) colsum_flush(cs, p.colsum, nw, p.N, lane);
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

template <bool AK, bool BK>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * TILE_ELEMS];  // [stage][A|B]
  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  const TileSlot ts = tile_slot(p, nwg);
  const int bid = ts.bid;
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
  const int a_mn = AK ? p.a_r : p.a_c, a_k = AK ? min(p.K, p.a_c) : min(p.K, p.a_r);
  const int b_mn = BK ? p.b_r : p.b_c, b_k = BK ? min(p.K, p.b_c) : min(p.K, p.b_r);
  g_load<AK>(ra, A, p.lda, m0, 0, a_mn, a_k);
  g_load<BK>(rb, B, p.ldb, n0, 0, b_mn, b_k);
  s_store<AK>(ra, smem);
  s_store<BK>(rb, smem + TILE_ELEMS);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      g_load<AK>(ra, A, p.lda, m0, (kt + 1) * BKT, a_mn, a_k);
      g_load<BK>(rb, B, p.ldb, n0, (kt + 1) * BKT, b_mn, b_k);
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
        if (aux_out) aux_out[(long long)m * p.ld_aux_out + n] = f2bf(p.aux_deriv ? act_grad(v, p.act) : v);
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

// =====================================================================================
// v2: LDS-DMA pipeline.  Operand tiles stream HBM/L2 -> LDS with buffer_load_dwordx4 ... lds
// (no VGPR round trip, no ds_write), STAGES-deep ring with ONE raw s_barrier per k-tile and a
// counted vmcnt that keeps STAGES-2 tiles in flight across it.  The buffer descriptor's
// num_records bounds every operand, so out-of-range rows / k-rows land in LDS as zeros (the
// M/N/K edges need no predicates).  Because the DMA writes LDS lane-linearly (1 KiB per
// wave-instruction), the bank swizzle is applied to the per-lane SOURCE address and read back
// with the same involution.  Epilogue: the f32 tile goes through LDS so that bias / residual /
// aux / C traffic is 16-B-per-lane row-contiguous.
// =====================================================================================



template <int NL>
__device__ __forceinline__ void issue_tile(const void* base, unsigned long long total, unsigned long long off,
                                           const int* voff, bf16_t* lds_tile, int wave) {
  // descriptor whose base is `off` bytes into the operand and whose range ends with it
  const unsigned long long left = off < total ? total - off : 0ull;
  const unsigned nrec = left > 0xffffffffull ? 0xffffffffu : (unsigned)left;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)base + off), 0, nrec, 0x00020000);
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const int j = wave * NL + i;  // wave-instruction index: 1 KiB of the tile
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t)(lds_tile + j * 512), 16, voff[i], 0, 0, 0);
  }
}

// buffer descriptor whose base is `off` bytes into the operand and whose range ends with it
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned long long total,
                                                            unsigned long long off) {
  const unsigned long long left = off < total ? total - off : 0ull;
  const unsigned nrec = left > 0xffffffffull ? 0xffffffffu : (unsigned)left;
  return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)base + off), 0, nrec, 0x00020000);
}


template <int KB, int STAGES>
struct V2Cfg {
  static constexpr int TILE = BM * KB;                  // bf16 elements per operand per stage
  static constexpr int PIPE = STAGES * 2 * TILE;        // pipeline ring (elements)
  static constexpr int EPI = 4 * 32 * 64 * 2;           // epilogue: 4 waves x [32][64] f32 (as bf16 units)
  static constexpr int SMEM = PIPE > EPI ? PIPE : EPI;
  static constexpr int WGS = (160 * 1024) / (SMEM * 2) > 4 ? 4 : (160 * 1024) / (SMEM * 2);
};

template <int KB, int STAGES, bool AK, bool BK>
__global__ __launch_bounds__(NT, (V2Cfg<KB, STAGES>::WGS)) void gemm2_kernel(GemmArgs p, unsigned long long a_bytes,
                                                                          unsigned long long b_bytes) {
  using Cfg = V2Cfg<KB, STAGES>;
  constexpr int NL = KB / 16;
  __shared__ __attribute__((aligned(16))) bf16_t smem[Cfg::SMEM];
  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  const TileSlot ts = tile_slot(p, nwg);
  const int bid = ts.bid;
  const int group = GROUP_M * tiles_n;
  const int gid = bid / group, first_m = gid * GROUP_M;
  const int gsz = min(tiles_m - first_m, GROUP_M);
  const int tm = first_m + (bid % group) % gsz;
  const int tn = (bid % group) / gsz;
  const int m0 = tm * BM, n0 = tn * BN;

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 1, wc = wid & 1;

  // Per-lane source byte offsets relative to the tile origin of the current k-tile.  The
  // descriptor base itself moves (64-bit scalar math) with the tile origin and k, so the
  // 32-bit voffsets stay small for operands of any size, and num_records = bytes left in the
  // operand makes every out-of-range lane read zeros.
  int va[NL], vb[NL];
  dma_offsets<KB, AK>(va, p.lda, wid, lane);
  dma_offsets<KB, BK>(vb, p.ldb, wid, lane);
  const unsigned long long a_org = AK ? (unsigned long long)m0 * p.lda * 2 : (unsigned long long)m0 * 2;
  const unsigned long long b_org = BK ? (unsigned long long)n0 * p.ldb * 2 : (unsigned long long)n0 * 2;
  const unsigned long long a_step = AK ? KB * 2ull : (unsigned long long)KB * p.lda * 2;
  const unsigned long long b_step = BK ? KB * 2ull : (unsigned long long)KB * p.ldb * 2;
  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // split-K: each split owns a contiguous run of k-tiles (the host only splits plain
  // f32-accumulating products, whose partial tiles are combined with f32 atomics)
  const int nk_all = (p.K + KB - 1) / KB;
  const int splits = ts.splits;
  const int per = (nk_all + splits - 1) / splits;
  const int kt0 = ts.split * per;
  const int nk = max(0, min(nk_all, kt0 + per) - kt0);
#define DPC_ISSUE(it_)                                                                              \
  do {                                                                                              \
    bf16_t* base_ = smem + ((it_) % STAGES) * 2 * Cfg::TILE;                                        \
    const unsigned long long ktg_ = (unsigned long long)(kt0 + (it_));                              \
    issue_tile<NL>(p.A, a_bytes, a_org + a_step * ktg_, va, base_, wid);                            \
    issue_tile<NL>(p.B, b_bytes, b_org + b_step * ktg_, vb, base_ + Cfg::TILE, wid);                \
  } while (0)
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) DPC_ISSUE(s);

  for (int kt = 0; kt < nk; ++kt) {
    // tile kt landed for THIS wave: the tiles issued after it (at most STAGES-2, fewer at the
    // tail) may stay in flight -- 2*NL loads each
    const int after = min(STAGES - 2, nk - 1 - kt);
    if (STAGES >= 4 && after >= 2) wait_vm<(STAGES >= 4 ? 4 * NL : 0)>();
    else if (STAGES >= 3 && after >= 1) wait_vm<(STAGES >= 3 ? 2 * NL : 0)>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();  // ... and for every wave; also: all waves finished tile kt-1
    asm volatile("" ::: "memory");
    if (kt + STAGES - 1 < nk) DPC_ISSUE(kt + STAGES - 1);
    const bf16_t* la = smem + (kt % STAGES) * 2 * Cfg::TILE;
    const bf16_t* lb = la + Cfg::TILE;
#pragma unroll
    for (int ks = 0; ks < KB / 32; ++ks) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag_k<KB, AK>(la, wr * 64 + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = frag_k<KB, BK>(lb, wc * 64 + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }

  // ---------------- epilogue through LDS, two passes of 32 rows per wave: the f32 tile is
  // re-read row-contiguously so bias / residual / aux / C move 16 B per lane
  epi_tile<4, (Cfg::WGS <= 2)>(p, acc, reinterpret_cast<float*>(smem) + wid * 32 * 64, splits, m0 + wr * 64, n0 + wc * 64, lane);
}

// =====================================================================================
// v3: large tiles.  A 128x128 tile re-reads each operand byte from L2 once per 128 output
// columns: at the MFMA rate that is ~39 TB/s of L2->LDS traffic chip-wide, the whole L2
// bandwidth, so v2 is L2-bound (PMC: WAIT_ANY 44 %).  v3 keeps v2's LDS-DMA pipeline,
// swizzles and epilogue but runs 8 waves on a 256x256 (or 256x128) tile: half (3/4) the
// L2 bytes per FLOP, and each wave owns a 128x64 (64x64) sub-tile, so per k-step a wave
// reads 12 (8) fragments for 32 (16) MFMAs.  mn-major operand tiles wider than 128 are
// stored as 128-column halves so the v2 transposed-read swizzle applies unchanged.
template <int BM_, int BN_, int WM, int WN, int KB, int STAGES>
struct V3Cfg {
  static constexpr int NW = WM * WN, NTH = 64 * NW;
  static constexpr int WTM = BM_ / WM, WTN = BN_ / WN;
  static constexpr int FM = WTM / 16, FN = WTN / 16;
  static constexpr int TA = BM_ * KB, TB = BN_ * KB;        // bf16 elements per stage
  static constexpr int NLA = TA / 512 / NW, NLB = TB / 512 / NW;  // 1-KiB DMA instr per wave
  static constexpr int PIPE = STAGES * (TA + TB);
  static constexpr int EPI = NW * 32 * WTN * 2;              // [32][WTN] f32 per wave
  static constexpr int SMEM = PIPE > EPI ? PIPE : EPI;
  static constexpr int WGS = (160 * 1024) / (SMEM * 2) >= 2 ? 2 : 1;
  static_assert(WTN == 64 && (WTM == 64 || WTM == 128), "wave tile 64x64 or 128x64");
  static_assert(NLA * 512 * NW == TA && NLB * 512 * NW == TB, "DMA split");
  static_assert(SMEM * 2 <= 160 * 1024, "LDS");
};



template <int BM_, int BN_, int WM, int WN, int KB, int STAGES, bool AK, bool BK>
__global__ __launch_bounds__((V3Cfg<BM_, BN_, WM, WN, KB, STAGES>::NTH), (V3Cfg<BM_, BN_, WM, WN, KB, STAGES>::WGS)) void gemm3_kernel(
    GemmArgs p, unsigned long long a_bytes, unsigned long long b_bytes) {
  using Cfg = V3Cfg<BM_, BN_, WM, WN, KB, STAGES>;
  constexpr int FM = Cfg::FM, FN = Cfg::FN, NLA = Cfg::NLA, NLB = Cfg::NLB;
  __shared__ __attribute__((aligned(16))) bf16_t smem[Cfg::SMEM];
  const int tiles_m = (p.M + BM_ - 1) / BM_, tiles_n = (p.N + BN_ - 1) / BN_;
  const int nwg = tiles_m * tiles_n;
  const TileSlot ts = tile_slot(p, nwg);
  const int bid = ts.bid;
  const int group = GROUP_M * tiles_n;
  const int gid = bid / group, first_m = gid * GROUP_M;
  const int gsz = min(tiles_m - first_m, GROUP_M);
  const int tm = first_m + (bid % group) % gsz;
  const int tn = (bid % group) / gsz;
  const int m0 = tm * BM_, n0 = tn * BN_;

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid / WN, wc = wid % WN;

  int va[NLA], vb[NLB];
  dma_offsets3<KB, AK, NLA>(va, p.lda, wid, lane);
  dma_offsets3<KB, BK, NLB>(vb, p.ldb, wid, lane);
  const unsigned long long a_org = AK ? (unsigned long long)m0 * p.lda * 2 : (unsigned long long)m0 * 2;
  const unsigned long long b_org = BK ? (unsigned long long)n0 * p.ldb * 2 : (unsigned long long)n0 * 2;
  const unsigned long long a_step = AK ? KB * 2ull : (unsigned long long)KB * p.lda * 2;
  const unsigned long long b_step = BK ? KB * 2ull : (unsigned long long)KB * p.ldb * 2;
  floatx4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int nk_all = (p.K + KB - 1) / KB;
  const int splits = ts.splits;
  const int per = (nk_all + splits - 1) / splits;
  const int kt0 = ts.split * per;
  const int nk = max(0, min(nk_all, kt0 + per) - kt0);
#define DPC_ISSUE3(it_)                                                                             \
  do {                                                                                              \
    bf16_t* base_ = smem + ((it_) % STAGES) * (Cfg::TA + Cfg::TB);                                  \
    const unsigned long long ktg_ = (unsigned long long)(kt0 + (it_));                              \
    issue_tile<NLA>(p.A, a_bytes, a_org + a_step * ktg_, va, base_, wid);                           \
    issue_tile<NLB>(p.B, b_bytes, b_org + b_step * ktg_, vb, base_ + Cfg::TA, wid);                 \
  } while (0)
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) DPC_ISSUE3(s);

  constexpr int PER_TILE = NLA + NLB;  // DMA instructions per wave per k-tile
  for (int kt = 0; kt < nk; ++kt) {
    const int after = min(STAGES - 2, nk - 1 - kt);
    if (STAGES >= 4 && after >= 2) wait_vm<(STAGES >= 4 ? 2 * PER_TILE : 0)>();
    else if (STAGES >= 3 && after >= 1) wait_vm<(STAGES >= 3 ? PER_TILE : 0)>();
    else wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + STAGES - 1 < nk) DPC_ISSUE3(kt + STAGES - 1);
    const bf16_t* la = smem + (kt % STAGES) * (Cfg::TA + Cfg::TB);
    const bf16_t* lb = la + Cfg::TA;
#pragma unroll
    for (int ks = 0; ks < KB / 32; ++ks) {
      bf16x8 fa[FM], fb[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) fb[j] = frag3<KB, BK>(lb, wc * Cfg::WTN + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i) fa[i] = frag3<KB, AK>(la, wr * Cfg::WTM + i * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }
#undef DPC_ISSUE3

  // ---------------- epilogue (as v2): WTM/32 passes of 32 rows per wave through LDS
  epi_tile<FM, (FM == 4 && Cfg::WGS == 1)>(p, acc, reinterpret_cast<float*>(smem) + wid * 32 * 64, splits, m0 + wr * Cfg::WTM, n0 + wc * 64, lane);
}

// (v5, the 256x256 eight-wave ping-pong kernel, was removed in round 5: no tuned-table entry and
// no policy branch chose it once v7 took the weight gradients)

}  // namespace dpc

using namespace dpc;

template <int BM_, int BN_, int WM, int WN, int KB, int STAGES>
static void launch_v3(const GemmArgs* a, dim3 grid, hipStream_t stream, unsigned long long ab,
                      unsigned long long bb) {
  constexpr int NTH = V3Cfg<BM_, BN_, WM, WN, KB, STAGES>::NTH;
  if (a->a_kmaj && a->b_kmaj)
    hipLaunchKernelGGL((gemm3_kernel<BM_, BN_, WM, WN, KB, STAGES, true, true>), grid, dim3(NTH), 0, stream, *a, ab, bb);
  else if (a->a_kmaj)
    hipLaunchKernelGGL((gemm3_kernel<BM_, BN_, WM, WN, KB, STAGES, true, false>), grid, dim3(NTH), 0, stream, *a, ab, bb);
  else if (!a->b_kmaj)
    hipLaunchKernelGGL((gemm3_kernel<BM_, BN_, WM, WN, KB, STAGES, false, false>), grid, dim3(NTH), 0, stream, *a, ab, bb);
  else
    hipLaunchKernelGGL((gemm3_kernel<BM_, BN_, WM, WN, KB, STAGES, false, true>), grid, dim3(NTH), 0, stream, *a, ab, bb);
}

static inline long long operand_bytes(long long rows, long long cols, long long ld) {
  // bytes a tile load may legitimately touch: [rows][ld], 16-B chunks up to roundup8(cols)
  if (rows <= 0 || cols <= 0) return 0;
  return ((rows - 1) * ld + ((cols + 7) / 8) * 8) * 2;
}

template <int KB, int STAGES>
static void launch_v2(const GemmArgs* a, dim3 grid, hipStream_t stream, unsigned long long ab,
                      unsigned long long bb) {
  if (a->a_kmaj && a->b_kmaj) hipLaunchKernelGGL((gemm2_kernel<KB, STAGES, true, true>), grid, dim3(NT), 0, stream, *a, ab, bb);
  else if (a->a_kmaj) hipLaunchKernelGGL((gemm2_kernel<KB, STAGES, true, false>), grid, dim3(NT), 0, stream, *a, ab, bb);
  else if (!a->b_kmaj) hipLaunchKernelGGL((gemm2_kernel<KB, STAGES, false, false>), grid, dim3(NT), 0, stream, *a, ab, bb);
  else hipLaunchKernelGGL((gemm2_kernel<KB, STAGES, false, true>), grid, dim3(NT), 0, stream, *a, ab, bb);
}

// -1: auto; 1: v1; 2: v2 KB64 x2 stages; 3: KB64 x3; 4: KB32 x3; 5: KB32 x4;
// 6-10: v3 (6: 256x256 KB64 x2, 7: 256x256 KB32 x4, 8: 256x128 KB64 x2, 9: 256x128 KB32 x4,
// 10: 256x128 KB32 x3); (11-14: v4 / v5 / v6, removed);
// 16 / 19 / 20: v7 (gemm7.hip: persistent one-wave-per-SIMD 256x256, 5-slot ring; DMA
// placement 0 / 1 / 2); 17: v7, one unit per workgroup; plain f32 products split K
static int g_gemm_impl = -1;
// XCD-aligned split-K mapping (tile_slot): measured ~6 % slower than the default mapping on
// the GPT-2 weight gradients, so off unless requested (sweeps)
static int g_xcd_split = 0;
// > 0: force this split-K count for plain f32 products (sweeps)
static int g_force_splits = 0;

DPC_API void dpc_gemm_set_impl(int impl) { g_gemm_impl = impl; }
DPC_API void dpc_gemm_set_xcd_split(int on) { g_xcd_split = on; }
DPC_API void dpc_gemm_set_splits(int s) { g_force_splits = s; }

static inline bool al(const void* p, int b) { return ((uintptr_t)p % b) == 0; }

// Per-class implementation override for sweeps, from the environment, e.g.
// DPC_GEMM_POLICY="fs=11,dl=4": fs / fl = forward (both k-major) with K <= / > 1024,
// ds / dl = dgrad (B mn-major) with K <= / > 2304, w = weight gradient (both mn-major).
static int g_policy[5] = {0, 0, 0, 0, 0};
static int g_policy_read = 0;
static int policy_impl(const GemmArgs* a) {
  if (!g_policy_read) {
    g_policy_read = 1;
    if (const char* e = getenv("DPC_GEMM_POLICY")) {
      const char* names[5] = {"fs", "fl", "ds", "dl", "w"};
      for (int c = 0; c < 5; ++c) {
        char key[8];
        snprintf(key, sizeof key, "%s=", names[c]);
        for (const char* q = e; (q = strstr(q, key)) != nullptr; ++q)
          if (q == e || q[-1] == ',') { g_policy[c] = atoi(q + strlen(key)); break; }
      }
    }
  }
  int c;
  if (a->a_kmaj && a->b_kmaj) c = a->K <= 1024 ? 0 : 1;
  else if (a->a_kmaj) c = a->K <= 2304 ? 2 : 3;
  else if (!a->b_kmaj) c = 4;
  else return 0;
  return g_policy[c];
}

extern "C" int dpc_gemm7(const GemmArgs* a, int persistent, int sched, int splits, hipStream_t stream, int wn);
extern "C" int dpc_gemm7_ok(const GemmArgs* a);

// GemmArgs::nt_store for every product (DPC_GEMM_NT: bit 0 bf16 outputs, bit 1 f32 outputs
// non-temporal; bits 2-3 the cache scope of the v7 / v9 epilogue stores: 0 none, 1 sc0, 2 sc1,
// 3 sc0 sc1).  Default 15 = nt + sc0 sc1: the epilogue's stores retire sooner, and the next
// tile's counted DMA waits -- which CDNA4's one in-order vmcnt makes wait for them too -- stall
// less.  Same box against nt alone (round 5, profiles/r5_epi/store_policy.log): up-projection
// fused 402 -> 384 us, down-projection fused 367 -> 349, plain up 283 -> 274, plain input
// gradient 300 -> 290; DDP 960.8K -> 971.6K (two runs each).  Bits 4-6: a separate scope for
// the f32 outputs (gemm.h:g_f32_pol) -- default 77 = the above for bf16 outputs, PLAIN stores for
// the f32 ones (the residual stream and the split-K slabs, which the next LayerNorm / the slab
// reduction read back at once from the Infinity Cache): DDP +0.45 % same box, three interleaved
// rounds (984.1 / 981.2 / 981.7K -> 989.7 / 984.5 / 985.5K, profiles/r5_epi/f32_store_scope.log).
static int gemm_nt_mode() {
  static int mode = -1;
  if (mode < 0) mode = getenv("DPC_GEMM_NT") ? atoi(getenv("DPC_GEMM_NT")) : 77;
  return mode;
}

DPC_API int dpc_gemm(const GemmArgs* a, hipStream_t stream) {
  if (a->M <= 0 || a->N <= 0) return 0;
  // aux_deriv: GELU' as the second output (v9 / v7 / v7-generic / v2 / v3 epilogues; v7d and the
  // LDS-staged residual epilogue are skipped by gemm7.hip)
  if (a->aux_deriv && (!a->aux_out || a->act != ACT_GELU)) return -1;
  const int tiles = ((a->M + BM - 1) / BM) * ((a->N + BN - 1) / BN);
  dim3 grid(tiles), block(NT);
  // v2 requirements: a k-major operand must hold exactly K (% 64) columns (its k-tail is not
  // zeroed by the descriptor), N % 4 == 0 and 16-B aligned f32 epilogue operands (vector
  // epilogue), every operand inside a 31-bit byte range.
  const long long ab = operand_bytes(a->a_r, a->a_c, a->lda);
  const long long bb = operand_bytes(a->b_r, a->b_c, a->ldb);
  const bool kmaj_ok = (!a->a_kmaj || (a->a_c == a->K && a->K % 64 == 0)) &&
                       (!a->b_kmaj || (a->b_c == a->K && a->K % 64 == 0));
  const bool v2_ok = kmaj_ok && a->N % 4 == 0 && ab > 0 && bb > 0 && a->K > 0 && a->ldc % 4 == 0 && a->ldr % 4 == 0 &&
                     a->ld_aux_in % 4 == 0 && a->ld_aux_out % 4 == 0 &&
                     al(a->C, a->out_f32 ? 16 : 8) && al(a->bias, 16) && al(a->residual, 16) &&
                     al(a->aux_in, 8) && al(a->aux_out, 8) && al(a->colsum, 4);
  int impl = g_gemm_impl;
  if (impl < 0 && a->impl > 0) impl = a->impl;
  const bool plain_any = !a->bias && !a->residual && !a->aux_in && !a->aux_out && !a->colsum && !a->act &&
                         !a->act_bwd;
  if (impl < 0 && plain_any && policy_impl(a) <= 0 && dpc_gemm7_ok(a)) {
    // products without a fused epilogue -- the QKV / out / LM-head forward, every input
    // gradient without act', the weight gradients (split K) -- run the persistent 4-wave
    // kernel (v7); GPT-2 small B=64 shapes on MI355X: 940-1,220 TF/s vs 640-940 for the
    // 8-wave / 128-wide kernels (bench/gemm_ab.py, profiles/r2_gemm/)
    impl = 20;
  }
  // forward epilogues that read nothing per element (bias / activation / aux_out: the FFN
  // products, whose table entries all name v9) default to v9's load-free epilogue when no table
  // entry covers the shape -- e.g. the down projection as a bias-only product since round 6 (its
  // residual add moved into the next LayerNorm), which the older policy sent to the 128 x 128
  // kernel at 366 us against ~280
  const bool fwd_epi = a->a_kmaj && a->b_kmaj && !plain_any && !a->residual && !a->accumulate && !a->aux_in &&
                       !a->colsum && !a->act_bwd && a->K % 64 == 0 && a->K >= 192;
  if (impl < 0 && fwd_epi && policy_impl(a) <= 0 && dpc_gemm7_ok(a)) impl = 26;
  if (impl < 0) {
    // Default per operand layout and depth, from the GPT-2 shape sweep on MI355X
    // (bench/kernels.py, profiles/kernels_r1_*.json): forward products with a short K
    // (<= 1024) are epilogue/prologue heavy and run best as 256x128 tiles two workgroups
    // per CU (impl 10); deep or mn-major products keep the 128x128 2-stage kernel (impl 2),
    // except dgrad at K <= 2304 and mid-size wgrad, where the 3-stage 32-deep ring wins.
    impl = 1;
    if (v2_ok) {
      impl = 2;
      if (a->a_kmaj && a->b_kmaj && a->K <= 1024) impl = 10;
      else if (a->a_kmaj && !a->b_kmaj && a->K <= 1024) impl = 10;  // dgrad + act' / colsum epilogue
      else if (a->a_kmaj && !a->b_kmaj && a->K <= 2304) impl = 4;
      else if (!a->a_kmaj && !a->b_kmaj && a->M > 2304 && a->M <= 4096) impl = 4;
      const int pol = policy_impl(a);
      if (pol > 0) impl = pol;
    }
  }
  // plain f32 products (weight gradients: small M x N, K = tokens) are split along K
  const bool plain = a->out_f32 && !a->bias && !a->residual && !a->aux_in && !a->aux_out &&
                     !a->colsum && !a->act && !a->act_bwd;
  if (g_gemm_impl < 0 && a->impl <= 0 && v2_ok && plain && !a->a_kmaj && !a->b_kmaj && policy_impl(a) <= 0) {
    // weight gradient: the split-K persistent kernel (v7, chosen above when its requirements
    // hold -- its own planner splits K to fill the chip however few tiles there are), else the
    // 2-stage 64-k kernel.  (Round 4: the pipeline stage proxy's micro-batch
    // out-projection weight gradient, 1024 x 1024 x 16368, off the table, fell to the 2-stage
    // kernel at 506 TF/s -- 8.7 ms of a 262 ms stage step, profiles/r4_pp/.)
    if (impl != 20) impl = 2;
  }
  if (impl >= 15 && impl <= 26) {  // v7 (gemm7.hip): 4-wave 256x256, split-K f32 products
    GemmArgs c = *a;
    c.ksplit = 0;
    c.nt_store = gemm_nt_mode();
    // (25: the split DMA interleave forced for plain products, SCHED 6; 20 / 22 pick it for
    // products with an mn-major operand; 26: v9, the 64-deep-stage kernel, which every other v7
    // placement takes for plain nt products)
    const int sched = impl == 19 ? 1 : (impl == 20 || impl == 17 || impl == 21 ? 2 : (impl == 22 ? 3 : (impl == 23 ? 4 : (impl == 24 ? 5 : (impl == 25 ? 6 : (impl == 26 ? 7 : 0))))));
    // 21: v8 -- 256x128 tiles, two persistent workgroups per CU (epilogue beside MFMAs)
    const int rc = dpc_gemm7(&c, impl != 17, sched, g_force_splits > 0 ? g_force_splits : 0, stream,
                             impl == 21 ? 64 : 128);
    if (rc >= 0) return rc;
    impl = v2_ok ? 2 : 1;  // requirements not met: the 128x128 kernels
  }
  if (impl >= 2 && !v2_ok) impl = 1;
  GemmArgs b = *a;  // dispatcher-owned copy: split-K mode is decided here
  b.ksplit = 0;
  b.nt_store = gemm_nt_mode();
  if (impl >= 2) {
    int bm = BM, bn = BN;
    if (impl >= 6) {
      bm = 256;  // (v3-v6)
      bn = (impl == 8 || impl == 9 || impl == 10) ? 128 : 256;
    }
    const int t = ((a->M + bm - 1) / bm) * ((a->N + bn - 1) / bn);
    const int nk = (a->K + BKT - 1) / BKT;
    int splits = 1;
    if (plain) {
      // Split-K count from a cost model fitted to the GPT-2 weight-gradient sweep on MI355X
      // (bench/wgrad_splits.py, profiles/r1_wgrad_splits.txt): time ~ rounds(s) / s + beta * s,
      // rounds = ceil(tiles * s / resident workgroups) (wave quantisation of the grid) and
      // beta * s the split-K partial-sum atomics relative to the K-proportional MFMA work.
      // resident workgroups per launch round: 256 CUs x workgroups per CU (LDS-bound, V2Cfg::WGS)
      const int slots = impl >= 6 || impl == 3 ? 256 : (impl == 4 ? 768 : 512);  // (v3-v6: 1 WG/CU)
      const double beta = 0.0056 * 32768.0 / (double)a->K;
      double best = 1e30;
      for (int s = 1; s <= 16 && (s == 1 || nk / s >= 8); ++s) {
        const long long rounds = ((long long)t * s + slots - 1) / slots;
        const double cost = (double)rounds / s + beta * s;
        if (cost < best - 1e-9) { best = cost; splits = s; }
      }
      if (g_force_splits > 0) splits = g_force_splits;
    }
    if (splits > 1 && !a->accumulate)
      hipMemset2DAsync(a->C, (size_t)a->ldc * 4, 0, (size_t)a->N * 4, (size_t)a->M, stream);
    dim3 g(t * splits);  // 1-D: tile_slot() maps block -> (split, tile)
    b.ksplit = splits > 1 ? (g_xcd_split ? -splits : splits) : 0;
    switch (impl) {
      case 3: launch_v2<64, 3>(&b, g, stream, ab, bb); break;
      case 4: launch_v2<32, 3>(&b, g, stream, ab, bb); break;
      case 10: launch_v3<256, 128, 4, 2, 32, 3>(&b, g, stream, ab, bb); break;
      case 2: launch_v2<64, 2>(&b, g, stream, ab, bb); break;
      default: return 1;  // (5-9, 11-14: removed implementations, chosen by no table or policy)
    }
    return (int)hipGetLastError();
  }
  if (a->a_kmaj && a->b_kmaj) hipLaunchKernelGGL((gemm_kernel<true, true>), grid, block, 0, stream, b);
  else if (a->a_kmaj && !a->b_kmaj) hipLaunchKernelGGL((gemm_kernel<true, false>), grid, block, 0, stream, b);
  else if (!a->a_kmaj && !a->b_kmaj) hipLaunchKernelGGL((gemm_kernel<false, false>), grid, block, 0, stream, b);
  else hipLaunchKernelGGL((gemm_kernel<false, true>), grid, block, 0, stream, b);
  return (int)hipGetLastError();
}
