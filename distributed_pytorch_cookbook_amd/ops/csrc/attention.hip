// Flash attention (forward + backward) for gfx950: head_dim 32, 64 or 128 natively (template HD),
// bf16 in / bf16 out, f32 online softmax, causal + optional key-padding mask.
//
// Replaces the reference's materialised attention (/root/reference/models/gpt.py:75-100: q@k,
// host-built causal mask copied H2D every layer, masked_fill, fp32 softmax, @v, head merge)
// with O(S) kernels that read q/k/v straight out of the fused QKV projection ([T, 3*H*hd],
// token-major) and write the merged-head output [T, H*hd] -- no permute/clone copies.
//
// MFMA layout (v_mfma_f32_32x32x16_bf16; C/D: col = lane & 31,
// row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)):
//   forward  S^T = K Q^T   -> the query sits on the lane, so the row max / row sum are
//            lane-local (+ one xor-32 shuffle) and the O^T = V^T P^T accumulator is
//            rescaled without any cross-lane traffic.  The S^T accumulator registers are
//            the B operand of the PV product directly (pairs packed to bf16); V^T comes
//            from LDS through ds_read_b64_tr_b16 (transposing read).
//   backward dK/dV kernel: S = Q K^T and dP = dO V^T with the key on the lane (K, V rows
//            live in registers for the whole sweep over queries); P / dS registers feed
//            dV^T += dO^T P and dK^T += Q^T dS with dO^T / Q^T via transposing reads.
//            dQ kernel: S^T, dP^T with the query on the lane, dQ^T += K^T dS^T.
//            No float atomics: each output is owned by exactly one wave.
//
// Pipeline (every kernel): the streamed 64-row tiles (K/V, or Q/dO + their per-row lse /
// delta) arrive by LDS-DMA into a 4-slot ring, issued from inline asm two tiles ahead, so the
// only wait is a counted vmcnt + barrier per tile at the top of the loop.  Inside a wave the
// work of adjacent 32-row sub-blocks is software-pipelined: the score MFMAs of sub-block
// j+1 sit in the same basic block as the softmax VALU of sub-block j (independent, so the
// scheduler interleaves them), then the accumulate MFMAs of j -- a wave alternates MFMA and
// VALU work on its own instead of relying on lock-stepped partner waves.
//
// LDS image of a tile: the [64 rows][HD] bf16 tile is stored as 128-B physical rows (HD=64:
// one row each; HD=32: two rows each) with the 16-B chunk swizzle
//   chunk ^ (((prow >> 1) & 7) ^ (((prow >> 1) & 1) << 2))
// which is conflict free for the ds_read_b128 row reads and the tr_b16 column reads at both
// head sizes.
#include "common.h"

#include <cstdio>
#include <cstdlib>
#include <type_traits>

namespace dpc {

struct AttnArgs {
  const void* q; const void* k; const void* v;  // bf16, row = token (n*S + s), head h at col h*hd
  void* o;                                      // bf16 [T][ld_o]
  float* lse;                                   // f32 [N*H][S] (natural log of scaled scores)
  const unsigned char* pad;                     // [N][S], 1 = padded key (masked), optional
  const void* dout;                             // bwd: dO bf16 [T][ld_o]
  void* dq; void* dk; void* dv;                 // bwd: bf16 outputs, row stride ld_dqkv
  float* delta;                                 // bwd: f32 [2][N*H][S]: delta, then lse in log2 units
  long long ld_qkv, ld_o, ld_dqkv;
  int N, S, H;
  float scale;
  int causal;
  int hd;                                       // head_dim: 32, 64 or 128
  int order;                                    // backward block order (set by the launcher: DPC_ATTN_ORDER)
};

constexpr int KT = 64;       // keys (or queries) per staged tile
constexpr int QB = 128;      // rows per workgroup (4 waves x 32)
constexpr int NSLOT = 4;     // LDS ring depth: tiles t (read), t+1 (landed), t+2, t+3 (in flight)
constexpr float LOG2E = 1.4426950408889634f;

template <int HD>
struct AT {
  static_assert(HD == 32 || HD == 64 || HD == 128, "head_dim 32, 64 or 128");
  static constexpr int TILE = KT * HD;   // elements of one 64-row tile
  static constexpr int NPW = HD / 32;    // 1-KiB DMA pieces per wave per tile (4 waves)
  static constexpr int NST = HD / 16;    // k-steps of a product over head_dim (32x32x16)
  static constexpr int NDT = HD / 32;    // 32-column blocks of an HD-wide accumulator
};

typedef short4_t __attribute__((address_space(3))) * lds4_t;
typedef __attribute__((address_space(3))) void* lds_void_t;

__device__ __forceinline__ int aswz(int prow) {
  const int a = (prow >> 1) & 7;
  return a ^ ((a & 1) << 2);
}
// element offset of (row, 16-B chunk) in the LDS image of a tile
template <int HD>
__device__ __forceinline__ int toff(int row, int chunk) {
  const int e = row * HD + chunk * 8;
  const int prow = e >> 6, pch = (e >> 3) & 7;
  return (prow << 6) + ((pch ^ aswz(prow)) << 3);
}

// ---- LDS-DMA from inline asm (buffer_load ... lds; M0 = the wave's LDS destination).
// Issued from asm so that the compiler does not wait for it before every LDS read: the
// kernels wait with explicit counted s_waitcnt at the ring boundary.
// M0 is declared clobbered rather than saved / restored around each piece: the save / restore pair
// was 2 of the ~13 scalar instructions per MFMA the forward issues (rocprofv3 SQ_INSTS_SALU,
// profiles/r5_attn/pmc_final.txt), and with the clobber the compiler itself keeps any value of its
// own out of M0 across the DMA (today it uses M0 for nothing in these kernels, so the clobber
// costs no instruction: the gfx950 asm is identical with and without it).
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, int voff, const void* lds) {
  const unsigned la = (unsigned)(uintptr_t)(lds_void_t)lds;
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               :
               : "v"(voff), "s"(rs), "s"(la)
               : "memory", "m0");
}
__device__ __forceinline__ void dma4(__amdgpu_buffer_rsrc_t rs, int voff, const void* lds) {
  const unsigned la = (unsigned)(uintptr_t)(lds_void_t)lds;
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dword %0, %1, 0 offen lds"
               :
               : "v"(voff), "s"(rs), "s"(la)
               : "memory", "m0");
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// Make the compiler wait for the kernel's own register loads (the per-row operands held for
// the whole sweep) HERE, before any LDS-DMA is in flight: left to itself it places that
// s_waitcnt at the first use -- inside the tile loop -- and, not counting the asm DMA, as
// vmcnt(0), which drains the ring's prefetch on every iteration.
template <int N>
__device__ __forceinline__ void pin_loaded(const bf16x8 (&x)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" ::"v"(x[i]));
}
__device__ __forceinline__ void pin_loaded(float x) { asm volatile("" ::"v"(x)); }

__device__ __forceinline__ void ring_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Descriptor of rows row0 .. S-1 of a [S][ld] operand (rows past S, or all of them if !valid, read
// as zeros).  32-bit offsets: the host guarantees (S + 256) * ld_bytes < 2^32 (attn_args_ok) --
// the 64-bit form (multiplies, a 64-bit clamp through VALU compares) was ~20 scalar instructions
// per descriptor, two descriptors per tile step.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const void* base, unsigned ld_bytes, int row0, int S,
                                                           bool valid) {
  const unsigned span = (unsigned)S * ld_bytes;
  const unsigned off = (unsigned)row0 * ld_bytes;
  // (readfirstlane: left alone, the compiler forms the clamp as a VALU saturating subtract and the
  // whole descriptor in VGPRs, which the DMA asm's "s" operand cannot take)
  const unsigned nrec = __builtin_amdgcn_readfirstlane((valid && off < span) ? span - off : 0u);
  return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)base + off), 0, nrec, 0x00020000);
}

// The DMA writes lane-linearly -- piece g (wave wid, instruction i: g = wid * NPW + i) fills
// physical rows 8g .. 8g+7, lane l slot (l & 7) of physical row 8g + (l >> 3) -- so the chunk
// swizzle moves to the SOURCE address: the lane fetches the logical (row, chunk) that the
// swizzle maps to its slot.  v: the lane's byte offsets relative to the tile's first row.
template <int HD>
__device__ __forceinline__ void dma_voff(int (&v)[AT<HD>::NPW], long long ld, int wid, int lane) {
#pragma unroll
  for (int i = 0; i < AT<HD>::NPW; ++i) {
    const int prow = 8 * (wid * AT<HD>::NPW + i) + (lane >> 3);
    const int e = prow * 64 + (((lane & 7) ^ aswz(prow)) << 3);
    const int row = e / HD, chunk = (e % HD) >> 3;
    v[i] = (int)((long long)row * ld * 2 + chunk * 16);
  }
}

// one 64-row tile (rows >= S, or the whole tile if !valid, land as zeros)
template <int HD>
__device__ __forceinline__ void tile_dma(const bf16_t* base, long long ld, int row0, int S, bool valid,
                                         const int (&v)[AT<HD>::NPW], bf16_t* lds, int wid) {
  const __amdgpu_buffer_rsrc_t rs = rows_rsrc(base, (unsigned)(ld * 2), row0, S, valid);
#pragma unroll
  for (int i = 0; i < AT<HD>::NPW; ++i) dma16(rs, v[i], lds + (wid * AT<HD>::NPW + i) * 512);
}

// Row fragment (A or B operand of 32x32x16): lane holds X[row0 + (lane & 31)][16 st + 8 h .. +7]
template <int HD>
__device__ __forceinline__ bf16x8 row_frag(const bf16_t* lds, int row0, int st, int lane) {
  return *reinterpret_cast<const bf16x8*>(lds + toff<HD>(row0 + (lane & 31), 2 * st + (lane >> 5)));
}

// Transposed fragment: lane gets X[rows r0 + 16 s + 8 (j >> 2) + 4 h + (j & 3)][col c0 + (lane & 31)]
// i.e. the permuted k order of an accumulator-as-operand k-step s.
template <int HD>
__device__ __forceinline__ bf16x8 tr_frag(const bf16_t* lds, int r0, int s, int c0, int lane) {
  const int h = lane >> 5, g2 = (lane >> 4) & 1, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
  const int row = r0 + 16 * s + 4 * h + q;
  const int col = c0 + 16 * g2 + 4 * p;
  const bf16_t* a0 = lds + toff<HD>(row, col >> 3) + (col & 7);
  const bf16_t* a1 = lds + toff<HD>(row + 8, col >> 3) + (col & 7);
  short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4_t)a0);
  short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4_t)a1);
  typedef short short8_t __attribute__((ext_vector_type(8)));
  short8_t s8 = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, s8);
}

// Accumulator registers 8s..8s+7 -> bf16 operand fragment of k-step s.
__device__ __forceinline__ bf16x8 acc_frag(const floatx16& x, int s) {
  uint4 u;
  u.x = pack2bf(x[8 * s + 0], x[8 * s + 1]);
  u.y = pack2bf(x[8 * s + 2], x[8 * s + 3]);
  u.z = pack2bf(x[8 * s + 4], x[8 * s + 5]);
  u.w = pack2bf(x[8 * s + 6], x[8 * s + 7]);
  return __builtin_bit_cast(bf16x8, u);
}

__device__ __forceinline__ int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// Row-per-lane epilogue stores, widened: lane (row = lane & 31, hh = lane >> 5) holds the 4
// bf16 at columns 8 g + 4 hh .. +3 of column group g (wa: group g, wb: group g + 1, g even).
// One v_permlane32_swap per dword (lanes 32..63 of wa <-> lanes 0..31 of wb) leaves lanes 0..31
// with columns 8 g .. 8 g + 7 and lanes 32..63 with 8 g + 8 .. 8 g + 15 of the SAME row, so the
// pair leaves in one 16-B store per lane instead of two 8-B ones: half the store instructions
// of a store-issue-bound tail (cdna_hip_programming.md T21).  Lanes l and l + 32 hold the same
// row, so a row guard (key / query < S) keeps both or neither active.
// (plain stores: the nt / sc0 sc1 nt scopes that speed up the GEMM epilogues measured 5-10 %
// slower here -- O, dQ, dK, dV are re-read at once by the next GEMM; profiles/r5_epi/attn_store_policy.log)
__device__ __forceinline__ void store_pair16(bf16_t* row, int g, int hh, uint2 wa, uint2 wb) {
  const auto s0 = __builtin_amdgcn_permlane32_swap(wa.x, wb.x, false, false);
  const auto s1 = __builtin_amdgcn_permlane32_swap(wa.y, wb.y, false, false);
  *reinterpret_cast<uint4*>(row + 8 * g + 8 * hh) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
}

// raw v_exp_f32 (2^x): inputs here are <= ~8 or -inf, no denormal range reduction needed
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// v_max3_f32.  This file is built with -fno-honor-nans (nothing here produces a NaN), so
// fmaxf on MFMA results needs no canonicalising v_max and pairs fold into v_max3.
__device__ __forceinline__ float max3f(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }

// 64-key padding bitmask of the tile starting at key k0 (bit i = key k0+i is padded); wave-uniform
__device__ __forceinline__ unsigned long long pad_bits(const unsigned char* pad, int k0, int S, int lane) {
  if (!pad) return 0ull;
  const int k = k0 + lane;
  return __ballot(k < S && pad[k] != 0);
}

__device__ __forceinline__ bf16x8 load_row8(const bf16_t* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}

#define MFMA32(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_bf16((a), (b), (c), 0, 0, 0)

// x *= a in place, element by element (inline asm with tied operands): written as plain C++
// inside the lazy-rescale branch, hipcc gave the rescaled accumulator new registers and paid
// 16 v_mov_b64 on EVERY tile to merge the two versions after the branch (round-5 asm of
// attn_fwd2_kernel); a v_mul_f32 per element also avoids v_pk_mul_f32, which costs extra
// issue cycles beside MFMAs (MI355X_MICROARCH.md, cycle constants)
__device__ __forceinline__ void scale16(floatx16& x, float a) {
#pragma unroll
  for (int i = 0; i < 16; ++i) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x[i]) : "v"(a));
}

// x[r] = 0 if v > K, in place (v_cmp + v_cndmask on the element's own register: a C++ select in
// one arm of a branch gave the element a new register and both arms a copy back)
template <int K>
__device__ __forceinline__ void zero_if_gt(floatx16& x, int r, int v) {
  asm volatile("v_cmp_lt_i32_e32 vcc, %1, %2\n\tv_cndmask_b32_e64 %0, %0, 0, vcc"
               : "+v"(x[r])
               : "n"(K), "v"(v)
               : "vcc");
}

// x *= a when `up` (a wave ballot, SGPR pair) is non-zero.  The branch sits INSIDE the asm statement, so the
// compiler sees straight-line code and has no join after which to copy the accumulator (a C++
// branch around scale16 gave both O accumulators new registers and a copy back on the path that
// did not rescale: 16 v_mov_b64 on most tiles, round-6 listing of attn_fwd2_kernel).  The s_nops
// keep the MFMA-result -> VALU and VALU -> MFMA-SrcC distances on the (rare) taken path, which the
// hazard recognizer cannot see inside asm.
#define DPC_RS_MUL(i) "v_mul_f32 %" #i ", %" #i ", %16\n\t"
__device__ __forceinline__ void scale16_if(floatx16& x, float a, unsigned long long up) {
  asm volatile(
      "s_cmp_eq_u64 %17, 0\n\t"
      "s_cbranch_scc1 .Ldpc_rs%=\n\t"
      "s_nop 7\n\ts_nop 7\n\t"
      DPC_RS_MUL(0) DPC_RS_MUL(1) DPC_RS_MUL(2) DPC_RS_MUL(3) DPC_RS_MUL(4) DPC_RS_MUL(5) DPC_RS_MUL(6)
      DPC_RS_MUL(7) DPC_RS_MUL(8) DPC_RS_MUL(9) DPC_RS_MUL(10) DPC_RS_MUL(11) DPC_RS_MUL(12)
      DPC_RS_MUL(13) DPC_RS_MUL(14) DPC_RS_MUL(15)
      "s_nop 7\n"
      ".Ldpc_rs%=:"
      : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),
        "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15])
      : "v"(a), "s"(up)
      : "scc");
}
#undef DPC_RS_MUL

// The plain tile's whole lazy-rescale update, when the ballot `up` is non-zero: mn = max(m, mx), alpha = 2^(m - mn),
// m = mn, l *= alpha, x *= alpha (the first O accumulator); alpha is returned for the others
// (scale16_if).  Nothing of it runs on the tiles that keep the running max (most of them): fwd2
// formed alpha and selected m / l on every tile.  m = -inf (a block's first tile) gives alpha = 0
// on zero accumulators; up is never set with mx = -inf.  s_nop 0 after v_exp: gfx950's
// transcendental-result wait state; v_swap_b32 leaves m = mn and alpha in a (one temporary).
#define DPC_RS_MUL(i) "v_mul_f32 %" #i ", %" #i ", %17\n\t"
__device__ __forceinline__ float rescale16_if(floatx16& x, float& m, float& l, float mx, unsigned long long up) {
  float a;
  asm volatile(
      "s_cmp_eq_u64 %20, 0\n\t"
      "s_cbranch_scc1 .Ldpc_ru%=\n\t"
      "s_nop 7\n\ts_nop 7\n\t"
      "v_max_f32 %17, %16, %19\n\t"
      "v_sub_f32 %16, %16, %17\n\t"
      "v_exp_f32 %16, %16\n\t"
      "s_nop 0\n\t"
      "v_swap_b32 %16, %17\n\t"
      "v_mul_f32 %18, %18, %17\n\t"
      DPC_RS_MUL(0) DPC_RS_MUL(1) DPC_RS_MUL(2) DPC_RS_MUL(3) DPC_RS_MUL(4) DPC_RS_MUL(5) DPC_RS_MUL(6)
      DPC_RS_MUL(7) DPC_RS_MUL(8) DPC_RS_MUL(9) DPC_RS_MUL(10) DPC_RS_MUL(11) DPC_RS_MUL(12)
      DPC_RS_MUL(13) DPC_RS_MUL(14) DPC_RS_MUL(15)
      "s_nop 7\n"
      ".Ldpc_ru%=:"
      : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),
        "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]),
        "+v"(m), "=&v"(a), "+v"(l)
      : "v"(mx), "s"(up)
      : "scc");
  return a;
}
#undef DPC_RS_MUL

__device__ __forceinline__ void zero16(floatx16& x) {
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = 0.f;
}

// XCD-aware work id (1-D grid of nblk * N * H workgroups): workgroup b runs on XCD b % 8, and
// the bijective remap gives every XCD a contiguous run of ids, so all the q- (or key-) blocks
// of one (batch, head) -- which read the same K/V (Q/dO) rows -- share one XCD's L2.
// Returns (bh, i): i = block index within the head.
__device__ __forceinline__ int g7_local_attn(int b, int grid) {
  const int xcd = b & 7, q = grid >> 3, r = grid & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}
// order 1 (the backward kernels' default, DPC_ATTN_ORDER): block-major over the whole grid in launch
// order -- every (batch, head)'s heaviest causal block first, the lightest last, so the grid's
// tail is light blocks -- at the cost of the L2 sharing of one head's rows across its blocks
__device__ __forceinline__ void work_order1(int nblk, int& bh, int& i) {
  const int nbh = gridDim.x / nblk;
  i = blockIdx.x / nbh;
  bh = blockIdx.x - i * nbh;
}
__device__ __forceinline__ void xcd_work(int nblk, int& bh, int& i) {
  const int b = blockIdx.x, nwg = gridDim.x, xcd = b & 7, q = nwg >> 3, r = nwg & 7;
  const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
  bh = t / nblk;
  i = t - bh * nblk;
}

// ------------------------------------------------------------------ forward
// Workgroup = 128 queries (4 waves x 32, query on the lane), sweeping 64-key tiles.  Per tile
// and wave: S^T of the NEXT tile (2 x NST MFMAs) overlaps this tile's softmax, then
// O^T += V^T P^T (4 x NDT MFMAs).
// PIPE: 0 = plain order, 1 = next tile's S^T beside this tile's softmax, 2 = 1 + the tile's
// LDS fragments read up front and the MFMA / VALU interleave pinned (sched_group_barrier)
template <int HD, int PIPE, int OCC>
__global__ __launch_bounds__(256, OCC) void attn_fwd_kernel(AttnArgs p) {
  using A = AT<HD>;
  __shared__ __attribute__((aligned(16))) bf16_t smem[NSLOT * 2 * A::TILE];  // [slot][K|V]
  const int S = p.S, H = p.H;
  const int nqb = (S + QB - 1) / QB;
  int bh, bi;
  xcd_work(nqb, bh, bi);
  const int qb = nqb - 1 - bi;  // heaviest causal blocks of a head first
  const int n = bh / H, h = bh % H;
  const int lane = threadIdx.x & 63, hh = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q0 = qb * QB + wid * 32;
  const int q = q0 + (lane & 31);
  const long long tok0 = (long long)n * S;
  const bf16_t* Q = static_cast<const bf16_t*>(p.q) + h * HD;
  const bf16_t* K = static_cast<const bf16_t*>(p.k) + tok0 * p.ld_qkv + h * HD;
  const bf16_t* V = static_cast<const bf16_t*>(p.v) + tok0 * p.ld_qkv + h * HD;

  bf16x8 qf[A::NST];
#pragma unroll
  for (int st = 0; st < A::NST; ++st)
    qf[st] = q < S ? load_row8(Q + (tok0 + q) * p.ld_qkv + 16 * st + 8 * hh) : bf16x8{};
  pin_loaded(qf);
  const float c = p.scale * LOG2E;
  const int kend = p.causal ? min(S, qb * QB + QB) : S;
  const int ntiles = (kend + KT - 1) / KT;
  // this wave's last tile holding a key it may attend to
  const int last_w = p.causal ? min(ntiles - 1, max(0, min(q0 + 31, S - 1)) / KT) : ntiles - 1;
  const unsigned char* pad = p.pad ? p.pad + (long long)n * S : nullptr;

  int dv[A::NPW];
  dma_voff<HD>(dv, p.ld_qkv, wid, lane);
  auto issue = [&](int t) {
    bf16_t* st = smem + (t % NSLOT) * 2 * A::TILE;
    const bool valid = t < ntiles;
    tile_dma<HD>(K, p.ld_qkv, t * KT, S, valid, dv, st, wid);
    tile_dma<HD>(V, p.ld_qkv, t * KT, S, valid, dv, st + A::TILE, wid);
  };
  // S^T = K Q^T of the tile in LDS at lk (keys on the accumulator rows, query on the lane)
  auto qk = [&](floatx16 (&s)[2], const bf16_t* lk) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      zero16(s[kb]);
#pragma unroll
      for (int st = 0; st < A::NST; ++st)
        s[kb] = MFMA32(row_frag<HD>(lk, kb * 32, st, lane), qf[st], s[kb]);
    }
  };

  float m = -INFINITY, l = 0.f;
  floatx16 o[A::NDT];
#pragma unroll
  for (int d = 0; d < A::NDT; ++d) zero16(o[d]);

  issue(0);
  issue(1);
  issue(2);
  vm_wait<4 * A::NPW>();  // tile 0 landed (tiles 1, 2 may fly)
  ring_barrier();
  // one tile: scores of tile t in sc; the next tile's land in sn (ping-pong, no copies)
  auto step = [&](int t, floatx16 (&sc)[2], floatx16 (&sn)[2]) {
    vm_wait<2 * A::NPW>();  // this wave's pieces of tile t+1 landed (t+2 may fly)
    ring_barrier();         // ... every wave's; and every wave is done with tile t-1's slot
    issue(t + 3);
    const bf16_t* lkn = smem + ((t + 1) % NSLOT) * 2 * A::TILE;
    const bf16_t* lv = smem + (t % NSLOT) * 2 * A::TILE + A::TILE;
    if (t > last_w) return;  // wave-uniform
    if constexpr (PIPE == 0) qk(sc, lv - A::TILE);
    // PIPE 2: the next tile's K row fragments and this tile's V^T fragments, read before the
    // softmax so their LDS latency hides under it
    bf16x8 kfr[2][A::NST], vfr[2][2][A::NDT];
    if constexpr (PIPE == 2) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int st = 0; st < A::NST; ++st) kfr[kb][st] = row_frag<HD>(lkn, kb * 32, st, lane);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int ss = 0; ss < 2; ++ss)
#pragma unroll
          for (int d = 0; d < A::NDT; ++d) vfr[kb][ss][d] = tr_frag<HD>(lv, kb * 32, ss, d * 32, lane);
    }
    const int kt0 = t * KT;
    // Scores stay raw (unscaled) until the exponent: p = 2^(s*c - m) is one FMA + v_exp.
    const bool need_mask = (p.causal && kt0 + KT - 1 > q0) || (kt0 + KT > S) || pad;  // wave-uniform
    if (need_mask) {
      // key > lim is causal / past-the-end, pm is the tile's padding bitmask
      const unsigned long long pm = pad_bits(pad, kt0, S, lane);
      const int lim = (p.causal ? min(q, S - 1) : S - 1) - kt0;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kl = kb * 32 + acc_row(r, lane);
          if (kl > lim || ((pm >> kl) & 1ull)) sc[kb][r] = -INFINITY;
        }
    }
    // the tile max as four independent v_max3 chains joined at the end (depth 6 instead of one
    // 16-deep dependent chain in front of every exponential of the tile)
    float mq[4];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const floatx16& sq = sc[q4 >> 1];
      const int r0 = (q4 & 1) * 8;
      float v = max3f(sq[r0], sq[r0 + 1], sq[r0 + 2]);
      v = max3f(v, sq[r0 + 3], sq[r0 + 4]);
      v = max3f(v, sq[r0 + 5], sq[r0 + 6]);
      mq[q4] = fmaxf(v, sq[r0 + 7]);
    }
    float mx = fmaxf(max3f(mq[0], mq[1], mq[2]), mq[3]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64)) * c;  // scaled log2 units (c > 0)
    // lazy rescale: the running max only moves when the tile max exceeds it by > 2^8, so
    // p <= 256 (exact enough in f32 / bf16) and the O rescale is skipped on most tiles
    if (__ballot(mx > m + 8.f)) {
      const float mn = fmaxf(m, mx);
      const float alpha = (mn == -INFINITY) ? 1.f : fast_exp2(m - mn);
      m = mn;
      l *= alpha;
#pragma unroll
      for (int d = 0; d < A::NDT; ++d) scale16(o[d], alpha);
    }
    const float nmu = (m == -INFINITY) ? 0.f : -m;
    // ---- one basic block: next tile's S^T MFMAs || this tile's exponentials
    if constexpr (PIPE == 2) {
      float ls = 0.f;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        zero16(sn[kb]);
#pragma unroll
        for (int st = 0; st < A::NST; ++st) sn[kb] = MFMA32(kfr[kb][st], qf[st], sn[kb]);
      }
      bf16x8 pb[2][2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = fast_exp2(fmaf(sc[kb][r], c, nmu));
          sc[kb][r] = e;
          ls += e;
        }
        pb[kb][0] = acc_frag(sc[kb], 0);
        pb[kb][1] = acc_frag(sc[kb], 1);
#pragma unroll
        for (int ss = 0; ss < 2; ++ss)
#pragma unroll
          for (int d = 0; d < A::NDT; ++d) o[d] = MFMA32(vfr[kb][ss][d], pb[kb][ss], o[d]);
      }
      l += ls;
      // interleave: the 2 NST score MFMAs carry the first half's ~56 VALU, the first half's
      // 2 NDT PV MFMAs the second half's, then the last PV MFMAs
      constexpr int NQ = 2 * A::NST, NP = 2 * A::NDT;
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 56 / NQ, 0);
      }
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 56 / NP, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, NP, 0);
      return;
    }
    if constexpr (PIPE == 1) qk(sn, lkn);
    float ls = 0.f;
    bf16x8 pb[2][2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = fast_exp2(fmaf(sc[kb][r], c, nmu));
        sc[kb][r] = e;
        ls += e;
      }
      pb[kb][0] = acc_frag(sc[kb], 0);
      pb[kb][1] = acc_frag(sc[kb], 1);
    }
    l += ls;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss)
#pragma unroll
        for (int d = 0; d < A::NDT; ++d)
          o[d] = MFMA32(tr_frag<HD>(lv, kb * 32, ss, d * 32, lane), pb[kb][ss], o[d]);
  };
  floatx16 s0[2], s1[2];
  if constexpr (PIPE != 0) qk(s0, smem);
  for (int t = 0; t < ntiles; t += 2) {
    step(t, s0, s1);
    if (t + 1 < ntiles) step(t + 1, s1, s0);
  }
  vm_wait<0>();  // the pieces issued past the last tile (empty descriptors) drained

  l += __shfl_xor(l, 32, 64);  // the two lane halves summed different key rows
  if (q < S) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    bf16_t* O = static_cast<bf16_t*>(p.o) + (tok0 + q) * p.ld_o + h * HD;
#pragma unroll
    for (int d = 0; d < A::NDT; ++d)
#pragma unroll
      for (int g = 0; g < 4; g += 2) {
        uint2 wa, wb;
        wa.x = pack2bf(o[d][4 * g + 0] * inv, o[d][4 * g + 1] * inv);
        wa.y = pack2bf(o[d][4 * g + 2] * inv, o[d][4 * g + 3] * inv);
        wb.x = pack2bf(o[d][4 * g + 4] * inv, o[d][4 * g + 5] * inv);
        wb.y = pack2bf(o[d][4 * g + 6] * inv, o[d][4 * g + 7] * inv);
        store_pair16(O + d * 32, g, hh, wa, wb);
      }
    if (hh == 0) {
      const float lse = (l > 0.f) ? (m + log2f(l)) / LOG2E : INFINITY;
      p.lse[(long long)bh * S + q] = lse;
    }
  }
}

// ------------------------------------------------------------------ forward v2 (pair stream)
// Measured on the one-launch-per-128-query-block kernel above (bench/attn_one.py, GPT-2 small
// shape, scripts/attn_abl.sh): with its tile loop removed it still took 76 of its 267 us --
// every workgroup pays a Q load + ring fill + drain + store tail at S = 1024, where a block
// averages 8.5 key tiles -- and the causal triangle leaves blocks of 2 .. 16 tiles.
// Here a workgroup runs TWO 128-query blocks of one (batch, head): the heaviest and the
// lightest left (qa = nqb-1-pr, qb = pr), so every workgroup does the same work (2 nqb + 2
// tiles), the second block's K/V tiles are L2 hits, and the grid is halved.  Both blocks form
// ONE LDS-DMA stream -- Q(qa), KV(0) .. KV(na-1), Q(qb), KV(0) .. KV(nb-1) -- each element one
// ring slot (a Q element is the block's 128 query rows as two 64-row images, read into
// registers by the waves at the block start), so the ring never drains at the seam and no
// global load sits in front of the first MFMA.
// Softmax: the row sum comes from the PV MFMAs (a constant all-ones A operand: every row of
// that accumulator is sum_k P -- 4 more MFMAs per tile instead of 32 v_add), the half-wave max
// combine is a v_permlane32_swap (no LDS round trip), masks are 32-bit compares of
// compile-time key offsets.
// Persistent form: a grid of at most two workgroups per CU walks the pair items (item i:
// head bh = i / npr, pair pr = i % npr; workgroup b takes items local(b) + k * grid, where the
// workgroups of one XCD hold a contiguous run of locals, so the items an XCD runs at once share
// heads and K/V tiles in its L2) and the DMA stream runs on across items: the next item's Q
// and first K/V tiles land while the current one finishes, and its O stores drain under the
// next item's MFMAs.  (A grid of one workgroup per item is the non-persistent form.)
struct PairItem {
  int bh, blk0, blk1, len0, len;
};

template <int HD, int OCC, bool LMFMA>
__global__ __launch_bounds__(256, OCC) void attn_fwd2_kernel(AttnArgs p, int nitems) {
  using A = AT<HD>;
  __shared__ __attribute__((aligned(16))) bf16_t smem[NSLOT * 2 * A::TILE];  // [slot][K|V] or [slot][Q lo|Q hi]
  const int S = p.S, H = p.H;
  const int nqb = (S + QB - 1) / QB;
  const int npr = (nqb + 1) / 2;
  const int grid = gridDim.x;
  const int local = g7_local_attn(blockIdx.x, grid);
  const int lane = threadIdx.x & 63, hh = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  auto ntiles_of = [&](int qb) {
    const int kend = p.causal ? min(S, qb * QB + QB) : S;
    return (kend + KT - 1) / KT;
  };
  auto item = [&](int k) {  // k-th item of this workgroup
    PairItem it;
    const int id = local + k * grid;
    it.bh = id / npr;
    const int pr = id - it.bh * npr;
    it.blk0 = nqb - 1 - pr;
    it.blk1 = pr;
    it.len0 = 1 + ntiles_of(it.blk0);
    it.len = it.len0 + (it.blk1 != it.blk0 ? 1 + ntiles_of(it.blk1) : 0);
    return it;
  };
  const int nmine = local < nitems ? (nitems - local + grid - 1) / grid : 0;
  if (nmine == 0) return;
  int total = 0;
  for (int k = 0; k < nmine; ++k) total += item(k).len;

  int dv[A::NPW];
  dma_voff<HD>(dv, p.ld_qkv, wid, lane);
  // ---- issue cursor: (item, offset), wave-uniform.  The item's (batch, head) offset is formed
  // when the cursor enters the item (a division by H): per step it was ~20 of the ~200 scalar
  // instructions of a tile (rocprofv3 SQ_INSTS_SALU, profiles/r5_attn/pmc_final.txt)
  int is_k = 0, is_off = 0;
  PairItem is_it = item(0);
  long long is_hoff = 0;  // elements from q / k / v to row 0 of the item's (batch, head)
  auto enter = [&]() {
    const int n = is_it.bh / H, h = is_it.bh - n * H;
    is_hoff = (long long)n * S * p.ld_qkv + h * HD;
  };
  enter();
  auto issue_next = [&](int e) {
    bf16_t* st = smem + (e % NSLOT) * 2 * A::TILE;
    const bool valid = is_k < nmine;
    const bool second = is_off >= is_it.len0;
    const int i = is_off - (second ? is_it.len0 : 0);
    if (i == 0 || !valid) {  // Q rows of the block (or an empty element past the end)
      const bf16_t* base = static_cast<const bf16_t*>(p.q) + is_hoff;
      const int r0 = (second ? is_it.blk1 : is_it.blk0) * QB;
      tile_dma<HD>(base, p.ld_qkv, r0, S, valid, dv, st, wid);
      tile_dma<HD>(base, p.ld_qkv, r0 + KT, S, valid, dv, st + A::TILE, wid);
    } else {
      const bf16_t* K = static_cast<const bf16_t*>(p.k) + is_hoff;
      const bf16_t* V = static_cast<const bf16_t*>(p.v) + is_hoff;
      tile_dma<HD>(K, p.ld_qkv, (i - 1) * KT, S, true, dv, st, wid);
      tile_dma<HD>(V, p.ld_qkv, (i - 1) * KT, S, true, dv, st + A::TILE, wid);
    }
    if (valid && ++is_off == is_it.len) {
      is_off = 0;
      if (++is_k < nmine) {
        is_it = item(is_k);
        enter();
      }
    }
  };

  const float c = p.scale * LOG2E;
  bf16x8 qf[A::NST];
  float m = -INFINITY, l = 0.f;
  constexpr int NO = A::NDT + (LMFMA ? 1 : 0);  // O^T blocks (+ the row-sum block)
  floatx16 o[NO];
  int q0 = 0, q = 0, last_w = 0;
  // ---- consume cursor
  int c_k = 0, c_off = 0;
  PairItem c_it = is_it;
  int bh = c_it.bh, h = 0, n = 0;
  const unsigned char* pad = nullptr;
  bf16x8 ones;
#pragma unroll
  for (int i = 0; i < 8; ++i) ones[i] = (__bf16)1.0f;

  auto qk = [&](floatx16 (&s)[2], const bf16_t* lk) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      zero16(s[kb]);
#pragma unroll
      for (int st = 0; st < A::NST; ++st) s[kb] = MFMA32(row_frag<HD>(lk, kb * 32, st, lane), qf[st], s[kb]);
    }
  };
  auto finish = [&]() {  // the block's O and lse
    if constexpr (LMFMA) l = o[A::NDT][0];
    else l += __shfl_xor(l, 32, 64);  // the two lane halves summed different key rows
    if (q < S) {
      const float inv = l > 0.f ? __builtin_amdgcn_rcpf(l) : 0.f;
      // (the row offset is formed here, in 32 bits: a pointer held across the loop is
      // spilled, and its reload's vmcnt(0) would drain the ring)
      bf16_t* O = static_cast<bf16_t*>(p.o) + (long long)n * S * p.ld_o + h * HD + q * (int)p.ld_o;
#pragma unroll
      for (int d = 0; d < A::NDT; ++d)
#pragma unroll
        for (int g = 0; g < 4; g += 2) {
          uint2 wa, wb;
          wa.x = pack2bf(o[d][4 * g + 0] * inv, o[d][4 * g + 1] * inv);
          wa.y = pack2bf(o[d][4 * g + 2] * inv, o[d][4 * g + 3] * inv);
          wb.x = pack2bf(o[d][4 * g + 4] * inv, o[d][4 * g + 5] * inv);
          wb.y = pack2bf(o[d][4 * g + 6] * inv, o[d][4 * g + 7] * inv);
          store_pair16(O + d * 32, g, hh, wa, wb);
        }
      if (hh == 0) p.lse[(long long)bh * S + q] = (l > 0.f) ? (m + log2f(l)) / LOG2E : INFINITY;
    }
  };

  issue_next(0);
  issue_next(1);
  issue_next(2);
  // element e: (block start) read Q, S^T of KV(0) into sn;  (KV tile t) softmax of sc, S^T of
  // KV(t+1) into sn if this wave needs it, O^T += V^T P^T.
  auto step = [&](int e, floatx16 (&sc)[2], floatx16 (&sn)[2]) {
    vm_wait<2 * A::NPW>();  // this wave's pieces of element e+1 landed (e+2 may fly)
    ring_barrier();         // ... every wave's; every wave is done with element e-1's slot
    issue_next(e + 3);
    const bf16_t* ls = smem + (e % NSLOT) * 2 * A::TILE;
    const bf16_t* lsn = smem + ((e + 1) % NSLOT) * 2 * A::TILE;
    const PairItem cur = c_it;
    const bool second = c_off >= cur.len0;
    const int i = c_off - (second ? cur.len0 : 0);
    const int t = i - 1;
    if (++c_off == cur.len) {  // advance the consume cursor
      c_off = 0;
      if (++c_k < nmine) c_it = item(c_k);
    }
    if (i == 0) {  // a block starts: the previous one's O, then this one's Q and first scores
      if (e > 0) finish();
      if (!second) {  // ... of a new item
        bh = cur.bh;
        n = bh / H;
        h = bh - n * H;
        pad = p.pad ? p.pad + (long long)n * S : nullptr;
      }
      q0 = (second ? cur.blk1 : cur.blk0) * QB + wid * 32;
      q = q0 + (lane & 31);
      const int nt = ntiles_of(second ? cur.blk1 : cur.blk0);
      last_w = p.causal ? min(nt - 1, max(0, min(q0 + 31, S - 1)) / KT) : nt - 1;
#pragma unroll
      for (int st = 0; st < A::NST; ++st) qf[st] = row_frag<HD>(ls + (wid >> 1) * A::TILE, 32 * (wid & 1), st, lane);
      m = -INFINITY;
      l = 0.f;
#pragma unroll
      for (int d = 0; d < NO; ++d) zero16(o[d]);
      qk(sn, lsn);
      return;
    }
    if (t > last_w) return;  // wave-uniform
    const bf16_t* lv = ls + A::TILE;
    const int kt0 = t * KT;
    const bool need_mask = (p.causal && kt0 + KT - 1 > q0) || (kt0 + KT > S) || pad;  // wave-uniform
    if (need_mask) {
      // key kb*32 + (r&3) + 8(r>>2) + 4 hh of the tile is masked if it is > lim (causal /
      // past the end) or padded
      const int limh = (p.causal ? min(q, S - 1) : S - 1) - kt0 - 4 * hh;
      const unsigned long long pm = pad_bits(pad, kt0, S, lane) >> (4 * hh);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        const unsigned pk = (unsigned)(pm >> (32 * kb));
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kc = kb * 32 + (r & 3) + 8 * (r >> 2);
          const bool masked = (kc > limh) || ((pk >> ((r & 3) + 8 * (r >> 2))) & 1u);
          if (masked) sc[kb][r] = -INFINITY;
        }
      }
    }
    // the tile max as four independent v_max3 chains joined at the end (depth 6 instead of one
    // 16-deep dependent chain in front of every exponential of the tile)
    float mq[4];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const floatx16& sq = sc[q4 >> 1];
      const int r0 = (q4 & 1) * 8;
      float v = max3f(sq[r0], sq[r0 + 1], sq[r0 + 2]);
      v = max3f(v, sq[r0 + 3], sq[r0 + 4]);
      v = max3f(v, sq[r0 + 5], sq[r0 + 6]);
      mq[q4] = fmaxf(v, sq[r0 + 7]);
    }
    float mx = fmaxf(max3f(mq[0], mq[1], mq[2]), mq[3]);
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1])) * c;  // scaled log2 units (c > 0)
    }
    // lazy rescale: the running max only moves when the tile max exceeds it by > 2^8
    if (__ballot(mx > m + 8.f)) {
      const float mn = fmaxf(m, mx);
      const float alpha = (m == -INFINITY) ? 1.f : fast_exp2(m - mn);
      m = mn;
      if constexpr (!LMFMA) l *= alpha;
#pragma unroll
      for (int d = 0; d < NO; ++d) scale16(o[d], alpha);
    }
    const float nmu = (m == -INFINITY) ? 0.f : -m;
    if (t + 1 <= last_w) qk(sn, lsn);  // next tile's scores beside this tile's exponentials
    float lq[4] = {0.f, 0.f, 0.f, 0.f};  // (four independent partial row sums)
    bf16x8 pb[2][2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float ex = fast_exp2(fmaf(sc[kb][r], c, nmu));
        sc[kb][r] = ex;
        if constexpr (!LMFMA) lq[r & 3] += ex;
      }
      pb[kb][0] = acc_frag(sc[kb], 0);
      pb[kb][1] = acc_frag(sc[kb], 1);
    }
    if constexpr (!LMFMA) l += (lq[0] + lq[1]) + (lq[2] + lq[3]);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
#pragma unroll
        for (int d = 0; d < A::NDT; ++d)
          o[d] = MFMA32(tr_frag<HD>(lv, kb * 32, ss, d * 32, lane), pb[kb][ss], o[d]);
        if constexpr (LMFMA) o[A::NDT] = MFMA32(ones, pb[kb][ss], o[A::NDT]);
      }
  };
  floatx16 s0[2], s1[2];
  for (int e = 0; e < total; e += 2) {
    step(e, s0, s1);
    if (e + 1 < total) step(e + 1, s1, s0);
  }
  finish();
  vm_wait<0>();  // the pieces issued past the end (empty descriptors) drained
}

// Forward, round 6 (DPC_ATTN_VAR 9 / 10): attn_fwd2_kernel's pair stream, DMA ring and math with
// the consume side split by tile kind.  fwd2 ran ONE step body for every element (block start,
// masked tile, skipped tile, plain tile), and at its joins the compiler copied the score and O
// accumulators: 48 v_mov_b64 per plain tile in its gfx950 listing, ~1/4 of the tile's VALU.  Here,
// per block and wave, the leading tiles that need no mask and have a successor tile run in a
// two-tile unrolled loop of straight-line code (no mask, no skip, the next tile's scores always
// formed, the lazy rescale's branch inside asm: scale16_if); the block's other tiles -- the
// causal diagonal, past the end, padded, or skipped by this wave -- take the general body one
// at a time, with one explicit copy of the next scores each.
template <int HD, int OCC, bool LMFMA>
__global__ __launch_bounds__(256, OCC) void attn_fwd3_kernel(AttnArgs p, int nitems) {
  using A = AT<HD>;
  __shared__ __attribute__((aligned(16))) bf16_t smem[NSLOT * 2 * A::TILE];  // [slot][K|V] or [slot][Q lo|Q hi]
  const int S = p.S, H = p.H;
  const int nqb = (S + QB - 1) / QB;
  const int npr = (nqb + 1) / 2;
  const int grid = gridDim.x;
  const int local = g7_local_attn(blockIdx.x, grid);
  const int lane = threadIdx.x & 63, hh = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  auto ntiles_of = [&](int qb) {
    const int kend = p.causal ? min(S, qb * QB + QB) : S;
    return (kend + KT - 1) / KT;
  };
  auto item = [&](int k) {  // k-th item of this workgroup
    PairItem it;
    const int id = local + k * grid;
    it.bh = id / npr;
    const int pr = id - it.bh * npr;
    it.blk0 = nqb - 1 - pr;
    it.blk1 = pr;
    it.len0 = 1 + ntiles_of(it.blk0);
    it.len = it.len0 + (it.blk1 != it.blk0 ? 1 + ntiles_of(it.blk1) : 0);
    return it;
  };
  const int nmine = local < nitems ? (nitems - local + grid - 1) / grid : 0;
  if (nmine == 0) return;

  int dv[A::NPW];
  dma_voff<HD>(dv, p.ld_qkv, wid, lane);
  // ---- issue cursor (as attn_fwd2_kernel): element e+3 is issued while element e is consumed
  int is_k = 0, is_off = 0;
  PairItem is_it = item(0);
  long long is_hoff = 0;
  auto enter = [&]() {
    const int n = is_it.bh / H, h = is_it.bh - n * H;
    is_hoff = (long long)n * S * p.ld_qkv + h * HD;
  };
  enter();
  auto issue_next = [&](int e) {
    bf16_t* st = smem + (e % NSLOT) * 2 * A::TILE;
    const bool valid = is_k < nmine;
    const bool second = is_off >= is_it.len0;
    const int i = is_off - (second ? is_it.len0 : 0);
    if (i == 0 || !valid) {
      const bf16_t* base = static_cast<const bf16_t*>(p.q) + is_hoff;
      const int r0 = (second ? is_it.blk1 : is_it.blk0) * QB;
      tile_dma<HD>(base, p.ld_qkv, r0, S, valid, dv, st, wid);
      tile_dma<HD>(base, p.ld_qkv, r0 + KT, S, valid, dv, st + A::TILE, wid);
    } else {
      const bf16_t* K = static_cast<const bf16_t*>(p.k) + is_hoff;
      const bf16_t* V = static_cast<const bf16_t*>(p.v) + is_hoff;
      tile_dma<HD>(K, p.ld_qkv, (i - 1) * KT, S, true, dv, st, wid);
      tile_dma<HD>(V, p.ld_qkv, (i - 1) * KT, S, true, dv, st + A::TILE, wid);
    }
    if (valid && ++is_off == is_it.len) {
      is_off = 0;
      if (++is_k < nmine) {
        is_it = item(is_k);
        enter();
      }
    }
  };
  auto sync = [&](int e) {
    vm_wait<2 * A::NPW>();  // this wave's pieces of element e+1 landed (e+2 may fly)
    ring_barrier();         // ... every wave's; every wave is done with element e-1's slot
    issue_next(e + 3);
  };
  auto slot = [&](int e) -> const bf16_t* { return smem + (e % NSLOT) * 2 * A::TILE; };

  const float c = p.scale * LOG2E;
  bf16x8 qf[A::NST];
  float m = -INFINITY, l = 0.f;
  constexpr int NO = A::NDT + (LMFMA ? 1 : 0);  // O^T blocks (+ the row-sum block)
  floatx16 o[NO];
  int q0 = 0, q = 0, last_w = 0;
  int bh = 0, h = 0, n = 0;
  const unsigned char* pad = nullptr;
  bf16x8 ones;
#pragma unroll
  for (int i = 0; i < 8; ++i) ones[i] = (__bf16)1.0f;

  auto qk = [&](floatx16 (&s)[2], const bf16_t* lk) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      zero16(s[kb]);
#pragma unroll
      for (int st = 0; st < A::NST; ++st) s[kb] = MFMA32(row_frag<HD>(lk, kb * 32, st, lane), qf[st], s[kb]);
    }
  };
  auto finish = [&]() {  // the block's O and lse
    if constexpr (LMFMA) l = o[A::NDT][0];
    else l += __shfl_xor(l, 32, 64);
    if (q < S) {
      const float inv = l > 0.f ? __builtin_amdgcn_rcpf(l) : 0.f;
      bf16_t* O = static_cast<bf16_t*>(p.o) + (long long)n * S * p.ld_o + h * HD + q * (int)p.ld_o;
#pragma unroll
      for (int d = 0; d < A::NDT; ++d)
#pragma unroll
        for (int g = 0; g < 4; g += 2) {
          uint2 wa, wb;
          wa.x = pack2bf(o[d][4 * g + 0] * inv, o[d][4 * g + 1] * inv);
          wa.y = pack2bf(o[d][4 * g + 2] * inv, o[d][4 * g + 3] * inv);
          wb.x = pack2bf(o[d][4 * g + 4] * inv, o[d][4 * g + 5] * inv);
          wb.y = pack2bf(o[d][4 * g + 6] * inv, o[d][4 * g + 7] * inv);
          store_pair16(O + d * 32, g, hh, wa, wb);
        }
      if (hh == 0) p.lse[(long long)bh * S + q] = (l > 0.f) ? (m + log2f(l)) / LOG2E : INFINITY;
    }
  };
  // one KV tile (element e, tile t of the block): sc = this tile's raw scores -> P, O += V^T P^T,
  // and the next tile's scores into sn.  GEN: the general body (mask, C++ lazy branch, the next
  // scores only if this wave needs that tile); otherwise the plain straight-line body.
  auto tile = [&](auto gen, int e, int t, floatx16 (&sc)[2], floatx16 (&sn)[2]) {
    constexpr bool GEN = decltype(gen)::value;
    const bf16_t* ls = slot(e);
    const bf16_t* lv = ls + A::TILE;
    const int kt0 = t * KT;
    if constexpr (GEN) {
      const bool need_mask = (p.causal && kt0 + KT - 1 > q0) || (kt0 + KT > S) || pad;  // wave-uniform
      if (need_mask) {
        const int limh = (p.causal ? min(q, S - 1) : S - 1) - kt0 - 4 * hh;
        const unsigned long long pm = pad_bits(pad, kt0, S, lane) >> (4 * hh);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          const unsigned pk = (unsigned)(pm >> (32 * kb));
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int kc = kb * 32 + (r & 3) + 8 * (r >> 2);
            const bool masked = (kc > limh) || ((pk >> ((r & 3) + 8 * (r >> 2))) & 1u);
            if (masked) sc[kb][r] = -INFINITY;
          }
        }
      }
    }
    float mq[4];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const floatx16& sq = sc[q4 >> 1];
      const int r0 = (q4 & 1) * 8;
      float v = max3f(sq[r0], sq[r0 + 1], sq[r0 + 2]);
      v = max3f(v, sq[r0 + 3], sq[r0 + 4]);
      v = max3f(v, sq[r0 + 5], sq[r0 + 6]);
      mq[q4] = fmaxf(v, sq[r0 + 7]);
    }
    float mx = fmaxf(max3f(mq[0], mq[1], mq[2]), mq[3]);
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      mx = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1])) * c;  // scaled log2 units (c > 0)
    }
    // lazy rescale: the running max only moves when the tile max exceeds it by > 2^8
    if constexpr (GEN) {
      if (__ballot(mx > m + 8.f)) {
        const float mn = fmaxf(m, mx);
        const float alpha = (m == -INFINITY) ? 1.f : fast_exp2(m - mn);
        m = mn;
        if constexpr (!LMFMA) l *= alpha;
#pragma unroll
        for (int d = 0; d < NO; ++d) scale16(o[d], alpha);
      }
    } else {
      static_assert(!LMFMA, "plain tiles: the row sum in l");
      const unsigned long long up = __ballot(mx > m + 8.f);
      const float alpha = rescale16_if(o[0], m, l, mx, up);
#pragma unroll
      for (int d = 1; d < NO; ++d) scale16_if(o[d], alpha, up);
    }
    // (a plain tile has no masked score, so m is finite after its update)
    const float nmu = (!GEN || m != -INFINITY) ? -m : 0.f;
    if constexpr (GEN) {
      if (t + 1 <= last_w) qk(sn, slot(e + 1));
    } else {
      qk(sn, slot(e + 1));  // next tile's scores beside this tile's exponentials
    }
    float lq[4] = {0.f, 0.f, 0.f, 0.f};
    bf16x8 pb[2][2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float ex = fast_exp2(fmaf(sc[kb][r], c, nmu));
        sc[kb][r] = ex;
        if constexpr (!LMFMA) lq[r & 3] += ex;
      }
      pb[kb][0] = acc_frag(sc[kb], 0);
      pb[kb][1] = acc_frag(sc[kb], 1);
    }
    if constexpr (!LMFMA) l += (lq[0] + lq[1]) + (lq[2] + lq[3]);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
#pragma unroll
        for (int d = 0; d < A::NDT; ++d)
          o[d] = MFMA32(tr_frag<HD>(lv, kb * 32, ss, d * 32, lane), pb[kb][ss], o[d]);
        if constexpr (LMFMA) o[A::NDT] = MFMA32(ones, pb[kb][ss], o[A::NDT]);
      }
  };
  using Plain = std::integral_constant<bool, false>;
  using General = std::integral_constant<bool, true>;

  issue_next(0);
  issue_next(1);
  issue_next(2);
  floatx16 sA[2], sB[2];
  int e = 0;
  for (int k = 0; k < nmine; ++k) {
    const PairItem it = item(k);
    for (int half = 0; half < 2; ++half) {
      if (half == 1 && it.blk1 == it.blk0) break;
      const int blk = half ? it.blk1 : it.blk0;
      // ---- block start: the previous block's O, then this block's Q and first scores
      sync(e);
      const bf16_t* ls = slot(e);
      if (e > 0) finish();
      if (half == 0) {
        bh = it.bh;
        n = bh / H;
        h = bh - n * H;
        pad = p.pad ? p.pad + (long long)n * S : nullptr;
      }
      q0 = blk * QB + wid * 32;
      q = q0 + (lane & 31);
      const int nt = ntiles_of(blk);
      last_w = p.causal ? min(nt - 1, max(0, min(q0 + 31, S - 1)) / KT) : nt - 1;
#pragma unroll
      for (int st = 0; st < A::NST; ++st) qf[st] = row_frag<HD>(ls + (wid >> 1) * A::TILE, 32 * (wid & 1), st, lane);
      m = -INFINITY;
      l = 0.f;
#pragma unroll
      for (int d = 0; d < NO; ++d) zero16(o[d]);
      qk(sA, slot(e + 1));
      ++e;
      // ---- plain tiles: no mask (inside S, no padding, wholly at or below the wave's first
      // query) and followed by another tile of this wave
      int nf = pad ? 0 : min(last_w, S / KT);
      if (p.causal) nf = min(nf, (q0 + 1) / KT);
      int t = 0;
      for (; t + 2 <= nf; t += 2, e += 2) {
        sync(e);
        tile(Plain(), e, t, sA, sB);
        sync(e + 1);
        tile(Plain(), e + 1, t + 1, sB, sA);
      }
      if (t < nf) {
        sync(e);
        tile(Plain(), e, t, sA, sB);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) sA[kb] = sB[kb];
        ++e;
        ++t;
      }
      // ---- the rest of the block's tiles: masked, the wave's last, or skipped by this wave
      for (; t < nt; ++t, ++e) {
        sync(e);
        if (t <= last_w) {  // wave-uniform
          tile(General(), e, t, sA, sB);
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) sA[kb] = sB[kb];
        }
      }
    }
  }
  finish();
  vm_wait<0>();  // the pieces issued past the end (empty descriptors) drained
}

// ------------------------------------------------------------------ backward
// delta[n,h,s] = sum_d dO * O   (one HD/8-lane group per (token, head)), stored NEGATED (the
// dK / dV kernel's dP accumulator starts at -delta: an LDS read straight into it, no per-element
// sign flip), and the second half of the buffer the row's lse in log2 units (lse * log2 e) --
// the kernels then form p = 2^(s c - lse2) with one FMA and no per-element multiply
template <int HD>
__global__ __launch_bounds__(256) void attn_bwd_pre_kernel(AttnArgs p) {
  constexpr int G = HD / 8;
  const long long T = (long long)p.N * p.S;
  const long long row = ((long long)blockIdx.x * 256 + threadIdx.x) / G;  // (token, head)
  const int sub = threadIdx.x % G;
  float acc = 0.f;
  long long t = 0;
  int h = 0;
  if (row < T * p.H) {
    t = row / p.H;
    h = (int)(row % p.H);
    const bf16_t* o = static_cast<const bf16_t*>(p.o) + t * p.ld_o + h * HD + sub * 8;
    const bf16_t* d = static_cast<const bf16_t*>(p.dout) + t * p.ld_o + h * HD + sub * 8;
    float fo[8], fd[8];
    unpack8(*reinterpret_cast<const uint4*>(o), fo);
    unpack8(*reinterpret_cast<const uint4*>(d), fd);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += fo[i] * fd[i];
  }
#pragma unroll
  for (int o = 1; o < G; o <<= 1) acc += __shfl_xor(acc, o, 64);
  if (row < T * p.H && sub == 0) {
    const long long n = t / p.S, s = t % p.S;
    const long long i = (n * p.H + h) * p.S + s;
    p.delta[i] = -acc;
    p.delta[T * p.H + i] = p.lse[i] * LOG2E;  // (+inf stays +inf: a fully masked row)
  }
}

// dK, dV: workgroup = 128 keys (4 waves x 32, key on the lane), sweeping the 64-query tiles
// at or after the first key.  Per 32-query sub-block j: S, dP of sub-block j+1 (2 x NST
// MFMAs) overlap the P / dS arithmetic of j, then dV^T, dK^T += ... (4 x NDT MFMAs).
// ABL (dpc_attn_bwd_lab only; the library launches ABL = 0): per-workgroup cost ablations --
// 1 = no tile loop (the ring prologue stays), 2 = no per-row register loads, 4 = no epilogue
// stores, 8 = no ring prologue.  Outputs are wrong by design.
template <int HD, bool PIPE, int OCC, int ABL = 0>
__global__ __launch_bounds__(256, OCC) void attn_bwd_dkdv_kernel(AttnArgs p) {
  using A = AT<HD>;
  __shared__ __attribute__((aligned(16))) bf16_t smem[NSLOT * 2 * A::TILE];  // [slot][Q|dO]
  __shared__ __attribute__((aligned(16))) float srow[NSLOT][2][KT];          // [slot][lse|delta]
  const int S = p.S, H = p.H;
  const int nkb = (S + QB - 1) / QB;
  int bh, kb;
  if (p.order == 1) work_order1(nkb, bh, kb);
  else xcd_work(nkb, bh, kb);  // kb = 0 (the most queries under the causal mask) first
  const int n = bh / H, h = bh % H;
  const int lane = threadIdx.x & 63, hh = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int k0 = kb * QB + wid * 32;
  const int key = k0 + (lane & 31);
  const long long tok0 = (long long)n * S;
  const bf16_t* Q = static_cast<const bf16_t*>(p.q) + tok0 * p.ld_qkv + h * HD;
  const bf16_t* Kp = static_cast<const bf16_t*>(p.k) + h * HD;
  const bf16_t* Vp = static_cast<const bf16_t*>(p.v) + h * HD;
  const bf16_t* dO = static_cast<const bf16_t*>(p.dout) + tok0 * p.ld_o + h * HD;
  const float* lse = p.delta + (long long)p.N * H * S + (long long)bh * S;  // log2 units
  const float* delta = p.delta + (long long)bh * S;
  const bool key_ok = key < S && !(p.pad && p.pad[(long long)n * S + min(key, S - 1)]);

  bf16x8 kf[A::NST], vf[A::NST];
#pragma unroll
  for (int st = 0; st < A::NST; ++st) {
    kf[st] = bf16x8{};
    vf[st] = bf16x8{};
  }
  const float c = p.scale * LOG2E;
  floatx16 dvt[A::NDT], dkt[A::NDT];
#pragma unroll
  for (int d = 0; d < A::NDT; ++d) {
    zero16(dvt[d]);
    zero16(dkt[d]);
  }

  const int qt_begin = p.causal ? (kb * QB) / KT : 0;
  const int nqt = (S + KT - 1) / KT;
  const int count = nqt - qt_begin;

  // Q / dO tiles and their (lse, delta) rows by LDS-DMA (the rows: wave 0, one dword per lane)
  int vq[A::NPW], vd[A::NPW];
  dma_voff<HD>(vq, p.ld_qkv, wid, lane);
  dma_voff<HD>(vd, p.ld_o, wid, lane);
  auto issue = [&](int i) {
    const int slot = i % NSLOT, qt = qt_begin + i;
    const bool valid = i < count;
    bf16_t* st = smem + slot * 2 * A::TILE;
    tile_dma<HD>(Q, p.ld_qkv, qt * KT, S, valid, vq, st, wid);
    tile_dma<HD>(dO, p.ld_o, qt * KT, S, valid, vd, st + A::TILE, wid);
    if (wid == 0) {
      dma4(rows_rsrc(lse, 4, qt * KT, S, valid), lane * 4, &srow[slot][0][0]);
      dma4(rows_rsrc(delta, 4, qt * KT, S, valid), lane * 4, &srow[slot][1][0]);
    }
  };
  // S = Q K^T, dP - delta = dO V^T - delta of the 32-query sub-block at row r0 of the slot
  // (key on the lane): the dP accumulator starts at -delta of its query rows (the buffer holds
  // -delta: four LDS reads land in the accumulator as they are), so dS = P (dP - delta) needs no
  // subtraction
  auto sdp = [&](floatx16& sa, floatx16& dp, const bf16_t* lq, int r0) {
    zero16(sa);
    const float* drow = &srow[((lq - smem) / (2 * A::TILE))][1][0];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 d4 = *reinterpret_cast<const float4*>(drow + r0 + 8 * g + 4 * hh);
      dp[4 * g + 0] = d4.x;
      dp[4 * g + 1] = d4.y;
      dp[4 * g + 2] = d4.z;
      dp[4 * g + 3] = d4.w;
    }
#pragma unroll
    for (int st = 0; st < A::NST; ++st) {
      sa = MFMA32(row_frag<HD>(lq, r0, st, lane), kf[st], sa);
      dp = MFMA32(row_frag<HD>(lq + A::TILE, r0, st, lane), vf[st], dp);
    }
  };

  if (count > 0 && !(ABL & 8)) {
    // The workgroup's 128 K and V rows arrive by LDS-DMA as tile images in ring slots 2 / 3
    // (1-KiB coalesced pieces; per-lane 16-B row loads touched 32 lines per instruction), the
    // lanes read their row fragments from there, and only then does tile 2 reuse slot 2.
    if constexpr (!(ABL & 2)) {
      bf16_t* sk = smem + 2 * 2 * A::TILE;
      bf16_t* sv = smem + 3 * 2 * A::TILE;
      const bf16_t* K0 = Kp + tok0 * p.ld_qkv;
      const bf16_t* V0 = Vp + tok0 * p.ld_qkv;
      tile_dma<HD>(K0, p.ld_qkv, kb * QB, S, true, vq, sk, wid);
      tile_dma<HD>(K0, p.ld_qkv, kb * QB + KT, S, true, vq, sk + A::TILE, wid);
      tile_dma<HD>(V0, p.ld_qkv, kb * QB, S, true, vq, sv, wid);
      tile_dma<HD>(V0, p.ld_qkv, kb * QB + KT, S, true, vq, sv + A::TILE, wid);
    }
    issue(0);
    issue(1);
    if constexpr (!(ABL & 2)) {
      if (wid == 0) vm_wait<4 * A::NPW + 4>();  // K / V landed (tiles 0, 1 may fly)
      else vm_wait<4 * A::NPW>();
      ring_barrier();
      const bf16_t* sk = smem + 2 * 2 * A::TILE + (wid >> 1) * A::TILE;
#pragma unroll
      for (int st = 0; st < A::NST; ++st) {
        kf[st] = row_frag<HD>(sk, 32 * (wid & 1), st, lane);
        vf[st] = row_frag<HD>(sk + 2 * A::TILE, 32 * (wid & 1), st, lane);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every wave done with slots 2 / 3
      __builtin_amdgcn_sched_barrier(0);
      ring_barrier();
    }
    issue(2);
    if (wid == 0) vm_wait<4 * A::NPW + 4>();  // tile 0 landed (tiles 1, 2 may fly)
    else vm_wait<4 * A::NPW>();
    ring_barrier();
  }
  // sub-block (tile i, half hf): its S / dP in (sa, dp); the next sub-block's land in (san, dpn)
  auto half = [&](int i, int hf, floatx16& sa, floatx16& dp, floatx16& san, floatx16& dpn) {
    const int slot = i % NSLOT;
    const bf16_t* lq = smem + slot * 2 * A::TILE;
    const bf16_t* ldo = lq + A::TILE;
    // the next sub-block: second half of this tile, or first half of the next tile
    const bf16_t* nq = hf == 0 ? lq : smem + ((i + 1) % NSLOT) * 2 * A::TILE;
    const int nr0 = hf == 0 ? 32 : 0;
    const int qt0 = (qt_begin + i) * KT;
    const int qs0 = qt0 + 32 * hf;
    const bool active = !(p.causal && qs0 + 31 < k0);  // wave-uniform: some query >= some key
    if (!active) {
      if constexpr (PIPE) sdp(san, dpn, nq, nr0);
      return;
    }
    const bool diag = p.causal && qs0 < k0 + 31;  // wave-uniform: some key > some query
    // ---- one basic block: next S, dP MFMAs || this sub-block's P, dS
    if constexpr (PIPE) sdp(san, dpn, nq, nr0);
    else sdp(sa, dp, lq, 32 * hf);
    // P, dS.  The causal zeroing runs only on the sub-blocks that cross the diagonal, in place,
    // between the exponentials and the dS products: written as a select inside the element loop,
    // hipcc if-converted it into an add, a compare, an exec-mask AND and a select on EVERY element
    // of every sub-block, and as two loop copies it gave P new registers plus copies at the join.
    // Element (g, e) holds query qs0 + 8 g + 4 hh + e: masked when key - qs0 - 4 hh > 8 g + e.
    sfor<4>([&](auto G) {
      constexpr int g = decltype(G)::value;
      const float4 l4 = *reinterpret_cast<const float4*>(&srow[slot][0][32 * hf + 8 * g + 4 * hh]);
      const float lv[4] = {l4.x, l4.y, l4.z, l4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) sa[4 * g + e] = fast_exp2(fmaf(sa[4 * g + e], c, -lv[e]));
    });
    if (diag) {
      // (a padded key's P only reaches this lane's own dK / dV column: zeroed at the store)
      const int kd = key - qs0 - 4 * hh;
      sfor<16>([&](auto R) {
        constexpr int r = decltype(R)::value;
        zero_if_gt<8 * (r >> 2) + (r & 3)>(sa, r, kd);
      });
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) dp[r] = sa[r] * dp[r];
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      const bf16x8 pb = acc_frag(sa, ss);
      const bf16x8 db = acc_frag(dp, ss);
#pragma unroll
      for (int d = 0; d < A::NDT; ++d) {
        dvt[d] = MFMA32(tr_frag<HD>(ldo, 32 * hf, ss, d * 32, lane), pb, dvt[d]);
        dkt[d] = MFMA32(tr_frag<HD>(lq, 32 * hf, ss, d * 32, lane), db, dkt[d]);
      }
    }
  };
  floatx16 sa0, dp0, sa1, dp1;
  if constexpr (PIPE) sdp(sa0, dp0, smem, 0);
  for (int i = 0; i < ((ABL & 1) ? 0 : count); ++i) {
    if (wid == 0) vm_wait<2 * A::NPW + 2>();  // tile i+1 landed (i+2 may fly)
    else vm_wait<2 * A::NPW>();
    ring_barrier();
    issue(i + 3);
    half(i, 0, sa0, dp0, sa1, dp1);
    half(i, 1, sa1, dp1, sa0, dp0);
  }
  vm_wait<0>();

  if (key < S && !(ABL & 4)) {
    bf16_t* dK = static_cast<bf16_t*>(p.dk) + (tok0 + key) * p.ld_dqkv + h * HD;
    bf16_t* dV = static_cast<bf16_t*>(p.dv) + (tok0 + key) * p.ld_dqkv + h * HD;
    auto wk = [&](int d, int g) {  // (padded key: dK = dV = 0)
      uint2 w = make_uint2(0u, 0u);
      if (key_ok) {
        w.x = pack2bf(dkt[d][4 * g + 0] * p.scale, dkt[d][4 * g + 1] * p.scale);
        w.y = pack2bf(dkt[d][4 * g + 2] * p.scale, dkt[d][4 * g + 3] * p.scale);
      }
      return w;
    };
    auto wv = [&](int d, int g) {
      uint2 u = make_uint2(0u, 0u);
      if (key_ok) {
        u.x = pack2bf(dvt[d][4 * g + 0], dvt[d][4 * g + 1]);
        u.y = pack2bf(dvt[d][4 * g + 2], dvt[d][4 * g + 3]);
      }
      return u;
    };
#pragma unroll
    for (int d = 0; d < A::NDT; ++d)
#pragma unroll
      for (int g = 0; g < 4; g += 2) {
        store_pair16(dK + d * 32, g, hh, wk(d, g), wk(d, g + 1));
        store_pair16(dV + d * 32, g, hh, wv(d, g), wv(d, g + 1));
      }
  }
}

// dQ: workgroup = 128 queries (4 waves x 32, query on the lane), sweeping the key tiles up to
// the last query.  Per 32-key sub-block j: S^T, dP^T of j+1 overlap dS^T of j, then
// dQ^T += K^T dS^T (2 x NDT MFMAs).
// PRE: the delta pre-pass fused in (the default): the kernel also loads its query rows of O,
// forms delta = rowsum(dO * O) itself (each lane holds half of a row, the other half on lane
// ^ 32) and writes delta and the log2-unit lse rows that the dK / dV kernel -- launched after
// it -- streams.  Saves attn_bwd_pre_kernel's pass over O and dO (the dQ kernel holds dO anyway).
template <int HD, bool PIPE, int OCC, int ABL = 0, bool PRE = false>  // (ABL: as attn_bwd_dkdv_kernel)
__global__ __launch_bounds__(256, OCC) void attn_bwd_dq_kernel(AttnArgs p) {
  using A = AT<HD>;
  __shared__ __attribute__((aligned(16))) bf16_t smem[NSLOT * 2 * A::TILE];  // [slot][K|V]
  const int S = p.S, H = p.H;
  const int nqb = (S + QB - 1) / QB;
  int bh, bi;
  if (p.order == 1) work_order1(nqb, bh, bi);
  else xcd_work(nqb, bh, bi);
  const int qb = nqb - 1 - bi;
  const int n = bh / H, h = bh % H;
  const int lane = threadIdx.x & 63, hh = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q0 = qb * QB + wid * 32;
  const int q = q0 + (lane & 31);
  const long long tok0 = (long long)n * S;
  const bf16_t* Q = static_cast<const bf16_t*>(p.q) + h * HD;
  const bf16_t* K = static_cast<const bf16_t*>(p.k) + tok0 * p.ld_qkv + h * HD;
  const bf16_t* V = static_cast<const bf16_t*>(p.v) + tok0 * p.ld_qkv + h * HD;
  const bf16_t* dO = static_cast<const bf16_t*>(p.dout) + h * HD;
  const unsigned char* pad = p.pad ? p.pad + (long long)n * S : nullptr;

  bf16x8 qf[A::NST], df[A::NST];
#pragma unroll
  for (int st = 0; st < A::NST; ++st) {
    qf[st] = (q < S && !(ABL & 2)) ? load_row8(Q + (tok0 + q) * p.ld_qkv + 16 * st + 8 * hh) : bf16x8{};
    df[st] = (q < S && !(ABL & 2)) ? load_row8(dO + (tok0 + q) * p.ld_o + 16 * st + 8 * hh) : bf16x8{};
  }
  const float c = p.scale * LOG2E;
  float lse2, dl;
  if constexpr (PRE) {
    const bf16_t* Op = static_cast<const bf16_t*>(p.o) + h * HD;
    float acc = 0.f;
    if (q < S) {
#pragma unroll
      for (int st = 0; st < A::NST; ++st) {
        const bf16x8 of = load_row8(Op + (tok0 + q) * p.ld_o + 16 * st + 8 * hh);
        float fo[8], fd[8];
        unpack8(__builtin_bit_cast(uint4, of), fo);
        unpack8(__builtin_bit_cast(uint4, df[st]), fd);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc = fmaf(fo[i], fd[i], acc);
      }
    }
    dl = acc + __shfl_xor(acc, 32, 64);  // (the row's other half on lane ^ 32)
    // (+inf stays +inf: a fully masked row)
    lse2 = q < S ? p.lse[(long long)bh * S + q] * LOG2E : INFINITY;
    if (q < S && hh == 0) {
      p.delta[(long long)bh * S + q] = -dl;  // (negated: attn_bwd_pre_kernel)
      p.delta[(long long)p.N * H * S + (long long)bh * S + q] = lse2;
    }
  } else {
    lse2 = q < S ? p.delta[(long long)p.N * H * S + (long long)bh * S + q] : INFINITY;
    dl = q < S ? -p.delta[(long long)bh * S + q] : 0.f;
  }
  pin_loaded(qf);
  pin_loaded(df);
  pin_loaded(lse2);
  pin_loaded(dl);
  floatx16 dqt[A::NDT];
#pragma unroll
  for (int d = 0; d < A::NDT; ++d) zero16(dqt[d]);

  const int kend = p.causal ? min(S, qb * QB + QB) : S;
  const int ntiles = (kend + KT - 1) / KT;

  int dv[A::NPW];
  dma_voff<HD>(dv, p.ld_qkv, wid, lane);
  auto issue = [&](int t) {
    bf16_t* st = smem + (t % NSLOT) * 2 * A::TILE;
    const bool valid = t < ntiles;
    tile_dma<HD>(K, p.ld_qkv, t * KT, S, valid, dv, st, wid);
    tile_dma<HD>(V, p.ld_qkv, t * KT, S, valid, dv, st + A::TILE, wid);
  };
  // S^T = K Q^T, dP^T - delta = V dO^T - delta of the 32-key sub-block at row r0 of the slot
  // (the dP accumulator starts at -delta of this lane's query)
  auto sdp = [&](floatx16& sa, floatx16& dp, const bf16_t* lk, int r0) {
    zero16(sa);
#pragma unroll
    for (int r = 0; r < 16; ++r) dp[r] = -dl;
#pragma unroll
    for (int st = 0; st < A::NST; ++st) {
      sa = MFMA32(row_frag<HD>(lk, r0, st, lane), qf[st], sa);
      dp = MFMA32(row_frag<HD>(lk + A::TILE, r0, st, lane), df[st], dp);
    }
  };

  if (!(ABL & 8)) {
    issue(0);
    issue(1);
    issue(2);
    vm_wait<4 * A::NPW>();  // tile 0 landed (tiles 1, 2 may fly)
    ring_barrier();
  }
  auto half = [&](int t, int hf, floatx16& sa, floatx16& dp, floatx16& san, floatx16& dpn) {
    const bf16_t* lk = smem + (t % NSLOT) * 2 * A::TILE;
    const bf16_t* nk = hf == 0 ? lk : smem + ((t + 1) % NSLOT) * 2 * A::TILE;
    const int nr0 = hf == 0 ? 32 : 0;
    const int kt0 = t * KT;
    const int ks0 = kt0 + 32 * hf;
    const bool active = !(p.causal && ks0 > q0 + 31);  // wave-uniform: some key <= some query
    if (!active) {
      if constexpr (PIPE) sdp(san, dpn, nk, nr0);
      return;
    }
    const bool need_mask = (p.causal && ks0 + 31 > q0) || (ks0 + 32 > S) || pad;  // wave-uniform
    // ---- one basic block: next S^T, dP^T MFMAs || this sub-block's dS^T
    if constexpr (PIPE) sdp(san, dpn, nk, nr0);
    else sdp(sa, dp, lk, 32 * hf);
    if (need_mask) {
      const unsigned long long pm = pad_bits(pad, kt0, S, lane);
      const int lim = (p.causal ? min(q, S - 1) : S - 1) - kt0;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kl = 32 * hf + acc_row(r, lane);
        float pv = fast_exp2(fmaf(sa[r], c, -lse2));
        pv = (kl > lim || ((pm >> kl) & 1ull)) ? 0.f : pv;
        dp[r] = pv * dp[r];
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) dp[r] = fast_exp2(fmaf(sa[r], c, -lse2)) * dp[r];
    }
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      const bf16x8 db = acc_frag(dp, ss);
#pragma unroll
      for (int d = 0; d < A::NDT; ++d)
        dqt[d] = MFMA32(tr_frag<HD>(lk, 32 * hf, ss, d * 32, lane), db, dqt[d]);
    }
  };
  floatx16 sa0, dp0, sa1, dp1;
  if constexpr (PIPE) sdp(sa0, dp0, smem, 0);
  for (int t = 0; t < ((ABL & 1) ? 0 : ntiles); ++t) {
    vm_wait<2 * A::NPW>();  // this wave's pieces of tile t+1 landed (t+2 may fly)
    ring_barrier();         // ... every wave's; and every wave is done with tile t-1's slot
    issue(t + 3);
    half(t, 0, sa0, dp0, sa1, dp1);
    half(t, 1, sa1, dp1, sa0, dp0);
  }
  vm_wait<0>();

  if (q < S && !(ABL & 4)) {
    bf16_t* dQ = static_cast<bf16_t*>(p.dq) + (tok0 + q) * p.ld_dqkv + h * HD;
#pragma unroll
    for (int d = 0; d < A::NDT; ++d)
#pragma unroll
      for (int g = 0; g < 4; g += 2) {
        uint2 wa, wb;
        wa.x = pack2bf(dqt[d][4 * g + 0] * p.scale, dqt[d][4 * g + 1] * p.scale);
        wa.y = pack2bf(dqt[d][4 * g + 2] * p.scale, dqt[d][4 * g + 3] * p.scale);
        wb.x = pack2bf(dqt[d][4 * g + 4] * p.scale, dqt[d][4 * g + 5] * p.scale);
        wb.y = pack2bf(dqt[d][4 * g + 6] * p.scale, dqt[d][4 * g + 7] * p.scale);
        store_pair16(dQ + d * 32, g, hh, wa, wb);
      }
  }
}

// kernel variant (env DPC_ATTN_VAR="<fwd>,<bwd>", measured on MI355X: bench/attn_one.py):
// 0 = software-pipelined, 2 workgroups / CU; 1 = plain order, 2 / CU; 2 = plain, 3 / CU;
// 3 = pipelined, 3 / CU; 4 (forward only) = pipelined + fragments up front + pinned interleave;
// forward only: 5 / 6 = pair stream (attn_fwd2_kernel) with / without the MFMA row sum,
// 7 / 8 = the same on a persistent grid, 9 = 6 with the tile loop split by kind (attn_fwd3_kernel;
// its MFMA-row-sum form spilled 80 registers and ran 272 us, so it is not built).
// Defaults per head size (GPT-2 small shape, B=64 S=1023 H=12, profiles/r2_attn/, round 6:
// profiles/r6_attn/):  hd 64: forward 9, backward 1;  hd 32: forward 6 (S < 512) / 9, backward 2.
static int g_attn_env[2] = {-2, -2};
static int attn_var(int hd, int bwd, int S = 0) {
  if (g_attn_env[0] == -2) {
    g_attn_env[0] = g_attn_env[1] = -1;
    if (const char* e = getenv("DPC_ATTN_VAR")) sscanf(e, "%d,%d", &g_attn_env[0], &g_attn_env[1]);
  }
  if (g_attn_env[bwd] >= 0) return g_attn_env[bwd];
  // hd 32 forward (round 6, profiles/r6_attn/hd32_fwd_variants.log): the pair streams beat the
  // per-block kernel (2) -- fwd2 (6) at the reference CLI default S = 255 (16.9 vs 18.2 us),
  // fwd3 (9) at S = 1023 (111.3 vs 120.5 us)
  if (hd == 32) return bwd ? 2 : (S < 512 ? 6 : 9);
  return bwd ? 1 : 9;
}

#define DPC_ATTN_SWITCH(var, KERNEL, ...)                                                   \
  switch (var) {                                                                           \
    case 0: hipLaunchKernelGGL((KERNEL<HD, true, 2>), __VA_ARGS__); break;                  \
    case 1: hipLaunchKernelGGL((KERNEL<HD, false, 2>), __VA_ARGS__); break;                 \
    case 3: hipLaunchKernelGGL((KERNEL<HD, true, 3>), __VA_ARGS__); break;                  \
    default: hipLaunchKernelGGL((KERNEL<HD, false, 3>), __VA_ARGS__); break;                \
  }

// head_dim 128 (e.g. main-single.py --head_dim 128; 96 and other sizes over 64 are padded up to
// it): the same kernels at one workgroup per CU -- the 4-slot ring of K|V (or Q|dO) tiles is
// 4 x 2 x 16 KiB = 128 KiB of LDS, and the doubled Q / O (K, V, dK, dV) register rows need the
// 512-register budget.  (Correctness path; the GPT-2 presets run hd 64.)
static int launch_fwd128(const AttnArgs* a, hipStream_t stream) {
  dim3 grid((unsigned)(((a->S + QB - 1) / QB) * a->N * a->H));
  hipLaunchKernelGGL((attn_fwd_kernel<128, 1, 1>), grid, dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}
static int launch_bwd128(const AttnArgs* a, hipStream_t stream) {
  dim3 grid((unsigned)(((a->S + QB - 1) / QB) * a->N * a->H));
  hipLaunchKernelGGL((attn_bwd_dq_kernel<128, false, 1, 0, true>), grid, dim3(256), 0, stream, *a);
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<128, false, 1>), grid, dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

template <int HD>
static int launch_fwd(const AttnArgs* a, hipStream_t stream) {
  const int var = attn_var(HD, 0, a->S);
  dim3 grid((unsigned)(((a->S + QB - 1) / QB) * a->N * a->H));  // 1-D: xcd_work() maps it
  if (var >= 5 && var <= 9) {  // pair stream (attn_fwd2_kernel); 7, 8: persistent grid; 9: = 6 with
    // the tile loop split by kind (attn_fwd3_kernel)
    const int nqb = (a->S + QB - 1) / QB;
    const int nitems = ((nqb + 1) / 2) * a->N * a->H;
    dim3 g2((unsigned)((var == 7 || var == 8) && nitems > 512 ? 512 : nitems));
    if (var == 9) hipLaunchKernelGGL((attn_fwd3_kernel<HD, 2, false>), g2, dim3(256), 0, stream, *a, nitems);
    else if (var == 5 || var == 8) hipLaunchKernelGGL((attn_fwd2_kernel<HD, 2, true>), g2, dim3(256), 0, stream, *a, nitems);
    else hipLaunchKernelGGL((attn_fwd2_kernel<HD, 2, false>), g2, dim3(256), 0, stream, *a, nitems);
  } else if (var == 4) hipLaunchKernelGGL((attn_fwd_kernel<HD, 2, 2>), grid, dim3(256), 0, stream, *a);
  else DPC_ATTN_SWITCH(var, attn_fwd_kernel, grid, dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

// The shipped backward (variant 1 at hd 64, 2 at hd 32): the dQ kernel first, with the delta
// pre-pass fused in (it writes delta / lse2 for the dK / dV kernel); DPC_ATTN_PRE=1 (or a forced
// variant) keeps the separate pre-pass kernel and the dK / dV -> dQ order.
template <int HD>
static int launch_bwd(const AttnArgs* a, hipStream_t stream) {
  const int var = attn_var(HD, 1);
  static int pre_env = -1;
  if (pre_env < 0) pre_env = getenv("DPC_ATTN_PRE") ? atoi(getenv("DPC_ATTN_PRE")) : 0;
  dim3 grid((unsigned)(((a->S + QB - 1) / QB) * a->N * a->H));
  // (round 4 measured persistent pair-stream forms of both kernels -- one LDS-DMA stream of
  // (heaviest, lightest) block pairs per workgroup -- bitwise equal but slower: bwd 754 -> 798 us
  // with the dK / dV stream, 770 -> 954 us with the dQ stream, DDP step -0.8 % / -4 %
  // (profiles/r4_attn/); removed)
  if (!pre_env && var == (HD == 32 ? 2 : 1)) {
    if (HD == 32) hipLaunchKernelGGL((attn_bwd_dq_kernel<HD, false, 3, 0, true>), grid, dim3(256), 0, stream, *a);
    else hipLaunchKernelGGL((attn_bwd_dq_kernel<HD, false, 2, 0, true>), grid, dim3(256), 0, stream, *a);
    DPC_ATTN_SWITCH(var, attn_bwd_dkdv_kernel, grid, dim3(256), 0, stream, *a);
    return (int)hipGetLastError();
  }
  const long long rows = (long long)a->N * a->S * a->H;
  dim3 gpre((unsigned)((rows * (HD / 8) + 255) / 256));
  hipLaunchKernelGGL(attn_bwd_pre_kernel<HD>, gpre, dim3(256), 0, stream, *a);
  DPC_ATTN_SWITCH(var, attn_bwd_dkdv_kernel, grid, dim3(256), 0, stream, *a);
  DPC_ATTN_SWITCH(var, attn_bwd_dq_kernel, grid, dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

}  // namespace dpc

using namespace dpc;

// Host-side checks: the kernels assume 16-B aligned rows (ld % 8 == 0) and head_dim 32 / 64 / 128.
static bool attn_args_ok(const AttnArgs* a, bool bwd) {
  if (a->hd != 32 && a->hd != 64 && a->hd != 128) return false;
  if (a->N <= 0 || a->S <= 0 || a->H <= 0) return false;
  if (a->ld_qkv % 8 || a->ld_o % 8 || (bwd && a->ld_dqkv % 8)) return false;
  // (rows_rsrc's 32-bit offsets: one sequence's rows of Q / K / V / O / dO span < 4 GiB)
  const long long ld = a->ld_qkv > a->ld_o ? a->ld_qkv : a->ld_o;
  if (((long long)a->S + 256) * ld * 2 >= 0xffffffffll) return false;
  return true;
}

DPC_API int dpc_attn_fwd(const AttnArgs* a, hipStream_t stream) {
  if (!attn_args_ok(a, false)) return (int)hipErrorInvalidValue;
  if (a->hd == 128) return launch_fwd128(a, stream);
  return a->hd == 32 ? launch_fwd<32>(a, stream) : launch_fwd<64>(a, stream);
}

// Lab entry (bench/attn_lab.py): one backward kernel (which: 0 = delta / lse pre-pass, 1 = dK / dV,
// 2 = dQ) of the hd-64 shipped variant (plain order, 2 workgroups per CU) with the
// per-workgroup cost ablation bits ABL (attn_bwd_dkdv_kernel).
template <int ABL>
static void attn_lab_launch(const AttnArgs* a, int which, hipStream_t stream) {
  dim3 grid((unsigned)(((a->S + QB - 1) / QB) * a->N * a->H));
  if (which == 1) hipLaunchKernelGGL((attn_bwd_dkdv_kernel<64, false, 2, ABL>), grid, dim3(256), 0, stream, *a);
  else hipLaunchKernelGGL((attn_bwd_dq_kernel<64, false, 2, ABL>), grid, dim3(256), 0, stream, *a);
}
DPC_API int dpc_attn_bwd_lab(const AttnArgs* a, int which, int abl, hipStream_t stream) {
  if (!attn_args_ok(a, true) || a->hd != 64) return (int)hipErrorInvalidValue;
  if (which == 0) {
    const long long rows = (long long)a->N * a->S * a->H;
    hipLaunchKernelGGL(attn_bwd_pre_kernel<64>, dim3((unsigned)((rows * 8 + 255) / 256)), dim3(256), 0, stream, *a);
    return (int)hipGetLastError();
  }
  switch (abl) {
    case 0: attn_lab_launch<0>(a, which, stream); break;
    case 1: attn_lab_launch<1>(a, which, stream); break;
    case 2: attn_lab_launch<2>(a, which, stream); break;
    case 4: attn_lab_launch<4>(a, which, stream); break;
    case 6: attn_lab_launch<6>(a, which, stream); break;
    case 3: attn_lab_launch<3>(a, which, stream); break;
    case 5: attn_lab_launch<5>(a, which, stream); break;
    case 7: attn_lab_launch<7>(a, which, stream); break;
    case 15: attn_lab_launch<15>(a, which, stream); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}


// backward block order (DPC_ATTN_ORDER: 1 heaviest-first over the grid, the default; 0 per-XCD
// head-major).  Measured round 5 (profiles/r5_attn/bwd_order.log, same box, interleaved): dQ + dK/dV
// 601-608 -> 556-563 us, DDP 982.6K / 984.8K -> 994.3K / 993.0K.  Head-major left heavy blocks
// (the first key block of a head sweeps all 16 query tiles, the last one 2) among the last
// launched, a tail of up to one heavy block per slot; the lost L2 sharing of a head's Q / dO
// rows costs less (they stay in the 256 MB Infinity Cache).
static int g_attn_order = -1;
static int attn_order() {
  if (g_attn_order < 0) g_attn_order = getenv("DPC_ATTN_ORDER") ? atoi(getenv("DPC_ATTN_ORDER")) : 1;
  return g_attn_order;
}
DPC_API void dpc_attn_set_order(int v) { g_attn_order = v; }  // (tests / A/B; -1: the env again)

DPC_API int dpc_attn_bwd(const AttnArgs* a_in, hipStream_t stream) {
  AttnArgs b = *a_in;
  b.order = attn_order();
  const AttnArgs* a = &b;
  if (!attn_args_ok(a, true)) return (int)hipErrorInvalidValue;
  if (a->hd == 128) return launch_bwd128(a, stream);
  return a->hd == 32 ? launch_bwd<32>(a, stream) : launch_bwd<64>(a, stream);
}
