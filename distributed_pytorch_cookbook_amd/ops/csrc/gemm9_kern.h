// v9: the persistent one-wave-per-SIMD 256 x 256 GEMM of v7 with 64-deep k-stages in a
// two-buffer LDS ring (2 x 64 KiB) instead of 32-deep slices in a 5-slot ring.
//
// Why (bench/g7lab.hip, profiles/r3_gemm/lab/): in v7 a k-major operand's 32-deep slice makes
// every LDS-DMA piece 16 rows x 64 B -- half cache lines, the "fragment-shaped" load the
// cdna_hip_programming.md GEMM notes price at +12..28 % of the load path -- and the nt products
// (both operands k-major: every GPT-2 forward) paid for their DMA twice what nn products did
// (8192^3: no-DMA ablation +33 % nt vs +15 % nn).  With 64-deep stages a k-major piece is 8
// rows x 128 B, whole lines, at the same bytes per MFMA.
//
// Schedule of body t (stage t in buffer t % 2; fragments of stage t, k-step 0 in set F0):
//   phase 0: per MFMA group i, the k-step-1 fragments of stage t (row i of A, column block i
//            of B) are read into F1 while row i's 8 MFMAs run on F0;
//   mid:     vmcnt(stage t+1 landed) + s_barrier -- every wave has read all of stage t, so
//            its buffer is free;
//   phase 1: per group i, stage t+1's k-step-0 fragments into F0 beside the MFMAs on F1, and
//            in group i the DMA pair i of stage t+2 into buffer t % 2 (its M0 write and its two
//            loads in separate MFMA gaps, as v7 SCHED 6).
// One barrier per 64-deep stage (2,048 MFMA cycles per SIMD), a stage's DMA issued one body
// before it is waited for; the same register budget as v7 (two fragment sets).
//   RAW: stage t+1 is read in phase 1 of body t, after the mid barrier that every wave enters
//        after its own counted vmcnt for stage t+1's pieces.
//   WAR: stage t+2 overwrites buffer t % 2 in phase 1 of body t, after the mid barrier: every
//        read of stage t (k-step 0 in phase 1 of body t-1, k-step 1 in phase 0 of body t) is
//        older than that barrier, and each wave waits lgkmcnt(0) before entering it (the k-step-1
//        fragments are consumed only after it, so the compiler's own waits would come too late).
// Epilogue: v7's MODE 0 (plain bf16 / f32 products) or MODE 1 without per-element reads (the
// up-projection forward: bias + GELU + the pre-activation aux_out); the stores of a full tile may
// stay in flight through the next tile's first mid wait (stage 1 was issued before them).
#pragma once
#include "gemm7_kern.h"

namespace dpc {

constexpr int G9_KB = 64;
constexpr int G9_TA = 256 * G9_KB;          // elements per operand per stage (32 KiB)
constexpr int G9_SLOT = 2 * G9_TA;          // A + B (64 KiB)
constexpr int G9_NL = G9_TA / 512 / 4;      // 1-KiB pieces per wave per operand per stage (8)

// EPI 0: plain products; EPI 4: split-K partial tiles into the f32 workspace slab of their
// k-range (as v7 EPI 4: unit = split * tiles + tile, pl.nk = stages per split, pl.nk_all =
// stages of the whole product -- whole stages past it are issued with empty descriptors).
// ER (early release; 0 = the schedule above, the library launches 4 -- DPC_G9_ER /
// DPC_G9_FWD_ER): phase 0 reads ALL of stage t's k-step-1 fragments
// in its first ER groups (16 / ER reads per group, one per MFMA gap), then lgkmcnt(0) + an extra
// barrier -- every wave is done with stage t's buffer -- and the DMA of stage t+2 starts right
// there (pairs in phase 0 groups ER..7, the rest in phase 1), instead of in phase 1.  A stage's
// pieces then have ~1.5-1.75 bodies (3,000-3,600 MFMA cycles) to land before the mid wait that
// needs them, instead of 0.5-1 body: the round-4 lab had v9's main loop at ~70 % MFMA use with
// the DMA the only large ablation (no-DMA +57 % on the QKV forward).
//   RAW: unchanged (mid wait = this wave's stage t+1 pieces; the stage t+2 pieces issued in
//        phase 0 -- 2 (8 - ER) loads -- may stay in flight).
//   WAR: stage t+2 lands in buffer t % 2 only after the early barrier, which every wave enters
//        after lgkmcnt(0) on its last read of stage t (k-step 0 was read in body t-1).
template <int EPI, bool AK, bool BK, int ABL = 0, int ER = 0>
__global__ __launch_bounds__(256, 1) void gemm9_kernel(GemmArgs p, unsigned long long a_bytes,
                                                       unsigned long long b_bytes, G7Plan pl) {
  static_assert(EPI == 0 || EPI == 1 || EPI == 4, "v9: plain products, load-free forward epilogues, split-K slabs");
  static_assert(ER == 0 || ER == 2 || ER == 4, "v9: early release over 2 or 4 groups");
  constexpr int P0 = ER ? 8 - ER : 0;  // DMA pairs of stage t+2 issued in phase 0
  constexpr int NJ = 8;
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * G9_SLOT];
  // EPI 1: the bias of a tile's 256 columns per wave, by unit parity -- DMA'd when the issue
  // cursor enters the unit (two units ahead of its epilogue: the host requires >= 3 stages per
  // unit so that unit u+2's copy lands after unit u's epilogue read the same buffer)
  __shared__ __attribute__((aligned(16))) float sbias[EPI == 1 ? 2 * 4 * 256 : 4];

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int ar = wr * 128, bc = wc * 128;

  const int local = g7_local(blockIdx.x, pl.grid);
  const int nmine = local < pl.units ? (pl.units - local + pl.grid - 1) / pl.grid : 0;
  if (nmine == 0) return;
  unsigned long long clk_t0 = 0, clk_r0 = 0;
  if constexpr ((ABL & 128) != 0) {
    clk_t0 = __builtin_amdgcn_s_memtime();
    clk_r0 = __builtin_amdgcn_s_memrealtime();
  }

  int va[G9_NL], vb[G9_NL];
  dma_offsets3<G9_KB, AK, G9_NL>(va, p.lda, wid, lane);
  dma_offsets3<G9_KB, BK, G9_NL>(vb, p.ldb, wid, lane);
  const unsigned long long a_step = AK ? 128ull : 64ull * p.lda * 2;
  const unsigned long long b_step = BK ? 128ull : 64ull * p.ldb * 2;

  // ---- DMA issue cursor (unit, stage, buffer, byte offsets), wave-uniform (pl.nk = stages per
  // unit here)
  int is_u = 0, is_k = 0, is_buf = 0, is_kt0 = 0;
  unsigned long long is_aoff = 0, is_boff = 0;
  const int ntiles = pl.tiles_m * pl.tiles_n;
  // the bias copy of unit ui: one 1-KiB piece per wave (columns past N read as zeros); issued
  // between operand pieces, it only adds a younger op to the counted waits before it
  auto bias_dma = [&](int ui, int n0) G7_AI {
    if constexpr (EPI == 1) {
      // (no bias: an empty descriptor, the copy reads zeros -- the epilogue adds without a branch)
      const long long rem = p.bias ? (long long)(p.N - n0) * 4 : 0;
      const unsigned nb = rem <= 0 ? 0u : (rem > 1024 ? 1024u : (unsigned)rem);
      const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(p.bias ? p.bias + n0 : p.bias), 0, nb, 0x00020000);
      g7_m0(reinterpret_cast<const bf16_t*>(sbias + ((ui & 1) * 4 + wid) * 256));
      g7_ld<0>(rs, lane * 16);
    }
  };
  auto set_org = [&](int ui) {
    const int uu = local + ui * pl.grid;
    const int sp = uu / ntiles;
    int m0, n0;
    g7_tile(pl, uu - sp * ntiles, m0, n0);
    is_kt0 = sp * pl.nk;
    is_aoff = (AK ? (unsigned long long)m0 * p.lda * 2 : (unsigned long long)m0 * 2) + a_step * is_kt0;
    is_boff = (BK ? (unsigned long long)n0 * p.ldb * 2 : (unsigned long long)n0 * 2) + b_step * is_kt0;
    bias_dma(ui, n0);
  };
  set_org(0);
  __amdgpu_buffer_rsrc_t rsa, rsb;
  const bf16_t* is_lds = smem;
  auto prep = [&]() {
    const bool valid = is_u < nmine && is_kt0 + is_k < pl.nk_all;
    const unsigned long long la = a_bytes - is_aoff, lb = b_bytes - is_boff;
    const unsigned na = valid ? ((la >> 32) ? 0xffffffffu : (unsigned)la) : 0u;
    const unsigned nb = valid ? ((lb >> 32) ? 0xffffffffu : (unsigned)lb) : 0u;
    rsa = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.A + is_aoff), 0, na, 0x00020000);
    rsb = __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.B + is_boff), 0, nb, 0x00020000);
    is_lds = smem + is_buf * G9_SLOT;
  };
  auto advance = [&]() {
    is_buf ^= 1;
    is_aoff += a_step;
    is_boff += b_step;
    if (++is_k == pl.nk) {
      is_k = 0;
      ++is_u;
      if (is_u < nmine) set_org(is_u);
    }
  };
  // pair q (0..7) of a stage: pieces 2q, 2q+1 of A (q < 4) or of B; step 0 = M0, 1 / 2 = loads
  auto dma = [&](int q, int step) G7_AI {
    if constexpr ((ABL & 2) != 0) return;
    const bool isa = q < 4;
    const int i = 2 * (isa ? q : q - 4);
    const bf16_t* dst = is_lds + (isa ? 0 : G9_TA) + (wid * G9_NL + i) * 512;
    if (step == 0) g7_m0(dst);
    else if (step == 1) g7_ld<0>(isa ? rsa : rsb, isa ? va[i] : vb[i]);
    else g7_ld<1024>(isa ? rsa : rsb, (isa ? va[i + 1] : vb[i + 1]) - 1024);
  };
  auto stage_all = [&]() {  // a whole stage at once (prologue)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      dma(q, 0);
      dma(q, 1);
      dma(q, 2);
    }
  };

  // prologue: stages 0 and 1; stage 0 landed -> its k-step-0 fragments
  prep();
  stage_all();
  advance();
  prep();
  stage_all();
  advance();
  prep();
  g7_wait<2 * G9_NL>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  bf16x8 a0[8], b0[NJ], a1[8], b1[NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i) a0[i] = frag3<G9_KB, AK>(smem, ar + 16 * i, 0, lane);
#pragma unroll
  for (int j = 0; j < NJ; ++j) b0[j] = frag3<G9_KB, BK>(smem + G9_TA, bc + 16 * j, 0, lane);

  floatx4 acc[8][NJ];
  int rd = 0;      // buffer of the stage being computed
  int credit = 0;  // the first mid wait of a tile may leave the last epilogue's stores in flight

  auto mf = [&](int i, int j, const bf16x8* ac, const bf16x8* bcur, bool first) G7_AI {
    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bcur[j], ac[i], first ? floatx4{0.f, 0.f, 0.f, 0.f} : acc[i][j],
                                                        0, 0, 0);
  };
#define G9_SB __builtin_amdgcn_sched_barrier(0)
  // phase 0, group i: fragments of k-step 1 (same buffer) into (a1, b1), MFMAs on (a0, b0)
#define G9_G0(i, FIRST)                                                                             \
  do {                                                                                              \
    mf(i, 0, a0, b0, FIRST); G9_SB;                                                                 \
    if (!(ABL & 32)) a1[i] = frag3<G9_KB, AK>(lc, ar + 16 * i, 1, lane);                            \
    G9_SB; mf(i, 1, a0, b0, FIRST); G9_SB;                                                          \
    if (!(ABL & 32)) b1[i] = frag3<G9_KB, BK>(lc + G9_TA, bc + 16 * i, 1, lane);                    \
    G9_SB;                                                                                          \
    _Pragma("unroll") for (int j_ = 2; j_ < 8; ++j_) { mf(i, j_, a0, b0, FIRST); G9_SB; }           \
  } while (0)
  // phase 1, group i: stage t+1's k-step-0 fragments into (a0, b0), MFMAs on (a1, b1), DMA pair i
#define G9_G1(i)                                                                                    \
  do {                                                                                              \
    mf(i, 0, a1, b1, false); G9_SB;                                                                 \
    if (!(ABL & 32) && !LASTB) a0[i] = frag3<G9_KB, AK>(ln, ar + 16 * i, 0, lane);                  \
    G9_SB; mf(i, 1, a1, b1, false); G9_SB;                                                          \
    if (!(ABL & 32) && !LASTB) b0[i] = frag3<G9_KB, BK>(ln + G9_TA, bc + 16 * i, 0, lane);          \
    G9_SB; mf(i, 2, a1, b1, false); G9_SB;                                                          \
    dma(i, 0);                                                                                      \
    G9_SB; mf(i, 3, a1, b1, false); G9_SB;                                                          \
    dma(i, 1);                                                                                      \
    G9_SB; mf(i, 4, a1, b1, false); G9_SB;                                                          \
    dma(i, 2);                                                                                      \
    if ((i) == 7) advance();                                                                        \
    G9_SB; mf(i, 5, a1, b1, false); G9_SB;                                                          \
    if ((i) == 7) prep();                                                                           \
    G9_SB; mf(i, 6, a1, b1, false); G9_SB;                                                          \
    mf(i, 7, a1, b1, false); G9_SB;                                                                 \
  } while (0)
  // early-release phase 0: group i < ER reads 16 / ER fragments of k-step 1 (one per MFMA gap);
  // groups ER..7 carry the DMA pairs 0 .. P0-1 of stage t+2
#define G9_E0(i, FIRST)                                                                             \
  do {                                                                                              \
    if constexpr ((i) < ER) {                                                                       \
      constexpr int NR = 16 / ER, R0 = (i) * NR;                                                    \
      _Pragma("unroll") for (int j_ = 0; j_ < 8; ++j_) {                                            \
        mf(i, j_, a0, b0, FIRST); G9_SB;                                                            \
        if (j_ < NR && !(ABL & 32)) {                                                               \
          const int r_ = R0 + j_;                                                                   \
          if (r_ < 8) a1[r_ & 7] = frag3<G9_KB, AK>(lc, ar + 16 * (r_ & 7), 1, lane);               \
          else b1[r_ & 7] = frag3<G9_KB, BK>(lc + G9_TA, bc + 16 * (r_ & 7), 1, lane);              \
        }                                                                                           \
        G9_SB;                                                                                      \
      }                                                                                             \
      if constexpr ((i) == ER - 1) {                                                                \
        /* every wave done reading stage t: its buffer may take stage t+2 */                      \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                          \
        G9_SB;                                                                                      \
        if (!(ABL & 16)) __builtin_amdgcn_s_barrier();                                              \
        asm volatile("" ::: "memory");                                                              \
      }                                                                                             \
    } else {                                                                                        \
      mf(i, 0, a0, b0, FIRST); G9_SB; mf(i, 1, a0, b0, FIRST); G9_SB;                               \
      mf(i, 2, a0, b0, FIRST); G9_SB;                                                               \
      dma((i) - ER, 0);                                                                             \
      G9_SB; mf(i, 3, a0, b0, FIRST); G9_SB;                                                        \
      dma((i) - ER, 1);                                                                             \
      G9_SB; mf(i, 4, a0, b0, FIRST); G9_SB;                                                        \
      dma((i) - ER, 2);                                                                             \
      G9_SB; mf(i, 5, a0, b0, FIRST); G9_SB; mf(i, 6, a0, b0, FIRST); G9_SB;                        \
      mf(i, 7, a0, b0, FIRST); G9_SB;                                                               \
    }                                                                                               \
  } while (0)
  // early-release phase 1: group i reads stage t+1's k-step-0 fragments; groups 0 .. 7-P0 carry the
  // remaining DMA pairs P0 .. 7, and the group after the last pair advances the cursor
#define G9_E1(i)                                                                                    \
  do {                                                                                              \
    mf(i, 0, a1, b1, false); G9_SB;                                                                 \
    if (!(ABL & 32) && !LASTB) a0[i] = frag3<G9_KB, AK>(ln, ar + 16 * i, 0, lane);                  \
    G9_SB; mf(i, 1, a1, b1, false); G9_SB;                                                          \
    if (!(ABL & 32) && !LASTB) b0[i] = frag3<G9_KB, BK>(ln + G9_TA, bc + 16 * i, 0, lane);          \
    G9_SB; mf(i, 2, a1, b1, false); G9_SB;                                                          \
    if constexpr ((i) < 8 - P0) dma(P0 + (i), 0);                                                   \
    G9_SB; mf(i, 3, a1, b1, false); G9_SB;                                                          \
    if constexpr ((i) < 8 - P0) dma(P0 + (i), 1);                                                   \
    G9_SB; mf(i, 4, a1, b1, false); G9_SB;                                                          \
    if constexpr ((i) < 8 - P0) dma(P0 + (i), 2);                                                   \
    if constexpr ((i) == 8 - P0) advance();                                                         \
    G9_SB; mf(i, 5, a1, b1, false); G9_SB;                                                          \
    if constexpr ((i) == 8 - P0) prep();                                                            \
    G9_SB; mf(i, 6, a1, b1, false); G9_SB;                                                          \
    mf(i, 7, a1, b1, false); G9_SB;                                                                 \
  } while (0)
#define G9_EBODY(FIRST, CREDIT, LASTB_)                                                             \
  do {                                                                                              \
    constexpr bool LASTB = (LASTB_);                                                                \
    const bf16_t* lc = smem + rd * G9_SLOT;                                                         \
    const bf16_t* ln = smem + (rd ^ 1) * G9_SLOT;                                                   \
    G9_E0(0, FIRST); G9_E0(1, FIRST); G9_E0(2, FIRST); G9_E0(3, FIRST);                             \
    G9_E0(4, FIRST); G9_E0(5, FIRST); G9_E0(6, FIRST); G9_E0(7, FIRST);                             \
    /* mid: stage t+1 landed (younger: the 2 P0 pieces of stage t+2 issued in phase 0, and in  */ \
    /* a tile's first body the last epilogue's stores between the two)                         */ \
    if (ABL & 64) {                                                                                 \
    } else if ((CREDIT) && credit > 0) {                                                            \
      if (pl.store_cnt >= 48) g7_wait<63>(); /* (the counter's limit: stage t+1 still done) */       \
      else g7_wait<31 + 2 * P0>();                                                                  \
    } else {                                                                                        \
      g7_wait<2 * P0>();                                                                            \
    }                                                                                               \
    G9_SB;                                                                                          \
    if (!(ABL & 16)) __builtin_amdgcn_s_barrier();                                                  \
    asm volatile("" ::: "memory");                                                                  \
    G9_E1(0); G9_E1(1); G9_E1(2); G9_E1(3); G9_E1(4); G9_E1(5); G9_E1(6); G9_E1(7);                 \
    rd ^= 1;                                                                                        \
  } while (0)
#define G9_BODY(FIRST, CREDIT, LASTB_)                                                              \
  do {                                                                                              \
    constexpr bool LASTB = (LASTB_);                                                                \
    const bf16_t* lc = smem + rd * G9_SLOT;                                                         \
    const bf16_t* ln = smem + (rd ^ 1) * G9_SLOT;                                                   \
    G9_G0(0, FIRST); G9_G0(1, FIRST); G9_G0(2, FIRST); G9_G0(3, FIRST);                             \
    G9_G0(4, FIRST); G9_G0(5, FIRST); G9_G0(6, FIRST); G9_G0(7, FIRST);                             \
    /* mid: stage t+1 landed (younger: nothing, or the last epilogue's stores) */                   \
    if (ABL & 64) {                                                                                 \
    } else if ((CREDIT) && credit > 0) {                                                            \
      if (pl.store_cnt >= 48) g7_wait<63>();                                                        \
      else g7_wait<31>();                                                                           \
    } else {                                                                                        \
      g7_wait<0>();                                                                                 \
    }                                                                                               \
    /* WAR: this wave's reads of stage t (k-step 1, not yet consumed) completed before the    */ \
    /* barrier, after which stage t+2 may land in its buffer                                   */ \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                              \
    G9_SB;                                                                                          \
    if (!(ABL & 16)) __builtin_amdgcn_s_barrier();                                                  \
    asm volatile("" ::: "memory");                                                                  \
    G9_G1(0); G9_G1(1); G9_G1(2); G9_G1(3); G9_G1(4); G9_G1(5); G9_G1(6); G9_G1(7);                 \
    rd ^= 1;                                                                                        \
  } while (0)

  for (int u = 0; u < nmine; ++u) {
    if constexpr (ER != 0) {
      if constexpr (EPI == 1) {  // (the last body's fragment reads moved after the epilogue, below)
        G9_EBODY(true, true, false);
        credit = 0;
        for (int k = 1; k < pl.nk - 1; ++k) G9_EBODY(false, false, false);
        G9_EBODY(false, false, true);
      } else {
        G9_EBODY(true, true, false);
        credit = 0;
        for (int k = 1; k < pl.nk; ++k) G9_EBODY(false, false, false);
      }
    } else {
      if constexpr (EPI == 1) {
        // the unit's last body reads no k-step-0 fragments of the next unit: those 64 registers
        // stay free through the epilogue (its bias and GELU temporaries would spill otherwise,
        // and a spill reload there is waited for with vmcnt(0) -- behind the stores); they are
        // read after it (the host guarantees nk >= 3)
        G9_BODY(true, true, false);
        credit = 0;
        for (int k = 1; k < pl.nk - 1; ++k) G9_BODY(false, false, false);
        G9_BODY(false, false, true);
      } else {
        G9_BODY(true, true, false);
        credit = 0;
        for (int k = 1; k < pl.nk; ++k) G9_BODY(false, false, false);
      }
    }
    const int uu = local + u * pl.grid;
    int m0, n0;
    g7_tile(pl, uu % ntiles, m0, n0);
    if (pl.debug & 1) {
    } else if constexpr (EPI == 4) {
      GemmArgs q = p;  // the k-range's slab: [M][N] f32 at ws + split * M * N
      q.C = static_cast<float*>(p.ws) + (long long)(uu / ntiles) * p.M * p.N;
      q.ldc = p.N;
      q.out_f32 = 1;
      g7_epilogue<0, NJ>(q, acc, m0 + ar, n0 + bc, lane, 0);
    } else if constexpr (EPI == 1) {
      // forward epilogue that reads nothing per element (bias, activation, the pre-activation
      // aux_out; no residual / accumulate): its 32 + 32 stores stay in flight into the next tile
      // (the lane index recomputed by an opaque mbcnt: the epilogue's per-lane offsets are derived
      // here, not hoisted out of the unit loop into registers the main loop would have to carry)
      int elane;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(elane));
      // (measured round 5: MODE 0's whole-line store layout for both outputs -- lanes l, l ^ 8
      // trading a chunk so one store writes 8 rows x 128 B -- was SLOWER here than these 16-row
      // x 64-B stores, 448.6 vs 405.5 us on the GPT-2 up-projection, bench/epi_decomp.py)
      const float* lb = sbias + ((u & 1) * 4 + wid) * 256 + bc;
      // full tile, bf16 output, the default store policy: check-free, branch-free stores
      constexpr int SP = G_SP_DEFAULT;
      if (m0 + 256 <= p.M && n0 + 256 <= p.N && !p.out_f32 && g_sp_default(p.nt_store)) {
        if (p.act == ACT_GELU && p.aux_deriv)  // (the FFN up-projection of training: GELU' as aux_out)
          g7_epilogue<1, NJ, true, true, ACT_GELU, true, true, SP>(p, acc, m0 + ar, n0 + bc, elane, 0, lb);
        else if (p.act == ACT_GELU) g7_epilogue<1, NJ, true, true, ACT_GELU, true, false, SP>(p, acc, m0 + ar, n0 + bc, elane, 0, lb);
        else if (p.act == ACT_RELU) g7_epilogue<1, NJ, true, true, ACT_RELU, true, false, SP>(p, acc, m0 + ar, n0 + bc, elane, 0, lb);
        else g7_epilogue<1, NJ, true, true, 0, true, false, SP>(p, acc, m0 + ar, n0 + bc, elane, 0, lb);
      } else {
        g7_epilogue<1, NJ, true, true>(p, acc, m0 + ar, n0 + bc, elane, 0, lb);
      }
    } else {
      // (ABL 512: the epilogue's VALU without its stores; ABL 1024: non-temporal stores -- lab only)
      g7_epilogue<0, NJ>(p, acc, m0 + ar, n0 + bc, lane, (ABL & 512) ? 4 : ((ABL & 1024) ? 16 : 0));
    }
    credit = (pl.store_cnt > 0 && m0 + 256 <= p.M && n0 + 256 <= p.N) ? 1 : 0;
    if constexpr (EPI == 1) {
      if (u + 1 < nmine) {  // the next unit's stage 0 (buffer rd, retired by the last mid wait)
        // (lane offsets from an opaque mbcnt again: a value kept from before the stores would be
        // a spill reload here, waited for with vmcnt(0) behind all of them)
        int flane;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(flane));
        const bf16_t* lc = smem + rd * G9_SLOT;
#pragma unroll
        for (int i = 0; i < 8; ++i) a0[i] = frag3<G9_KB, AK>(lc, ar + 16 * i, 0, flane);
#pragma unroll
        for (int j = 0; j < NJ; ++j) b0[j] = frag3<G9_KB, BK>(lc + G9_TA, bc + 16 * j, 0, flane);
      }
    }
    if constexpr ((ABL & 2048) != 0) credit = 0;  // (lab: the next tile waits for the stores at once)
  }
#undef G9_G0
#undef G9_G1
#undef G9_BODY
#undef G9_E0
#undef G9_E1
#undef G9_EBODY
#undef G9_SB
  g7_wait<0>();  // the empty-descriptor DMA issued past the end drained before exit
  if constexpr ((ABL & 128) != 0) {
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x < 2048) {
      g7_clk[2 * blockIdx.x] = t1 - clk_t0;
      g7_clk[2 * blockIdx.x + 1] = r1 - clk_r0;
    }
  }
}

}  // namespace dpc
