// v7: persistent 256x256 bf16 MFMA GEMM, one 4-wave workgroup per CU, one wave per SIMD.
//
// Why this shape (MI355X, measured with bench/gemm_ab.py): the 8-wave ping-pong kernels
// (v5/v6) pay two workgroup barriers per 16 MFMAs and re-read 12 fragments per 32 MFMAs; on
// short-K products (K = 768: the QKV / out / up / LM-head forward products of GPT-2 small) they
// also drain the whole pipeline at every tile -- prologue latency + a 128 KiB store burst per
// CU with the matrix pipe idle -- and ran at ~680 TF/s against hipBLASLt's ~1,200.  Here:
//   * each wave owns a 128x128 output tile: 8 x 8 accumulators of v_mfma_f32_16x16x32_bf16
//     (256 accumulator registers; a 512-register wave, one per SIMD), i.e. 16 fragment reads
//     per 64 MFMAs (0.25 / MFMA vs 0.375) and ONE workgroup barrier per 32-deep k-slice
//     (1,024 MFMA cycles per SIMD);
//   * the k-slices of all the tiles a workgroup owns form one stream: an NS-slot LDS ring
//     (32 KiB per slot: A 256x32 + B 256x32) filled by LDS-DMA (buffer_load ... lds) DIST =
//     NS-1 slices ahead, never drained at a tile boundary, so the next tile's first slices are
//     in flight while the previous tile's epilogue runs;
//   * fragments of slice q+1 are read into a second register set while the MFMAs of slice q
//     run (two named sets, the loop unrolled by two);
//   * the MFMA operands are swapped (C^T = B A^T): lane l of a 16x16 accumulator holds output
//     row l & 15 and four CONSECUTIVE columns 4 (l >> 4) + r, so the epilogue works straight
//     from registers -- no LDS staging, no barrier: 16-B f32 stores, and for bf16 outputs
//     v_permlane16_swap pairs two fragments' 8-B halves into one 16-B store per lane.
// LDS images and fragment reads are the v3 ones (gemm.h): k-major [rows][32] with the 16-B
// chunk swizzle, mn-major [k][128-column halves] read with ds_read_b64_tr_b16.
//
// Synchronisation (per slice q, every wave):  body(q) = MFMAs on frags(q) | reads of frags(q+1)
// from slot (q+1) % NS | DMA of slice q+DIST into slot (q+DIST) % NS | epilogue if q ends a
// tile;  then vmcnt(slice q+2 landed) + s_barrier.
//   RAW: slot (q+2) is read in body(q+1), after this barrier, which every wave enters after its
//        own counted vmcnt for slice q+2 (its DMA pieces are older than the count).
//   WAR: slot (q+DIST) % NS held slice q-1, read in body(q-2) and consumed by the MFMAs of
//        body(q-1), i.e. retired before every wave passed barrier(q-1) -- before any wave
//        can be in body(q).
// Reference: every nn.Linear of /root/reference/models/gpt.py:29-30,60-64,219.
#include "gemm9_kern.h"
// every kernel instantiation below is compiled in gemm7_part*.hip (ops/gen_gemm_parts.py)
#include "gemm7_extern.inc"

using namespace dpc;

// ---- resident-CU budget.  v7 / v8 are persistent: their grid is sized to fill every CU
// (one / two 160 KiB workgroups each), so a kernel already resident on a CU -- an RCCL
// collective on the comm stream -- would hold back that CU's GEMM workgroup until the
// collective ends, and that workgroup's whole share of the tiles would then run as a second
// round (the product's time roughly doubled, SURVEY.md §5.8 rule 4).  While the engines have
// a collective in flight they reserve R CUs (parallel/transport.py; DPC_CU_RESERVE): the grid
// shrinks to CUs - R workgroups, the XCD remap (g7_local) stays bijective for any grid, and the
// tiles redistribute over the workgroups that are resident.
static int g7_reserve = 0;
static int g7_cus = 0;

static int g7_cu_count() {
  if (g7_cus <= 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      g7_cus = n;
    else
      g7_cus = 256;
  }
  return g7_cus;
}

DPC_API void dpc_set_cu_reserve(int r) { g7_reserve = r < 0 ? 0 : r; }
DPC_API int dpc_get_cu_reserve() { return g7_reserve; }

static inline long long g7_operand_bytes(long long rows, long long cols, long long ld) {
  if (rows <= 0 || cols <= 0) return 0;
  return ((rows - 1) * ld + ((cols + 7) / 8) * 8) * 2;
}

static int g_last_kernel = 0;  // (dpc_gemm_last_kernel, below)

template <int EPI, int SCHED, int WN = 128>
static void g7_launch(const GemmArgs* a, const G7Plan& pl, hipStream_t stream, unsigned long long ab,
                      unsigned long long bb) {
  dim3 grid(pl.grid), block(256);
  g_last_kernel = 700 + EPI + (WN == 64 ? 50 : 0);
  if (a->a_kmaj && a->b_kmaj) hipLaunchKernelGGL((gemm7_kernel<EPI, SCHED, true, true, WN>), grid, block, 0, stream, *a, ab, bb, pl);
  else if (a->a_kmaj) hipLaunchKernelGGL((gemm7_kernel<EPI, SCHED, true, false, WN>), grid, block, 0, stream, *a, ab, bb, pl);
  else if (!a->b_kmaj) hipLaunchKernelGGL((gemm7_kernel<EPI, SCHED, false, false, WN>), grid, block, 0, stream, *a, ab, bb, pl);
  else hipLaunchKernelGGL((gemm7_kernel<EPI, SCHED, false, true, WN>), grid, block, 0, stream, *a, ab, bb, pl);
}

// SCHED 3 / 4 pre-bias the voffset of the k-th piece of a group by -k KiB: it must hold that
// many bytes of rows before it (k-major: 16 rows per piece, mn-major: 4 k-rows per piece)
static bool g7_bias_ok(const GemmArgs* a, long long bytes = 1024) {
  auto ok = [bytes](bool kmaj, long long ld) { return kmaj ? ld * 2 * 16 >= bytes : ld * 2 * 4 >= bytes; };
  return ok(a->a_kmaj, a->lda) && ok(a->b_kmaj, a->ldb);
}

// The shipped schedule: two DMA pieces at the head of every even MFMA group, issued under one
// M0 write (SCHED 3) where the operands allow it, else one M0 write per piece (SCHED 2).
// Same-box A/B on MI355X (profiles/r3_gemm/ab22_*): +3 to +7 % on every GPT-2 product and on
// 8192^3 (1252 -> 1330 TF/s nt).  DPC_G7_PAIR=0 restores SCHED 2.
// v7 products with an mn-major operand (input and weight gradients) take the split interleave
// (SCHED 6: one M0 / DMA instruction per MFMA gap): same-box bench/g7lab A/B +4..8 % on nn and
// tn (8192^3 nn 1331 -> 1409, tn 1335 -> 1437 TF/s; GPT-2 out / up / LM-head input gradients
// +5.4 / +4.8 / +5.1 %), within 1 % on nt (profiles/r3_gemm/lab_sched6.log).  DPC_G7_SPLIT=0
// keeps the pairs.
static bool g7_split_sched(const GemmArgs* a) {
  static int env = -1;
  if (env < 0) env = getenv("DPC_G7_SPLIT") ? atoi(getenv("DPC_G7_SPLIT")) : 1;
  return env && (!a->a_kmaj || !a->b_kmaj);
}

template <int EPI, int WN = 128>
static void g7_launch_s(const GemmArgs* a, const G7Plan& pl, hipStream_t stream, unsigned long long ab,
                        unsigned long long bb) {
  static int pair_env = -1;
  if (pair_env < 0) pair_env = getenv("DPC_G7_PAIR") ? atoi(getenv("DPC_G7_PAIR")) : 1;
  if (WN == 128 && g7_bias_ok(a) && g7_split_sched(a)) g7_launch<EPI, 6, WN>(a, pl, stream, ab, bb);
  else if (pair_env && g7_bias_ok(a)) g7_launch<EPI, 3, WN>(a, pl, stream, ab, bb);
  else g7_launch<EPI, 2, WN>(a, pl, stream, ab, bb);
}

// v7d (deferred GELU epilogues): the forward up-projection form (both operands k-major) and
// the input-gradient form (A k-major, B n-major) with the paired-M0 DMA schedule
template <int EPI>
static bool g7d_launch(const GemmArgs* a, const G7Plan& pl, hipStream_t stream, unsigned long long ab,
                       unsigned long long bb) {
  dim3 grid(pl.grid), block(256);
  if (!g7_bias_ok(a)) return false;
  g_last_kernel = 750 + EPI;
  if (EPI == 5 && a->a_kmaj && a->b_kmaj) {
    hipLaunchKernelGGL((gemm7d_kernel<5, 3, true, true>), grid, block, 0, stream, *a, ab, bb, pl);
    return true;
  }
  if (EPI == 6 && a->a_kmaj && !a->b_kmaj) {
    hipLaunchKernelGGL((gemm7d_kernel<6, 3, true, false>), grid, block, 0, stream, *a, ab, bb, pl);
    return true;
  }
  if (EPI == 7 && a->a_kmaj && a->b_kmaj && pl.nk >= 34) {
    hipLaunchKernelGGL((gemm7d_kernel<7, 3, true, true>), grid, block, 0, stream, *a, ab, bb, pl);
    return true;
  }
  return false;
}

// Returns -1 if the product does not meet v7's requirements (caller falls back), else the
// hipError_t of the launch.  Requirements: k-major operands hold exactly K (% 64 == 0) columns,
// those of dpc_gemm7_ok.
// splits: 1 = none, > 1 forced, 0 = automatic (plain f32 products only: the tiles are too few to
// fill the chip, e.g. weight gradients -- K = tokens, M x N = a weight).
// Whether v7 takes this product: k-major operands hold exactly K columns with K % 32 == 0 (a
// slice never straddles a row end; mn-major operands end at row K, so their last slice reads
// zeros past it), N % 8 == 0, 16-B aligned C / bias / residual, 8-B aligned aux.
static int g7_act_lds = -1;  // -1: DPC_G7_ACTLDS (default on); 0 / 1 forced (A/B sweeps)
DPC_API void dpc_gemm7_set_act_lds(int v) { g7_act_lds = v; }
// lab switches for interleaved same-process A/Bs (bench/epi_decomp.py): variant k = v, -1 default
//   (none wired at the moment; round 5 used key 0 for the v9 EPI 1 store-layout A/B)
static int g_variant[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
// the kernel family + epilogue of the last product dpc_gemm7 launched (tests assert a forced
// implementation really ran instead of falling back): 900 + EPI for v9, 700 + EPI for v7
// (+ 50 for v8), 750 + EPI for v7d
DPC_API int dpc_gemm_last_kernel() { return g_last_kernel; }
DPC_API void dpc_gemm_set_variant(int k, int v) {
  if (k >= 0 && k < 8) g_variant[k] = v;
}
static int g7_res_lds = -1;  // -1: DPC_G7_RESLDS (default on); 0 / 1 forced (A/B sweeps)
DPC_API void dpc_gemm7_set_res_lds(int v) { g7_res_lds = v; }

DPC_API int dpc_gemm7_ok(const GemmArgs* a) {
  const long long ab = g7_operand_bytes(a->a_r, a->a_c, a->lda);
  const long long bb = g7_operand_bytes(a->b_r, a->b_c, a->ldb);
  auto al = [](const void* q, int b) { return ((uintptr_t)q % b) == 0; };
  const bool kmaj_ok = (!a->a_kmaj || (a->a_c == a->K && a->K % 32 == 0)) &&
                       (!a->b_kmaj || (a->b_c == a->K && a->K % 32 == 0)) &&
                       (a->a_kmaj || a->a_r == a->K) && (a->b_kmaj || a->b_r == a->K);
  return kmaj_ok && a->K > 0 && ab > 0 && bb > 0 && a->N % 8 == 0 && a->ldc % 8 == 0 && a->ldr % 4 == 0 &&
         a->ld_aux_in % 4 == 0 && a->ld_aux_out % 4 == 0 && al(a->C, 16) && al(a->bias, 16) &&
         al(a->residual, 16) && al(a->aux_in, 8) && al(a->aux_out, 8) && al(a->colsum, 4);
}

// splits: 1 = none, > 1 forced, 0 = automatic (plain f32 products only: the tiles are too few to
// fill the chip, e.g. weight gradients -- K = tokens, M x N = a weight).
// wn: 128 = v7 (256 x 256 tiles, one workgroup per CU), 64 = v8 (256 x 128 tiles, two per CU;
// split-K through workspace slabs only)
DPC_API int dpc_gemm7(const GemmArgs* a, int persistent, int sched, int splits, hipStream_t stream, int wn) {
  g_last_kernel = 0;
  if (a->M <= 0 || a->N <= 0) return 0;
  if (!dpc_gemm7_ok(a)) return -1;
  const long long ab = g7_operand_bytes(a->a_r, a->a_c, a->lda);
  const long long bb = g7_operand_bytes(a->b_r, a->b_c, a->ldb);
  const bool v8 = wn == 64;
  G7Plan pl{};
  pl.tile_n = v8 ? 128 : 256;
  pl.tiles_m = (a->M + 255) / 256;
  pl.tiles_n = (a->N + pl.tile_n - 1) / pl.tile_n;
  const int tiles = pl.tiles_m * pl.tiles_n;
  pl.nk_all = (a->K + G7_KB - 1) / G7_KB;
  const bool plain = !a->bias && !a->act_bwd && !a->aux_out && !a->act && !a->residual && !a->colsum;
  const bool splittable = plain && a->out_f32;
  int s = splits > 0 ? splits : 1;
  auto slab_fits = [&](int c) {
    return a->ws && (long long)c * a->M * a->N * 4 <= a->ws_bytes && a->ldc % 4 == 0 && ((uintptr_t)a->ws % 16) == 0;
  };
  const int cus = std::max(8, g7_cu_count() - g7_reserve);  // CUs the grid may occupy
  if (splits <= 0 && splittable) {
    // fill the chip (few tiles) or even out the last round (wave quantisation): time ~ rounds
    // * (slices per unit + the split epilogue) [+ the slab reduction].  Units are in k-slices
    // (~0.7 us at the measured MFMA rate).  The split epilogue: 256 KiB of f32 adds per CU at
    // the chip's memory-side atomic rate, ~40 slices, or the same bytes as plain slab stores,
    // ~12, plus a reduction pass over (c + 1) M x N f32 at ~5 TB/s.
    double best = 1e30;
    for (int c = 1; c <= 32; ++c) {
      const int per = 2 * ((pl.nk_all + 2 * c - 1) / (2 * c));
      if (c > 1 && per < 16) break;
      // (v8: two 256 x 128 units per CU at once, each half a v7 unit's MFMA work)
      const int rounds = v8 ? (tiles * c + 2 * cus - 1) / (2 * cus) : (tiles * c + cus - 1) / cus;
      double cost = (double)rounds * per;
      if (c > 1 && slab_fits(c)) {
        const double red_us = (double)(c + 1 + a->accumulate) * a->M * a->N * 4 / 5e6;
        cost += rounds * 12.0 + red_us / 0.7;
      } else if (c > 1) {
        if (v8) continue;  // v8 splits through workspace slabs only (no atomic epilogue)
        cost += rounds * 40.0;
      }
      if (cost < best - 1e-9) { best = cost; s = c; }
    }
  }
  if (s > 1 && (!splittable || (v8 && !slab_fits(s)))) return -1;
  // slab split (workspace for every k-range's partial tile) when the caller passed one that is
  // large enough; otherwise f32 atomics into C
  const bool slab = s > 1 && slab_fits(s);
  // the input-gradient epilogue (act', column sums) carries no forward operation
  if ((a->act_bwd || a->colsum) && (a->bias || a->act || a->aux_out || a->residual || a->accumulate)) return -1;
  pl.splits = s;
  pl.nk = 2 * ((pl.nk_all + 2 * s - 1) / (2 * s));  // even: a unit starts on register set 0
  pl.units = tiles * s;
  // persistent: one workgroup per CU streams its units through one ring; otherwise one unit
  // per workgroup
  const int slots = v8 ? 2 * cus : cus;  // workgroups resident at once
  pl.grid = (persistent && pl.units > slots) ? slots : pl.units;
  // vector-memory ops an epilogue issues per lane, for the store credit: only epilogues that
  // read nothing per element and issue every store of a full tile (no column-sum atomics)
  const bool no_loads = !a->residual && !a->act_bwd && !a->accumulate && !a->colsum;
  pl.store_cnt = (no_loads && (s == 1 || slab) && !v8) ? ((a->out_f32 || slab ? 64 : 32) + (a->aux_out ? 32 : 0)) : 0;
  static int dbg = -1;
  if (dbg < 0) dbg = getenv("DPC_G7_DEBUG") ? atoi(getenv("DPC_G7_DEBUG")) : 0;
  pl.debug = dbg;
  if (dbg & 13) pl.store_cnt = 0;
  // v7 input-gradient epilogue with an act' operand: the operand staged through LDS by DMA
  bool act_lds = false;
  // (g7_epilogue_act_lds; DPC_G7_ACTLDS=0 or dpc_gemm7_set_act_lds(0) keeps the per-lane reads)
  {
    static int env = -1;
    if (env < 0) env = getenv("DPC_G7_ACTLDS") ? atoi(getenv("DPC_G7_ACTLDS")) : 1;
    const int on = g7_act_lds >= 0 ? g7_act_lds : env;
    // (ACT_MUL: EPI 10, compiled for the default store policy only -- another policy takes EPI 3)
    act_lds = on && !v8 && s == 1 && a->act_bwd && a->aux_in && !a->out_f32 && a->ld_aux_in % 8 == 0 &&
              (a->act_bwd != ACT_MUL || g_sp_default(a->nt_store)) &&
              ((uintptr_t)a->aux_in % 16) == 0 && a->ld_aux_in <= (1 << 20);
  }
  // v7d: sched 5 (impl 24) takes the GELU / GELU' fused epilogues of full-depth products
  // (nk >= 18: at least 16 slices to spread a tile's deferred chunks over)
  if (sched == 5 && !v8 && s == 1 && pl.nk >= 18) {
    auto a16 = [](const void* q) { return ((uintptr_t)q % 16) == 0; };
    const bool dfwd = a->act == ACT_GELU && a->aux_out && !a->aux_deriv && !a->residual && !a->accumulate && !a->out_f32 &&
                      !a->act_bwd && !a->colsum && a->ld_aux_out % 8 == 0 && a16(a->aux_out);
    const bool dbwd = a->act_bwd == ACT_GELU && a->aux_in && !a->out_f32 && !a->accumulate && !a->bias && !a->act &&
                      !a->aux_out && !a->residual && a->ld_aux_in % 8 == 0 && a16(a->aux_in);
    const bool ddown = a->act == ACT_GELU && a->aux_out && !a->aux_deriv && a->residual && !a->accumulate && a->out_f32 &&
                       !a->act_bwd && !a->colsum && a->ld_aux_out % 8 == 0 && a16(a->aux_out) && a->ldr % 4 == 0 &&
                       a16(a->residual);  // (residual may alias C: a chunk is read, then written, by one lane)
    if (dfwd && g7d_launch<5>(a, pl, stream, ab, bb)) return (int)hipGetLastError();
    if (ddown && g7d_launch<7>(a, pl, stream, ab, bb)) return (int)hipGetLastError();
    if (dbwd && g7d_launch<6>(a, pl, stream, ab, bb)) return (int)hipGetLastError();
  }
  // v9 (64-deep stages, whole-line DMA pieces of the k-major operands) for the plain nt
  // products -- every GPT-2 forward projection: same-box bench/g7lab A/B +0.7..+8.7 % over v7
  // (8192^3 1383 -> 1429, out-projection 1045 -> 1136 TF/s; profiles/r3_gemm/lab_v9.log);
  // impl 26 forces it, DPC_G9=0 keeps v7 there.
  {
    static int g9_env = -1;
    if (g9_env < 0) g9_env = getenv("DPC_G9") ? atoi(getenv("DPC_G9")) : 1;
    const bool g9_ok = plain && !a->accumulate && s == 1 && !v8 && a->a_kmaj && a->b_kmaj && a->K % 64 == 0 &&
                       a->lda >= 64 && a->ldb >= 64;
    if (g9_ok && (sched == 7 || (g9_env && sched != 6 && sched != 5))) {
      G7Plan p9 = pl;
      p9.nk = a->K / 64;
      p9.nk_all = p9.nk;
      // early-release schedule (gemm9_kern.h ER): DPC_G9_ER = 0 / 2 / 4.  Default 4: same-box
      // bench/g7lab +2..5 % on the GPT-2 nt products (QKV 1142 -> 1169-1200, up 1166 -> 1200,
      // 8192^3 1494 -> 1546-1563 TF/s) and the DDP step 940.4K -> 945.9K tok/s over two
      // interleaved runs each (profiles/r4_er/)
      static int er_env = -1;
      if (er_env < 0) er_env = getenv("DPC_G9_ER") ? atoi(getenv("DPC_G9_ER")) : 4;
      if (er_env == 2)
        { g_last_kernel = 900; hipLaunchKernelGGL((gemm9_kernel<0, true, true, 0, 2>), dim3(p9.grid), dim3(256), 0, stream, *a, ab, bb, p9); }
      else if (er_env == 4)
        { g_last_kernel = 900; hipLaunchKernelGGL((gemm9_kernel<0, true, true, 0, 4>), dim3(p9.grid), dim3(256), 0, stream, *a, ab, bb, p9); }
      else
        { g_last_kernel = 900; hipLaunchKernelGGL((gemm9_kernel<0, true, true>), dim3(p9.grid), dim3(256), 0, stream, *a, ab, bb, p9); }
      return (int)hipGetLastError();
    }
    // plain input gradients (A k-major, B mn-major) on v9 only when the table asks for it (impl
    // 26): same-box A/B against v7 schedule 6 (the default for dX) +4-5 % on the out-projection
    // input gradients (K = N = D), -1..-3 % on the others (profiles/r4_g9/ab_*.log), so the
    // table gives it the square ones
    const bool g9_km = plain && !a->accumulate && s == 1 && !v8 && a->a_kmaj && !a->b_kmaj && a->K % 64 == 0 &&
                       a->lda >= 64 && a->ldb >= 128;
    if (g9_km && sched == 7) {
      G7Plan p9 = pl;
      p9.nk = a->K / 64;
      p9.nk_all = p9.nk;
      // (this path is built for ER 4 and ER 0 only: DPC_G9_ER=2 runs ER 0 here, so an ER-2 A/B
      // covers the nt forward products alone)
      static int er_km = -1;
      if (er_km < 0) er_km = getenv("DPC_G9_ER") ? atoi(getenv("DPC_G9_ER")) : 4;
      if (er_km == 4)
        { g_last_kernel = 900; hipLaunchKernelGGL((gemm9_kernel<0, true, false, 0, 4>), dim3(p9.grid), dim3(256), 0, stream, *a, ab, bb, p9); }
      else
        { g_last_kernel = 900; hipLaunchKernelGGL((gemm9_kernel<0, true, false>), dim3(p9.grid), dim3(256), 0, stream, *a, ab, bb, p9); }
      return (int)hipGetLastError();
    }
    // forward epilogues that read nothing per element (bias / activation / aux_out, no residual or
    // accumulate: the FFN up-projection) on v9 when the table asks for it (impl 26) or
    // DPC_G9_FWD=1: the 2 x 32 bf16 stores of a tile stay in flight into the next tile's stages
    // instead of draining beside the MFMAs of a 256 x 128 two-per-CU kernel (impl 10)
    static int g9f_env = -1;
    if (g9f_env < 0) g9f_env = getenv("DPC_G9_FWD") ? atoi(getenv("DPC_G9_FWD")) : 0;
    const bool g9_fwd = !plain && !a->residual && !a->accumulate && !a->act_bwd && !a->colsum && s == 1 && !v8 &&
                        a->a_kmaj && a->b_kmaj && a->K % 64 == 0 && a->K >= 192 && a->lda >= 64 && a->ldb >= 64 &&
                        (!a->aux_out || (a->ld_aux_out % 8 == 0 && ((uintptr_t)a->aux_out % 16) == 0));
    if (g9_fwd && (sched == 7 || g9f_env)) {
      G7Plan p9 = pl;
      p9.nk = a->K / 64;
      p9.nk_all = p9.nk;
      // the early-release schedule here too (DPC_G9_FWD_ER, default 4): same-box XL up-projection
      // 1,023 -> 1,046 TF/s, DDP 945.1K -> 947.7K, FSDP XL 88.5K -> 90.1K (profiles/r4_g9/)
      static int fer = -1;
      if (fer < 0) fer = getenv("DPC_G9_FWD_ER") ? atoi(getenv("DPC_G9_FWD_ER")) : 4;
      if (fer == 4)
        { g_last_kernel = 901; hipLaunchKernelGGL((gemm9_kernel<1, true, true, 0, 4>), dim3(p9.grid), dim3(256), 0, stream, *a, ab, bb, p9); }
      else
        { g_last_kernel = 901; hipLaunchKernelGGL((gemm9_kernel<1, true, true>), dim3(p9.grid), dim3(256), 0, stream, *a, ab, bb, p9); }
      return (int)hipGetLastError();
    }
    // weight gradients (both operands mn-major, split K through workspace slabs) on v9, with the
    // split count of v7's plan and the stages per split recomputed: measured SLOWER than v7
    // schedule 6 (GPT-2 small QKV / up weight gradients 0.205 -> 0.216 / 0.269 -> 0.285 ms, DDP
    // step -0.9 %; profiles/r3_gemm/v9_wgrad_negative.txt) -- the mn-major pieces were whole lines
    // already, and the two-buffer ring leaves the HBM-streamed operands less latency slack.
    // Off unless DPC_G9_WGRAD=1 (or impl 26).
    static int g9w_env = -1;
    if (g9w_env < 0) g9w_env = getenv("DPC_G9_WGRAD") ? atoi(getenv("DPC_G9_WGRAD")) : 0;
    if (slab && !v8 && !a->a_kmaj && !a->b_kmaj && a->lda >= 128 && a->ldb >= 128 &&
        (sched == 7 || (g9w_env && sched != 5))) {
      G7Plan p9 = pl;
      p9.nk_all = (a->K + 63) / 64;
      p9.nk = (p9.nk_all + s - 1) / s;
      { g_last_kernel = 904; hipLaunchKernelGGL((gemm9_kernel<4, false, false>), dim3(p9.grid), dim3(256), 0, stream, *a, ab, bb, p9); }
      const long long nq = (long long)a->M * (a->N / 4);
      const int blocks = (int)std::min<long long>((nq + 255) / 256, 4096);
      hipLaunchKernelGGL(g7_splitk_reduce, dim3(blocks), dim3(256), 0, stream, static_cast<float*>(a->C), a->ldc,
                         static_cast<const float*>(a->ws), a->M, a->N, s, a->accumulate, a->nt_store & 2);
      return (int)hipGetLastError();
    }
  }
  if (slab) {
    if (v8) g7_launch_s<4, 64>(a, pl, stream, ab, bb);
    else g7_launch_s<4>(a, pl, stream, ab, bb);
    const long long nq = (long long)a->M * (a->N / 4);
    const int blocks = (int)std::min<long long>((nq + 255) / 256, 4096);
    hipLaunchKernelGGL(g7_splitk_reduce, dim3(blocks), dim3(256), 0, stream, static_cast<float*>(a->C), a->ldc,
                       static_cast<const float*>(a->ws), a->M, a->N, s, a->accumulate, a->nt_store & 2);
  } else if (s > 1) {
    if (!a->accumulate) hipMemset2DAsync(a->C, (size_t)a->ldc * 4, 0, (size_t)a->N * 4, (size_t)a->M, stream);
    g7_launch_s<2>(a, pl, stream, ab, bb);
  } else if (v8) {
    if (plain && !a->accumulate) g7_launch_s<0, 64>(a, pl, stream, ab, bb);
    else if (!a->act_bwd && !a->colsum) g7_launch_s<1, 64>(a, pl, stream, ab, bb);
    else g7_launch_s<3, 64>(a, pl, stream, ab, bb);
  } else if (plain && !a->accumulate) {
    // the grouped-M0 forms replace the per-piece ones: SCHED 0 / 2 (one or two pieces per
    // group) -> pairs (3), SCHED 1 (four pieces at groups 0 and 4) -> quads (4)
    static int pair_env = -1;
    if (pair_env < 0) pair_env = getenv("DPC_G7_PAIR") ? atoi(getenv("DPC_G7_PAIR")) : 1;
    // (every DMA placement of the table's v7 choices -- 16 / 19 / 20 / 22 / 23 -- gives way to the
    // split interleave when an operand is mn-major: it beat each of them there)
    if ((sched == 6 || g7_split_sched(a)) && g7_bias_ok(a)) g7_launch<0, 6>(a, pl, stream, ab, bb);
    else if ((sched == 4 || (sched == 1 && pair_env)) && g7_bias_ok(a, 3072)) g7_launch<0, 4>(a, pl, stream, ab, bb);
    else if (sched == 1) g7_launch<0, 1>(a, pl, stream, ab, bb);
    else if ((sched == 3 || pair_env) && g7_bias_ok(a)) g7_launch<0, 3>(a, pl, stream, ab, bb);
    else if (sched == 2) g7_launch<0, 2>(a, pl, stream, ab, bb);
    else g7_launch<0, 0>(a, pl, stream, ab, bb);
  } else if (!a->act_bwd && !a->colsum) {
    // forward epilogue with an f32 residual into an f32 output: the residual staged through LDS
    // (g7_epilogue_res_lds; DPC_G7_RESLDS=0 or dpc_gemm7_set_res_lds(0) keeps the per-lane reads)
    static int res_env = -1;
    if (res_env < 0) res_env = getenv("DPC_G7_RESLDS") ? atoi(getenv("DPC_G7_RESLDS")) : 1;
    const bool res_lds = (g7_res_lds >= 0 ? g7_res_lds : res_env) && s == 1 && a->residual && a->out_f32 && !a->aux_deriv &&
                         !a->accumulate && a->ldr % 4 == 0 && ((uintptr_t)a->residual % 16) == 0 &&
                         a->ldr <= (1 << 20);
    if (res_lds) g7_launch_s<9>(a, pl, stream, ab, bb);
    else g7_launch_s<1>(a, pl, stream, ab, bb);
  } else if (act_lds) {
    // column sums through the workspace ([2 tiles_m][N] partials + g7_colsum_reduce) when the
    // caller passed one large enough, else f32 atomics from the epilogue
    const long long rows = 2ll * pl.tiles_m;
    const bool cs_ws = a->colsum && a->ws && rows * a->N * 4 <= a->ws_bytes && ((uintptr_t)a->ws % 16) == 0 &&
                       a->N % 4 == 0 && ((uintptr_t)a->colsum % 16) == 0;
    GemmArgs q = *a;
    if (!cs_ws) q.ws = nullptr;
    // (EPI 10: ACT_MUL with the default store policy compiled in)
    if (a->act_bwd == ACT_MUL) g7_launch_s<10>(&q, pl, stream, ab, bb);
    else g7_launch_s<8>(&q, pl, stream, ab, bb);
    if (cs_ws)
      hipLaunchKernelGGL(g7_colsum_reduce, dim3((unsigned)((a->N / 4 + 255) / 256), (unsigned)((rows + 15) / 16)),
                         dim3(256), 0, stream, a->colsum, static_cast<const float*>(a->ws), (int)rows, a->N);
  } else {
    g7_launch_s<3>(a, pl, stream, ab, bb);
  }
  return (int)hipGetLastError();
}
