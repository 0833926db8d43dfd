// MFMA bf16 GEMM for gfx950 with fused epilogues.
//
//   C[m,n] = alpha * sum_k A(m,k) * B(n,k)  (+ beta*C_old) (+ bias[n]) (act)
//
// A(m,k) is either "K-contiguous" (row-major [M][lda], the activation layout)
// or "M-contiguous" ([K][lda], i.e. a transposed view: wgrad's dY^T / X^T).
// B(n,k) likewise: K-contiguous ([N][ldb], torch [out,in] weights: forward)
// or N-contiguous ([K][ldb]: dgrad's W, wgrad's X).
//
// One kernel template covers forward (NT), dgrad (NN) and wgrad (TN): tiles
// are staged global->registers->LDS in their memory layout and the MFMA
// fragments are read with ds_read_b128 (K-contiguous images) or the gfx950
// transposing ds_read_b64_tr_b16 (M/N-contiguous images). Both LDS images are
// XOR-swizzled at 32-byte granularity so that either read is bank-conflict
// free (derivation in docs/KERNELS.md).
//
// MFMA: v_mfma_f32_16x16x32_bf16, 4 waves (2x2) per workgroup, 64-deep K tiles,
// double-buffered LDS with one barrier per K tile, register prefetch of the
// next tile issued before the MFMAs of the current one.
//
// Replaces the reference's Keras Dense MatMul+BiasAdd(+Relu) ops
// (reference: distributed_training_transformer/transformer_model.py:119-122,
// 165, 172-174, 333) and their gradients.
#pragma once
#include "tdg_common.h"
#include "tdg_gemm.h"
#include "tdg_reduce.h"
#include "gemm_pipe.h"

#include <cstdlib>
#include <type_traits>

namespace tdg {



// Grouped launch: up to MAXG same-shape problems in one grid (blockIdx.y =
// problem). Used for the weight gradients, deferred to the end of backward and
// issued per shape: long-K tiles for the whole chip without split-K slabs.
constexpr int MAXG = 32;
struct GemmGroup {
  const bf16_t* A[MAXG];
  const bf16_t* B[MAXG];
  void* C[MAXG];
};

template <int BM, int BN, int WM, int WN, int STAGES, bool A_KC, bool B_KC, int EPI,
          bool OUT_F32>
__global__ __launch_bounds__(WM* WN * 64) void gemm_kernel(
    const bf16_t* __restrict__ A, const bf16_t* __restrict__ B, void* __restrict__ Cv,
    const float* __restrict__ bias, const bf16_t* __restrict__ aux, int M, int N, int K, int lda,
    int ldb, int ldc, int ldaux, float alpha, float beta, int k_per_split, long long split_stride,
    const GemmGroup grp) {
  if (gridDim.y > 1) {
    A = grp.A[blockIdx.y];
    B = grp.B[blockIdx.y];
    Cv = grp.C[blockIdx.y];
  }
  constexpr int NW = WM * WN;
  constexpr int NT = NW * 64;
  constexpr int TM = BM / WM / 16;  // 16x16 subtiles per wave along M
  constexpr int TN = BN / WN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int SB = A_BYTES + B_BYTES;  // bytes per pipeline stage
  using GA = Glds<A_KC, BM, NW>;
  using GB = Glds<B_KC, BN, NW>;
  constexpr int PT = GA::P + GB::P;  // LDS-DMA instructions per wave per tile
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_m = cdiv(M, BM), tiles_n = cdiv(N, BN);
  const int nwg = tiles_m * tiles_n;
  // XCD-aware raster: xcd_remap gives each XCD a contiguous run of tile ids;
  // the run walks the SHORT output dimension fastest, so each XCD owns a band
  // of the larger operand (read from HBM once chip-wide) and re-reads only the
  // smaller one (L2-resident). Walking the long dimension fastest instead made
  // every XCD stream the whole large operand.
  const int t = xcd_remap(blockIdx.x, nwg);
  int tm, tn;
  if (tiles_n <= tiles_m) {
    tn = t % tiles_n;
    tm = t / tiles_n;
  } else {
    tm = t % tiles_m;
    tn = t / tiles_m;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  TDG_STAMP(0);

  // split-K range
  const int kb = blockIdx.z * k_per_split;
  const int ke = min(K, kb + k_per_split);
  const int nk = cdiv(ke - kb, BK);
  const bool ktail = ((ke - kb) % BK) != 0;

  GA ga;
  GB gb;
  ga.init(wid, lane);
  gb.init(wid, lane);

  // Epilogue operands (ReLU-mask aux, beta*C_old) of the wave's sub-tile are
  // loaded into registers HERE, before the first LDS-DMA: in the training
  // step they are cold in HBM (the ReLU input was written in forward), and
  // loaded after the MFMAs their latency sat fully exposed at the end of
  // every tile. Issued first, they are older than every DMA, so the
  // pipeline's vmcnt waits stay exact (they only also cover these loads).
  // Layout = the epilogue's 16-byte row chunks (EpiLds, tdg_gemm.h).
  using OutT = typename std::conditional<OUT_F32, float, bf16_t>::type;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int RPASS = OUT_F32 ? (WTM < 32 ? WTM : 32) : WTM;
  using Epi = EpiLds<EPI, OUT_F32, TM, TN, RPASS>;
  using EpiF = EpiLds<EPI_NONE, true, TM, TN, (WTM < 32 ? WTM : 32)>;  // split-K slabs
  static_assert(NW * Epi::BYTES <= STAGES * (BM + BN) * BK * 2 &&
                    NW * EpiF::BYTES <= STAGES * (BM + BN) * BK * 2,
                "epilogue images must fit in the pipeline LDS");
  const bool split = gridDim.z > 1;
  const bool vec = epi_vec_ok<EPI, OUT_F32>(Cv, ldc, aux, ldaux);
  constexpr bool SINGLE = RPASS == WTM;
  const bool pre_aux = SINGLE && EPI == EPI_DRELU && !split && vec && (ldaux % 8) == 0 &&
                       (reinterpret_cast<uintptr_t>(aux) & 15) == 0;
  const bool pre_c = SINGLE && beta != 0.f && !split && vec && ((ldc * (int)sizeof(OutT)) % 16) == 0;
  int4 aux_r[Epi::ITER], c_r[Epi::ITER];
#pragma unroll
  for (int t = 0; t < Epi::ITER; ++t) {
    const int m = m0 + wm * WTM + Epi::row_of(lane, t);
    const int n = n0 + wn * WTN + Epi::col_of(lane, t);
    const bool in = m < M && n + Epi::EPC <= N;
    if (pre_aux && in) aux_r[t] = *reinterpret_cast<const int4*>(aux + (size_t)m * ldaux + n);
    if (pre_c && in)
      c_r[t] = *reinterpret_cast<const int4*>(reinterpret_cast<const OutT*>(Cv) + (size_t)m * ldc + n);
  }

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Software pipeline. LDS: STAGES tiles in flight (LDS-DMA). Registers:
  // MFMA fragments one 32-deep k-step ahead (fa0/fb0 = step 0, fa1/fb1 =
  // step 1 of a 64-deep tile), so every ds_read is issued before the MFMAs
  // that hide its latency, and the single barrier per tile sits between the
  // two MFMA groups. The slot refilled after that barrier is the one of the
  // tile whose fragments are already all in registers, so all STAGES slots
  // hold live prefetches.
  static_assert(BK == 64, "two 32-deep k-steps per tile");
  const int abase = wm * (BM / WM), bbase = wn * (BN / WN);
#pragma unroll
  for (int s = 0; s < STAGES; ++s) {
    if (s < nk) {
      ga.issue(A, lda, M, ke, m0, kb + s * BK, smem + s * SB, wid);
      gb.issue(B, ldb, N, ke, n0, kb + s * BK, smem + s * SB + A_BYTES, wid);
    }
  }
  short8_t fa0[TM], fb0[TN], fa1[TM], fb1[TN];
  if (nk > 0) {
    if (nk >= STAGES)
      wait_vmcnt<(STAGES - 1) * PT>();
    else
      wait_vmcnt<0>();
    lds_barrier();
    TDG_STAMP(1);
    if (ktail && nk == 1) {
      GA::zero_ktail(smem, kb, ke, tid, NT);
      GB::zero_ktail(smem + A_BYTES, kb, ke, tid, NT);
      lds_barrier();
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) fa0[i] = frag<A_KC, BM>(smem, abase + 16 * i, 0, lane);
#pragma unroll
    for (int j = 0; j < TN; ++j) fb0[j] = frag<B_KC, BN>(smem + A_BYTES, bbase + 16 * j, 0, lane);
  }

  // LDS instructions of one k-step's fragment reads (for the counted waits)
  constexpr int STEP_OPS = TM * frag_ops<A_KC>() + TN * frag_ops<B_KC>();
  // MODE 3: steady state (tile kt + STAGES exists: refill, counted wait);
  // 2: tile kt + STAGES - 1 is the last one (counted wait, no refill);
  // 1: drain (wait for everything); 0: the last tile. Branch-free steady
  // state, the tail steps their own instantiations (docs/PERF.md "Round 4").
  auto kstep = [&](int kt, auto modec) {
    constexpr int MODE = decltype(modec)::value;
    const char* st = smem + (kt % STAGES) * SB;
#pragma unroll
    for (int i = 0; i < TM; ++i) fa1[i] = frag<A_KC, BM>(st, abase + 16 * i, 1, lane);
#pragma unroll
    for (int j = 0; j < TN; ++j) fb1[j] = frag<B_KC, BN>(st + A_BYTES, bbase + 16 * j, 1, lane);
    // step-0 fragments landed; the step-1 reads just issued stay in flight
    lgkm_wait<STEP_OPS>();
    tie_all(fa0);
    tie_all(fb0);
    prio_hi();
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(fb0[j], fa0[i], acc[i][j]);
    prio_lo();
    if constexpr (MODE >= 1) {
      // tile kt+1 landed (this wave's DMA), then everyone's; everyone is done
      // reading tile kt (its fragments are in registers)
      if constexpr (MODE >= 2) wait_vmcnt<(STAGES - 2) * PT>();
      else wait_vmcnt<0>();
      lds_barrier();
      const char* nx = smem + ((kt + 1) % STAGES) * SB;
      if constexpr (MODE <= 2) {  // (a K tail is only ever the last tile)
        if (ktail && kt + 1 == nk - 1) {
          GA::zero_ktail(const_cast<char*>(nx), kb + (kt + 1) * BK, ke, tid, NT);
          GB::zero_ktail(const_cast<char*>(nx) + A_BYTES, kb + (kt + 1) * BK, ke, tid, NT);
          lds_barrier();
        }
      }
      if constexpr (MODE == 3) {
        char* ns = smem + (kt % STAGES) * SB;
        ga.issue(A, lda, M, ke, m0, kb + (kt + STAGES) * BK, ns, wid);
        gb.issue(B, ldb, N, ke, n0, kb + (kt + STAGES) * BK, ns + A_BYTES, wid);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) fa0[i] = frag<A_KC, BM>(nx, abase + 16 * i, 0, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb0[j] = frag<B_KC, BN>(nx + A_BYTES, bbase + 16 * j, 0, lane);
      // (the step-1 fragments completed at the barrier's lgkmcnt(0))
    } else {
      lgkm_wait<0>();
    }
    tie_all(fa1);
    tie_all(fb1);
    prio_hi();
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(fb1[j], fa1[i], acc[i][j]);
    prio_lo();
  };
  {
    int kt = 0;
    for (; kt + STAGES < nk; ++kt) kstep(kt, std::integral_constant<int, 3>{});
    if (kt + STAGES - 1 < nk && kt + 1 < nk) kstep(kt++, std::integral_constant<int, 2>{});
    for (; kt + 1 < nk; ++kt) kstep(kt, std::integral_constant<int, 1>{});
    if (kt < nk) kstep(kt, std::integral_constant<int, 0>{});
  }

  TDG_STAMP(2);
  // ---------------- epilogue: per-wave LDS image over the pipeline stages
  // (EpiLds, tdg_gemm.h). Split-K partial products go unscaled into the f32
  // slab of split z.
  lds_barrier();  // all waves done with the pipeline stages
  const int mw0 = m0 + wm * WTM, nw0 = n0 + wn * WTN;
  if (split) {
    float* Cs = reinterpret_cast<float*>(Cv) + (size_t)blockIdx.z * split_stride;
    EpiF::run(smem + wid * EpiF::BYTES, acc, lane, Cs, ldc, M, N, mw0, nw0, 1.f, 0.f, nullptr,
              nullptr, 0, epi_vec_ok<EPI_NONE, true>(Cs, ldc, nullptr, 0));
  } else {
    Epi::template run_pre<true>(smem + wid * Epi::BYTES, acc, lane, Cv, ldc, M, N, mw0, nw0, alpha,
                                beta, bias, aux, ldaux, vec, aux_r, pre_aux, c_r, pre_c);
  }
#ifdef TDG_STAMPS
  TDG_STAMP(3);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  TDG_STAMP(4);
#endif
}

// ---------------------------------------------------------------------------
// 256x256-tile GEMM, any operand layout: 8 waves as 2 (M) x 4 (N), each wave a
// 128 x 64 block = 8 x 4 MFMA subtiles. A K-tile (64 deep) is processed in
// four phases, one output quadrant of every wave (4 x 2 subtiles x 2 k-steps =
// 16 MFMAs) each: (a0,b0) (a0,b1) (a1,b1) (a1,b0), where a0/a1 are the
// upper/lower 64 rows of a wave's block and b0/b1 its left/right 32 columns.
// So each phase reads only the operand half it adds and a K-tile's fragments
// stay in registers.
// The LDS-DMA stages the next K-tile one half-tile per phase, in consumption
// order: A-half 0 (the a0 rows of both wave rows), B-half 0, B-half 1, A-half 1
// -- i.e. a half-tile is a set of 128 non-contiguous rows / columns (2 x 64 of
// A, 4 x 32 of B), remapped on the global side. A half-tile image is 16 KiB in
// either layout (K-contiguous: 128 rows x 64 k; MN-contiguous: 64 k x 128
// columns, read with ds_read_b64_tr_b16). A phase that needs a new half waits
// vmcnt(4) (the two younger halves stay in flight) + one barrier; two LDS
// buffers. MFMA groups run at raised wave priority.
//
// Ragged grouping: one launch covers up to R256_MAXP problems in up to
// R256_MAXC shape classes sharing K (the deferred weight gradients of a whole
// model: 60+ long-K problems of 5 shapes -> ~700 tiles, one launch, no split-K).
// 128 FLOP per LDS byte vs 64 for 128x128 tiles.
constexpr int R256_MAXP = 64, R256_MAXC = 8;
struct R256Class {
  // t_first: tile index (within the problem) of the class's first tile -- a
  // class may cover a tile sub-range of a single problem, so a long list of
  // weight gradients can be cut into launches of exactly one wave of tiles
  int M, N, lda, ldb, ldc, tiles_m, tiles_n, tile_start, prob_start, t_first;
};
struct R256Args {
  const bf16_t* A[R256_MAXP];
  const bf16_t* B[R256_MAXP];
  void* C[R256_MAXP];
  // optional fused bias gradient of problem i: bias_out[i][m] (=|+=) sum_k A[m][k]
  // (row sums of the A operand over the whole K; only for A MN-contiguous)
  float* bias_out[R256_MAXP];
  R256Class cls[R256_MAXC];
  int ncls;
};

// Main-loop refill: every half-tile slot is refilled with the K-tile TWO
// steps ahead as soon as the phase after its last read has passed its
// barrier (A-half0 / B-half0 in phase 1, B-half1 in phase 2, A-half1 in
// phase 0 of the next step), not with the next K-tile one whole step later:
// the same 128 KiB of LDS keep 5-7 half-tiles (80-112 KiB) in flight instead
// of 2-4, each half issued 6-7 phases before its use instead of 3-4 (round 6:
// weight-gradient L2 hit rate 54 -> 65 %, profiles/r6/). Counted waits (per
// wave, 2 LDS-DMA instructions per half; issue order A1 of kt+1 | A0 B0 of
// kt+2 | B1 of kt+2 per step):
//   steady (kt+2 exists) 10 / 10 / 12, kt+1 last 10 / 10 / 8, last 4 / 2 / 0.
// (Measured and not kept, docs/PERF.md "Round 6": reading each phase's
// fragments behind the previous phase's MFMAs -- equal on the NT forwards,
// and with MN-contiguous operands, whose fragments are two transposing reads
// joined into one register quad, it spills inside the loop.)
template <bool A_KC, bool B_KC, int EPI, bool OUT_F32>
__global__ __launch_bounds__(512) void gemm256_kernel(const R256Args args,
                                                      const float* __restrict__ bias,
                                                      const bf16_t* __restrict__ aux, int K,
                                                      int ldaux, float alpha, float beta) {
  constexpr int NW = 8;
  constexpr int HB = 128 * BK * 2;  // bytes of one half-tile image
  constexpr int SB = 4 * HB;        // stage: A-half0, A-half1, B-half0, B-half1
  using GA = Glds<A_KC, 128, NW>;
  using GB = Glds<B_KC, 128, NW>;
  static_assert(GA::P == 2 && GB::P == 2, "half-tile = 2 pieces per wave");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;

  // ragged tile id -> (class, problem, tile); class fields picked with
  // constant indices (scalar selects, no private copy of the argument block)
  const int t0 = xcd_remap(blockIdx.x, gridDim.x);
  R256Class cl = args.cls[0];
#pragma unroll
  for (int i = 1; i < R256_MAXC; ++i)
    if (i < args.ncls && t0 >= args.cls[i].tile_start) cl = args.cls[i];
  const int M = cl.M, N = cl.N, lda = cl.lda, ldb = cl.ldb, ldc = cl.ldc;
  const int tpp = cl.tiles_m * cl.tiles_n;
  const int lt = t0 - cl.tile_start + cl.t_first;
  const int p = cl.prob_start + lt / tpp;
  const int t = lt % tpp;
  const bf16_t* __restrict__ A = args.A[p];
  const bf16_t* __restrict__ B = args.B[p];
  void* __restrict__ Cv = args.C[p];
  int tm, tn;
  if (cl.tiles_n <= cl.tiles_m) {
    tn = t % cl.tiles_n;
    tm = t / cl.tiles_n;
  } else {
    tm = t % cl.tiles_m;
    tn = t / cl.tiles_m;
  }
  // Fused bias gradient (weight-gradient launches): the tiles of the first
  // N-column also sum their A fragments over K -- the A operand is dY^T, so
  // its row sums are the bias gradient, read here from registers the MFMAs
  // already hold instead of a second pass over dY. Wave wn sums fragments
  // wn (rows 16wn.., half 0) and 4+wn (half 1) with v_dot2 against ones.
  float* __restrict__ bias_out = A_KC ? nullptr : args.bias_out[p];
  const bool do_bsum = bias_out != nullptr && tn == 0;
  float bsum0 = 0.f, bsum1 = 0.f;
  const int m0 = tm * 256, n0 = tn * 256;
  const int nk = K / BK;  // host guarantees K % 64 == 0
  TDG_STAMP(0);

  GA ga;
  GB gb;
  ga.init(wid, lane);
  gb.init(wid, lane);
  // Image row/column x (0..127) of a half-tile <- tile row/column:
  //   A-half hA: (x / 64) * 128 + hA * 64 + x % 64
  //   B-half hB: (x / 32) * 64 + hB * 32 + x % 32
  // (KC images remap rows, MC images remap 8-element column chunks.)
  // LDS-DMA through buffer resources: per lane and piece of every half-tile a
  // byte offset fixed for the whole K loop (VGPR), per K-tile one scalar
  // offset (k0 * 2 K-contiguous, k0 * ld * 2 MN-contiguous) -- no per-lane
  // 64-bit address is ever formed (as global_load_lds addresses, the
  // compiler strength-reduced them into eight loop-carried 64-bit pointers
  // and spilled). launch_256 checks every extent is below 2^31 bytes. Rows /
  // columns past the operand are clamped (KC: the last row, MC: column 0;
  // never stored).
  uint32_t a_off[2][2], b_off[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int xa = A_KC ? ga.row[i] : ga.col[i];
    const int xb = B_KC ? gb.row[i] : gb.col[i];
    const int ka = A_KC ? ga.col[i] : ga.row[i];
    const int kb = B_KC ? gb.col[i] : gb.row[i];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      int ma = m0 + (xa >> 6) * 128 + hh * 64 + (xa & 63);
      int nb = n0 + (xb >> 5) * 64 + hh * 32 + (xb & 31);
      if (A_KC) {
        ma = ma < M ? ma : M - 1;
        a_off[hh][i] = 2u * (uint32_t)(ma * lda + ka);
      } else {
        ma = ma < M ? ma : 0;
        a_off[hh][i] = 2u * (uint32_t)(ka * lda + ma);
      }
      if (B_KC) {
        nb = nb < N ? nb : N - 1;
        b_off[hh][i] = 2u * (uint32_t)(nb * ldb + kb);
      } else {
        nb = nb < N ? nb : 0;
        b_off[hh][i] = 2u * (uint32_t)(kb * ldb + nb);
      }
    }
  }
  const int nrec_a = 2 * (A_KC ? (M - 1) * lda + K : (K - 1) * lda + M);
  const int nrec_b = 2 * (B_KC ? (N - 1) * ldb + K : (K - 1) * ldb + N);
  const uint32_t kstep_a = A_KC ? BK * 2u : (uint32_t)BK * (uint32_t)lda * 2u;
  const uint32_t kstep_b = B_KC ? BK * 2u : (uint32_t)BK * (uint32_t)ldb * 2u;
  auto issue = [&](const bf16_t* X, int nrec, const uint32_t* offs, uint32_t soff, char* dst) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(X), (short)0, nrec, 0x00020000),
          (__attribute__((address_space(3))) void*)(dst + (wid * 2 + i) * 1024), 16, offs[i],
          (int)soff, 0, 0);
  };
  // half h of K-tile kt: 0 = A-half0, 1 = B-half0, 2 = B-half1, 3 = A-half1
  auto issue_half = [&](int kt, int h) {
    char* st = smem + (kt & 1) * SB;
    if (h == 0) issue(A, nrec_a, a_off[0], kstep_a * (uint32_t)kt, st + 0 * HB);
    else if (h == 1) issue(B, nrec_b, b_off[0], kstep_b * (uint32_t)kt, st + 2 * HB);
    else if (h == 2) issue(B, nrec_b, b_off[1], kstep_b * (uint32_t)kt, st + 3 * HB);
    else issue(A, nrec_a, a_off[1], kstep_a * (uint32_t)kt, st + 1 * HB);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // this wave's rows/columns inside the half-tile images: a-subtile i (0..3)
  // of half hA at wm*64 + 16i; b-subtile j (0..1) of half hB at wn*32 + 16j
  const int arow = wm * 64, brow = wn * 32;
  short8_t fa[8][2], fb[4][2];
  auto bias_sum = [&](int ph) {
    const bf16x2_t one = __builtin_bit_cast(bf16x2_t, 0x3f803f80);
    float bs = ph == 0 ? bsum0 : bsum1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i != wn) continue;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const short8_t f = ph == 0 ? fa[i][s2] : fa[4 + i][s2];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          bs = __builtin_amdgcn_fdot2_f32_bf16(
              __builtin_bit_cast(bf16x2_t, (short2_t){f[2 * e], f[2 * e + 1]}), one, bs, false);
      }
    }
    if (ph == 0) bsum0 = bs;
    else bsum1 = bs;
  };
  {
#pragma unroll
    for (int h = 0; h < 4; ++h) issue_half(0, h);
    if (nk > 1) {
#pragma unroll
      for (int h = 0; h < 3; ++h) issue_half(1, h);
    }
    // Fragment reads at immediate DS offsets: every read of a K-step is one
    // of six per-lane bases (+ the stage) plus a compile-time offset -- the
    // half image, the 32-deep k-step, the 4-row group of a transposing read
    // or the subtile row -- instead of a swizzled address computed per read
    // (~50 VALU per K-step and wave). The swizzle terms of frag<> (lds_off)
    // depend only on the lane there: K-contiguous images XOR the 32-byte
    // segment 2 s + (g >> 1) with (lane >> 1) & 3, one base per k-step s;
    // MN-contiguous images XOR the subtile's segment with (lane >> 2) & 3 |
    // (g & 1) << 2, one base per subtile.
    const int fg = lane >> 4, fcl = lane & 15, fq = fcl >> 2, fp = fcl & 3;
    const uint32_t lds0 = (uint32_t)(uintptr_t)smem;
    auto kc_base = [&](int row0, int s) -> uint32_t {
      return lds0 + (row0 + fcl) * (BK * 2) + (((2 * s + (fg >> 1)) ^ ((fcl >> 1) & 3)) << 5) + (fg & 1) * 16;
    };
    auto mn_base = [&](int sub) -> uint32_t {
      return lds0 + (8 * fg + fq) * 256 + 8 * fp + ((sub ^ (fq | ((fg & 1) << 2))) << 5);
    };
    uint32_t rba[4], rbb[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) rba[i] = A_KC ? kc_base(arow, i & 1) : mn_base((arow >> 4) + i);
#pragma unroll
    for (int j = 0; j < 2; ++j) rbb[j] = B_KC ? kc_base(brow, j) : mn_base((brow >> 4) + j);
    // fragment (subtile I, k-step S) of the half image at H * HB; b: bases of the stage
    auto frag_imm = [&](auto kcc, auto hc, auto ic, auto sc, const uint32_t* b) -> short8_t {
      constexpr bool KC = decltype(kcc)::value;
      constexpr int H = decltype(hc)::value, I = decltype(ic)::value, S = decltype(sc)::value;
      if constexpr (KC) {
        return lds_read_b128_at<H * HB + I * 16 * BK * 2>(b[S]);
      } else {
        return cat4(lds_read_tr16_at<H * HB + 8192 * S>(b[I]), lds_read_tr16_at<H * HB + 8192 * S + 1024>(b[I]));
      }
    };
    using AKCc = std::integral_constant<bool, A_KC>;
    using BKCc = std::integral_constant<bool, B_KC>;
    // MODE 3: K-tiles kt+1 and kt+2 exist; 2: kt+1 is the last; 1: kt is
    auto kstep_deep = [&](int kt, auto modec) {
      constexpr int MODE = decltype(modec)::value;
      const uint32_t stg = (uint32_t)(kt & 1) * SB;
      uint32_t ba[4], bb[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) ba[i] = rba[i] + stg;
#pragma unroll
      for (int j = 0; j < 2; ++j) bb[j] = rbb[j] + stg;
#pragma unroll
      for (int ph = 0; ph < 4; ++ph) {
        if (ph < 3) {
          if (ph == 0) wait_vmcnt<MODE == 1 ? 4 : 10>();
          else if (ph == 1) wait_vmcnt<MODE == 1 ? 2 : 10>();
          else wait_vmcnt<MODE == 3 ? 12 : (MODE == 2 ? 8 : 0)>();
          lds_barrier();
          if (kt == 0 && ph == 0) TDG_STAMP(1);
        }
        using C0 = std::integral_constant<int, 0>;
        using C1 = std::integral_constant<int, 1>;
        using C2 = std::integral_constant<int, 2>;
        using C3 = std::integral_constant<int, 3>;
        if (ph == 0) {
          static_for<4>([&](auto I) {
            fa[I][0] = frag_imm(AKCc{}, C0{}, I, C0{}, ba);
            fa[I][1] = frag_imm(AKCc{}, C0{}, I, C1{}, ba);
          });
          static_for<2>([&](auto J) {
            fb[J][0] = frag_imm(BKCc{}, C2{}, J, C0{}, bb);
            fb[J][1] = frag_imm(BKCc{}, C2{}, J, C1{}, bb);
          });
        } else if (ph == 1) {
          static_for<2>([&](auto J) {
            fb[2 + J][0] = frag_imm(BKCc{}, C3{}, J, C0{}, bb);
            fb[2 + J][1] = frag_imm(BKCc{}, C3{}, J, C1{}, bb);
          });
        } else if (ph == 2) {
          static_for<4>([&](auto I) {
            fa[4 + I][0] = frag_imm(AKCc{}, C1{}, I, C0{}, ba);
            fa[4 + I][1] = frag_imm(AKCc{}, C1{}, I, C1{}, ba);
          });
        }
        // refills: the slot read in the previous phase (every wave's reads of
        // it completed before this phase's barrier) takes K-tile kt + 2
        if constexpr (MODE >= 2) {
          if (ph == 0) issue_half(kt + 1, 3);
        }
        if constexpr (MODE == 3) {
          if (ph == 1) {
            issue_half(kt + 2, 0);
            issue_half(kt + 2, 1);
          } else if (ph == 2) {
            issue_half(kt + 2, 2);
          }
        }
        if (ph < 3) {
          lgkm_wait<0>();
          if (ph == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) tie_all(fa[i]);
#pragma unroll
            for (int j = 0; j < 2; ++j) tie_all(fb[j]);
          } else if (ph == 1) {
#pragma unroll
            for (int j = 2; j < 4; ++j) tie_all(fb[j]);
          } else {
#pragma unroll
            for (int i = 4; i < 8; ++i) tie_all(fa[i]);
          }
        }
        const int i0 = (ph < 2) ? 0 : 4;
        const int j0 = (ph == 0 || ph == 3) ? 0 : 2;
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[i0 + i][j0 + j] = mfma16(fb[j0 + j][s2], fa[i0 + i][s2], acc[i0 + i][j0 + j]);
        __builtin_amdgcn_s_setprio(0);
        if (do_bsum && (ph == 0 || ph == 2)) bias_sum(ph);
      }
    };
    int kt = 0;
    for (; kt + 2 < nk; ++kt) kstep_deep(kt, std::integral_constant<int, 3>{});
    if (kt + 1 < nk) kstep_deep(kt++, std::integral_constant<int, 2>{});
    kstep_deep(kt, std::integral_constant<int, 1>{});
  }
  if (do_bsum) {  // lanes l, l+16, l+32, l+48 hold disjoint K subsets of row l&15
    bsum0 += __shfl_xor(bsum0, 16, 64);
    bsum0 += __shfl_xor(bsum0, 32, 64);
    bsum1 += __shfl_xor(bsum1, 16, 64);
    bsum1 += __shfl_xor(bsum1, 32, 64);
    if (lane < 16) {
      const int mA = m0 + wm * 128 + 16 * wn + lane, mB = mA + 64;
      if (mA < M) bias_out[mA] = alpha * bsum0 + (beta != 0.f ? beta * bias_out[mA] : 0.f);
      if (mB < M) bias_out[mB] = alpha * bsum1 + (beta != 0.f ? beta * bias_out[mB] : 0.f);
    }
  }

  TDG_STAMP(2);
  // ---------------- epilogue: per-wave LDS image (EpiLds, tdg_gemm.h) over
  // the pipeline stages; the wave tile is rows wm*128.., columns wn*64..
  wait_vmcnt<0>();
  lds_barrier();
  {
    constexpr int RPASS = OUT_F32 ? 32 : 64;
    using Epi = EpiLds<EPI, OUT_F32, 8, 4, RPASS>;
    static_assert(8 * Epi::BYTES <= 2 * 4 * 128 * BK * 2, "epilogue images fit in the stages");
    Epi::run(smem + wid * Epi::BYTES, acc, lane, Cv, ldc, M, N, m0 + wm * 128, n0 + wn * 64, alpha,
             beta, bias, aux, ldaux, epi_vec_ok<EPI, OUT_F32>(Cv, ldc, aux, ldaux));
  }
#ifdef TDG_STAMPS
  TDG_STAMP(3);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  TDG_STAMP(4);
#endif
}

// ---------------------------------------------------------------------------
// Ragged weight-gradient launch on the software-pipelined main loop (Pipe,
// gemm_pipe.h) at ONE wave per SIMD: 256x256 tiles, 2 x 2 waves of 128 x 128
// (the 8 x 8 accumulator fragments live in AGPRs), 32-deep K tiles in an
// NS-slot LDS-DMA ring. Per FLOP a 128 x 128 wave tile reads 2/3 of the LDS
// fragment bytes of the lock-step kernel's 128 x 64, and nothing waits in
// bulk (fragment reads and DMA issue behind the MFMA rows). TN only (both
// operands token-major: dY^T, X), f32 out (alpha, beta), fused bias sums for
// the tiles of the first N-column (the wn == 0 waves sum their A fragments).
template <int NS>
__global__ __launch_bounds__(256) void wgrad_pipe_kernel(const R256Args args, int K, float alpha,
                                                         float beta) {
  constexpr int BM = 256, BN = 256, WM = 2, WN = 2;
  using P = Pipe<BM, BN, WM, WN, NS, false, false>;
  constexpr int TM = P::TM, TN = P::TN, A_BYTES = P::A_BYTES, PT = P::PT;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  static_assert(NS >= 3, "ring: refilled, being read, landed");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;

  const int t0 = xcd_remap(blockIdx.x, gridDim.x);
  R256Class cl = args.cls[0];
#pragma unroll
  for (int i = 1; i < R256_MAXC; ++i)
    if (i < args.ncls && t0 >= args.cls[i].tile_start) cl = args.cls[i];
  const int M = cl.M, N = cl.N, lda = cl.lda, ldb = cl.ldb, ldc = cl.ldc;
  const int tpp = cl.tiles_m * cl.tiles_n;
  const int lt = t0 - cl.tile_start + cl.t_first;
  const int p = cl.prob_start + lt / tpp;
  const int t = lt % tpp;
  int tm, tn;
  if (cl.tiles_n <= cl.tiles_m) {
    tn = t % cl.tiles_n;
    tm = t / cl.tiles_n;
  } else {
    tm = t % cl.tiles_m;
    tn = t / cl.tiles_m;
  }
  float* __restrict__ bias_out = args.bias_out[p];
  const bool do_bs = bias_out != nullptr && tn == 0 && wn == 0;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = K / PK;

  typename P::SA sa;
  typename P::SBt sb;
  // byte extents of the MN-contiguous operands ([K][ld]) for the buffer resources
  sa.init(args.A[p], lda, M, m0, (int)(((long long)(K - 1) * lda + M) * 2), wid, lane);
  sb.init(args.B[p], ldb, N, n0, (int)(((long long)(K - 1) * ldb + N) * 2), wid, lane);
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bs[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) bs[i] = 0.f;

  const int abase = wm * WTM, bbase = wn * WTN;
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) P::stage(sa, sb, smem, s, wid);
  wait_tiles<PT, NS - 2>(min(NS - 1, nk) - 1);
  __builtin_amdgcn_s_barrier();
  typename P::FA fa[TM];
  typename P::FBt fb[TN], fbn[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    lgkm_wait<15 - P::FBt::NI>();
    fb[j].read(smem + A_BYTES, bbase + 16 * j, lane);
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    lgkm_wait<15 - P::FA::NI>();
    fa[i].read(smem, abase + 16 * i, lane);
  }
  if (NS - 1 < nk) P::stage(sa, sb, smem, NS - 1, wid);
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    P::template ktile_bs<true>(kt, nk, fb, fbn, fa, acc, sa, sb, smem, lane, wid, abase, bbase, bs, do_bs);
    P::template ktile_bs<true>(kt + 1, nk, fbn, fb, fa, acc, sa, sb, smem, lane, wid, abase, bbase, bs, do_bs);
  }
  if (kt < nk)
    P::template ktile_bs<true>(kt, nk, fb, fbn, fa, acc, sa, sb, smem, lane, wid, abase, bbase, bs, do_bs);

  if (do_bs) {  // lanes l, l+16, l+32, l+48 hold disjoint k subsets of row l & 15
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      float b = bs[i];
      b += __shfl_xor(b, 16, 64);
      b += __shfl_xor(b, 32, 64);
      const int m = m0 + abase + 16 * i + lane;
      if (lane < 16 && m < M) bias_out[m] = alpha * b + (beta != 0.f ? beta * bias_out[m] : 0.f);
    }
  }

  lgkm_wait<0>();
  wait_vmcnt<0>();
  lds_barrier();
  {
    using Epi = EpiLds<EPI_NONE, true, TM, TN, 32>;
    static_assert(4 * Epi::BYTES <= NS * P::SB, "epilogue images fit in the stages");
    void* Cv = args.C[p];
    Epi::run(smem + wid * Epi::BYTES, acc, lane, Cv, ldc, M, N, m0 + wm * WTM, n0 + wn * WTN, alpha,
             beta, nullptr, nullptr, 0, epi_vec_ok<EPI_NONE, true>(Cv, ldc, nullptr, 0));
  }
}

// Split-K reduction: C = sum_z slab[z] (+beta*C) with the epilogue.
template <int EPI, bool OUT_F32>
__global__ void splitk_reduce_kernel(const float* __restrict__ ws, void* __restrict__ Cv,
                                     const float* __restrict__ bias, const bf16_t* __restrict__ aux,
                                     int M, int N, int ldc, int ldaux, int splits,
                                     long long split_stride, float alpha, float beta) {
  const long long total = (long long)M * N;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int m = (int)(idx / N), n = (int)(idx % N);
    const size_t o = (size_t)m * ldc + n;
    float v = 0.f;
    for (int z = 0; z < splits; ++z) v += ws[(size_t)z * split_stride + o];
    v *= alpha;
    if constexpr (EPI == EPI_BIAS) v += bias[n];
    if constexpr (EPI == EPI_BIAS_RELU) v = fmaxf(v + bias[n], 0.f);
    if constexpr (EPI == EPI_DRELU) {
      if (!(bf2f(aux[(size_t)m * ldaux + n]) > 0.f)) v = 0.f;
    }
    if constexpr (OUT_F32) {
      float* C = reinterpret_cast<float*>(Cv);
      if (beta != 0.f) v += beta * C[o];
      C[o] = v;
    } else {
      bf16_t* C = reinterpret_cast<bf16_t*>(Cv);
      if (beta != 0.f) v += beta * bf2f(C[o]);
      C[o] = f2bf(v);
    }
  }
}

}  // namespace tdg

// ============================================================================ host
using namespace tdg;

namespace {

template <int BM, int BN, int WM, int WN, int ST, bool AK, bool BKc, int EPI, bool F32>
void launch_cfg(const bf16_t* A, const bf16_t* B, void* C, const float* bias, const bf16_t* aux,
                int M, int N, int K, int lda, int ldb, int ldc, int ldaux, float alpha, float beta,
                int splits, float* ws, hipStream_t st, const GemmGroup* grp = nullptr, int G = 1) {
  static const GemmGroup kNoGroup{};
  const GemmGroup& gr = grp ? *grp : kNoGroup;
  const int tiles = cdiv(M, BM) * cdiv(N, BN);
  const int lds = ST * (BM + BN) * BK * 2;  // pipeline stages only (register epilogue)
  static bool attr_set = false;  // >64 KiB dynamic LDS needs the opt-in
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_kernel<BM, BN, WM, WN, ST, AK, BKc, EPI, F32>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)gemm_kernel<BM, BN, WM, WN, ST, AK, BKc, EPI_NONE, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  if (splits <= 1 || G > 1) {
    hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, ST, AK, BKc, EPI, F32>), dim3(tiles, G, 1),
                       dim3(WM * WN * 64), lds, st, A, B, C, bias, aux, M, N, K, lda, ldb, ldc,
                       ldaux, alpha, beta, K, 0LL, gr);
  } else {
    int kps = cdiv(cdiv(K, splits), BK) * BK;
    splits = cdiv(K, kps);
    const long long stride = (long long)M * ldc;
    hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, ST, AK, BKc, EPI_NONE, true>),
                       dim3(tiles, 1, splits), dim3(WM * WN * 64), lds, st, A, B, (void*)ws, bias,
                       aux, M, N, K, lda, ldb, ldc, ldaux, 1.f, 0.f, kps, stride, gr);
    const long long total = (long long)M * N;
    const int blocks = (int)std::min<long long>(4096, (total + 255) / 256);
    hipLaunchKernelGGL((splitk_reduce_kernel<EPI, F32>), dim3(blocks), dim3(256), 0, st, ws, C,
                       bias, aux, M, N, ldc, ldaux, splits, stride, alpha, beta);
  }
}

// Which (layout, epilogue) combinations have a 256x256 instantiation:
// forward NT (plain / bias / bias+relu; relu-backward for dgrads against a
// transposed weight copy), dgrad NN (plain / relu-backward), wgrad TN (f32 or
// bf16 out).
template <bool AK, bool BKc, int EPI, bool F32>
constexpr bool has_256() {
  if (AK && BKc) return !F32 || EPI == EPI_NONE;
  if (AK && !BKc) return !F32 && (EPI == EPI_NONE || EPI == EPI_DRELU);
  if (!AK && !BKc) return EPI == EPI_NONE;
  return false;
}

// gemm256_kernel addresses its operands through buffer resources (32-bit
// byte offsets): every class's operand extents must stay below 2^31 bytes
inline bool r256_offsets_ok(const R256Args& a, bool akc, bool bkc, int K) {
  for (int c = 0; c < a.ncls; ++c) {
    const R256Class& k = a.cls[c];
    const long long ea = akc ? (long long)(k.M - 1) * k.lda + K : (long long)(K - 1) * k.lda + k.M;
    const long long eb = bkc ? (long long)(k.N - 1) * k.ldb + K : (long long)(K - 1) * k.ldb + k.N;
    if (ea * 2 >= 0x7fffffffLL || eb * 2 >= 0x7fffffffLL) return false;
  }
  return true;
}

template <bool AK, bool BKc, int EPI, bool F32>
int launch_256(const R256Args& args, int tiles, const float* bias, const bf16_t* aux, int K,
               int ldaux, float alpha, float beta, hipStream_t st) {
  if constexpr (!has_256<AK, BKc, EPI, F32>()) {
    return -4;
  } else {
    if (K % BK != 0 || tiles <= 0) return -3;
    if (!r256_offsets_ok(args, AK, BKc, K)) return -9;
    constexpr int lds = 2 * 4 * 128 * BK * 2;  // 128 KiB: 2 stages x 4 half-tiles
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)gemm256_kernel<AK, BKc, EPI, F32>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr = true;
    }
    hipLaunchKernelGGL((gemm256_kernel<AK, BKc, EPI, F32>), dim3(tiles), dim3(512), lds, st, args,
                       bias, aux, K, ldaux, alpha, beta);
    return 0;
  }
}

// Ragged TN weight gradients on the one-wave-per-SIMD pipelined loop (f32 out).
template <int NS>
int launch_wgrad_pipe(const R256Args& args, int tiles, int K, float alpha, float beta,
                      hipStream_t st) {
  if (K % PK != 0 || K <= 0 || tiles <= 0) return -3;
  for (int c = 0; c < args.ncls; ++c) {
    const R256Class& cl = args.cls[c];
    if (cl.lda % 8 || cl.ldb % 8) return -6;
    if (((long long)(K - 1) * cl.lda + cl.M) * 2 >= 0x7fffffffLL ||
        ((long long)(K - 1) * cl.ldb + cl.N) * 2 >= 0x7fffffffLL)
      return -9;
  }
  constexpr int lds = NS * (256 + 256) * PK * 2;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)wgrad_pipe_kernel<NS>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((wgrad_pipe_kernel<NS>), dim3(tiles), dim3(256), lds, st, args, K, alpha, beta);
  return 0;
}

// One shape class of G problems (G == 1: a plain GEMM). Returns the tile count.
inline int r256_single(R256Args& a, const bf16_t* const* A, const bf16_t* const* B,
                       void* const* C, int G, int M, int N, int lda, int ldb, int ldc) {
  a.ncls = 1;
  for (int i = 0; i < G; ++i) {
    a.A[i] = A[i];
    a.B[i] = B[i];
    a.C[i] = C[i];
  }
  R256Class& c = a.cls[0];
  c.M = M; c.N = N; c.lda = lda; c.ldb = ldb; c.ldc = ldc;
  c.tiles_m = cdiv(M, 256); c.tiles_n = cdiv(N, 256);
  c.tile_start = 0; c.prob_start = 0; c.t_first = 0;
  return G * c.tiles_m * c.tiles_n;
}

// Pipelined kernel (gemm_pipe.h): single problem, K % 32 == 0, operands
// addressable with 31-bit byte offsets. Returns false if not applicable.
template <int BM, int BN, int WM, int WN, int NS, bool AK, bool BKc, int EPI, bool F32>
bool launch_pipe(const bf16_t* A, const bf16_t* B, void* C, const float* bias, const bf16_t* aux,
                 int M, int N, int K, int lda, int ldb, int ldc, int ldaux, float alpha, float beta,
                 hipStream_t st) {
  if (K % PK != 0 || K <= 0) return false;
  const long long ab = AK ? (long long)(M - 1) * lda + K : (long long)(K - 1) * lda + M;
  const long long bb = BKc ? (long long)(N - 1) * ldb + K : (long long)(K - 1) * ldb + N;
  if (ab * 2 >= 0x7fffffffLL || bb * 2 >= 0x7fffffffLL) return false;
  if ((!AK && lda % 8) || (!BKc && ldb % 8)) return false;
  constexpr int lds = NS * (BM + BN) * PK * 2;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_pipe_kernel<BM, BN, WM, WN, NS, AK, BKc, EPI, F32>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const int tiles = cdiv(M, BM) * cdiv(N, BN);
  hipLaunchKernelGGL((gemm_pipe_kernel<BM, BN, WM, WN, NS, AK, BKc, EPI, F32>), dim3(tiles),
                     dim3(WM * WN * 64), lds,
                     st, A, B, C, bias, aux, M, N, K, lda, ldb, ldc, ldaux, alpha, beta,
                     (int)(ab * 2), (int)(bb * 2));
  return true;
}

template <bool AK, bool BKc, int EPI, bool F32>
void launch_tiles(int tile_cfg, const bf16_t* A, const bf16_t* B, void* C, const float* bias,
                  const bf16_t* aux, int M, int N, int K, int lda, int ldb, int ldc, int ldaux,
                  float alpha, float beta, int splits, float* ws, hipStream_t st,
                  const GemmGroup* grp = nullptr, int G = 1) {
  if (tile_cfg >= 20 && tile_cfg <= 26) {
    // software-pipelined kernel (one problem, no split-K); else cfg 0
    if (!grp && splits <= 1) {
      bool ok = false;
#define TDG_PIPE(ID, BM_, BN_, WM_, WN_, NS_)                                                      \
  case ID:                                                                                    \
    ok = launch_pipe<BM_, BN_, WM_, WN_, NS_, AK, BKc, EPI, F32>(A, B, C, bias, aux, M, N, K, lda, \
                                                                 ldb, ldc, ldaux, alpha, beta, st); \
    break;
      switch (tile_cfg) {
        TDG_PIPE(20, 256, 256, 2, 4, 4)
        TDG_PIPE(21, 256, 128, 2, 4, 6)
        TDG_PIPE(22, 128, 256, 2, 4, 6)
        // one wave per SIMD, 128x128 per wave (accumulators beyond 256 VGPRs)
        TDG_PIPE(23, 256, 256, 2, 2, 4)
        TDG_PIPE(24, 256, 256, 2, 2, 5)
        TDG_PIPE(25, 256, 128, 2, 2, 6)
        TDG_PIPE(26, 128, 256, 2, 2, 6)
        default: break;
      }
#undef TDG_PIPE
      if (ok) return;
    }
    // not applicable (K % 32, split-K, grouped): the deep-pipelined 8-wave
    // 128x128 tile, which takes K tails -- cfg 0 ran the big vocab dgrad (K =
    // 7010) at 0.6 PF/s
    tile_cfg = 13;
  }
  if (tile_cfg == 12) {
    // 256x256 tiles (K % 64 == 0, no split-K; MN-contiguous operands need
    // ld % 8 == 0); otherwise cfg 0
    if (splits <= 1 && (AK || lda % 8 == 0) && (BKc || ldb % 8 == 0)) {
      R256Args args{};
      const bf16_t* a1 = A;
      const bf16_t* b1 = B;
      void* c1 = C;
      const int tiles = grp ? r256_single(args, grp->A, grp->B, grp->C, G, M, N, lda, ldb, ldc)
                            : r256_single(args, &a1, &b1, &c1, 1, M, N, lda, ldb, ldc);
      if (launch_256<AK, BKc, EPI, F32>(args, tiles, bias, aux, K, ldaux, alpha, beta, st) == 0)
        return;
    }
    tile_cfg = 13;
  }
#define TDG_CFG(ID, BM_, BN_, WM_, WN_, ST_)                                                  \
  case ID:                                                                                    \
    launch_cfg<BM_, BN_, WM_, WN_, ST_, AK, BKc, EPI, F32>(A, B, C, bias, aux, M, N, K, lda, ldb, \
                                                          ldc, ldaux, alpha, beta, splits, ws,   \
                                                          st, grp, G);                           \
    break;
  // Tile table (BM, BN, waves M x N, pipeline stages). LDS = ST*(BM+BN)*128 B;
  // the table keeps >= 2 waves per SIMD resident (1 is latency-bound).
  switch (tile_cfg) {
    TDG_CFG(0, 128, 128, 2, 2, 2)
    TDG_CFG(1, 128, 64, 2, 2, 3)
    TDG_CFG(2, 64, 128, 2, 2, 3)
    TDG_CFG(3, 64, 64, 2, 2, 4)
    TDG_CFG(4, 128, 128, 2, 4, 3)
    TDG_CFG(5, 256, 128, 4, 2, 2)
    TDG_CFG(6, 128, 256, 2, 4, 2)
    TDG_CFG(7, 64, 128, 2, 2, 2)
    TDG_CFG(9, 256, 128, 4, 2, 3)
    TDG_CFG(10, 128, 256, 2, 4, 3)
    TDG_CFG(11, 128, 128, 2, 2, 4)
    // deeper pipelines for the latency-bound one-tile-per-CU shapes (8 waves)
    TDG_CFG(13, 128, 128, 2, 4, 4)
    TDG_CFG(14, 128, 128, 2, 4, 5)
    default:
      TDG_CFG(8, 64, 64, 2, 2, 2)
  }
#undef TDG_CFG
}

template <bool AK, bool BKc>
int dispatch_epi(int epi, bool f32, int tile_cfg, const bf16_t* A, const bf16_t* B, void* C,
                 const float* bias, const bf16_t* aux, int M, int N, int K, int lda, int ldb,
                 int ldc, int ldaux, float alpha, float beta, int splits, float* ws,
                 hipStream_t st) {
#define TDG_E(E, F)                                                                              \
  if (epi == E && f32 == F) {                                                                    \
    launch_tiles<AK, BKc, E, F>(tile_cfg, A, B, C, bias, aux, M, N, K, lda, ldb, ldc, ldaux,     \
                                alpha, beta, splits, ws, st);                                    \
    return 0;                                                                                    \
  }
  TDG_E(EPI_NONE, false)
  TDG_E(EPI_NONE, true)
  TDG_E(EPI_BIAS, false)
  TDG_E(EPI_BIAS, true)
  TDG_E(EPI_BIAS_RELU, false)
  TDG_E(EPI_DRELU, false)
#undef TDG_E
  return -1;
}

}  // namespace

// Per-layout entry points: each operand layout's instantiations are
// compiled in a translation unit of their own (gemm_<layout>.hip), so the
// build runs them in parallel.
#define TDG_GEMM_LAYOUT(NAME, AK, BKc)                                                          \
  namespace tdg {                                                                               \
  int gemm_##NAME(int epi, bool f32, int tile_cfg, const bf16_t* A, const bf16_t* B, void* C,    \
                  const float* bias, const bf16_t* aux, int M, int N, int K, int lda, int ldb,     \
                  int ldc, int ldaux, float alpha, float beta, int splits, float* ws,              \
                  hipStream_t st) {                                                              \
    return dispatch_epi<AK, BKc>(epi, f32, tile_cfg, A, B, C, bias, aux, M, N, K, lda, ldb, ldc,  \
                                 ldaux, alpha, beta, splits, ws, st);                             \
  }                                                                                             \
  int gemm_grouped_##NAME(const GemmGroup& g, int G, int M, int N, int K, int lda, int ldb,       \
                          int ldc, bool f32, float alpha, float beta, int tile_cfg,              \
                          hipStream_t st) {                                                      \
    if (f32)                                                                                    \
      launch_tiles<AK, BKc, EPI_NONE, true>(tile_cfg, g.A[0], g.B[0], g.C[0], nullptr, nullptr,  \
                                            M, N, K, lda, ldb, ldc, 0, alpha, beta, 1, nullptr,  \
                                            st, &g, G);                                           \
    else                                                                                        \
      launch_tiles<AK, BKc, EPI_NONE, false>(tile_cfg, g.A[0], g.B[0], g.C[0], nullptr, nullptr, \
                                             M, N, K, lda, ldb, ldc, 0, alpha, beta, 1, nullptr, \
                                             st, &g, G);                                          \
    return 0;                                                                                   \
  }                                                                                             \
  int gemm_ragged_##NAME(const R256Args& args, int tiles, int K, bool f32, float alpha,         \
                         float beta, int impl, hipStream_t st) {                                \
    if constexpr (!AK && !BKc) {                                                                \
      if (f32 && impl == 1) return launch_wgrad_pipe<4>(args, tiles, K, alpha, beta, st);       \
      if (f32 && impl == 2) return launch_wgrad_pipe<5>(args, tiles, K, alpha, beta, st);       \
    }                                                                                           \
    if (f32)                                                                                    \
      return launch_256<AK, BKc, EPI_NONE, true>(args, tiles, nullptr, nullptr, K, 0, alpha, beta, \
                                                st);                                             \
    return launch_256<AK, BKc, EPI_NONE, false>(args, tiles, nullptr, nullptr, K, 0, alpha, beta,  \
                                                st);                                             \
  }                                                                                             \
  }
