// Software-pipelined MFMA GEMM main loop (tile configs 20-22, gemm_impl.h).
//
// Why a second main loop: measured with csrc/lab/stream_lab.cpp
// (profiles/gemm/r3_stream_lab_work_modes_clock.txt), the LDS-DMA operand
// stream of a 128x128-tile GEMM alone moves 83-85 GB/s per CU, but with the
// MFMAs OR the fragment reads of the k-step added in the lock-step form of
// the older kernels (barrier -> reads -> wait -> MFMAs) it drops by ~25 %,
// with both by ~70 % -- at an unchanged clock, also from L2-resident operands:
// the phases of a K tile serialise. Here nothing waits in bulk:
//   * fragment reads are untracked inline asm with counted lgkmcnt waits
//     (PFrag): the compiler would otherwise drain the LDS-DMA ring before
//     every read;
//   * K tiles are 32 deep (one MFMA k-step) in an NS-slot LDS ring, NS-2 .. NS-1
//     tiles in flight, one barrier per K tile and no LDS drain at it (the
//     slot refilled in iteration kt is tile kt-1's, whose reads every wave has
//     consumed -- waited for -- before the barrier);
//   * the MFMAs of tile kt are issued per A fragment row i (TN MFMAs each);
//     behind each row the wave requests that row's fragment of tile kt+1
//     into the same registers (the B fragments of kt+1 are double-buffered)
//     and, spread over the rows, its share of tile kt+NS-1's LDS-DMA pieces,
//     so LDS reads, DMA issue and address arithmetic all run in the MFMA
//     shadow (each MFMA row waits only for its own fragment);
//   * the DMA goes through buffer_load ... lds with per-lane byte offsets
//     computed once and a scalar per-K-tile offset (no per-issue VALU).
// WM x WN waves: 2 x 4 for tiles 256x256 (wave tile 128x64), 256x128
// (128x32), 128x256 (64x64). Measured and not kept
// (profiles/gemm/r3s2_pipe_wave_layouts.txt): 128x128 with 2 x 4 waves, and
// 2 x 2 waves (one per SIMD, fewer LDS fragment bytes per FLOP) at 128x128 /
// 256x128 -- all slower than the lock-step 128x128 kernels at N = 512. Same operand layouts (K- or MN-contiguous,
// XOR-swizzled images, conflict-free fragment reads) and the same epilogue
// (EpiLds) as the other kernels. K % 32 == 0; one problem per launch.
#pragma once
#include "tdg_common.h"
#include "tdg_gemm.h"

namespace tdg {

constexpr int PK = 32;  // K-tile depth of the pipelined kernel

// Byte offset of (row, byte) in a PK-deep tile image.
//  KC: [R rows][32 k] -> 64-B rows; 16-B chunk ^= ((row >> 3) & 1) << 1
//      (every ds_read_b128 lane group of a 16-row fragment read then covers
//      all 16 bank slots: found by exhaustive search over row-bit XORs)
//  MC: [32 k rows][R]: the 32-B segment swizzle of the BK = 64 images
//      (lds_off<false, R>), rows are k.
template <bool KC, int R>
__device__ __forceinline__ int plds_off(int row, int byte) {
  if constexpr (KC) {
    const int ch = (byte >> 4) ^ (((row >> 3) & 1) << 1);
    return row * 64 + (ch << 4) + (byte & 15);
  } else {
    return lds_off<false, R>(row, byte);
  }
}

// LDS-DMA staging of one PK-deep operand tile through a buffer resource:
// per lane and piece a byte offset fixed for the whole K loop (rows /
// columns clamped to the operand), per K tile one scalar offset.
template <bool KC, int R, int NW>
struct PStage {
  static constexpr int BYTES = R * PK * 2;
  static constexpr int P = BYTES / (NW * 1024);  // pieces per wave per tile
  static_assert(BYTES % (NW * 1024) == 0, "tile must split into 1 KiB pieces per wave");
  // (the buffer descriptor is rebuilt per issue from uniform values: the
  // compiler hoists it, and the struct stays host-compilable)
  uint32_t voff[P];
  const bf16_t* base;
  int nrec;
  uint32_t kstep;  // bytes per K tile
  // X: operand base; ld in elements; len = rows (KC) / columns (MC) valid
  __device__ __forceinline__ void init(const bf16_t* X, int ld, int len, int mn0, int nrec_bytes,
                                       int wid, int lane) {
    base = X;
    nrec = nrec_bytes;
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const int piece = wid * P + i;
      if constexpr (KC) {
        const int r = piece * 16 + (lane >> 2);
        const int c = (lane & 3) ^ (((r >> 3) & 1) << 1);
        int mn = mn0 + r;
        mn = mn < len ? mn : len - 1;
        voff[i] = (uint32_t)(((long long)mn * ld + c * 8) * 2);
      } else {
        constexpr int RPP = 1024 / (R * 2);  // k rows per piece
        constexpr int CPR = R / 8;           // 16-B chunks per row
        const int r = piece * RPP + lane / CPR;
        const int pc = lane % CPR;
        const int c = (((pc >> 1) ^ ((r & 3) | (((r >> 3) & 1) << 2))) << 1) | (pc & 1);
        int mn = mn0 + c * 8;
        mn = mn < len ? mn : 0;  // fully past len: never stored
        voff[i] = (uint32_t)(((long long)r * ld + mn) * 2);
      }
    }
    kstep = KC ? PK * 2 : (uint32_t)PK * (uint32_t)ld * 2u;
  }
  __device__ __forceinline__ void issue(int i, int kt, char* lds, int wid) const {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(base), (short)0, nrec, 0x00020000), (__attribute__((address_space(3))) void*)(lds + (wid * P + i) * 1024), 16, voff[i],
        (int)(kstep * (uint32_t)kt), 0, 0);
  }
};

// MFMA operand fragment (16 rows / columns at `base`) of a PK-deep image:
// lane l holds X(base + (l & 15), 8 (l >> 4) + j), j < 8. UNTRACKED reads
// (inline asm, tdg_common.h): the compiler's waitcnt pass treats a plain LDS
// read as possibly aliasing every LDS-DMA in flight and puts an
// `s_waitcnt vmcnt(0)` in front of it, which drains the ring at every
// fragment read (the first version of this kernel did exactly that). The
// caller waits with a counted lgkmcnt and ties the registers before use.
template <bool KC, int R>
struct PFrag {
  static constexpr int NI = KC ? 1 : 2;  // LDS instructions per fragment
  short8_t v;       // KC
  short4_t lo, hi;  // MC (two transposing 8-byte reads)
  __device__ __forceinline__ void read(const char* lds, int base, int lane) {
    if constexpr (KC) {
      const int row = base + (lane & 15);
      v = lds_read_b128_async(lds + plds_off<true, R>(row, (lane >> 4) * 16));
    } else {
      const int g = lane >> 4, w = lane & 15, q = w >> 2, p = w & 3;
      const int krow = 8 * g + q;
      const int byte = (base + 4 * p) * 2;
      lo = lds_read_tr_async(lds + plds_off<false, R>(krow, byte));
      hi = lds_read_tr_async(lds + plds_off<false, R>(krow + 4, byte));
    }
  }
  __device__ __forceinline__ void tie_() {
    if constexpr (KC) {
      tie(v);
    } else {
      tie(lo);
      tie(hi);
    }
  }
  __device__ __forceinline__ short8_t get() const {
    if constexpr (KC) return v;
    else return cat4(lo, hi);
  }
};

// The K loop's pieces as static members of one class template (the pattern
// of EpiLds): clang's host pass failed substitution of free function templates
// taking the kernel's local operand-stage types for every kernel instantiation
// but the first, silently dropping those kernels' host handles.
template <int BM, int BN, int WM, int WN, int NS, bool A_KC, bool B_KC>
struct Pipe {
  static constexpr int NW = WM * WN;
  static constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);  // 16x16 fragments per wave
  static constexpr int A_BYTES = BM * PK * 2, SB = A_BYTES + BN * PK * 2;
  using SA = PStage<A_KC, BM, NW>;
  using SBt = PStage<B_KC, BN, NW>;
  static constexpr int PT = SA::P + SBt::P;  // LDS-DMA per wave per K tile

  // whole A+B tile kt into its ring slot (prologue), or piece q of this
  // wave's PT pieces (interleaved with the MFMAs)
  static __device__ __forceinline__ void stage(const SA& sa, const SBt& sb, char* smem, int kt,
                                               int wid) {
    char* st = smem + (kt % NS) * SB;
#pragma unroll
    for (int i = 0; i < SA::P; ++i) sa.issue(i, kt, st, wid);
#pragma unroll
    for (int i = 0; i < SBt::P; ++i) sb.issue(i, kt, st + A_BYTES, wid);
  }
  static __device__ __forceinline__ void stage_piece(const SA& sa, const SBt& sb, char* smem, int q,
                                                     int kt, int wid) {
    char* st = smem + (kt % NS) * SB;
    if (q < SA::P) sa.issue(q, kt, st, wid);
    else sb.issue(q - SA::P, kt, st + A_BYTES, wid);
  }

  // One K tile: MFMAs of tile kt with tile kt+1's fragment reads and tile
  // kt+NS-1's DMA pieces behind the MFMA rows. FB: this tile's B fragments,
  // FN: receives the next tile's (named buffers: the caller unrolls by two so
  // every array index stays a compile-time constant).
  using FA = PFrag<A_KC, BM>;
  using FBt = PFrag<B_KC, BN>;
  // LDS instructions a wave has issued after its read of A fragment i of a
  // tile, by the time row i of that tile's MFMAs is reached: A fragments
  // i+1.. of the same tile, the next tile's B fragments, A fragments ..i-1 of
  // the next tile -- the same for every i
  static constexpr int LGKM = (TM - 1) * FA::NI + TN * FBt::NI;
  // The counter is 4 bits: with more than 15 LDS instructions in flight it
  // no longer counts them -- a later counted wait passes early, the compiler
  // reuses the destination registers, and the late data lands on top of
  // whatever they hold by then (measured: wrong fragments, and an illegal
  // address once an address register was hit). So every read first waits
  // for at most 15 - NI in flight (free in the steady state whenever
  // LGKM <= 15 - NI); with LGKM > 15 (MN-contiguous A at 256 rows) fa[i],
  // older than LGKM >= 16 reads, has landed by row i anyway.
  template <typename F>
  static __device__ __forceinline__ void throttle() {
    lgkm_wait<15 - F::NI>();
  }

  static __device__ __forceinline__ void ktile(int kt, int nk, FBt (&FB)[TN],
                                               FBt (&FN)[TN], FA (&fa)[TM],
                                               f32x4 (&acc)[TM][TN], const SA& sa, const SBt& sb,
                                               char* smem, int lane, int wid, int abase,
                                               int bbase) {
    float none[TM];
    ktile_bs<false>(kt, nk, FB, FN, fa, acc, sa, sb, smem, lane, wid, abase, bbase, none, false);
  }
  // steady-state tile (1 <= kt <= nk - NS: the next tile exists, a tile is
  // refilled, NS - 3 tiles stay in flight): no runtime tail tests in the
  // body (docs/PERF.md "Round 4": tail branches inside the loop body)
  static __device__ __forceinline__ void ktile_s(int kt, int nk, FBt (&FB)[TN],
                                                 FBt (&FN)[TN], FA (&fa)[TM],
                                                 f32x4 (&acc)[TM][TN], const SA& sa, const SBt& sb,
                                                 char* smem, int lane, int wid, int abase,
                                                 int bbase) {
    float none[TM];
    ktile_bs<false, true>(kt, nk, FB, FN, fa, acc, sa, sb, smem, lane, wid, abase, bbase, none,
                          false);
  }
  // BS: also accumulate the sums over k of the A fragments (bs[i]: row
  // abase + 16 i + (lane & 15), this lane's k subset) when do_bs -- the fused
  // bias gradient of a weight-gradient tile (A = dY^T), from registers the
  // MFMAs already hold
  template <bool BS, bool STEADY = false>
  static __device__ __forceinline__ void ktile_bs(int kt, int nk, FBt (&FB)[TN],
                                                  FBt (&FN)[TN], FA (&fa)[TM],
                                                  f32x4 (&acc)[TM][TN], const SA& sa,
                                                  const SBt& sb, char* smem, int lane, int wid,
                                                  int abase, int bbase, float (&bs)[TM],
                                                  bool do_bs) {
    if (STEADY || kt + 1 < nk) {
      // tile kt+1 landed (this wave's pieces), then everyone's; every wave
      // also finished reading tile kt-1, whose slot is refilled below.
      // In flight after kt+1: tiles up to kt+NS-2 (kt = 0: NS-1)
      if constexpr (STEADY) wait_vmcnt<(NS - 3) * PT>();
      else wait_tiles<PT, NS - 2>(kt == 0 ? min(NS - 2, nk - 2) : min(NS - 3, nk - 2 - kt));
      __builtin_amdgcn_s_barrier();
    }
    const char* nx = smem + ((kt + 1) % NS) * SB;
    const int rt = kt - 1 + NS;  // tile refilled into tile kt-1's slot
    const bool refill = STEADY || (rt < nk && kt >= 1);
    // (the next tile's fragments are read unconditionally -- after the last
    // tile from a stale slot, never used -- so the compiler's lgkmcnt
    // bookkeeping stays exact: no branch around an LDS read)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      throttle<FBt>();
      FN[j].read(nx + A_BYTES, bbase + 16 * j, lane);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      lgkm_wait<LGKM>();  // fa[i] of this tile (and this tile's B fragments)
      fa[i].tie_();
      if (i == 0) {
#pragma unroll
        for (int j = 0; j < TN; ++j) FB[j].tie_();
      }
      const short8_t a = fa[i].get();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(FB[j].get(), a, acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
      if constexpr (BS) {
        if (do_bs) {
          const bf16x2_t one = __builtin_bit_cast(bf16x2_t, 0x3f803f80);
          float b = bs[i];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            b = __builtin_amdgcn_fdot2_f32_bf16(
                __builtin_bit_cast(bf16x2_t, (short2_t){a[2 * e], a[2 * e + 1]}), one, b, false);
          bs[i] = b;
        }
      }
      throttle<FA>();
      fa[i].read(nx, abase + 16 * i, lane);
      // this wave's DMA pieces of tile rt, spread over the MFMA rows
#pragma unroll
      for (int q = 0; q < PT; ++q)
        if (q * TM / PT == i && refill) stage_piece(sa, sb, smem, q, rt, wid);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
};

template <int BM, int BN, int WM, int WN, int NS, bool A_KC, bool B_KC, int EPI, bool OUT_F32>
__global__ __launch_bounds__(WM * WN * 64) void gemm_pipe_kernel(
    const bf16_t* __restrict__ A, const bf16_t* __restrict__ B, void* __restrict__ Cv,
    const float* __restrict__ bias, const bf16_t* __restrict__ aux, int M, int N, int K, int lda,
    int ldb, int ldc, int ldaux, float alpha, float beta, int a_bytes, int b_bytes) {
  using P = Pipe<BM, BN, WM, WN, NS, A_KC, B_KC>;
  constexpr int NW = P::NW, TM = P::TM, TN = P::TN, A_BYTES = P::A_BYTES, SB = P::SB, PT = P::PT;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  static_assert(NS >= 3, "ring: refilled, being read, landed");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_m = cdiv(M, BM), tiles_n = cdiv(N, BN);
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  int tm, tn;
  if (tiles_n <= tiles_m) {
    tn = t % tiles_n;
    tm = t / tiles_n;
  } else {
    tm = t % tiles_m;
    tn = t / tiles_m;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = K / PK;

  typename P::SA sa;
  typename P::SBt sb;
  sa.init(A, lda, M, m0, a_bytes, wid, lane);
  sb.init(B, ldb, N, n0, b_bytes, wid, lane);
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int abase = wm * WTM, bbase = wn * WTN;
  // prologue: NS-1 tiles in flight, tile 0 landed, its fragments requested
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) P::stage(sa, sb, smem, s, wid);
  wait_tiles<PT, NS - 2>(min(NS - 1, nk) - 1);
  __builtin_amdgcn_s_barrier();
  typename P::FA fa[TM];
  typename P::FBt fb[TN], fbn[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    lgkm_wait<15 - P::FBt::NI>();  // (prologue: at most 15 LDS reads in flight)
    fb[j].read(smem + A_BYTES, bbase + 16 * j, lane);
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    lgkm_wait<15 - P::FA::NI>();
    fa[i].read(smem, abase + 16 * i, lane);
  }

  // kt = 0 refills nothing (tile NS-1's slot was never used): issue it now
  if (NS - 1 < nk) P::stage(sa, sb, smem, NS - 1, wid);
  // tile 0, then steady-state pairs (odd kt: B fragments in fbn), then the
  // tail tiles with their runtime tests
  int kt = 0;
  if (nk > 0) P::ktile(kt++, nk, fb, fbn, fa, acc, sa, sb, smem, lane, wid, abase, bbase);
  for (; kt + 1 <= nk - NS; kt += 2) {
    P::ktile_s(kt, nk, fbn, fb, fa, acc, sa, sb, smem, lane, wid, abase, bbase);
    P::ktile_s(kt + 1, nk, fb, fbn, fa, acc, sa, sb, smem, lane, wid, abase, bbase);
  }
  for (; kt + 1 < nk; kt += 2) {
    P::ktile(kt, nk, fbn, fb, fa, acc, sa, sb, smem, lane, wid, abase, bbase);
    P::ktile(kt + 1, nk, fb, fbn, fa, acc, sa, sb, smem, lane, wid, abase, bbase);
  }
  if (kt < nk) P::ktile(kt, nk, fbn, fb, fa, acc, sa, sb, smem, lane, wid, abase, bbase);

  // ---------------- epilogue: per-wave LDS image over the pipeline stages
  // (the last tile's next-fragment reads, from a stale slot, are drained here)
  lgkm_wait<0>();
  wait_vmcnt<0>();
  lds_barrier();
  {
    using OutT = typename std::conditional<OUT_F32, float, bf16_t>::type;
    (void)sizeof(OutT);
    constexpr int RPASS = OUT_F32 ? (WTM < 32 ? WTM : 32) : (WTM > 64 ? 64 : WTM);
    using Epi = EpiLds<EPI, OUT_F32, TM, TN, RPASS>;
    static_assert(NW * Epi::BYTES <= NS * SB, "epilogue images fit in the stages");
    Epi::run(smem + wid * Epi::BYTES, acc, lane, Cv, ldc, M, N, m0 + wm * WTM, n0 + wn * WTN, alpha,
             beta, bias, aux, ldaux, epi_vec_ok<EPI, OUT_F32>(Cv, ldc, aux, ldaux));
  }
}

}  // namespace tdg
