// Shared pieces of the MFMA GEMM kernels (gemm.hip, fp8.hip): LDS tile
// image layout (XOR-swizzled), the LDS-DMA operand stager, counted waits and
// MFMA fragment reads.
#pragma once
#include "tdg_common.h"

#include <type_traits>

namespace tdg {

constexpr int BK = 64;

// Byte offset inside an LDS tile image.
//  KC (K-contiguous): [R rows][BK] -> 128-B rows; 32-B segment ^= (row>>1)&3
//  MC (MN-contiguous): [BK rows][R] -> R*2-B rows
//     R=128 (256-B rows): seg ^= (row&3) | ((row>>3)&1)<<2
//     R=64  (128-B rows): seg ^= ((row>>1)&1) | ((row>>3)&1)<<1
template <bool KC, int R>
__device__ __forceinline__ int lds_off(int row, int byte) {
  if constexpr (KC) {
    const int seg = (byte >> 5) ^ ((row >> 1) & 3);
    return row * (BK * 2) + (seg << 5) + (byte & 31);
  } else if constexpr (R >= 128) {
    const int seg = (byte >> 5) ^ ((row & 3) | (((row >> 3) & 1) << 2));
    return row * (R * 2) + (seg << 5) + (byte & 31);
  } else {
    static_assert(R == 64, "MN-contiguous tiles must be 64 or 128 wide");
    const int seg = (byte >> 5) ^ (((row >> 1) & 1) | (((row >> 3) & 1) << 1));
    return row * 128 + (seg << 5) + (byte & 31);
  }
}

// Direct global->LDS staging (global_load_lds_dwordx4) of one operand tile.
// One wave instruction writes 1 KiB of LDS linearly (wave-uniform base +
// 16*lane), so the XOR swizzle of the image is applied to the per-lane SOURCE
// address: lane l fetches the logical 16-byte chunk that belongs at physical
// position l of the piece. Out-of-range rows/columns are clamped to valid
// addresses (their outputs are never stored); the K tail of the last tile is
// zeroed in LDS after it lands (zero_ktail).
template <bool KC, int R, int NW>
struct Glds {
  static constexpr int BYTES = R * BK * 2;
  static constexpr int P = BYTES / (NW * 1024);  // pieces per wave per tile
  static_assert(BYTES % (NW * 1024) == 0, "tile must split into 1 KiB pieces per wave");
  static constexpr int RPP = KC ? 8 : 1024 / (R * 2);  // tile rows per piece
  static constexpr int CPR = KC ? 8 : R / 8;           // 16-byte chunks per tile row
  // per piece: element offset of this lane's chunk relative to (mn0, k0)
  int row[P];   // KC: mn row within tile; MC: k row within tile
  int col[P];   // KC: k element offset (chunk*8); MC: mn element offset
  __device__ __forceinline__ void init(int wid, int lane) {
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const int j = wid * P + i;
      const int r = j * RPP + lane / CPR;
      const int pc = lane % CPR;
      int c;
      if constexpr (KC) {
        c = (((pc >> 1) ^ ((r >> 1) & 3)) << 1) | (pc & 1);
      } else if constexpr (R >= 128) {
        c = (((pc >> 1) ^ ((r & 3) | (((r >> 3) & 1) << 2))) << 1) | (pc & 1);
      } else {
        c = (((pc >> 1) ^ (((r >> 1) & 1) | (((r >> 3) & 1) << 1))) << 1) | (pc & 1);
      }
      row[i] = r;
      col[i] = c * 8;
    }
  }
  // Issue the tile at (mn0, k0). len = M or N; kend = K bound; ld elements.
  __device__ __forceinline__ void issue(const bf16_t* __restrict__ X, int ld, int len, int kend,
                                        int mn0, int k0, char* lds, int wid) const {
#pragma unroll
    for (int i = 0; i < P; ++i) {
      long long off;
      if constexpr (KC) {
        int mn = mn0 + row[i];
        mn = mn < len ? mn : len - 1;
        int k = k0 + col[i];
        k = k < kend ? k : 0;  // fully past K: any valid chunk (zeroed later)
        off = (long long)mn * ld + k;
      } else {
        int k = k0 + row[i];
        k = k < kend ? k : kend - 1;  // zeroed later
        int mn = mn0 + col[i];
        mn = mn < len ? mn : 0;  // fully past len: never stored
        off = (long long)k * ld + mn;
      }
      __builtin_amdgcn_global_load_lds(
          (const void*)(X + off),
          (__attribute__((address_space(3))) void*)(lds + (wid * P + i) * 1024), 16, 0, 0);
    }
  }
  // Zero the k >= kend part of the tile image at k0 (last, partial tile).
  __device__ __forceinline__ static void zero_ktail(char* lds, int k0, int kend, int tid, int nt) {
    if constexpr (KC) {
      for (int id = tid; id < R * 8; id += nt) {
        const int r = id >> 3, c = id & 7;
        const int kk = k0 + c * 8;
        if (kk + 8 <= kend) continue;
        short8_t* p = reinterpret_cast<short8_t*>(lds + lds_off<KC, R>(r, c * 16));
        short8_t v = *p;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (kk + e >= kend) v[e] = 0;
        *p = v;
      }
    } else {
      for (int id = tid; id < BK * (R / 8); id += nt) {
        const int r = id / (R / 8), c = id % (R / 8);
        if (k0 + r < kend) continue;
        *reinterpret_cast<short8_t*>(lds + lds_off<KC, R>(r, c * 16)) =
            short8_t{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
  }
};

// Epilogue stores write-through (sc1) by default: measured 8192x2048x512
// 25.1 -> 22.8 us, 8192x512x512 10.3 -> 10.0 us (csrc/lab/gemm_lab.cpp): the
// output lines are not left dirty in the XCD L2 for the kernel-end write-back,
// and the consumer kernel runs on other XCDs anyway.
#ifndef TDG_EPI_SC1
#define TDG_EPI_SC1 1
#endif
#ifndef TDG_GEMM_PRIO
#define TDG_GEMM_PRIO 1
#endif
__device__ __forceinline__ void prio_hi() {
  if (TDG_GEMM_PRIO) __builtin_amdgcn_s_setprio(1);
}
__device__ __forceinline__ void prio_lo() {
  if (TDG_GEMM_PRIO) __builtin_amdgcn_s_setprio(0);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// The same vmcnt wait as a builtin: unlike the asm form, the compiler's
// waitcnt pass sees it, so registers loaded from global memory before the N
// younger operations are known complete after it (no vmcnt(0) of its own
// before their first use, e.g. inside a loop that also has LDS-DMA in flight).
template <int N>
__device__ __forceinline__ void wait_vmcnt_known() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// vmcnt wait leaving `n` younger tiles (PT LDS-DMA each) in flight
template <int PT, int NMAX>
__device__ __forceinline__ void wait_tiles(int n) {
  static_assert(NMAX <= 6 && PT * NMAX <= 63, "vmcnt range");
  if (NMAX >= 6 && n >= 6) { wait_vmcnt<(NMAX >= 6 ? 6 * PT : 0)>(); return; }
  if (NMAX >= 5 && n >= 5) { wait_vmcnt<(NMAX >= 5 ? 5 * PT : 0)>(); return; }
  if (NMAX >= 4 && n >= 4) { wait_vmcnt<(NMAX >= 4 ? 4 * PT : 0)>(); return; }
  if (NMAX >= 3 && n >= 3) { wait_vmcnt<(NMAX >= 3 ? 3 * PT : 0)>(); return; }
  if (NMAX >= 2 && n >= 2) { wait_vmcnt<(NMAX >= 2 ? 2 * PT : 0)>(); return; }
  if (NMAX >= 1 && n >= 1) { wait_vmcnt<PT>(); return; }
  wait_vmcnt<0>();
}

// Workgroup barrier that does NOT drain in-flight LDS-DMA (no vmcnt(0)).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// MFMA operand fragment for 16 rows/cols starting at `base` within the tile,
// k-step s (32 deep). Lane l holds X(base + (l&15), 32s + 8(l>>4) + j), j<8.
template <bool KC, int R>
__device__ __forceinline__ short8_t frag(const char* lds, int base, int s, int lane) {
  if constexpr (KC) {
    const int row = base + (lane & 15);
    const int byte = (s * 4 + (lane >> 4)) * 16;
    return lds_read_b128_async(lds + lds_off<KC, R>(row, byte));
  } else {
    const int g = lane >> 4, w = lane & 15, q = w >> 2, p = w & 3;
    const int krow = s * 32 + 8 * g + q;
    const int byte = (base + 4 * p) * 2;
    const short4_t lo = lds_read_tr_async(lds + lds_off<KC, R>(krow, byte));
    const short4_t hi = lds_read_tr_async(lds + lds_off<KC, R>(krow + 4, byte));
    return cat4(lo, hi);
  }
}

// LDS instructions one frag<KC>() issues (MN-contiguous: two transposing reads)
template <bool KC>
constexpr int frag_ops() {
  return KC ? 1 : 2;
}

// ---------------------------------------------------------------- epilogue
// The GEMM kernels issue their MFMAs with the operands swapped
// (mfma16(b_frag, a_frag)), so every 16x16 accumulator holds the TRANSPOSED
// sub-tile: lane l has C[m = base_m + (l & 15)][n = base_n + 4 (l >> 4) + r],
// r = 0..3 -- four consecutive output columns of one row: one 8-byte (bf16)
// or 16-byte (f32) LDS write per sub-tile in the epilogue image (EpiLds
// below; the untransposed layout needed one 2-byte write per element), or --
// epi_store4, the simple fallback -- a direct store from registers.
enum Epi : int {
  EPI_NONE = 0,       // alpha*acc (+beta*C)
  EPI_BIAS = 1,       // alpha*acc + bias[n]
  EPI_BIAS_RELU = 2,  // relu(alpha*acc + bias[n])
  EPI_DRELU = 3,      // alpha*acc * (aux[m,n] > 0)      (ReLU backward fused in dgrad)
};

// 4 bias values of columns n..n+3 (clamped to N-1 past the edge).
template <int EPI>
__device__ __forceinline__ f32x4 load_bias4(const float* __restrict__ bias, int n, int N) {
  f32x4 b = {0.f, 0.f, 0.f, 0.f};
  if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU) {
    if (n + 4 <= N && (reinterpret_cast<uintptr_t>(bias + n) & 15) == 0) {
      b = *reinterpret_cast<const f32x4*>(bias + n);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) b[r] = bias[min(n + r, N - 1)];
    }
  }
  return b;
}

// Whether the 4-wide vector path is legal for this launch (alignment of C,
// its row stride and the ReLU-mask operand).
template <int EPI, bool OUT_F32>
__device__ __forceinline__ bool epi_vec_ok(const void* C, int ldc, const bf16_t* aux, int ldaux) {
  constexpr int ES = OUT_F32 ? 4 : 2;
  bool ok = (ldc % 4) == 0 && (reinterpret_cast<uintptr_t>(C) % (4 * ES)) == 0;
  if constexpr (EPI == EPI_DRELU) ok = ok && (ldaux % 4) == 0 && (reinterpret_cast<uintptr_t>(aux) & 7) == 0;
  return ok;
}

// Store C[m][n..n+3] = epilogue(alpha * a) (+ beta * C_old).
template <int EPI, bool OUT_F32>
__device__ __forceinline__ void epi_store4(void* __restrict__ Cv, int ldc, int M, int N, int m, int n,
                                           const f32x4& a, float alpha, float beta, const f32x4& bn,
                                           const bf16_t* __restrict__ aux, int ldaux, bool vec) {
  if (m >= M || n >= N) return;
  float v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    v[r] = alpha * a[r];
    if constexpr (EPI == EPI_BIAS) v[r] += bn[r];
    if constexpr (EPI == EPI_BIAS_RELU) v[r] = fmaxf(v[r] + bn[r], 0.f);
  }
  const size_t off = (size_t)m * ldc + n;
  if (vec && n + 4 <= N) {
    if constexpr (EPI == EPI_DRELU) {
      const short4_t x = *reinterpret_cast<const short4_t*>(aux + (size_t)m * ldaux + n);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (!(bf2f((bf16_t)x[r]) > 0.f)) v[r] = 0.f;
    }
    if constexpr (OUT_F32) {
      f32x4* cp = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(Cv) + off);
      f32x4 o = {v[0], v[1], v[2], v[3]};
      if (beta != 0.f) o += beta * *cp;
      *cp = o;
    } else {
      short4_t* cp = reinterpret_cast<short4_t*>(reinterpret_cast<bf16_t*>(Cv) + off);
      if (beta != 0.f) {
        const short4_t old = *cp;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += beta * bf2f((bf16_t)old[r]);
      }
      short4_t o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(v[r]);
      *cp = o;
    }
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (n + r >= N) break;
      float x = v[r];
      if constexpr (EPI == EPI_DRELU) {
        if (!(bf2f(aux[(size_t)m * ldaux + n + r]) > 0.f)) x = 0.f;
      }
      if constexpr (OUT_F32) {
        float* cp = reinterpret_cast<float*>(Cv) + off + r;
        if (beta != 0.f) x += beta * *cp;
        *cp = x;
      } else {
        bf16_t* cp = reinterpret_cast<bf16_t*>(Cv) + off + r;
        if (beta != 0.f) x += beta * bf2f(*cp);
        *cp = f2bf(x);
      }
    }
  }
}

// Epilogue through a per-wave LDS image (what the kernels use). The direct
// store above writes 16 rows x 8-16 bytes per wave instruction; measured on
// MI355X (csrc/lab/gemm_lab.cpp stamps) that store stream is issue-bound at
// ~20-35 GB/s per CU -- 3.7 us for a 256x256 bf16 tile. Here each lane's 4
// consecutive columns go to a padded row-major image as ONE 8-byte (bf16) or
// 16-byte (f32) LDS write, are read back as 16-byte row chunks, and leave as
// fully coalesced 16-byte stores (8 lanes per 128-byte row for bf16).
// RPASS rows of the wave tile per pass (the image is reused across passes);
// pre_aux / pre_c: optional epilogue operands prefetched in the chunk layout
// (one int4 per lane per chunk iteration), single-pass only.
template <int EPI, bool OUT_F32, int TM, int TN, int RPASS>
struct EpiLds {
  static constexpr int ES = OUT_F32 ? 4 : 2;
  static constexpr int SP = TN * 16 * ES + 16;  // padded image row (bytes)
  static constexpr int CPR = TN * 16 * ES / 16;  // 16-byte chunks per row
  static constexpr int EPC = 16 / ES;            // elements per chunk
  static constexpr int ITER = RPASS * CPR / 64;  // chunk iterations per lane per pass
  static constexpr int BYTES = RPASS * SP;       // image bytes per wave
  static_assert(RPASS % 16 == 0 && (TM * 16) % RPASS == 0, "passes of whole 16-row sub-tiles");
  static_assert((RPASS * CPR) % 64 == 0, "whole chunk iterations");

  // m_of / n_of: row / column of chunk iteration t (pass 0) -- for prefetch.
  __device__ static __forceinline__ int row_of(int lane, int t) { return (lane + 64 * t) / CPR; }
  __device__ static __forceinline__ int col_of(int lane, int t) { return ((lane + 64 * t) % CPR) * EPC; }

  __device__ static __forceinline__ void run(char* wimg, const f32x4 (&acc)[TM][TN], int lane,
                                             void* __restrict__ Cv, int ldc, int M, int N, int mw0,
                                             int nw0, float alpha, float beta,
                                             const float* __restrict__ bias,
                                             const bf16_t* __restrict__ aux, int ldaux, bool vec) {
    int4 none[ITER];
    run_pre<false>(wimg, acc, lane, Cv, ldc, M, N, mw0, nw0, alpha, beta, bias, aux, ldaux, vec,
                   none, false, none, false);
  }
  // With operands prefetched in the chunk layout (arrays indexed by constants
  // only after unrolling: no private-memory copies).
  template <bool PRE>
  __device__ static __forceinline__ void run_pre(char* wimg, const f32x4 (&acc)[TM][TN], int lane,
                                                 void* __restrict__ Cv, int ldc, int M, int N,
                                                 int mw0, int nw0, float alpha, float beta,
                                                 const float* __restrict__ bias,
                                                 const bf16_t* __restrict__ aux, int ldaux, bool vec,
                                                 const int4 (&pre_aux)[ITER], bool use_aux,
                                                 const int4 (&pre_c)[ITER], bool use_c) {
    const int g = lane >> 4, r16 = lane & 15;
    // 16-byte chunk path: C rows 16-byte aligned, the ReLU mask likewise
    bool vok = vec && ((ldc * ES) % 16) == 0 && (reinterpret_cast<uintptr_t>(Cv) & 15) == 0;
    if constexpr (EPI == EPI_DRELU)
      vok = vok && (ldaux % EPC) == 0 && (reinterpret_cast<uintptr_t>(aux) % (2 * EPC)) == 0;
#if TDG_EPI_SC1
    const WtBuf wt(Cv, ((size_t)(M - 1) * ldc + N) * ES);
#endif
    f32x4 bn[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) bn[j] = load_bias4<EPI>(bias, nw0 + 16 * j + 4 * g, N);
    using VecT = typename std::conditional<OUT_F32, f32x4, short8_t>::type;
    // Epilogue operands not prefetched by the caller (ReLU mask, beta * C_old)
    // are loaded per pass BEFORE the image is written, all ITER chunks in
    // flight at once. Loaded inside the store loop, each chunk's load sat
    // behind its own s_waitcnt vmcnt(0): ITER (8-16) serial memory round trips
    // per wave at the end of every tile (measured ISA of gemm256<NN, DRELU>).
    // Out-of-range chunks load the operand's first chunk instead (branch-free;
    // the value is never used).
    constexpr bool AUX8 = EPI == EPI_DRELU && EPC == 8;
    const bool loc_aux = AUX8 && !(PRE && use_aux) && vok;
    const bool loc_c = !(PRE && use_c) && beta != 0.f && vok;
#pragma unroll
    for (int p = 0; p < TM * 16 / RPASS; ++p) {
      int4 la[ITER], lc[ITER];
      if (loc_aux || loc_c) {
#pragma unroll
        for (int t = 0; t < ITER; ++t) {
          const int id = lane + 64 * t;
          const int m = mw0 + p * RPASS + id / CPR, n = nw0 + (id % CPR) * EPC;
          const bool in = m < M && n + EPC <= N;
          if (loc_aux) {
            const bf16_t* a = in ? aux + (size_t)m * ldaux + n : aux;
            la[t] = *reinterpret_cast<const int4*>(a);
          }
          if (loc_c) {
            const char* c = in ? reinterpret_cast<const char*>(Cv) + ((size_t)m * ldc + n) * ES
                               : reinterpret_cast<const char*>(Cv);
            lc[t] = *reinterpret_cast<const int4*>(c);
          }
        }
      }
      // 1) accumulators (alpha, bias, relu applied) -> image
#pragma unroll
      for (int ii = 0; ii < RPASS / 16; ++ii) {
        const int i = p * (RPASS / 16) + ii;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[r] = alpha * acc[i][j][r];
            if constexpr (EPI == EPI_BIAS) v[r] += bn[j][r];
            if constexpr (EPI == EPI_BIAS_RELU) v[r] = fmaxf(v[r] + bn[j][r], 0.f);
          }
          char* dst = wimg + (16 * ii + r16) * SP + (16 * j + 4 * g) * ES;
          if constexpr (OUT_F32) {
            *reinterpret_cast<f32x4*>(dst) = f32x4{v[0], v[1], v[2], v[3]};
          } else {
            short4_t w;
#pragma unroll
            for (int r = 0; r < 4; ++r) w[r] = (short)f2bf(v[r]);
            *reinterpret_cast<short4_t*>(dst) = w;
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-local image complete
      // 2) image -> 16-byte row chunks -> global
#pragma unroll
      for (int t = 0; t < ITER; ++t) {
        const int id = lane + 64 * t;
        const int row = id / CPR, ch = id % CPR;
        const int m = mw0 + p * RPASS + row;
        const int n = nw0 + ch * EPC;
        // vector types only (a reinterpret_cast of a local array would put
        // it in private memory)
        VecT vals = *reinterpret_cast<const VecT*>(wimg + row * SP + ch * 16);
        if (m >= M || n >= N) continue;
        char* cp = reinterpret_cast<char*>(Cv) + ((size_t)m * ldc + n) * ES;
        if (vok && n + EPC <= N) {
          if constexpr (EPI == EPI_DRELU) {
            if constexpr (EPC == 8) {
              // vok: either the caller prefetched the mask or la[] holds it
              const short8_t x = __builtin_bit_cast(short8_t, (PRE && use_aux) ? pre_aux[t] : la[t]);
#pragma unroll
              for (int e = 0; e < 8; ++e)
                if (!(bf2f((bf16_t)x[e]) > 0.f)) vals[e] = 0;
            } else {
              const short4_t x = *reinterpret_cast<const short4_t*>(aux + (size_t)m * ldaux + n);
#pragma unroll
              for (int e = 0; e < 4; ++e)
                if (!(bf2f((bf16_t)x[e]) > 0.f)) vals[e] = 0;
            }
          }
          if (beta != 0.f) {
            const VecT old = __builtin_bit_cast(VecT, (PRE && use_c) ? pre_c[t] : lc[t]);
            if constexpr (OUT_F32) {
              vals += beta * old;
            } else {
#pragma unroll
              for (int e = 0; e < 8; ++e)
                vals[e] = (short)f2bf(bf2f((bf16_t)vals[e]) + beta * bf2f((bf16_t)old[e]));
            }
          }
#if TDG_EPI_SC1
          // write-through (sc1): nothing left dirty in the XCD's L2 for the
          // end-of-kernel write-back
          wt.st16(cp, vals);
#else
          *reinterpret_cast<VecT*>(cp) = vals;
#endif
        } else {
#pragma unroll
          for (int e = 0; e < EPC; ++e) {
            if (n + e >= N) break;
            float v = OUT_F32 ? (float)vals[e] : bf2f((bf16_t)vals[e]);
            if constexpr (EPI == EPI_DRELU) {
              if (!(bf2f(aux[(size_t)m * ldaux + n + e]) > 0.f)) v = 0.f;
            }
            if constexpr (OUT_F32) {
              float* c = reinterpret_cast<float*>(cp) + e;
              if (beta != 0.f) v += beta * *c;
              *c = v;
            } else {
              bf16_t* c = reinterpret_cast<bf16_t*>(cp) + e;
              if (beta != 0.f) v += beta * bf2f(*c);
              *c = f2bf(v);
            }
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // image reads done before the next pass
    }
  }
};

// Fragments read with lds_read_tr_async are not tracked by the compiler:
// make every later use wait for them (see tdg_common.h).
template <int N>
__device__ __forceinline__ void tie_all(short8_t (&f)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) tie(f[i]);
}

}  // namespace tdg
