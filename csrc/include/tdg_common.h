// Common device helpers for the gfx950 (CDNA4 / MI355X) kernels.
//
// Everything here is written for 64-lane wavefronts, MFMA 16x16x32 bf16 matrix
// cores and the 64-bank LDS of gfx950. No portability layer: this is CDNA4 code.
#pragma once
#include <hip/hip_runtime.h>
#include <utility>
#include <stdint.h>

namespace tdg {

// Diagnostic build only (csrc/lab/*.cpp, -DTDG_STAMPS): wave 0 of every
// workgroup records s_memrealtime (100 MHz) at phase boundaries, one slot per
// lane (vector stores), so a single launch yields per-workgroup timelines.
#ifdef TDG_STAMPS
__device__ unsigned long long* tdg_stamps;
#define TDG_STAMP(i)                                                                      \
  do {                                                                                    \
    if (threadIdx.x < 64)                                                                 \
      tdg_stamps[(((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 512 + (i) * 64 + threadIdx.x] =                     \
          __builtin_amdgcn_s_memrealtime();                                               \
  } while (0)
#else
#define TDG_STAMP(i) \
  do {               \
  } while (0)
#endif

typedef uint16_t bf16_t;  // raw bf16 bits in memory

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4_t __attribute__((ext_vector_type(4)));
typedef short short8_t __attribute__((ext_vector_type(8)));
typedef short short2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

typedef __attribute__((address_space(3))) short4_t lds_short4;

constexpr int WAVE = 64;

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// Round-to-nearest-even f32 -> bf16 via the plain cast: hipcc -O3 emits the
// gfx950 v_cvt_pk_bf16_f32 for it (keeps NaN a NaN, pairs adjacent converts).
__device__ __forceinline__ bf16_t f2bf(float f) {
  return __builtin_bit_cast(bf16_t, (__bf16)f);
}

// Two floats -> one packed bf16 pair (lo = a) in ONE v_cvt_pk_bf16_f32; the
// `f2bf(a) | f2bf(b) << 16` form converts each alone and then shifts and ors
// (4 instructions per pair).
__device__ __forceinline__ uint32_t pack2bf(float a, float b) {
  const bf16x2_t v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

__host__ __device__ __forceinline__ int cdiv(int a, int b) { return (a + b - 1) / b; }

// ---------------------------------------------------------------- reductions
// Whole-wave sum / max without the LDS crossbar: DPP row rotations (by 8, 4,
// 2, 1 within each 16-lane row: pairs combine symmetrically, every lane of a
// row ends with the same value), then the GFX9 row broadcasts (row_bcast:15
// into rows 1 and 3, row_bcast:31 into rows 2 and 3) and lane 63 read out as
// a scalar -- the bitwise-same value in every lane. The __shfl_xor butterfly
// compiles to ds_bpermute_b32, whose lanes l and l + 32 hit the same LDS bank
// on every step (the LayerNorm backward's 14 % conflict cycles,
// profiles/r4/pmc_base_end_round4.txt).
// Every lane of the wave must be active.
template <int CTRL, int ROWS = 0xF, bool BC = true>
__device__ __forceinline__ float dpp_f(float v, float old = 0.f) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old),
                                                               __builtin_bit_cast(int, v), CTRL, ROWS,
                                                               0xF, BC));
}
__device__ __forceinline__ float lane63(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<0x128>(v);  // row_ror:8
  v += dpp_f<0x124>(v);  // row_ror:4
  v += dpp_f<0x122>(v);  // row_ror:2
  v += dpp_f<0x121>(v);  // row_ror:1
  v += dpp_f<0x142, 0xA, false>(v);  // row_bcast:15 -> rows 1, 3
  v += dpp_f<0x143, 0xC, false>(v);  // row_bcast:31 -> rows 2, 3
  return lane63(v);
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_f<0x128>(v, v));
  v = fmaxf(v, dpp_f<0x124>(v, v));
  v = fmaxf(v, dpp_f<0x122>(v, v));
  v = fmaxf(v, dpp_f<0x121>(v, v));
  v = fmaxf(v, dpp_f<0x142, 0xA, false>(v, v));
  v = fmaxf(v, dpp_f<0x143, 0xC, false>(v, v));
  return lane63(v);
}

// f32 max without the canonicalising v_max_f32 x, x that fmaxf puts in front
// of every operand the compiler cannot prove quiet (MFMA results, permlane
// outputs: two extra VALU per fmaxf in the softmax row max). Operands are
// never signalling NaNs here.
__device__ __forceinline__ float vmax(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// Per lane position, the four 16-lane rows combined (lanes l, l ^ 16, l ^ 32,
// l ^ 48: the xor-16 / xor-32 butterfly of __shfl_xor) on v_permlane16_swap /
// v_permlane32_swap -- VALU ops, no ds_bpermute round trip through the LDS
// crossbar. Each swap takes the value and a copy made by an asm move with an
// early-clobber output (a distinct register the compiler cannot fold back
// into the operand: a swap of one register with itself only rotates it).
// swap16: row pairs (0,1), (2,3) exchange -> op gives the xor-16 combine in
// every lane; swap32: halves exchange -> xor-32.
template <class Op>
__device__ __forceinline__ float rows_reduce(float v, Op op) {
  // (elements copied out before the bit casts: __builtin_bit_cast of a vector
  // element r[1] read element 0 -- the clang front end took the vector's
  // address; that, not the swap, was the earlier "miscompile")
  float t;
  asm("v_mov_b32 %0, %1" : "=&v"(t) : "v"(v));
  auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v),
                                            __builtin_bit_cast(unsigned, t), false, false);
  unsigned r0 = r[0], r1 = r[1];
  v = op(__builtin_bit_cast(float, r0), __builtin_bit_cast(float, r1));
  asm("v_mov_b32 %0, %1" : "=&v"(t) : "v"(v));
  r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v),
                                       __builtin_bit_cast(unsigned, t), false, false);
  r0 = r[0];
  r1 = r[1];
  return op(__builtin_bit_cast(float, r0), __builtin_bit_cast(float, r1));
}
__device__ __forceinline__ float rows_max(float v) {
  return rows_reduce(v, [](float a, float b) { return vmax(a, b); });
}
__device__ __forceinline__ float rows_sum(float v) {
  return rows_reduce(v, [](float a, float b) { return a + b; });
}

// ---------------------------------------------------------------- Philox4x32-10
// Counter-based RNG: dropout masks are a pure function of (seed, offset,
// element index) so backward regenerates them instead of storing them.
struct Philox {
  static __host__ __device__ __forceinline__ void round(uint32_t& c0, uint32_t& c1, uint32_t& c2,
                                                        uint32_t& c3, uint32_t k0, uint32_t k1) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0;
    const uint32_t h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
    const uint32_t n0 = h1 ^ c1 ^ k0;
    const uint32_t n2 = h0 ^ c3 ^ k1;
    c0 = n0; c1 = l1; c2 = n2; c3 = l0;
  }
  // Returns 4 uint32 random words for counter (idx_lo, idx_hi, off_lo, off_hi).
  static __host__ __device__ __forceinline__ void gen(uint64_t seed, uint64_t offset, uint64_t idx,
                                                      uint32_t out[4]) {
    uint32_t c0 = (uint32_t)idx, c1 = (uint32_t)(idx >> 32);
    uint32_t c2 = (uint32_t)offset, c3 = (uint32_t)(offset >> 32);
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      round(c0, c1, c2, c3, k0, k1);
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
  }
};

// Keep-mask for element `e` of a dropout site: one Philox call covers 8
// consecutive elements (block e/8); element e draws the 16-bit half (e % 2)
// of word (e % 8) / 2 and is kept iff it is >= thresh = rint(p * 2^16)
// (dropout_thresh; keep probability within 2^-17 of 1 - p). Half-word draws
// halve the generator work per element: at D = 1024 the mask's Philox rounds,
// not memory, bounded the LayerNorm kernels.
__host__ __device__ __forceinline__ uint32_t dropout_thresh(float p) {
  return (uint32_t)fminf(65536.f, rintf(p * 65536.f));
}
__device__ __forceinline__ uint32_t half_draw(const uint32_t r[4], int j) {  // j in [0, 8)
  return (r[j >> 1] >> (16 * (j & 1))) & 0xffffu;
}
__device__ __forceinline__ bool dropout_keep(uint64_t seed, uint64_t offset, uint64_t e,
                                             uint32_t thresh) {
  uint32_t r[4];
  Philox::gen(seed, offset, e >> 3, r);
  return half_draw(r, (int)(e & 7)) >= thresh;
}

// Dropout stream offset: a device-resident counter (advanced once per forward,
// so HIP-graph replays draw fresh masks) times 4096 dropout sites + site id.
__device__ __forceinline__ uint64_t rng_offset(const long long* ctr, uint64_t site) {
  return (ctr ? (uint64_t)ctr[0] * 4096ull : 0ull) + site;
}
__device__ __forceinline__ bool dropout_keep(uint64_t seed, const long long* ctr, uint64_t site,
                                             uint64_t e, uint32_t thresh) {
  return dropout_keep(seed, rng_offset(ctr, site), e, thresh);
}

// keep bits of the n (<= 8) consecutive elements e0.. (all in one 8-block:
// e0 % 8 + n <= 8), bit i = element e0 + i: one Philox call
template <int N>
__device__ __forceinline__ uint32_t dropout_keep_run(uint64_t seed, uint64_t offset, uint64_t e0,
                                                     uint32_t thresh) {
  uint32_t r[4];
  Philox::gen(seed, offset, e0 >> 3, r);
  const int j0 = (int)(e0 & 7);
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) m |= (half_draw(r, j0 + i) >= thresh ? 1u : 0u) << i;
  return m;
}

// ---------------------------------------------------------------- MFMA
__device__ __forceinline__ f32x4 mfma16(const short8_t& a, const short8_t& b, const f32x4& c) {
#ifdef TDG_ABLATE_MFMA  // lab-only ablation: operands consumed, no matrix work
  asm volatile("" ::"v"(a), "v"(b));
  return c;
#else
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
#endif
}

// ds_read_b64_tr_b16: per 16-lane group, reads 4 rows x 16 columns (16-bit) and
// delivers lane i column i (row q in element q). `p` is this lane's address:
// row (base + (lane&15)>>2), columns 4*(lane&3)..+3.
__device__ __forceinline__ short4_t lds_read_tr(const void* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(p));
}

// The same read as inline asm, for kernels that stage tiles with LDS-DMA
// (global_load_lds). The compiler's waitcnt pass treats the builtin above as
// possibly aliasing every in-flight LDS-DMA and puts an `s_waitcnt vmcnt(0)`
// in front of it -- which drains the DMA prefetch of the NEXT tile before the
// current one can be read (measured: the whole multi-stage pipeline collapses
// to one tile in flight). The asm form is invisible to that pass; in exchange
// the caller owns the wait: `lgkm_wait<N>()` then `tie()` on every fragment
// before its first use (the tie orders the consuming MFMAs after the wait).
__device__ __forceinline__ short4_t lds_read_tr_async(const void* p) {
  short4_t r;
  // low 32 bits of a generic pointer into LDS = the LDS byte address
  const uint32_t a = (uint32_t)(uintptr_t)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a) : "memory");
  return r;
}

// 16-byte LDS read, likewise untracked (a tracked read mixed into an untracked
// stream makes the pass fall back to lgkmcnt(0) at loop boundaries).
__device__ __forceinline__ short8_t lds_read_b128_async(const void* p) {
  short8_t r;
  const uint32_t a = (uint32_t)(uintptr_t)p;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a) : "memory");
  return r;
}

// 8-byte LDS reads, likewise untracked: plain and transposing-bytes (gfx950
// ds_read_b64_tr_b8: lanes 2r, 2r+1 of a 16-lane group pass the two 8-byte
// halves of row r of an 8-row x 16-byte block; lane i receives column i, one
// byte per row -- verified on the box, scripts/probes/fp8_attn_layout.hip)
__device__ __forceinline__ long lds_read_b64_async(const void* p) {
  long r;
  const uint32_t a = (uint32_t)(uintptr_t)p;
  asm volatile("ds_read_b64 %0, %1" : "=v"(r) : "v"(a) : "memory");
  return r;
}
// ... at a compile-time byte offset from a 32-bit LDS address (the DS
// instruction's 16-bit offset field: no v_add per read for the constant part
// of a fragment address)
template <int OFF>
__device__ __forceinline__ long lds_read_b64_at(uint32_t a) {
  static_assert(OFF >= 0 && OFF < 65536, "DS offset field");
  long r;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF) : "memory");
  return r;
}
// 8-byte LDS store at a compile-time offset, untracked like the reads above
// (a later lgkmcnt wait -- e.g. lds_barrier -- covers it)
template <int OFF>
__device__ __forceinline__ void lds_write_b64_at(uint32_t a, long v) {
  static_assert(OFF >= 0 && OFF < 65536, "DS offset field");
  asm volatile("ds_write_b64 %0, %1 offset:%2" ::"v"(a), "v"(v), "i"(OFF) : "memory");
}
template <int OFF>
__device__ __forceinline__ long lds_read_tr8_at(uint32_t a) {
  static_assert(OFF >= 0 && OFF < 65536, "DS offset field");
  long r;
  asm volatile("ds_read_b64_tr_b8 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF) : "memory");
  return r;
}
template <int OFF>
__device__ __forceinline__ short8_t lds_read_b128_at(uint32_t a) {
  static_assert(OFF >= 0 && OFF < 65536, "DS offset field");
  short8_t r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF) : "memory");
  return r;
}
template <int OFF>
__device__ __forceinline__ short4_t lds_read_tr16_at(uint32_t a) {
  static_assert(OFF >= 0 && OFF < 65536, "DS offset field");
  short4_t r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF) : "memory");
  return r;
}
// f(std::integral_constant<int, I>{}) for I = 0 .. N-1 (compile-time indices
// for the offset-immediate reads)
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}
__device__ __forceinline__ long lds_read_tr8_async(const void* p) {
  long r;
  const uint32_t a = (uint32_t)(uintptr_t)p;
  asm volatile("ds_read_b64_tr_b8 %0, %1" : "=v"(r) : "v"(a) : "memory");
  return r;
}

template <int N>
__device__ __forceinline__ void lgkm_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N < 15 ? N : 15) : "memory");
}

template <typename T>
__device__ __forceinline__ void tie(T& x) {
  asm volatile("" : "+v"(x));
}

__device__ __forceinline__ short8_t cat4(short4_t a, short4_t b) {
  short8_t r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}

__device__ __forceinline__ short pack_bf(float f) { return (short)f2bf(f); }

// Pack 8 f32 -> 8 bf16 (as MFMA operand)
__device__ __forceinline__ short8_t pack8(float a0, float a1, float a2, float a3, float a4, float a5,
                                          float a6, float a7) {
  short8_t r;
  r[0] = pack_bf(a0); r[1] = pack_bf(a1); r[2] = pack_bf(a2); r[3] = pack_bf(a3);
  r[4] = pack_bf(a4); r[5] = pack_bf(a5); r[6] = pack_bf(a6); r[7] = pack_bf(a7);
  return r;
}

// ---------------------------------------------------------------- stores
// Write-through (sc1) vector stores into one buffer (< 2 GiB): the lines are
// not left dirty in the XCD's L2, so the end-of-kernel L2 write-back has
// nothing to do for them. Worth it for large outputs consumed by a later
// kernel (on other XCDs anyway): measured on the GEMM epilogue 25.1 -> 22.8
// us for a 32 MB output (csrc/lab/gemm_lab.cpp).
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
struct WtBuf {
  __amdgpu_buffer_rsrc_t r;
  const char* base;
  bool ok;  // buffers past 31-bit offsets fall back to plain stores (uniform branch)
  __device__ __forceinline__ WtBuf(const void* p, size_t bytes)
      : r(__builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0,
                                             (int)(bytes < 0x7fffffffull ? bytes : 0x7fffffffull),
                                             0x00020000)),
        base(static_cast<const char*>(p)),
        ok(bytes <= 0x7fffffffull) {}
  template <typename T>
  __device__ __forceinline__ void st16(void* p, const T& v) const {
    static_assert(sizeof(T) == 16, "16-byte value");
    if (ok)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), r,
                                             (int)(static_cast<const char*>(p) - base), 0, 16);
    else
      *static_cast<T*>(p) = v;
  }
  template <typename T>
  __device__ __forceinline__ void st8(void* p, const T& v) const {
    static_assert(sizeof(T) == 8, "8-byte value");
    if (ok)
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), r,
                                            (int)(static_cast<const char*>(p) - base), 0, 16);
    else
      *static_cast<T*>(p) = v;
  }
  __device__ __forceinline__ void st4(void* p, uint32_t v) const {
    if (ok)
      __builtin_amdgcn_raw_buffer_store_b32(v, r, (int)(static_cast<const char*>(p) - base), 0, 16);
    else
      *static_cast<uint32_t*>(p) = v;
  }
};

// XCD-aware bijective block remap (blocks b and b+8 share an XCD under the
// observed round-robin dispatch): give each XCD a contiguous chunk of tiles so
// neighbouring tiles share that XCD's L2. Speed-only; any placement is correct.
// OCP e4m3 (gfx950 native fp8): saturating pack of two floats into the low
// (HI=false) or high 16 bits of `old`; amax as the bit pattern of |v| (non-
// negative floats order like their bits), spread over AMAX_SPREAD words that
// sit AMAX_STRIDE words (one 128-byte line) apart: atomics execute at the
// memory side per line, so thousands of producer blocks on the 2 lines of 64
// consecutive words serialised (the e4m3-emitting LayerNorm took 20.8 vs
// 11.6 us). A slot is AMAX_WORDS words; producers call amax_word(slot, b).
constexpr float E4M3_MAX = 448.f;
constexpr int AMAX_SPREAD = 64;
constexpr int AMAX_STRIDE = 32;
constexpr int AMAX_WORDS = AMAX_SPREAD * AMAX_STRIDE;
__device__ __forceinline__ unsigned* amax_word(unsigned* slot, int b) {
  return slot + (b & (AMAX_SPREAD - 1)) * AMAX_STRIDE;
}
template <bool HI>
__device__ __forceinline__ int pack2_e4m3(float a, float b, int old) {
  a = fminf(fmaxf(a, -E4M3_MAX), E4M3_MAX);
  b = fminf(fmaxf(b, -E4M3_MAX), E4M3_MAX);
  return __builtin_amdgcn_cvt_pk_fp8_f32(a, b, old, HI);
}
// OCP e5m2 (gfx950 bf8): the gradient format of the fp8 backward
constexpr float E5M2_MAX_F = 57344.f;
template <bool HI>
__device__ __forceinline__ int pack2_e5m2c(float a, float b, int old) {
  a = fminf(fmaxf(a, -E5M2_MAX_F), E5M2_MAX_F);
  b = fminf(fmaxf(b, -E5M2_MAX_F), E5M2_MAX_F);
  return __builtin_amdgcn_cvt_pk_bf8_f32(a, b, old, HI);
}
__device__ __forceinline__ void atomic_amax(unsigned* p, float v) {
  atomicMax(p, __float_as_uint(fabsf(v)));
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  constexpr int NX = 8;
  if (nwg <= NX) return bid;
  const int q = nwg / NX, r = nwg % NX;
  const int x = bid % NX, i = bid / NX;
  const int base = (x < r) ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + i;
}

}  // namespace tdg
