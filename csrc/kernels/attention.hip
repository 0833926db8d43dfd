// Flash-style fused multi-head attention for gfx950 (forward + backward).
//
// Replaces the reference's scaled_dot_product_attention
// (reference: distributed_training_transformer/transformer_model.py:73-109):
//   softmax(Q K^T / sqrt(dk) + mask*-1e9) V
// with the [B,h,Lq,Lk] score tensor never materialised. Padding masks are
// per-batch key lengths (right-padded PAD=0 tokens, transformer_model.py:56-62)
// and the look-ahead mask (transformer_model.py:65-70) is causal tile skipping
// plus an in-tile compare; masked logits contribute exactly 0 probability, as
// exp(-1e9) does in the reference.
//
// Design (CDNA4): one workgroup = 4 waves = 64 query rows (forward / dQ) or
// 64 key rows (dK/dV) of one (batch, head). MFMA v_mfma_f32_16x16x32_bf16.
// Forward computes S^T = K Q^T so that every lane owns one query row (lane&15)
// and 4 key positions per 16-key tile: the row softmax is register-local plus
// two cross-lane xors, and the P accumulators feed the P^T operand of
// O^T = V^T P^T directly (keys permuted consistently on both operands), the V
// operand coming from the transposing ds_read_b64_tr_b16. K/V tiles are staged
// through one XOR-swizzled LDS image that is conflict-free both for the
// 16-byte row reads and for the transposed reads (docs/KERNELS.md).
// Backward: two kernels (dK/dV with key rows on lanes, dQ with query rows on
// lanes), each recomputing P from the forward's log-sum-exp; no atomics, so
// gradients are bitwise deterministic.
#include "tdg_common.h"
#include "tdg_attn.h"

#include <cstdlib>
#include "tdg_gemm.h"


namespace tdg {

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LOG2_448 = 8.807354922057604f;  // log2(448): the e4m3 P scale

// v_exp_f32 as is: libm's exp2f wraps it in a denormal-range fix-up (compare,
// select, ldexp: 4 more VALU per element); softmax weights below 2^-126
// flushed to zero change nothing at bf16 P.
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
// ok ? exp2(x) : 0 as a select: exp2 computed for every lane (x is finite or
// -inf on the masked side, never NaN). Written as the conditional expression,
// the compiler branched around each element's exp (exec-mask save / restore,
// ~10 instructions per element on every masked tile).
__device__ __forceinline__ float masked_exp2(float x, bool ok) {
  float e = fast_exp2(x);
  asm volatile("" : "+v"(e));
  return ok ? e : 0.f;
}

// Row-per-lane store of a 16x16-MFMA output row: lane (g, cl) holds columns
// 16 dt + 4 g .. +3 (dt < DT) of its row as packed bf16 pairs lo[dt] / hi[dt].
// For each dt pair, v_permlane16_swap exchanges the odd 16-lane groups' dt
// half with the even groups' dt + 1 half, after which every lane holds 16
// contiguous bytes -- columns 16 (dt + (g & 1)) + 8 (g >> 1) .. +7 -- and
// writes them with one dwordx4: half the store instructions of the 8-byte
// form, whose tail was store-issue-bound (the guide's T21). Every lane of
// the wave must call it (the swaps); `store` masks the lane's row.
template <int DT>
__device__ __forceinline__ void store_row16(bf16_t* __restrict__ row, const uint32_t (&lo)[DT],
                                            const uint32_t (&hi)[DT], int g, bool store) {
  if constexpr (DT % 2 == 0) {
#pragma unroll
    for (int d = 0; d < DT; d += 2) {
      const auto r0 = __builtin_amdgcn_permlane16_swap(lo[d], lo[d + 1], false, false);
      const auto r1 = __builtin_amdgcn_permlane16_swap(hi[d], hi[d + 1], false, false);
      if (store)
        *reinterpret_cast<uint4*>(row + 16 * (d + (g & 1)) + 8 * (g >> 1)) =
            make_uint4(r0[0], r1[0], r0[1], r1[1]);
    }
  } else {
#pragma unroll
    for (int d = 0; d < DT; ++d)
      if (store) *reinterpret_cast<uint2*>(row + 16 * d + 4 * g) = make_uint2(lo[d], hi[d]);
  }
}
// (the packing of an accumulator: 4 values, times sc)
__device__ __forceinline__ void pack_acc(const f32x4& v, float sc, uint32_t& lo, uint32_t& hi) {
  lo = pack2bf(v[0] * sc, v[1] * sc);
  hi = pack2bf(v[2] * sc, v[3] * sc);
}

// 16-byte global load from an always-valid (clamped) address, zero where
// !ok: a select instead of an exec-mask branch around every prologue load
__device__ __forceinline__ short8_t ld8_or0(const bf16_t* p, bool ok) {
  const short8_t v = *reinterpret_cast<const short8_t*>(p);
  const short8_t z = {0, 0, 0, 0, 0, 0, 0, 0};
  return ok ? v : z;
}

// Key window and logit scale of batch row b. A row with NO valid key
// (kv_len == 0: an all-PAD sequence) gets the reference's numerics: its
// padding mask adds -1e9 to every logit, which in fp32 leaves them all equal
// (transformer_model.py:101-105), so the softmax is uniform over ALL Lk keys
// (padding included) -- reproduced by attending to all Lk keys with a zero
// logit scale for P. The backward is TF's autograd of that graph: dS =
// P (dP - delta) with the uniform P, and dQ / dK keep the real scale (the
// mask add passes the gradient through). In causal attention such a row's
// look-ahead mask is covered by the padding mask too (the reference combines
// them with a maximum, transformer_model.py:361-362): all keys, causal off.
__device__ __forceinline__ void key_window(const AttnArgs& a, int b, int& klim, float& scale,
                                           bool& causal) {
  klim = a.Lk;
  scale = a.scale;
  causal = a.causal != 0;
  if (a.kv_len) {
    const int n = a.kv_len[b];
    if (n > 0) {
      klim = min(klim, n);
    } else {
      scale = 0.f;
      causal = false;
    }
  }
}
// (block, head, batch) of this workgroup over a (blocks, H, B) grid; with
// a.xcd the linear order is xcd_remap'd (tdg_common.h), so the XCD that ran
// the projection GEMM tiles of a batch element's rows (their run of tile ids
// covers whole row bands) also runs that element's attention workgroups
__device__ __forceinline__ void attn_coords(const AttnArgs& a, int& xb, int& h, int& b) {
  const int gx = gridDim.x, gy = gridDim.y;
  int t = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  if (a.xcd) t = xcd_remap(t, gx * gy * gridDim.z);
  xb = t % gx;
  h = (t / gx) % gy;
  b = t / (gx * gy);
}
constexpr int QB = 64;  // rows per workgroup
constexpr int KB = 64;  // keys per tile

template <int HD>
struct ATile {
  static constexpr int RB = HD * 2;                       // bytes per row
  static constexpr int SEGS = HD / 16 > 0 ? HD / 16 : 1;  // 32-byte segments per row
  static constexpr int RPB = 128 / HD;                    // rows per 256-B bank row
  static constexpr int BYTES = 64 * RB;
  static constexpr int KS = HD >= 32 ? HD / 32 : 1;       // 32-deep MFMA steps over head dim
  static constexpr int DT = HD / 16;                      // 16-wide tiles over head dim
  __device__ static __forceinline__ int off(int row, int byte) {
    const int seg = (byte >> 5) ^ ((row / RPB) & (SEGS - 1));
    return row * RB + (seg << 5) + (byte & 31);
  }
  // Stage 64 rows (row0..row0+63, rows >= nrows zero) of a [L, ...] tensor,
  // in two halves so that callers can issue the global loads of several
  // tiles before the first LDS write (one memory latency, not one per tile).
  template <int NT = 256>
  struct Chunks {
    static constexpr int CPR = HD / 8;
    static constexpr int TOTAL = 64 * CPR;
    static constexpr int NI = (TOTAL + NT - 1) / NT;
    short8_t v[NI];
  };
  template <int NT = 256>
  __device__ static __forceinline__ void fetch(Chunks<NT>& c, const bf16_t* __restrict__ base,
                                               long long sl, int row0, int nrows, int tid) {
    using C = Chunks<NT>;
#pragma unroll
    for (int i = 0; i < C::NI; ++i) {
      const int id = tid + i * NT;
      const int row = id / C::CPR, cc = id % C::CPR;
      if constexpr (C::TOTAL % NT == 0) {  // (rows past nrows: clamped load, zeroed)
        const int r = min(row0 + row, nrows - 1);
        c.v[i] = ld8_or0(base + (long long)r * sl + cc * 8, row0 + row < nrows);
      } else {
        c.v[i] = short8_t{0, 0, 0, 0, 0, 0, 0, 0};
        if (id < C::TOTAL && row0 + row < nrows)
          c.v[i] = *reinterpret_cast<const short8_t*>(base + (long long)(row0 + row) * sl + cc * 8);
      }
    }
  }
  template <int NT = 256>
  __device__ static __forceinline__ void put(char* lds, const Chunks<NT>& c, int tid) {
    using C = Chunks<NT>;
#pragma unroll
    for (int i = 0; i < C::NI; ++i) {
      const int id = tid + i * NT;
      if (C::TOTAL % NT != 0 && id >= C::TOTAL) break;
      const int row = id / C::CPR, cc = id % C::CPR;
      *reinterpret_cast<short8_t*>(lds + off(row, cc * 16)) = c.v[i];
    }
  }
  template <int NT = 256>
  __device__ static __forceinline__ void load(char* lds, const bf16_t* __restrict__ base,
                                              long long sl, int row0, int nrows, int tid) {
    Chunks<NT> c;
    fetch<NT>(c, base, sl, row0, nrows, tid);
    put<NT>(lds, c, tid);
  }
  // Row fragment: lane holds X[rbase + (lane&15)][32s + 8(lane>>4) + j]
  __device__ static __forceinline__ short8_t frag_row(const char* lds, int rbase, int s, int lane) {
    const int row = rbase + (lane & 15);
    const int c = 4 * s + (lane >> 4);
    if constexpr (HD < 32) {
      const short8_t z = {0, 0, 0, 0, 0, 0, 0, 0};
      const short8_t v =
          *reinterpret_cast<const short8_t*>(lds + off(row, (c & (HD / 8 - 1)) * 16));
      return c < HD / 8 ? v : z;
    } else {
      return *reinterpret_cast<const short8_t*>(lds + off(row, c * 16));
    }
  }
  // The same row fragment read untracked (tdg_common.h lds_read_b128_async):
  // for loops with LDS-DMA in flight, where the compiler would put a
  // vmcnt(0) before a tracked read; the caller waits (lgkm_wait) and ties.
  __device__ static __forceinline__ short8_t frag_row_async(const char* lds, int rbase, int s, int lane) {
    static_assert(HD >= 32, "untracked row fragments: hd >= 32");
    const int row = rbase + (lane & 15);
    const int c = 4 * s + (lane >> 4);
    return lds_read_b128_async(lds + off(row, c * 16));
  }
  // Offset-immediate forms (tdg_common.h lds_read_*_at): the lane part of
  // the address once per tile, the row base in the DS offset field.
  // row_off: frag_row_async's lane part for row bases that are multiples of
  // 8 (the swizzle term is then the lane's own); frag_row_at<RBASE>(tile
  // address + row_off(s, lane)) == frag_row_async(tile, RBASE, s, lane).
  __device__ static __forceinline__ uint32_t row_off(int s, int lane) {
    return (uint32_t)off(lane & 15, (4 * s + (lane >> 4)) * 16);
  }
  template <int RBASE>
  __device__ static __forceinline__ short8_t frag_row_at(uint32_t a) {
    static_assert(RBASE % 8 == 0, "row base: multiple of 8");
    return lds_read_b128_at<RBASE * RB>(a);
  }
  // tr_off: frag_tr_async's lane part (rows 4 g + q of k-step 0: the swizzle
  // term is the same at + 16 and + 32 s2 rows)
  __device__ static __forceinline__ uint32_t tr_off(int dt, int lane) {
    const int g = lane >> 4, w = lane & 15, q = w >> 2, p = w & 3;
    return (uint32_t)off(4 * g + q, (16 * dt + 4 * p) * 2);
  }
  template <int S2>
  __device__ static __forceinline__ void frag_tr_at(uint32_t a, short4_t& lo, short4_t& hi) {
    lo = lds_read_tr16_at<32 * S2 * RB>(a);
    hi = lds_read_tr16_at<(32 * S2 + 16) * RB>(a);
  }
  // Transposed fragment, untracked, as its two 8-byte halves (tie both
  // after the wait, then cat4)
  __device__ static __forceinline__ void frag_tr_async(const char* lds, int s2, int dt, int lane,
                                                       short4_t& lo, short4_t& hi) {
    const int g = lane >> 4, w = lane & 15, q = w >> 2, p = w & 3;
    const int r1 = 32 * s2 + 4 * g + q;
    const int byte = (16 * dt + 4 * p) * 2;
    lo = lds_read_tr_async(lds + off(r1, byte));
    hi = lds_read_tr_async(lds + off(r1 + 16, byte));
  }
  // Transposed fragment over 32 rows (k-step s2 of a 64-row tile), head-dim
  // columns 16dt..16dt+15. Element j of lane group g is row
  // 32s2 + (j<4 ? 4g+j : 16+4g+j-4) (the key/query permutation that matches
  // the accumulator layout of a 16x16 MFMA output), column 16dt + (lane&15).
  __device__ static __forceinline__ short8_t frag_tr(const char* lds, int s2, int dt, int lane) {
    const int g = lane >> 4, w = lane & 15, q = w >> 2, p = w & 3;
    const int r1 = 32 * s2 + 4 * g + q;
    const int byte = (16 * dt + 4 * p) * 2;
    return cat4(lds_read_tr(lds + off(r1, byte)), lds_read_tr(lds + off(r1 + 16, byte)));
  }
};

// Load a head-row fragment straight from global: X[row][32s + 8g + j]
template <int HD>
__device__ __forceinline__ short8_t gfrag(const bf16_t* __restrict__ rowp, bool valid, int s,
                                          int lane) {
  const int c = 4 * s + (lane >> 4);
  if constexpr (HD >= 64) {  // (c < HD / 8 always; rowp is a clamped, valid row)
    return ld8_or0(rowp + c * 8, valid);
  } else {
    short8_t v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (valid && c < HD / 8) v = *reinterpret_cast<const short8_t*>(rowp + c * 8);
    return v;
  }
}



// One key tile of the online softmax for the lane's query row (swapped
// QK^T: s[t][r] = S[key = k0 + 16t + 4g + r][row], raw logits). m is the
// running max in the scaled log2 domain (max of c*S), l the running sum.
// Per element: a max, one FMA, one exp2, one add (and the mask compare only
// on tiles that need it: the key-window edge, the causal diagonal); the
// O rescale runs only when some lane's max grew (exact: alpha = 1 otherwise).
// Writes the tile's P as bf16 MFMA operands (pairs of 16-key tiles).
// Does the key tile [k0, k0 + kt) need the per-element mask for a wave whose
// first query row is wq0 (wave-uniform)?
__device__ __forceinline__ bool tile_masked(int k0, int kt, int klim, bool causal, int wq0) {
  return k0 + kt > klim || (causal && k0 + kt - 1 > wq0);
}

// (split in two so that LDS reads can be issued between them: the max part
// has the cross-lane shuffles, the exp part no LDS access)
// (a masked tile is scaled while masking -- masked logits -inf, the others
// c*S -- so that c = 0, the zero logit scale of a kv_len = 0 row, never meets
// an infinity in a product; unmasked tiles keep raw logits and fold c into
// the exp's FMA)
// (KPERM: the e4m3 kernel's key order, accumulator (t, g, r) = key
// 32 (t >> 1) + 8 g + 4 (t & 1) + r -- see attn_fwd_fp8_kernel)
template <int NT16, int DT, bool KPERM = false>
__device__ __forceinline__ void softmax_max(f32x4 (&s)[NT16], float& m, float& l, f32x4 (&oacc)[DT],
                                            bool masked, int k0, int klim, bool causal, int qrow,
                                            int g, float c) {
  if (masked) {
    // key = lane base + a constant per (t, r): valid iff the constant <= the
    // lane's limit (last valid key, the causal diagonal) minus the base --
    // one compare against an inline constant per element
    const int kb = k0 + (KPERM ? 8 * g : 4 * g);
    const int lim = (causal ? min(klim - 1, qrow) : klim - 1) - kb;
#pragma unroll
    for (int t = 0; t < NT16; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int off = KPERM ? 32 * (t >> 1) + 4 * (t & 1) + r : 16 * t + r;
        s[t][r] = off <= lim ? s[t][r] * c : -INFINITY;
      }
  }
  // (asm max3 chain: no canonicalising moves on the MFMA results)
  float tmax = vmax3(s[0][0], s[0][1], s[0][2]);
  tmax = vmax(tmax, s[0][3]);
#pragma unroll
  for (int t = 1; t < NT16; ++t) {
    tmax = vmax3(tmax, s[t][0], s[t][1]);
    tmax = vmax3(tmax, s[t][2], s[t][3]);
  }
  tmax = rows_max(tmax);
  const float mn = vmax(m, masked ? tmax : tmax * c);
  if (__ballot(mn > m)) {  // wave-uniform: rescale only when a row max grew
    const float alpha = fast_exp2(m - mn);  // m = -inf (nothing yet): 0, and O, l are 0
#pragma unroll
    for (int i = 0; i < DT; ++i) oacc[i] *= alpha;
    l *= alpha;
    m = mn;
  }
}
// cs: c for a raw (unmasked) tile, 1 for a masked (already scaled) one
template <int NT16>
__device__ __forceinline__ void softmax_exp(f32x4 (&s)[NT16], float m, float& l,
                                            short8_t (&pf)[NT16 / 2], float cs) {
  const float nm = m == -INFINITY ? 0.f : -m;  // all masked so far: exp2(-inf) = 0, no NaN
  float rs = 0.f;
#pragma unroll
  for (int t = 0; t < NT16; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float p = fast_exp2(fmaf(s[t][r], cs, nm));
      s[t][r] = p;
      rs += p;
    }
  l += rs;
#pragma unroll
  for (int s2 = 0; s2 < NT16 / 2; ++s2)
    pf[s2] = pack8(s[2 * s2][0], s[2 * s2][1], s[2 * s2][2], s[2 * s2][3], s[2 * s2 + 1][0],
                   s[2 * s2 + 1][1], s[2 * s2 + 1][2], s[2 * s2 + 1][3]);
}
template <int NT16, int DT>
__device__ __forceinline__ void softmax_tile(f32x4 (&s)[NT16], float& m, float& l,
                                             f32x4 (&oacc)[DT], short8_t (&pf)[NT16 / 2],
                                             bool masked, int k0, int klim, bool causal, int qrow,
                                             int g, float c) {
  softmax_max<NT16, DT>(s, m, l, oacc, masked, k0, klim, causal, qrow, g, c);
  softmax_exp<NT16>(s, m, l, pf, masked ? 1.f : c);
}

// ============================================================================ forward
// NWV waves per workgroup, U 16-query subtiles per wave (16 U NWV queries per
// workgroup; 8 x 1 covers a whole <= 128-query sequence, so K/V are read from
// HBM once per (batch, head)). Each K / V fragment read from LDS feeds U
// MFMAs: with U = 1 the fragment reads alone saturate the LDS at the MFMA
// rate (1 KiB per 16-cycle MFMA per wave), U = 2 halves them.
// KT keys per LDS tile (64 or 128: one load phase and one barrier pair for a
// whole <= 128-key sequence).
template <int HD, int NWV, int KT, int U>
__global__ __launch_bounds__(NWV * 64) __attribute__((amdgpu_waves_per_eu(2))) void attn_fwd_kernel(AttnArgs a) {
  using T = ATile<HD>;
  constexpr int QBW = 16 * NWV * U;
  constexpr int NT16 = KT / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ldsK = smem;
  char* ldsV = smem + (KT / 64) * T::BYTES;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, cl = lane & 15;
  int xb, h, b;
  attn_coords(a, xb, h, b);
  const int q0 = xb * QBW;
  int qrow[U];
#pragma unroll
  for (int u = 0; u < U; ++u) qrow[u] = q0 + 16 * (U * w + u) + cl;
  int klim;
  float scl;
  bool causal;
  key_window(a, b, klim, scl, causal);
  if (causal) klim = min(klim, q0 + QBW);

  TDG_STAMP(0);
  short8_t qf[U][T::KS];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bf16_t* qp = a.q + b * a.q_sb + (long long)min(qrow[u], a.Lq - 1) * a.q_sl + h * a.q_sh;
#pragma unroll
    for (int s = 0; s < T::KS; ++s) qf[u][s] = gfrag<HD>(qp, qrow[u] < a.Lq, s, lane);
  }

  const bf16_t* kb = a.k + b * a.k_sb + h * a.k_sh;
  const bf16_t* vb = a.v + b * a.v_sb + h * a.v_sh;
  const float c = scl * LOG2E;
  constexpr int KTILE = KT;
  const int wq0 = q0 + 16 * U * w;

  f32x4 oacc[U][T::DT];
  float m[U], l[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    m[u] = -INFINITY;
    l[u] = 0.f;
#pragma unroll
    for (int i = 0; i < T::DT; ++i) oacc[u][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // K / V tiles staged global -> registers -> LDS; the NEXT tile's loads are
  // issued right after the current one is in LDS, so they are in flight
  // during this tile's MFMAs (every load of a tile in flight before the
  // first LDS write, one memory latency per tile at most)
  typename T::template Chunks<NWV * 64> ck[KT / 64], cv[KT / 64];
  auto fetch_kv = [&](int kk0) {
#pragma unroll
    for (int h64 = 0; h64 < KT / 64; ++h64) {
      T::template fetch<NWV * 64>(ck[h64], kb, a.k_sl, kk0 + 64 * h64, a.Lk, tid);
      T::template fetch<NWV * 64>(cv[h64], vb, a.v_sl, kk0 + 64 * h64, a.Lk, tid);
    }
  };
  if (klim > 0) fetch_kv(0);
  for (int k0 = 0; k0 < klim; k0 += KT) {
#pragma unroll
    for (int h64 = 0; h64 < KT / 64; ++h64) {
      T::template put<NWV * 64>(ldsK + h64 * T::BYTES, ck[h64], tid);
      T::template put<NWV * 64>(ldsV + h64 * T::BYTES, cv[h64], tid);
    }
    __syncthreads();
    if (k0 == 0) TDG_STAMP(1);
    if (k0 + KT < klim) fetch_kv(k0 + KT);
    f32x4 s[U][NT16];
#pragma unroll
    for (int t = 0; t < NT16; ++t) {
#pragma unroll
      for (int u = 0; u < U; ++u) s[u][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < T::KS; ++ks) {
        const short8_t kfr = T::frag_row(ldsK, 16 * t, ks, lane);
#pragma unroll
        for (int u = 0; u < U; ++u) s[u][t] = mfma16(kfr, qf[u][ks], s[u][t]);
      }
    }
    short8_t pf[U][NT16 / 2];
#pragma unroll
    for (int u = 0; u < U; ++u)
      softmax_tile<NT16, T::DT>(s[u], m[u], l[u], oacc[u], pf[u], tile_masked(k0, KTILE, klim, causal, wq0),
                                k0, klim, causal, qrow[u], g, c);
#pragma unroll
    for (int s2 = 0; s2 < NT16 / 2; ++s2) {
#pragma unroll
      for (int dt = 0; dt < T::DT; ++dt) {
        const short8_t vfr = T::frag_tr(ldsV, s2, dt, lane);
#pragma unroll
        for (int u = 0; u < U; ++u) oacc[u][dt] = mfma16(vfr, pf[u][s2], oacc[u][dt]);
      }
    }
    __syncthreads();
  }
  TDG_STAMP(2);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    float lu = l[u];
    lu = rows_sum(lu);
    const bool ok = qrow[u] < a.Lq;
    const float inv = lu > 0.f ? 1.f / lu : 0.f;
    bf16_t* op = a.out + b * a.o_sb + (long long)qrow[u] * a.o_sl + h * a.o_sh;
    uint32_t lo[T::DT], hi[T::DT];
#pragma unroll
    for (int dt = 0; dt < T::DT; ++dt) pack_acc(oacc[u][dt], inv, lo[dt], hi[dt]);  // columns 16dt + 4g + r
    store_row16<T::DT>(op, lo, hi, g, ok);
    if (ok && g == 0)
      a.lse[((long long)b * a.H + h) * a.Lq + qrow[u]] = lu > 0.f ? m[u] + log2f(lu) : INFINITY;
  }
#ifdef TDG_STAMPS
  TDG_STAMP(3);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  TDG_STAMP(4);
#endif
}

// ============================================================================ forward, long sequences
// hd = 64, Lq > 128. The K / V tiles (64 keys) stream through an NS-slot LDS
// ring by LDS-DMA (Glds: the ATile<64> image is the GEMM's K-contiguous
// 64-row image), NS-1 tiles in flight and one barrier per tile -- instead of
// global -> register -> LDS with one tile of register prefetch, which left
// the 512-key sequences latency-bound (0.31 PF/s). NWV waves x U 16-query
// subtiles per wave; the K / V fragment reads are shared by the U subtiles.
template <int NWV, int U, int NS>
__global__ __launch_bounds__(NWV * 64) __attribute__((amdgpu_waves_per_eu(2))) void attn_fwd_pipe_kernel(AttnArgs a) {
  constexpr int HD = 64;
  using T = ATile<HD>;
  using G = Glds<true, 64, NWV>;  // 64 rows x 64 head-dim elements
  constexpr int QBW = 16 * NWV * U;
  constexpr int NT16 = 4;             // 16-key tiles per 64-key tile
  constexpr int SLOT = 2 * T::BYTES;  // K image, V image
  constexpr int PT = 2 * G::P;        // LDS-DMA per wave per tile
  static_assert(NS >= 3, "ring: refilled, being read, landed");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, cl = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  int xb, h, b;
  attn_coords(a, xb, h, b);
  const int q0 = xb * QBW;
  int qrow[U];
#pragma unroll
  for (int u = 0; u < U; ++u) qrow[u] = q0 + 16 * (U * w + u) + cl;
  int klim;
  float scl;
  bool causal;
  key_window(a, b, klim, scl, causal);
  if (causal) klim = min(klim, q0 + QBW);
  const int nkt = (klim + 63) / 64;

  short8_t qf[U][T::KS];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bf16_t* qp = a.q + b * a.q_sb + (long long)min(qrow[u], a.Lq - 1) * a.q_sl + h * a.q_sh;
#pragma unroll
    for (int s = 0; s < T::KS; ++s) qf[u][s] = gfrag<HD>(qp, qrow[u] < a.Lq, s, lane);
  }
  const bf16_t* kb = a.k + b * a.k_sb + h * a.k_sh;
  const bf16_t* vb = a.v + b * a.v_sb + h * a.v_sh;
  G gs;
  gs.init(w, lane);
  auto issue = [&](int kt) {
    char* slot = smem + (kt % NS) * SLOT;
    gs.issue(kb, (int)a.k_sl, a.Lk, HD, 64 * kt, 0, slot, w);
    gs.issue(vb, (int)a.v_sl, a.Lk, HD, 64 * kt, 0, slot + T::BYTES, w);
  };
  // prologue tiles issued unconditionally (clamped rows past the sequence,
  // never read) so the DMA count behind the Q loads is a constant
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) issue(s);
  wait_vmcnt_known<(NS - 1) * PT>();  // Q fragments in registers

  const float c = scl * LOG2E;
  constexpr int KTILE = 64;
  const int wq0 = q0 + 16 * U * w;
  f32x4 oacc[U][T::DT];
  float m[U], l[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    m[u] = -INFINITY;
    l[u] = 0.f;
#pragma unroll
    for (int i = 0; i < T::DT; ++i) oacc[u][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  for (int kt = 0; kt < nkt; ++kt) {
    // tile kt landed (this wave's DMA, then everyone's); every wave is past
    // its reads of tile kt-1, whose slot takes tile kt+NS-1
    wait_tiles<PT, NS - 2>(min(NS - 2, nkt - 1 - kt));
    lds_barrier();
    if (kt + NS - 1 < nkt) issue(kt + NS - 1);
    const char* ldsK = smem + (kt % NS) * SLOT;
    const char* ldsV = ldsK + T::BYTES;
    const int k0 = 64 * kt;
    // all LDS reads of the tile untracked (a tracked read would get a
    // vmcnt(0) for the DMA in flight), with counted waits: K fragments in
    // two halves, V fragments issued between the softmax's max and exp parts
    short8_t kfr[NT16][T::KS];
#pragma unroll
    for (int t = 0; t < NT16; ++t)
#pragma unroll
      for (int ks = 0; ks < T::KS; ++ks) kfr[t][ks] = T::frag_row_async(ldsK, 16 * t, ks, lane);
    f32x4 s[U][NT16];
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      if (half == 0) lgkm_wait<NT16 * T::KS / 2>();
      else lgkm_wait<0>();
#pragma unroll
      for (int t = half * NT16 / 2; t < (half + 1) * NT16 / 2; ++t) {
#pragma unroll
        for (int ks = 0; ks < T::KS; ++ks) tie(kfr[t][ks]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          s[u][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < T::KS; ++ks) s[u][t] = mfma16(kfr[t][ks], qf[u][ks], s[u][t]);
        }
      }
    }
    const bool msk = tile_masked(k0, KTILE, klim, causal, wq0);
#pragma unroll
    for (int u = 0; u < U; ++u)
      softmax_max<NT16, T::DT>(s[u], m[u], l[u], oacc[u], msk, k0, klim, causal, qrow[u], g, c);
    short4_t vlo[NT16 / 2][T::DT], vhi[NT16 / 2][T::DT];
#pragma unroll
    for (int s2 = 0; s2 < NT16 / 2; ++s2)
#pragma unroll
      for (int dt = 0; dt < T::DT; ++dt) T::frag_tr_async(ldsV, s2, dt, lane, vlo[s2][dt], vhi[s2][dt]);
    short8_t pf[U][NT16 / 2];
#pragma unroll
    for (int u = 0; u < U; ++u) softmax_exp<NT16>(s[u], m[u], l[u], pf[u], msk ? 1.f : c);
#pragma unroll
    for (int s2 = 0; s2 < NT16 / 2; ++s2) {
      if (s2 == 0) lgkm_wait<2 * T::DT>();
      else lgkm_wait<0>();
#pragma unroll
      for (int dt = 0; dt < T::DT; ++dt) {
        tie(vlo[s2][dt]);
        tie(vhi[s2][dt]);
        const short8_t vfr = cat4(vlo[s2][dt], vhi[s2][dt]);
#pragma unroll
        for (int u = 0; u < U; ++u) oacc[u][dt] = mfma16(vfr, pf[u][s2], oacc[u][dt]);
      }
    }
  }
  wait_vmcnt<0>();  // (nothing in flight on the exit paths; keeps the grid drained)
#pragma unroll
  for (int u = 0; u < U; ++u) {
    float lu = l[u];
    lu = rows_sum(lu);
    const bool ok = qrow[u] < a.Lq;
    const float inv = lu > 0.f ? 1.f / lu : 0.f;
    bf16_t* op = a.out + b * a.o_sb + (long long)qrow[u] * a.o_sl + h * a.o_sh;
    uint32_t lo[T::DT], hi[T::DT];
#pragma unroll
    for (int dt = 0; dt < T::DT; ++dt) pack_acc(oacc[u][dt], inv, lo[dt], hi[dt]);
    store_row16<T::DT>(op, lo, hi, g, ok);
    if (ok && g == 0)
      a.lse[((long long)b * a.H + h) * a.Lq + qrow[u]] = lu > 0.f ? m[u] + log2f(lu) : INFINITY;
  }
}

// ============================================================================ forward, e4m3
// BASELINE config 5's fp8 attention: Q, K, V are the e4m3 copies the fp8
// input projections emit (per-tensor scales sq, sk, sv), S^T = K Q^T and
// O^T = V^T P^T on v_mfma_f32_16x16x32_fp8_fp8, P quantised as e4m3(P * 448)
// (P <= 1 against the running max), softmax in f32. hd = 64, > 128 queries;
// the structure of attn_fwd_pipe_kernel: 8 waves x 16 queries, K / V tiles of
// 64 keys (64-byte rows, 4 KiB each) in an NS-slot LDS-DMA ring, waves 0-3
// staging K and 4-7 V (one 1 KiB piece per wave per tile), untracked counted
// LDS reads. Images: 8-byte chunk c of row r stored at c ^ 2 ((r >> 2) & 3)
// (the K row reads and the V transposing reads both conflict-free). The PV
// product needs each lane group's 8 keys consecutive (ds_read_b64_tr_b8 gives
// 8 consecutive V rows): the K image is filled in a permuted key order so
// that the S accumulator (t, g, r) is key 32 (t >> 1) + 8 g + 4 (t & 1) + r,
// which makes the P registers the PV B operand as they stand. The backward
// stays bf16 (it recomputes P from the bf16 Q, K and this LSE).
template <int NS, int U>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(U == 2 ? 4 : 2))) void attn_fwd_fp8_kernel(AttnArgs a) {
  // U 16-query subtiles per wave (16 U queries): every K / V fragment feeds U
  // MFMAs and each wave carries U independent softmax chains (U = 2: one
  // round of 4 waves per SIMD at seq 512 instead of 1.33 rounds of 6)
  constexpr int NWV = 8, HD = 64, RB = 64, TB = 64 * RB, SLOT = 2 * TB, QBW = 16 * U * NWV;
  constexpr int NT16 = 4, DT = 4;
  static_assert(NS >= 3, "ring: refilled, being read, landed");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint8_t* q8 = reinterpret_cast<const uint8_t*>(a.q);
  const uint8_t* k8 = reinterpret_cast<const uint8_t*>(a.k);
  const uint8_t* v8 = reinterpret_cast<const uint8_t*>(a.v);
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, cl = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  int xb, h, b;
  attn_coords(a, xb, h, b);
  const int q0 = xb * QBW;
  const int wq0 = q0 + 16 * U * w;
  int qrow[U];
#pragma unroll
  for (int u = 0; u < U; ++u) qrow[u] = wq0 + 16 * u + cl;
  int klim;
  float scl;
  bool causal;
  key_window(a, b, klim, scl, causal);
  if (causal) klim = min(klim, q0 + QBW);
  const int nkt = (klim + 63) / 64;
  // (causal: the wave's last key tile; later tiles are staged for the other
  // waves but skipped here)
  const int wkt = causal ? min(nkt, (wq0 + 16 * U + 63) / 64) : nkt;

  // Q fragments (B operand of S^T): lane (g, q) holds Q[q][32 ks + 8 g .. +7]
  long qf[U][2];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint8_t* qp = q8 + b * a.q_sb + (long long)min(qrow[u], a.Lq - 1) * a.q_sl + h * a.q_sh;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      qf[u][ks] = qrow[u] < a.Lq ? *reinterpret_cast<const long*>(qp + 32 * ks + 8 * g) : 0;
  }
  // staging: wave w < 4 fills K image rows 16w.., w >= 4 V image rows 16(w-4)..
  const bool isv = w >= 4;
  const int rho = 16 * (w & 3) + (lane >> 2);
  // K image row rho = 16 t + 4 g + r holds key 32 t1 + 8 g + 4 t0 + r
  const int kin = isv ? rho : ((rho & 0x23) | ((rho & 0x0C) << 1) | ((rho & 0x10) >> 2));
  const int chunk = (lane & 3) ^ ((rho >> 2) & 3);  // 16-byte source chunk of the swizzled row
  const uint8_t* src0 = (isv ? v8 + b * a.v_sb + h * a.v_sh : k8 + b * a.k_sb + h * a.k_sh) + 16 * chunk;
  const long long sl = isv ? a.v_sl : a.k_sl;
  char* dst0 = smem + (isv ? TB : 0) + (w & 3) * 1024;
  // DMA source: a 32-bit byte offset stepped by 64 rows per tile (no 64-bit
  // multiply per issue); only the tiles that reach past Lk clamp their row
  const uint8_t* srcb = src0 + (long long)kin * sl;
  const uint32_t step = (uint32_t)(64 * sl);
  const int klast = a.Lk - 1 - kin;  // (64 kt > klast: this lane's row is clamped)
  auto issue = [&](int kt, auto slc) {
    constexpr int SL = decltype(slc)::value;
    const uint8_t* sp = 64 * kt <= klast ? srcb + (uint32_t)kt * step : src0 + (long long)(a.Lk - 1) * sl;
    __builtin_amdgcn_global_load_lds((const void*)sp,
                                     (__attribute__((address_space(3))) void*)(dst0 + SL * SLOT), 16, 0, 0);
  };
  // prologue tiles issued unconditionally (clamped rows, never read) so the
  // DMA count behind the Q loads is a constant
  static_for<NS - 1>([&](auto sc) { issue(decltype(sc)::value, sc); });
  wait_vmcnt_known<NS - 1>();

  // lane parts of the fragment addresses (the swizzle term (row >> 2) & 3 is
  // the same for every 16-row K tile t and both 32-row V halves s2); the ring
  // slot and the tile rows are immediate offsets (the tile loop is unrolled
  // by NS, so tile kt's slot kt % NS is a constant)
  const uint32_t sbase = (uint32_t)(uintptr_t)smem;
  uint32_t ka[2], va[DT];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) ka[ks] = sbase + cl * RB + 8 * ((4 * ks + g) ^ (((cl >> 2) & 3) << 1));
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    const int row = 8 * g + (cl >> 1);
    va[dt] = sbase + TB + row * RB + 8 * ((2 * dt + (cl & 1)) ^ (((row >> 2) & 3) << 1));
  }
  const float inv_qk = 1.f / (a.sq8[0] * a.sk8[0]);
  const float c = scl * LOG2E * inv_qk;
  f32x4 oacc[U][DT];
  float m[U], l[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    m[u] = -INFINITY;
    l[u] = 0.f;
#pragma unroll
    for (int i = 0; i < DT; ++i) oacc[u][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  auto tile = [&](int kt, auto slc) {
    constexpr int SL = decltype(slc)::value;
    wait_tiles<1, NS - 2>(min(NS - 2, nkt - 1 - kt));
    lds_barrier();
    if (kt + NS - 1 < nkt) issue(kt + NS - 1, std::integral_constant<int, (SL + NS - 1) % NS>{});
    if (kt >= wkt) return;  // (wave-uniform)
    const int k0 = 64 * kt;
    // S^T: K rows 16 t + cl, hd bytes 32 ks + 8 g (8-byte chunk 4 ks + g);
    // lane part of the address ka[ks], slot and 16 t rows immediate offsets
    long kfr[NT16][2];
    static_for<NT16>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      kfr[t][0] = lds_read_b64_at<SL * SLOT + 16 * t * RB>(ka[0]);
      kfr[t][1] = lds_read_b64_at<SL * SLOT + 16 * t * RB>(ka[1]);
    });
    f32x4 s[U][NT16];
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      if (half == 0) lgkm_wait<NT16>();
      else lgkm_wait<0>();
#pragma unroll
      for (int t = half * 2; t < half * 2 + 2; ++t) {
        tie(kfr[t][0]);
        tie(kfr[t][1]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          s[u][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
            s[u][t] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(kfr[t][ks], qf[u][ks], s[u][t], 0, 0, 0);
        }
      }
    }
    const bool msk = tile_masked(k0, 64, klim, causal, wq0);
#pragma unroll
    for (int u = 0; u < U; ++u)
      softmax_max<NT16, DT, true>(s[u], m[u], l[u], oacc[u], msk, k0, klim, causal, qrow[u], g, c);
    // V^T fragments: lane pair (2 r8 + hh) of group g passes V row 32 s2 + 8 g + r8,
    // 8-byte chunk 2 dt + hh; lane i receives hd column 16 dt + i, keys 8 g .. +7
    long vfr[2][DT];
    static_for<DT>([&](auto dc) {
      constexpr int dt = decltype(dc)::value;
      vfr[0][dt] = lds_read_tr8_at<SL * SLOT>(va[dt]);
      vfr[1][dt] = lds_read_tr8_at<SL * SLOT + 32 * RB>(va[dt]);
    });
    // P448 = 448 exp2(c S - m) = exp2(c S - m + log2 448) (f32 row sum l of
    // P448), then e4m3(P448) in PV operand order: P <= 1 against the running
    // max, so P448 <= 448 needs no clamp and the 448 costs no multiply
    const float cs = msk ? 1.f : c;
    long pf[U][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float nm = (m[u] == -INFINITY ? 0.f : -m[u]) + LOG2_448;
#pragma unroll
      for (int t = 0; t < NT16; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[u][t][r] = fast_exp2(fmaf(s[u][t][r], cs, nm));
      float rs = s[u][0][0];
#pragma unroll
      for (int i = 1; i < 4 * NT16; ++i) rs += s[u][i / 4][i % 4];
      l[u] += rs;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        // (the first convert of each word writes its low half: its old value
        // is any register, the high half is written next -- no zeroing move)
        int lo = __builtin_amdgcn_cvt_pk_fp8_f32(s[u][2 * s2][0], s[u][2 * s2][1],
                                                 __builtin_bit_cast(int, s[u][2 * s2][0]), false);
        lo = __builtin_amdgcn_cvt_pk_fp8_f32(s[u][2 * s2][2], s[u][2 * s2][3], lo, true);
        int hi = __builtin_amdgcn_cvt_pk_fp8_f32(s[u][2 * s2 + 1][0], s[u][2 * s2 + 1][1],
                                                 __builtin_bit_cast(int, s[u][2 * s2 + 1][0]), false);
        hi = __builtin_amdgcn_cvt_pk_fp8_f32(s[u][2 * s2 + 1][2], s[u][2 * s2 + 1][3], hi, true);
        pf[u][s2] = (long)(uint32_t)lo | ((long)hi << 32);
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      if (s2 == 0) lgkm_wait<DT>();
      else lgkm_wait<0>();
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        tie(vfr[s2][dt]);
#pragma unroll
        for (int u = 0; u < U; ++u)
          oacc[u][dt] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(vfr[s2][dt], pf[u][s2], oacc[u][dt], 0, 0, 0);
      }
    }
  };
  int kt = 0;
  for (; kt + NS <= nkt; kt += NS) static_for<NS>([&](auto sc) { tile(kt + decltype(sc)::value, sc); });
  static_for<NS - 1>([&](auto sc) {
    if (kt + decltype(sc)::value < nkt) tile(kt + decltype(sc)::value, sc);
  });
  wait_vmcnt<0>();
  // e4m3 copy of O for the e4m3 output projection: from the bf16-rounded
  // values (what quantising the bf16 O gives), wave amax -> one atomic
  const float so = a.out8 ? a.so8[0] : 0.f;
  float am = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    float lu = l[u];
    lu = rows_sum(lu);
    const bool valid = qrow[u] < a.Lq;
    const float inv = lu > 0.f ? 1.f / (lu * a.sv8[0]) : 0.f;  // (lu: the row sum of P448)
    const long long ooff = b * a.o_sb + (long long)qrow[u] * a.o_sl + h * a.o_sh;
    bf16_t* op = a.out + ooff;
    // (8-byte stores: the 16-byte form of store_row16 measured 4 % slower here,
    // 739 vs 708 us per step over 18 calls, profiles/r4/ab_grouped_tiles_fp8_kstats.txt)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      bf16_t e[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) e[r] = f2bf(oacc[u][dt][r] * inv);
      if (valid) {
        const uint32_t lo = (uint32_t)e[0] | ((uint32_t)e[1] << 16);
        const uint32_t hi = (uint32_t)e[2] | ((uint32_t)e[3] << 16);
        *reinterpret_cast<uint2*>(op + 16 * dt + 4 * g) = make_uint2(lo, hi);
      }
      if (a.out8) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = bf2f(e[r]);
          am = fmaxf(am, valid ? fabsf(v[r]) : 0.f);
        }
        int w8 = pack2_e4m3<false>(v[0] * so, v[1] * so, 0);
        w8 = pack2_e4m3<true>(v[2] * so, v[3] * so, w8);
        if (valid) *reinterpret_cast<int*>(a.out8 + ooff + 16 * dt + 4 * g) = w8;
      }
    }
    if (valid && g == 0)
      a.lse[((long long)b * a.H + h) * a.Lq + qrow[u]] = lu > 0.f ? m[u] + (log2f(lu) - LOG2_448) : INFINITY;
  }
  if (a.out8) {
    am = wave_max(am);
    if (lane == 0) atomic_amax(amax_word(a.amax8, blockIdx.x + 7 * blockIdx.y + 13 * blockIdx.z), am);
  }
}

// ============================================================================ dK, dV
// 4 waves, U 16-key subtiles per wave (64 U keys per workgroup): every Q / dO
// fragment read from LDS feeds U MFMAs.
template <int HD, int U>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void attn_bwd_dkdv_kernel(AttnArgs a) {
  using T = ATile<HD>;
  constexpr int KBW = 64 * U;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ldsQ = smem;
  char* ldsO = smem + T::BYTES;  // dO tile
  float* ldsL = reinterpret_cast<float*>(smem + 2 * T::BYTES);
  float* ldsD = ldsL + QB;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, cl = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // (wave-uniform: scalar branches)
  int xb, h, b;
  attn_coords(a, xb, h, b);
  const int k0 = xb * KBW;
  int key[U];
#pragma unroll
  for (int u = 0; u < U; ++u) key[u] = k0 + 16 * (U * w + u) + cl;
  int klim;
  float scl;
  bool causal;
  key_window(a, b, klim, scl, causal);
  const float c = scl * LOG2E;

  f32x4 dk[U][T::DT], dv[U][T::DT];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int i = 0; i < T::DT; ++i) dk[u][i] = dv[u][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (k0 < klim) {
    short8_t kf[U][T::KS], vf[U][T::KS];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int krow = min(key[u], a.Lk - 1);
      const bf16_t* kp = a.k + b * a.k_sb + (long long)krow * a.k_sl + h * a.k_sh;
      const bf16_t* vp = a.v + b * a.v_sb + (long long)krow * a.v_sl + h * a.v_sh;
#pragma unroll
      for (int s = 0; s < T::KS; ++s) {
        kf[u][s] = gfrag<HD>(kp, key[u] < a.Lk, s, lane);
        vf[u][s] = gfrag<HD>(vp, key[u] < a.Lk, s, lane);
      }
    }
    const bf16_t* qb = a.q + b * a.q_sb + h * a.q_sh;
    const bf16_t* ob = a.dout + b * a.do_sb + h * a.do_sh;
    const float* lse = a.lse + ((long long)b * a.H + h) * a.Lq;
    const float* del = a.delta + ((long long)b * a.H + h) * a.Lq;
    const int qstart = causal ? (k0 / QB) * QB : 0;
    // Q / dO / lse / delta of query block q0+QB are loaded into registers
    // while block q0 is computed (register prefetch, single LDS buffer)
    typename T::template Chunks<256> cq, co;
    float lv = INFINITY, dlv = 0.f;
    auto fetch_q = [&](int qq0) {
      T::template fetch<256>(cq, qb, a.q_sl, qq0, a.Lq, tid);
      T::template fetch<256>(co, ob, a.do_sl, qq0, a.Lq, tid);
      if (tid < QB) {
        const int q = qq0 + tid;
        lv = q < a.Lq ? lse[q] : INFINITY;
        dlv = q < a.Lq ? del[q] : 0.f;
      }
    };
    if (qstart < a.Lq) fetch_q(qstart);
    for (int q0 = qstart; q0 < a.Lq; q0 += QB) {
      T::template put<256>(ldsQ, cq, tid);
      T::template put<256>(ldsO, co, tid);
      if (tid < QB) {
        ldsL[tid] = lv;
        ldsD[tid] = dlv;
      }
      __syncthreads();
      if (q0 + QB < a.Lq) fetch_q(q0 + QB);
      // S[q][key] and dP[q][key]: rows q = q0 + 16t + 4g + r, col key (lane)
      short8_t pf[U][2], dsf[U][2];
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        f32x4 p[U][2], ds[U][2];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          const int t = 2 * s2 + tt;
          f32x4 sv[U], dpv[U];
#pragma unroll
          for (int u = 0; u < U; ++u) sv[u] = dpv[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < T::KS; ++ks) {
            const short8_t qfr = T::frag_row(ldsQ, 16 * t, ks, lane);
            const short8_t ofr = T::frag_row(ldsO, 16 * t, ks, lane);
#pragma unroll
            for (int u = 0; u < U; ++u) {
              sv[u] = mfma16(qfr, kf[u][ks], sv[u]);
              dpv[u] = mfma16(ofr, vf[u][ks], dpv[u]);
            }
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int ql = 16 * t + 4 * g + r;
            const int q = q0 + ql;
            const float lq = ldsL[ql], dq = ldsD[ql];
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const bool ok = (key[u] < klim) & (q < a.Lq) & (!causal | (key[u] <= q));  // (no short circuit: no branches)
              const float pv = masked_exp2(sv[u][r] * c - lq, ok);
              p[u][tt][r] = pv;
              ds[u][tt][r] = pv * (dpv[u][r] - dq);
            }
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          pf[u][s2] = pack8(p[u][0][0], p[u][0][1], p[u][0][2], p[u][0][3], p[u][1][0], p[u][1][1],
                            p[u][1][2], p[u][1][3]);
          dsf[u][s2] = pack8(ds[u][0][0], ds[u][0][1], ds[u][0][2], ds[u][0][3], ds[u][1][0],
                             ds[u][1][1], ds[u][1][2], ds[u][1][3]);
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
        for (int dt = 0; dt < T::DT; ++dt) {
          const short8_t ot = T::frag_tr(ldsO, s2, dt, lane);
          const short8_t qt = T::frag_tr(ldsQ, s2, dt, lane);
#pragma unroll
          for (int u = 0; u < U; ++u) {
            dv[u][dt] = mfma16(ot, pf[u][s2], dv[u][dt]);
            dk[u][dt] = mfma16(qt, dsf[u][s2], dk[u][dt]);
          }
        }
      }
      __syncthreads();
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool ok = key[u] < a.Lk;
    bf16_t* dkp = a.dk + b * a.dk_sb + (long long)key[u] * a.dk_sl + h * a.dk_sh;
    bf16_t* dvp = a.dv + b * a.dv_sb + (long long)key[u] * a.dv_sl + h * a.dv_sh;
    uint32_t lo[T::DT], hi[T::DT];
#pragma unroll
    for (int dt = 0; dt < T::DT; ++dt) pack_acc(dk[u][dt], a.scale, lo[dt], hi[dt]);
    store_row16<T::DT>(dkp, lo, hi, g, ok);
#pragma unroll
    for (int dt = 0; dt < T::DT; ++dt) pack_acc(dv[u][dt], 1.f, lo[dt], hi[dt]);
    store_row16<T::DT>(dvp, lo, hi, g, ok);
  }
}

// ============================================================================ dQ
// 4 waves, U 16-query subtiles per wave (64 U queries per workgroup): every
// K / V fragment read from LDS feeds U MFMAs.
template <int HD, int U>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void attn_bwd_dq_kernel(AttnArgs a) {
  using T = ATile<HD>;
  constexpr int QBW = 64 * U;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ldsK = smem;
  char* ldsV = smem + T::BYTES;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, cl = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // (wave-uniform: scalar branches)
  int xb, h, b;
  attn_coords(a, xb, h, b);
  const int q0 = xb * QBW;
  int qrow[U];
#pragma unroll
  for (int u = 0; u < U; ++u) qrow[u] = q0 + 16 * (U * w + u) + cl;
  int klim;
  float scl;
  bool causal;
  key_window(a, b, klim, scl, causal);
  if (causal) klim = min(klim, q0 + QBW);
  const float c = scl * LOG2E;
  short8_t qf[U][T::KS], of[U][T::KS];
  float L[U], D[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool qvalid = qrow[u] < a.Lq;
    const int qr = min(qrow[u], a.Lq - 1);
    const bf16_t* qp = a.q + b * a.q_sb + (long long)qr * a.q_sl + h * a.q_sh;
    const bf16_t* dop = a.dout + b * a.do_sb + (long long)qr * a.do_sl + h * a.do_sh;
#pragma unroll
    for (int s = 0; s < T::KS; ++s) {
      qf[u][s] = gfrag<HD>(qp, qvalid, s, lane);
      of[u][s] = gfrag<HD>(dop, qvalid, s, lane);
    }
    const long long bh = ((long long)b * a.H + h) * a.Lq + qr;
    L[u] = a.lse[bh];
    // delta = rowsum(dO * O) of this lane's query row, from the dO fragments
    // already in registers and the matching O fragments (the 4 lane groups g
    // hold disjoint head-dim slices); written for the dK/dV kernel, which runs
    // after this one -- no separate delta pass over O and dO
    float d = 0.f;
    const bf16_t* opr = a.o + b * a.o_sb + (long long)qr * a.o_sl + h * a.o_sh;
#pragma unroll
    for (int s = 0; s < T::KS; ++s) {
      const short8_t ov = gfrag<HD>(opr, qvalid, s, lane);
#pragma unroll
      for (int e = 0; e < 8; ++e) d += bf2f((bf16_t)of[u][s][e]) * bf2f((bf16_t)ov[e]);
    }
    d = rows_sum(d);
    if (qvalid && g == 0) a.delta[bh] = d;
    D[u] = d;
  }
  const bf16_t* kb = a.k + b * a.k_sb + h * a.k_sh;
  const bf16_t* vb = a.v + b * a.v_sb + h * a.v_sh;
  f32x4 dq[U][T::DT];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int i = 0; i < T::DT; ++i) dq[u][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // K / V of key block k0+KB in registers while block k0 is computed
  typename T::template Chunks<256> ck, cv;
  if (klim > 0) {
    T::template fetch<256>(ck, kb, a.k_sl, 0, a.Lk, tid);
    T::template fetch<256>(cv, vb, a.v_sl, 0, a.Lk, tid);
  }
  for (int k0 = 0; k0 < klim; k0 += KB) {
    T::template put<256>(ldsK, ck, tid);
    T::template put<256>(ldsV, cv, tid);
    __syncthreads();
    if (k0 + KB < klim) {
      T::template fetch<256>(ck, kb, a.k_sl, k0 + KB, a.Lk, tid);
      T::template fetch<256>(cv, vb, a.v_sl, k0 + KB, a.Lk, tid);
    }
    short8_t dsf[U][2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      f32x4 ds[U][2];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const int t = 2 * s2 + tt;
        f32x4 sv[U], dpv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) sv[u] = dpv[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < T::KS; ++ks) {
          const short8_t kfr = T::frag_row(ldsK, 16 * t, ks, lane);
          const short8_t vfr = T::frag_row(ldsV, 16 * t, ks, lane);
#pragma unroll
          for (int u = 0; u < U; ++u) {
            sv[u] = mfma16(kfr, qf[u][ks], sv[u]);
            dpv[u] = mfma16(vfr, of[u][ks], dpv[u]);
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = k0 + 16 * t + 4 * g + r;
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const bool ok = (qrow[u] < a.Lq) & (key < klim) & (!causal | (key <= qrow[u]));  // (no short circuit)
            const float pv = masked_exp2(sv[u][r] * c - L[u], ok);
            ds[u][tt][r] = pv * (dpv[u][r] - D[u]);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        dsf[u][s2] = pack8(ds[u][0][0], ds[u][0][1], ds[u][0][2], ds[u][0][3], ds[u][1][0],
                           ds[u][1][1], ds[u][1][2], ds[u][1][3]);
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
      for (int dt = 0; dt < T::DT; ++dt) {
        const short8_t kt = T::frag_tr(ldsK, s2, dt, lane);
#pragma unroll
        for (int u = 0; u < U; ++u) dq[u][dt] = mfma16(kt, dsf[u][s2], dq[u][dt]);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    bf16_t* dqp = a.dq + b * a.dq_sb + (long long)qrow[u] * a.dq_sl + h * a.dq_sh;
    uint32_t lo[T::DT], hi[T::DT];
#pragma unroll
    for (int dt = 0; dt < T::DT; ++dt) pack_acc(dq[u][dt], a.scale, lo[dt], hi[dt]);
    store_row16<T::DT>(dqp, lo, hi, g, qrow[u] < a.Lq);
  }
}

// ============================================================================ backward, long sequences, pipelined
// hd = 64, the dQ / dK,dV kernels above with their streamed operand tiles in
// an NS-slot LDS-DMA ring (as attn_fwd_pipe_kernel): dK/dV streams Q, dO and
// the tile's lse / delta (one 4-byte-per-lane DMA per wave: wave 0 lse, wave 1
// delta, the others a scratch copy so every wave's DMA count is the same),
// dQ streams K and V.
// e5m2 copy of a 4-wave workgroup's gradient tile (the hd-64 pipelined
// backward kernels): lane (g, cl) of wave w holds rows rows[u] (u < U),
// columns 16 dt + 4 g .. +3 of one head. Writes the e5m2 values of the
// bf16-rounded x * sc, records their |max| (one atomic per wave) and, when
// part != null, the columns' sums over the workgroup's valid rows into
// part[0..63] (shuffles over the 16 rows of a lane group, then the 4 waves
// through `red`, 1 KiB of LDS). Every thread of the workgroup must call it.
template <int U>
__device__ __forceinline__ void attn_emit_g8(const f32x4 (&x)[U][4], float sc, const int (&rows)[U],
                                             int nrows, uint8_t* base8, long long sl, float s8,
                                             unsigned* amax, float* part, float* red, int lane,
                                             int w) {
  const int g = lane >> 4;
  float cs[4][4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) cs[dt][r] = 0.f;
  float am = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool ok = rows[u] < nrows;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = ok ? bf2f(f2bf(x[u][dt][r] * sc)) : 0.f;
        cs[dt][r] += v[r];
        am = fmaxf(am, fabsf(v[r]));
      }
      int w8 = pack2_e5m2c<false>(v[0] * s8, v[1] * s8, 0);
      w8 = pack2_e5m2c<true>(v[2] * s8, v[3] * s8, w8);
      if (ok) *reinterpret_cast<int*>(base8 + (long long)rows[u] * sl + 16 * dt + 4 * g) = w8;
    }
  }
#pragma unroll
  for (int sh = 32; sh >= 1; sh >>= 1) am = fmaxf(am, __shfl_xor(am, sh, 64));
  if (lane == 0) atomic_amax(amax_word(amax, blockIdx.x + 5 * blockIdx.y + 11 * blockIdx.z + w), am);
  if (!part) return;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int sh = 1; sh < 16; sh <<= 1) cs[dt][r] += __shfl_xor(cs[dt][r], sh, 64);
  __syncthreads();  // (the caller's LDS reads are done)
  if ((lane & 15) == 0) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[w * 64 + 16 * dt + 4 * g + r] = cs[dt][r];
  }
  __syncthreads();
  if (threadIdx.x < 64)
    part[threadIdx.x] = red[threadIdx.x] + red[64 + threadIdx.x] + red[128 + threadIdx.x] +
                        red[192 + threadIdx.x];
  __syncthreads();
}

template <int U, int NS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void attn_bwd_dkdv_pipe_kernel(AttnArgs a) {
  constexpr int HD = 64;
  using T = ATile<HD>;
  using G = Glds<true, 64, 4>;
  constexpr int KBW = 64 * U;
  constexpr int SLOT = 2 * T::BYTES + 3 * 256;  // Q, dO images, lse, delta, scratch
  constexpr int PT = 2 * G::P + 1;
  static_assert(NS >= 3, "ring: refilled, being read, landed");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, cl = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  int xb, h, b;
  attn_coords(a, xb, h, b);
  const int k0 = xb * KBW;
  int key[U];
#pragma unroll
  for (int u = 0; u < U; ++u) key[u] = k0 + 16 * (U * w + u) + cl;
  int klim;
  float scl;
  bool causal;
  key_window(a, b, klim, scl, causal);
  const float c = scl * LOG2E;
  const int kmaxw = k0 + 16 * U * (w + 1) - 1;  // the wave's last key

  f32x4 dk[U][T::DT], dv[U][T::DT];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int i = 0; i < T::DT; ++i) dk[u][i] = dv[u][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int qstart = causal ? (k0 / 64) * 64 : 0;
  const int nqt = k0 < klim && qstart < a.Lq ? (a.Lq - qstart + 63) / 64 : 0;
  short8_t kf[U][T::KS], vf[U][T::KS];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int krow = min(key[u], a.Lk - 1);
    const bf16_t* kp = a.k + b * a.k_sb + (long long)krow * a.k_sl + h * a.k_sh;
    const bf16_t* vp = a.v + b * a.v_sb + (long long)krow * a.v_sl + h * a.v_sh;
#pragma unroll
    for (int s = 0; s < T::KS; ++s) {
      kf[u][s] = gfrag<HD>(kp, key[u] < a.Lk, s, lane);
      vf[u][s] = gfrag<HD>(vp, key[u] < a.Lk, s, lane);
    }
  }
  const bf16_t* qb = a.q + b * a.q_sb + h * a.q_sh;
  const bf16_t* ob = a.dout + b * a.do_sb + h * a.do_sh;
  const float* vecs = (w == 1 ? a.delta : a.lse) + ((long long)b * a.H + h) * a.Lq;
  const int voff = 2 * T::BYTES + 256 * min(w, 2);
  G gs;
  gs.init(w, lane);
  auto issue = [&](int it) {
    const int q0 = qstart + 64 * it;
    char* slot = smem + (it % NS) * SLOT;
    gs.issue(qb, (int)a.q_sl, a.Lq, HD, q0, 0, slot, w);
    gs.issue(ob, (int)a.do_sl, a.Lq, HD, q0, 0, slot + T::BYTES, w);
    __builtin_amdgcn_global_load_lds((const void*)(vecs + min(q0 + lane, a.Lq - 1)),
                                     (__attribute__((address_space(3))) void*)(slot + voff), 4, 0, 0);
  };
  // prologue tiles issued unconditionally (clamped rows, never read) so the
  // DMA count behind the K / V fragment loads is a constant
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) issue(s);
  wait_vmcnt_known<(NS - 1) * PT>();

  uint32_t roff[T::KS], troff[T::DT];  // lane parts of the fragment addresses
#pragma unroll
  for (int ks = 0; ks < T::KS; ++ks) roff[ks] = T::row_off(ks, lane);
#pragma unroll
  for (int dt = 0; dt < T::DT; ++dt) troff[dt] = T::tr_off(dt, lane);
  for (int it = 0; it < nqt; ++it) {
    wait_tiles<PT, NS - 2>(min(NS - 2, nqt - 1 - it));
    lds_barrier();
    if (it + NS - 1 < nqt) issue(it + NS - 1);
    const uint32_t slotQ = (uint32_t)(uintptr_t)smem + (uint32_t)((it % NS) * SLOT);
    const uint32_t slotO = slotQ + T::BYTES;
    const char* ldsL = smem + (it % NS) * SLOT + 2 * T::BYTES;  // lse, then delta (64 floats each)
    const int q0 = qstart + 64 * it;
    // untracked LDS reads with counted waits (a tracked read would get a
    // vmcnt(0) for the DMA in flight); the next 16-query tile's Q / dO
    // fragments and lse / delta are requested before this one is used; row
    // bases in the DS offset field
    uint32_t qra[T::KS], ora[T::KS];
#pragma unroll
    for (int ks = 0; ks < T::KS; ++ks) {
      qra[ks] = slotQ + roff[ks];
      ora[ks] = slotO + roff[ks];
    }
    const uint32_t lda4 = (uint32_t)(uintptr_t)ldsL + 16 * g;
    short8_t pf[U][2], dsf[U][2];
    short8_t qfr[2][T::KS], ofr[2][T::KS];
    f32x4 l4[2], d4[2];
#pragma unroll
    for (int ks = 0; ks < T::KS; ++ks) {
      qfr[0][ks] = T::template frag_row_at<0>(qra[ks]);
      ofr[0][ks] = T::template frag_row_at<0>(ora[ks]);
    }
    l4[0] = __builtin_bit_cast(f32x4, lds_read_b128_at<0>(lda4));
    d4[0] = __builtin_bit_cast(f32x4, lds_read_b128_at<256>(lda4));
    constexpr int RPT = 2 * T::KS + 2;  // LDS reads per 16-query tile
    f32x4 p[U][2], ds[U][2];
    static_for<4>([&](auto tc) {
      constexpr int t = decltype(tc)::value, tt = t & 1, s2 = t >> 1, cb = t & 1, nb = cb ^ 1;
      if constexpr (t < 3) {
#pragma unroll
        for (int ks = 0; ks < T::KS; ++ks) {
          qfr[nb][ks] = T::template frag_row_at<16 * (t + 1)>(qra[ks]);
          ofr[nb][ks] = T::template frag_row_at<16 * (t + 1)>(ora[ks]);
        }
        l4[nb] = __builtin_bit_cast(f32x4, lds_read_b128_at<64 * (t + 1)>(lda4));
        d4[nb] = __builtin_bit_cast(f32x4, lds_read_b128_at<256 + 64 * (t + 1)>(lda4));
        lgkm_wait<RPT>();
      } else {
        lgkm_wait<0>();
      }
#pragma unroll
      for (int ks = 0; ks < T::KS; ++ks) {
        tie(qfr[cb][ks]);
        tie(ofr[cb][ks]);
      }
      tie(l4[cb]);
      tie(d4[cb]);
      f32x4 sv[U], dpv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) sv[u] = dpv[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < T::KS; ++ks) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          sv[u] = mfma16(qfr[cb][ks], kf[u][ks], sv[u]);
          dpv[u] = mfma16(ofr[cb][ks], vf[u][ks], dpv[u]);
        }
      }
      // the whole 16-query subtile valid for every key of the wave (a
      // wave-uniform test): no per-element masking
      const int qs0 = q0 + 16 * t;
      const bool full = kmaxw < klim && qs0 + 15 < a.Lq && (!causal || kmaxw <= qs0);
      if (full) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const float pv = fast_exp2(sv[u][r] * c - l4[cb][r]);
            p[u][tt][r] = pv;
            ds[u][tt][r] = pv * (dpv[u][r] - d4[cb][r]);
          }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = qs0 + 4 * g + r;
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const bool ok = (key[u] < klim) & (q < a.Lq) & (!causal | (key[u] <= q));  // (no short circuit: no branches)
            const float pv = masked_exp2(sv[u][r] * c - l4[cb][r], ok);
            p[u][tt][r] = pv;
            ds[u][tt][r] = pv * (dpv[u][r] - d4[cb][r]);
          }
        }
      }
      if constexpr (tt == 1) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          pf[u][s2] = pack8(p[u][0][0], p[u][0][1], p[u][0][2], p[u][0][3], p[u][1][0], p[u][1][1],
                            p[u][1][2], p[u][1][3]);
          dsf[u][s2] = pack8(ds[u][0][0], ds[u][0][1], ds[u][0][2], ds[u][0][3], ds[u][1][0],
                             ds[u][1][1], ds[u][1][2], ds[u][1][3]);
        }
      }
    });
    // dV^T += dO^T P, dK^T += Q^T dS: transposed fragments, next requested
    // before this one is used
    uint32_t otra[T::DT], qtra[T::DT];
#pragma unroll
    for (int dt = 0; dt < T::DT; ++dt) {
      otra[dt] = slotO + troff[dt];
      qtra[dt] = slotQ + troff[dt];
    }
    short4_t olo[2], ohi[2], qlo[2], qhi[2];
    T::template frag_tr_at<0>(otra[0], olo[0], ohi[0]);
    T::template frag_tr_at<0>(qtra[0], qlo[0], qhi[0]);
    static_for<2 * T::DT>([&](auto ic) {
      constexpr int i = decltype(ic)::value, s2 = i / T::DT, dt = i % T::DT, cb = i & 1, nb = cb ^ 1;
      if constexpr (i + 1 < 2 * T::DT) {
        T::template frag_tr_at<(i + 1) / T::DT>(otra[(i + 1) % T::DT], olo[nb], ohi[nb]);
        T::template frag_tr_at<(i + 1) / T::DT>(qtra[(i + 1) % T::DT], qlo[nb], qhi[nb]);
        lgkm_wait<4>();
      } else {
        lgkm_wait<0>();
      }
      tie(olo[cb]);
      tie(ohi[cb]);
      tie(qlo[cb]);
      tie(qhi[cb]);
      const short8_t ot = cat4(olo[cb], ohi[cb]);
      const short8_t qt = cat4(qlo[cb], qhi[cb]);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        dv[u][dt] = mfma16(ot, pf[u][s2], dv[u][dt]);
        dk[u][dt] = mfma16(qt, dsf[u][s2], dk[u][dt]);
      }
    });
  }
  wait_vmcnt<0>();
  if (!a.skip_bf16) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool ok = key[u] < a.Lk;
    bf16_t* dkp = a.dk + b * a.dk_sb + (long long)key[u] * a.dk_sl + h * a.dk_sh;
    bf16_t* dvp = a.dv + b * a.dv_sb + (long long)key[u] * a.dv_sl + h * a.dv_sh;
    uint32_t lo[T::DT], hi[T::DT];
#pragma unroll
    for (int dt = 0; dt < T::DT; ++dt) pack_acc(dk[u][dt], a.scale, lo[dt], hi[dt]);
    store_row16<T::DT>(dkp, lo, hi, g, ok);
#pragma unroll
    for (int dt = 0; dt < T::DT; ++dt) pack_acc(dv[u][dt], 1.f, lo[dt], hi[dt]);
    store_row16<T::DT>(dvp, lo, hi, g, ok);
  }
  }
  if (a.dk8) {  // e5m2 dK / dV (+ amax, + bias-gradient partials)
    const float s8 = a.sg8[0];
    float* red = reinterpret_cast<float*>(smem);
    float* prow = a.cs_part ? a.cs_part + ((long long)b * a.cs_np + xb) * a.cs_ld + h * 64 : nullptr;
    attn_emit_g8<U>(dk, a.scale, key, a.Lk, a.dk8 + b * a.dk_sb + h * a.dk_sh, a.dk_sl, s8, a.amaxg8,
                    prow ? prow + a.cs_k : nullptr, red, lane, w);
    attn_emit_g8<U>(dv, 1.f, key, a.Lk, a.dv8 + b * a.dv_sb + h * a.dv_sh, a.dv_sl, s8, a.amaxg8,
                    prow ? prow + a.cs_v : nullptr, red, lane, w);
  }
}

template <int U, int NS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void attn_bwd_dq_pipe_kernel(AttnArgs a) {
  constexpr int HD = 64;
  using T = ATile<HD>;
  using G = Glds<true, 64, 4>;
  constexpr int QBW = 64 * U;
  constexpr int SLOT = 2 * T::BYTES;
  constexpr int PT = 2 * G::P;
  static_assert(NS >= 3, "ring: refilled, being read, landed");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, cl = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  int xb, h, b;
  attn_coords(a, xb, h, b);
  const int q0 = xb * QBW;
  int qrow[U];
#pragma unroll
  for (int u = 0; u < U; ++u) qrow[u] = q0 + 16 * (U * w + u) + cl;
  const int qminw = q0 + 16 * U * w;  // the wave's first query
  int klim;
  float scl;
  bool causal;
  key_window(a, b, klim, scl, causal);
  if (causal) klim = min(klim, q0 + QBW);
  const float c = scl * LOG2E;
  const int nkt = (klim + 63) / 64;
  const bf16_t* kb = a.k + b * a.k_sb + h * a.k_sh;
  const bf16_t* vb = a.v + b * a.v_sb + h * a.v_sh;
  short8_t qf[U][T::KS], of[U][T::KS];
  float L[U], D[U];
  short8_t ov[U][T::KS];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool qvalid = qrow[u] < a.Lq;
    const int qr = min(qrow[u], a.Lq - 1);
    const bf16_t* qp = a.q + b * a.q_sb + (long long)qr * a.q_sl + h * a.q_sh;
    const bf16_t* dop = a.dout + b * a.do_sb + (long long)qr * a.do_sl + h * a.do_sh;
#pragma unroll
    for (int s = 0; s < T::KS; ++s) {
      qf[u][s] = gfrag<HD>(qp, qvalid, s, lane);
      of[u][s] = gfrag<HD>(dop, qvalid, s, lane);
    }
    const long long bh = ((long long)b * a.H + h) * a.Lq + qr;
    L[u] = a.lse[bh];
    const bf16_t* opr = a.o + b * a.o_sb + (long long)qr * a.o_sl + h * a.o_sh;
#pragma unroll
    for (int s = 0; s < T::KS; ++s) ov[u][s] = gfrag<HD>(opr, qvalid, s, lane);
  }
  G gs;
  gs.init(w, lane);
  auto issue = [&](int kt) {
    char* slot = smem + (kt % NS) * SLOT;
    gs.issue(kb, (int)a.k_sl, a.Lk, HD, 64 * kt, 0, slot, w);
    gs.issue(vb, (int)a.v_sl, a.Lk, HD, 64 * kt, 0, slot + T::BYTES, w);
  };
  // prologue tiles issued unconditionally (clamped rows, never read) so the
  // DMA count behind the Q / dO / O / lse loads is a constant
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) issue(s);
  wait_vmcnt_known<(NS - 1) * PT>();
  // delta = rowsum(dO * O) of the lane's query row (the 4 lane groups hold
  // disjoint head-dim slices), written for the dK/dV kernel, which runs after
#pragma unroll
  for (int u = 0; u < U; ++u) {
    float d = 0.f;
#pragma unroll
    for (int s = 0; s < T::KS; ++s)
#pragma unroll
      for (int e = 0; e < 8; ++e) d += bf2f((bf16_t)of[u][s][e]) * bf2f((bf16_t)ov[u][s][e]);
    d = rows_sum(d);
    if (qrow[u] < a.Lq && g == 0) a.delta[((long long)b * a.H + h) * a.Lq + qrow[u]] = d;
    D[u] = d;
  }
  f32x4 dq[U][T::DT];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int i = 0; i < T::DT; ++i) dq[u][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint32_t roff[T::KS], troff[T::DT];  // lane parts of the fragment addresses
#pragma unroll
  for (int ks = 0; ks < T::KS; ++ks) roff[ks] = T::row_off(ks, lane);
#pragma unroll
  for (int dt = 0; dt < T::DT; ++dt) troff[dt] = T::tr_off(dt, lane);

  for (int kt = 0; kt < nkt; ++kt) {
    wait_tiles<PT, NS - 2>(min(NS - 2, nkt - 1 - kt));
    lds_barrier();
    if (kt + NS - 1 < nkt) issue(kt + NS - 1);
    const uint32_t slotK = (uint32_t)(uintptr_t)smem + (uint32_t)((kt % NS) * SLOT);
    const uint32_t slotV = slotK + T::BYTES;
    const int k0 = 64 * kt;
    // untracked LDS reads with counted waits, next 16-key tile requested
    // before this one is used; row bases in the DS offset field
    uint32_t kra[T::KS], vra[T::KS];
#pragma unroll
    for (int ks = 0; ks < T::KS; ++ks) {
      kra[ks] = slotK + roff[ks];
      vra[ks] = slotV + roff[ks];
    }
    short8_t dsf[U][2];
    short8_t kfr[2][T::KS], vfr[2][T::KS];
#pragma unroll
    for (int ks = 0; ks < T::KS; ++ks) {
      kfr[0][ks] = T::template frag_row_at<0>(kra[ks]);
      vfr[0][ks] = T::template frag_row_at<0>(vra[ks]);
    }
    constexpr int RPT = 2 * T::KS;
    f32x4 ds[U][2];
    static_for<4>([&](auto tc) {
      constexpr int t = decltype(tc)::value, tt = t & 1, s2 = t >> 1, cb = t & 1, nb = cb ^ 1;
      if constexpr (t < 3) {
#pragma unroll
        for (int ks = 0; ks < T::KS; ++ks) {
          kfr[nb][ks] = T::template frag_row_at<16 * (t + 1)>(kra[ks]);
          vfr[nb][ks] = T::template frag_row_at<16 * (t + 1)>(vra[ks]);
        }
        lgkm_wait<RPT>();
      } else {
        lgkm_wait<0>();
      }
#pragma unroll
      for (int ks = 0; ks < T::KS; ++ks) {
        tie(kfr[cb][ks]);
        tie(vfr[cb][ks]);
      }
      f32x4 sv[U], dpv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) sv[u] = dpv[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < T::KS; ++ks) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          sv[u] = mfma16(kfr[cb][ks], qf[u][ks], sv[u]);
          dpv[u] = mfma16(vfr[cb][ks], of[u][ks], dpv[u]);
        }
      }
      // the whole 16-key subtile valid for every query of the wave (a
      // wave-uniform test): no per-element masking
      const int ks0 = k0 + 16 * t;
      const bool full = qminw + 16 * U <= a.Lq && ks0 + 15 < klim && (!causal || ks0 + 15 <= qminw);
      if (full) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int u = 0; u < U; ++u)
            ds[u][tt][r] = fast_exp2(sv[u][r] * c - L[u]) * (dpv[u][r] - D[u]);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = ks0 + 4 * g + r;
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const bool ok = (qrow[u] < a.Lq) & (key < klim) & (!causal | (key <= qrow[u]));  // (no short circuit)
            const float pv = masked_exp2(sv[u][r] * c - L[u], ok);
            ds[u][tt][r] = pv * (dpv[u][r] - D[u]);
          }
        }
      }
      if constexpr (tt == 1) {
#pragma unroll
        for (int u = 0; u < U; ++u)
          dsf[u][s2] = pack8(ds[u][0][0], ds[u][0][1], ds[u][0][2], ds[u][0][3], ds[u][1][0],
                             ds[u][1][1], ds[u][1][2], ds[u][1][3]);
      }
    });
    uint32_t ktra[T::DT];
#pragma unroll
    for (int dt = 0; dt < T::DT; ++dt) ktra[dt] = slotK + troff[dt];
    short4_t klo[2], khi[2];
    T::template frag_tr_at<0>(ktra[0], klo[0], khi[0]);
    static_for<2 * T::DT>([&](auto ic) {
      constexpr int i = decltype(ic)::value, s2 = i / T::DT, dt = i % T::DT, cb = i & 1, nb = cb ^ 1;
      if constexpr (i + 1 < 2 * T::DT) {
        T::template frag_tr_at<(i + 1) / T::DT>(ktra[(i + 1) % T::DT], klo[nb], khi[nb]);
        lgkm_wait<2>();
      } else {
        lgkm_wait<0>();
      }
      tie(klo[cb]);
      tie(khi[cb]);
      const short8_t kt2 = cat4(klo[cb], khi[cb]);
#pragma unroll
      for (int u = 0; u < U; ++u) dq[u][dt] = mfma16(kt2, dsf[u][s2], dq[u][dt]);
    });
  }
  wait_vmcnt<0>();
  if (!a.skip_bf16) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    bf16_t* dqp = a.dq + b * a.dq_sb + (long long)qrow[u] * a.dq_sl + h * a.dq_sh;
    uint32_t lo[T::DT], hi[T::DT];
#pragma unroll
    for (int dt = 0; dt < T::DT; ++dt) pack_acc(dq[u][dt], a.scale, lo[dt], hi[dt]);
    store_row16<T::DT>(dqp, lo, hi, g, qrow[u] < a.Lq);
  }
  }
  if (a.dq8) {  // e5m2 dQ (+ amax, + bias-gradient partials)
    float* prow = a.cs_part ? a.cs_part + ((long long)b * a.cs_np + xb) * a.cs_ld + h * 64 + a.cs_q
                            : nullptr;
    attn_emit_g8<U>(dq, a.scale, qrow, a.Lq, a.dq8 + b * a.dq_sb + h * a.dq_sh, a.dq_sl, a.sg8[0],
                    a.amaxg8, prow, reinterpret_cast<float*>(smem), lane, w);
  }
}

// ============================================================================ fused backward, short sequences
// Lq, Lk <= 128: one workgroup (8 waves) per (batch, head) computes dQ, dK
// and dV together, with delta = rowsum(dO*O) computed in the prologue.
// Phase 1 (key rows on lanes, wave w owns keys 16w..16w+15): S^T and dP^T
// from the Q / dO tiles in LDS and the wave's K / V fragments in registers,
// P recomputed from the forward log-sum-exp, dS = P (dP - delta); dV^T and
// dK^T accumulate over all queries. dS is then written as bf16 into the LDS
// the Q / dO tiles used: a [key][query] image whose transposing read is
// exactly the B-operand layout of phase 2. Phase 2 (query rows on lanes,
// wave w owns queries 16w..16w+15): dQ^T = K^T dS^T.
// Versus the three-kernel path (delta, dK/dV, dQ): every tile is read from
// HBM once and there is one launch instead of three.
// U: 16-key (phase 1) / 16-query (phase 2) subtiles per wave, 8 / U waves.
// U = 2 reads every Q / dO / K fragment from LDS once for two MFMAs (the
// U = 1 loops issue one LDS read per MFMA).
// dS^T image of the fused backward: 128 key rows x 128 queries (bf16, 256-B
// rows). ATile<128>'s 32-byte segment swizzle (segment ^ row & 7) keeps the
// transposing dQ-phase reads conflict-free, but the key-row-per-lane 8-byte
// stores of a 16-lane group (one row each, the same column) then land on only
// 4 bank positions (a 256-B row is 0 mod 32 banks): 4-way conflicts. Rows with
// bit 3 set also swap the 16-byte halves of each segment: 2-way for the stores,
// the reads (8 consecutive rows per 32-lane half, bit 3 constant) unchanged.
struct DsImg {
  static constexpr int RB = 256;
  __device__ static __forceinline__ int off(int row, int byte) {
    const int seg = (byte >> 5) ^ (row & 7);
    return row * RB + (seg << 5) + ((byte & 31) ^ (((row >> 3) & 1) << 4));
  }
  // ATile<128>::frag_tr with this image's offsets
  __device__ static __forceinline__ short8_t frag_tr(const char* lds, int s2, int dt, int lane) {
    const int g = lane >> 4, w = lane & 15, q = w >> 2, p = w & 3;
    const int r1 = 32 * s2 + 4 * g + q;
    const int byte = (16 * dt + 4 * p) * 2;
    return cat4(lds_read_tr(lds + off(r1, byte)), lds_read_tr(lds + off(r1 + 16, byte)));
  }
};

// dO tile of the fused backward with the output-projection dgrad (FDO):
// dO_bh [128 x 64] = dY_b [128 rows, d] @ Wo[:, 64 h .. 64 h + 63], K = d,
// on 8 waves as 4 x 2 of 32 x 32 -- the main loop of gemm_impl.h's
// gemm_kernel (3 LDS-DMA stages of 64-deep K tiles, swapped-operand MFMAs,
// the same k order per element as the standalone NN dgrad, so the bf16 dO is
// bitwise that kernel's). Uses smem[0, 3 * 24 KiB); returns the accumulators.
constexpr int FDO_STAGES = 3, FDO_SB = (128 + 64) * BK * 2;
__device__ __forceinline__ void fdo_tile(const AttnArgs& a, int b, int h, char* smem, int wid,
                                         int lane, f32x4 (&acc)[2][2]) {
  constexpr int NW = 8, BM = 128, BN = 64, WN = 2, TM = 2, TN = 2, STAGES = FDO_STAGES;
  constexpr int A_BYTES = BM * BK * 2, SB = FDO_SB;
  using GA = Glds<true, BM, NW>;
  using GB = Glds<false, BN, NW>;
  constexpr int PT = GA::P + GB::P;
  const int wm = wid / WN, wn = wid % WN;
  const int K = a.fdo_d;
  const bf16_t* Y = reinterpret_cast<const bf16_t*>(a.fdo_dy) + (size_t)b * a.Lq * a.fdo_ldy;
  const bf16_t* W = reinterpret_cast<const bf16_t*>(a.fdo_w) + 64 * h;
  GA ga;
  GB gb;
  ga.init(wid, lane);
  gb.init(wid, lane);
  const int nk = K / BK;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < STAGES; ++st) {
    if (st < nk) {
      ga.issue(Y, a.fdo_ldy, a.Lq, K, 0, st * BK, smem + st * SB, wid);
      gb.issue(W, a.fdo_ldw, BN, K, 0, st * BK, smem + st * SB + A_BYTES, wid);
    }
  }
  const int abase = wm * (BM / 4), bbase = wn * (BN / WN);
  short8_t fa0[TM], fb0[TN], fa1[TM], fb1[TN];
  if (nk >= STAGES)
    wait_vmcnt<(STAGES - 1) * PT>();
  else
    wait_vmcnt<0>();
  lds_barrier();
#pragma unroll
  for (int i = 0; i < TM; ++i) fa0[i] = frag<true, BM>(smem, abase + 16 * i, 0, lane);
#pragma unroll
  for (int j = 0; j < TN; ++j) fb0[j] = frag<false, BN>(smem + A_BYTES, bbase + 16 * j, 0, lane);
  constexpr int STEP_OPS = TM * frag_ops<true>() + TN * frag_ops<false>();
  auto kstep = [&](int kt, auto modec) {
    constexpr int MODE = decltype(modec)::value;
    const char* st = smem + (kt % STAGES) * SB;
#pragma unroll
    for (int i = 0; i < TM; ++i) fa1[i] = frag<true, BM>(st, abase + 16 * i, 1, lane);
#pragma unroll
    for (int j = 0; j < TN; ++j) fb1[j] = frag<false, BN>(st + A_BYTES, bbase + 16 * j, 1, lane);
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
      if constexpr (MODE >= 2) wait_vmcnt<(STAGES - 2) * PT>();
      else wait_vmcnt<0>();
      lds_barrier();
      const char* nx = smem + ((kt + 1) % STAGES) * SB;
      if constexpr (MODE == 3) {
        char* ns = smem + (kt % STAGES) * SB;
        ga.issue(Y, a.fdo_ldy, a.Lq, K, 0, (kt + STAGES) * BK, ns, wid);
        gb.issue(W, a.fdo_ldw, BN, K, 0, (kt + STAGES) * BK, ns + A_BYTES, wid);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) fa0[i] = frag<true, BM>(nx, abase + 16 * i, 0, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb0[j] = frag<false, BN>(nx + A_BYTES, bbase + 16 * j, 0, lane);
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
  int kt = 0;
  for (; kt + STAGES < nk; ++kt) kstep(kt, std::integral_constant<int, 3>{});
  if (kt + STAGES - 1 < nk && kt + 1 < nk) kstep(kt++, std::integral_constant<int, 2>{});
  for (; kt + 1 < nk; ++kt) kstep(kt, std::integral_constant<int, 1>{});
  if (kt < nk) kstep(kt, std::integral_constant<int, 0>{});
  lds_barrier();  // the stages are free for the attention's images
}

template <int HD, int U, bool FDO = false>
__global__ __launch_bounds__(512 / U) __attribute__((amdgpu_waves_per_eu(U == 1 ? (HD <= 64 ? 4 : 2) : 2))) void attn_bwd_fused_kernel(AttnArgs a) {
  static_assert(!FDO || (HD == 64 && U == 1), "in-kernel dO: hd 64, 8 waves");
  using T = ATile<HD>;
  using TS = DsImg;  // dS image: 128 key rows x 128 queries (bf16)
  constexpr int R = 128;
  constexpr int NT = 512 / U;  // threads
  constexpr int TB = R * T::RB;  // bytes of one 128-row tile image
  constexpr int SB = R * TS::RB;  // dS image bytes (32 KiB)
  constexpr int ALIAS = 2 * TB >= SB;  // dS fits over Q + dO
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ldsQ = smem;
  char* ldsO = smem + TB;
  char* ldsK = smem + 2 * TB;
  char* ldsS = ALIAS ? smem : smem + 3 * TB;
  float* ldsL = reinterpret_cast<float*>(smem + (ALIAS ? 3 * TB : 3 * TB + SB));
  float* ldsD = ldsL + R;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, cl = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // (wave-uniform: scalar branches)
  const int bh = a.xcd ? xcd_remap(blockIdx.x, gridDim.x) : blockIdx.x;
  const int b = bh / a.H, h = bh % a.H;
  int klim;
  float scl;
  bool causal;
  key_window(a, b, klim, scl, causal);
  const float c = scl * LOG2E;

  // ---- prologue. Every global load is issued before any is used (one
  // memory latency): this wave's K / V register fragments for phase 1, the
  // Q / dO / K tile chunks, O chunks for delta, and lse.
  TDG_STAMP(0);
  const bf16_t* qb = a.q + b * a.q_sb + h * a.q_sh;
  const bf16_t* ob = a.dout + b * a.do_sb + h * a.do_sh;
  const bf16_t* kbp = a.k + b * a.k_sb + h * a.k_sh;
  const bf16_t* obo = a.o + b * a.o_sb + h * a.o_sh;
  int key[U];
#pragma unroll
  for (int u = 0; u < U; ++u) key[u] = 16 * (U * w + u) + cl;
  short8_t kf[U][T::KS], vf[U][T::KS];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int krow = min(key[u], a.Lk - 1);
    const bf16_t* kp = kbp + (long long)krow * a.k_sl;
    const bf16_t* vp = a.v + b * a.v_sb + (long long)krow * a.v_sl + h * a.v_sh;
#pragma unroll
    for (int ks = 0; ks < T::KS; ++ks) {
      kf[u][ks] = gfrag<HD>(kp, key[u] < a.Lk, ks, lane);
      vf[u][ks] = gfrag<HD>(vp, key[u] < a.Lk, ks, lane);
    }
  }
  {
    constexpr int CPR = HD / 8;  // 16-byte chunks per row
    constexpr int TOTAL = R * CPR;
    constexpr int NI = (TOTAL + NT - 1) / NT;
    short8_t vq[NI], vo[NI], vk[NI], vx[NI];
    const short8_t z = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int id = tid + i * NT;
      const int row = id / CPR, cc = id % CPR;
      vq[i] = vo[i] = vk[i] = vx[i] = z;
      if constexpr (TOTAL % NT == 0) {  // (clamped rows, zeroed: no branch per load)
        const int rq = min(row, a.Lq - 1), rk = min(row, a.Lk - 1);
        vq[i] = ld8_or0(qb + (long long)rq * a.q_sl + cc * 8, row < a.Lq);
        if constexpr (!FDO) vo[i] = ld8_or0(ob + (long long)rq * a.do_sl + cc * 8, row < a.Lq);
        vx[i] = ld8_or0(obo + (long long)rq * a.o_sl + cc * 8, row < a.Lq);
        vk[i] = ld8_or0(kbp + (long long)rk * a.k_sl + cc * 8, row < a.Lk);
      } else {
        if (id < TOTAL && row < a.Lq) {
          vq[i] = *reinterpret_cast<const short8_t*>(qb + (long long)row * a.q_sl + cc * 8);
          if constexpr (!FDO) vo[i] = *reinterpret_cast<const short8_t*>(ob + (long long)row * a.do_sl + cc * 8);
          vx[i] = *reinterpret_cast<const short8_t*>(obo + (long long)row * a.o_sl + cc * 8);
        }
        if (id < TOTAL && row < a.Lk)
          vk[i] = *reinterpret_cast<const short8_t*>(kbp + (long long)row * a.k_sl + cc * 8);
      }
    }
    const float lse_v = (tid < R && tid < a.Lq) ? a.lse[((long long)b * a.H + h) * a.Lq + tid] : INFINITY;
    if constexpr (FDO) {
      // dO from the in-kernel output-projection dgrad (rows >= Lq zero, as
      // the loads above give them), into its image; then read back in the
      // chunk layout for delta
      f32x4 acc[2][2];
      fdo_tile(a, b, h, smem, w, lane, acc);
      const int wm = w / 2, wn = w % 2;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int m = 32 * wm + 16 * i + cl, n = 32 * wn + 16 * j + 4 * g;
          short4_t o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = m < a.Lq ? (short)f2bf(acc[i][j][r]) : (short)0;
          *reinterpret_cast<short4_t*>(ldsO + T::off(m, n * 2)) = o;
        }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int id = tid + i * NT;
        const int row = id / CPR, cc = id % CPR;
        if (id < TOTAL) vo[i] = *reinterpret_cast<const short8_t*>(ldsO + T::off(row, cc * 16));
      }
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int id = tid + i * NT;
      const int row = id / CPR, cc = id % CPR;
      if (id < TOTAL) {
        *reinterpret_cast<short8_t*>(ldsQ + T::off(row, cc * 16)) = vq[i];
        if constexpr (!FDO) *reinterpret_cast<short8_t*>(ldsO + T::off(row, cc * 16)) = vo[i];
        *reinterpret_cast<short8_t*>(ldsK + T::off(row, cc * 16)) = vk[i];
      }
      // delta[row] = sum_d dO * O: partial over this chunk, then over the
      // CPR consecutive lanes holding the row (xor shuffles)
      float d = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) d += bf2f((bf16_t)vo[i][e]) * bf2f((bf16_t)vx[i][e]);
#pragma unroll
      for (int o = 1; o < CPR; o <<= 1) d += __shfl_xor(d, o, 64);
      if (id < TOTAL && cc == 0) ldsD[row] = row < a.Lq ? d : 0.f;
    }
    if (tid < R) ldsL[tid] = lse_v;
  }
  __syncthreads();
  TDG_STAMP(1);

  // ---- phase 1: this wave's U x 16 keys against all queries
  f32x4 dk[U][T::DT], dv[U][T::DT];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int i = 0; i < T::DT; ++i) dk[u][i] = dv[u][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  // P and dS of [q = 16t + 4g + r][key], packed to bf16 pairs as produced
  uint32_t pk[U][8][2], dk2[U][8][2];
  const bool active = 16 * U * w < klim;  // wave-uniform
  if (active) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const bool live = 16 * t < a.Lq && (!causal || 16 * t + 15 >= 16 * U * w);  // uniform
      if (!live) {  // (no query of the tile attends to the wave's keys: P = dS = 0)
#pragma unroll
        for (int u = 0; u < U; ++u) pk[u][t][0] = pk[u][t][1] = dk2[u][t][0] = dk2[u][t][1] = 0u;
        continue;
      }
      f32x4 sv[U], dpv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) sv[u] = dpv[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < T::KS; ++ks) {
        const short8_t qfr = T::frag_row(ldsQ, 16 * t, ks, lane);
        const short8_t ofr = T::frag_row(ldsO, 16 * t, ks, lane);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          sv[u] = mfma16(qfr, kf[u][ks], sv[u]);
          dpv[u] = mfma16(ofr, vf[u][ks], dpv[u]);
        }
      }
      // lse / delta of queries 16t + 4g .. +3: one 16-byte LDS read each
      const f32x4 l4 = *reinterpret_cast<const f32x4*>(ldsL + 16 * t + 4 * g);
      const f32x4 d4 = *reinterpret_cast<const f32x4*>(ldsD + 16 * t + 4 * g);
      // every (query, key) of this 16-query tile valid for the wave's keys
      // (wave-uniform): no per-element masks
      const int kmaxw = 16 * U * (w + 1) - 1;
      const bool full = kmaxw < klim && 16 * t + 15 < a.Lq && (!causal || kmaxw <= 16 * t);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float pv[4], dv4[4];
        const bool kvalid = key[u] < klim;
        if (full) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            pv[r] = fast_exp2(sv[u][r] * c - l4[r]);
            dv4[r] = pv[r] * (dpv[u][r] - d4[r]);
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int q = 16 * t + 4 * g + r;
            const bool ok = kvalid & (q < a.Lq) & (!causal | (key[u] <= q));  // (no short circuit: no branches)
            pv[r] = masked_exp2(sv[u][r] * c - l4[r], ok);
            dv4[r] = pv[r] * (dpv[u][r] - d4[r]);
          }
        }
        pk[u][t][0] = pack2bf(pv[0], pv[1]);
        pk[u][t][1] = pack2bf(pv[2], pv[3]);
        dk2[u][t][0] = pack2bf(dv4[0], dv4[1]);
        dk2[u][t][1] = pack2bf(dv4[2], dv4[3]);
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      if (32 * s2 >= a.Lq) break;
      short8_t pf[U], dsf[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        pf[u] = __builtin_bit_cast(short8_t, make_uint4(pk[u][2 * s2][0], pk[u][2 * s2][1],
                                                        pk[u][2 * s2 + 1][0], pk[u][2 * s2 + 1][1]));
        dsf[u] = __builtin_bit_cast(short8_t, make_uint4(dk2[u][2 * s2][0], dk2[u][2 * s2][1],
                                                         dk2[u][2 * s2 + 1][0], dk2[u][2 * s2 + 1][1]));
      }
#pragma unroll
      for (int dt = 0; dt < T::DT; ++dt) {
        const short8_t otr = T::frag_tr(ldsO, s2, dt, lane);
        const short8_t qtr = T::frag_tr(ldsQ, s2, dt, lane);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          dv[u][dt] = mfma16(otr, pf[u], dv[u][dt]);
          dk[u][dt] = mfma16(qtr, dsf[u], dk[u][dt]);
        }
      }
    }
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int t = 0; t < 8; ++t) dk2[u][t][0] = dk2[u][t][1] = 0u;
  }
  TDG_STAMP(2);
  __syncthreads();  // everyone done with Q / dO (the dS image aliases them)
  // dS^T image: row = key, bytes (16t + 4g) * 2 .. +8 = queries 16t+4g .. +3
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int t = 0; t < 8; ++t)
      *reinterpret_cast<uint2*>(ldsS + TS::off(key[u], (16 * t + 4 * g) * 2)) = make_uint2(dk2[u][t][0], dk2[u][t][1]);
  // dK, dV out (key rows on lanes)
  const float sc = a.scale;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool ok = key[u] < a.Lk;
    bf16_t* dkp = a.dk + b * a.dk_sb + (long long)key[u] * a.dk_sl + h * a.dk_sh;
    bf16_t* dvp = a.dv + b * a.dv_sb + (long long)key[u] * a.dv_sl + h * a.dv_sh;
    uint32_t lo[T::DT], hi[T::DT];
#pragma unroll
    for (int dt = 0; dt < T::DT; ++dt) pack_acc(dk[u][dt], sc, lo[dt], hi[dt]);
    store_row16<T::DT>(dkp, lo, hi, g, ok);
#pragma unroll
    for (int dt = 0; dt < T::DT; ++dt) pack_acc(dv[u][dt], 1.f, lo[dt], hi[dt]);
    store_row16<T::DT>(dvp, lo, hi, g, ok);
  }
  __syncthreads();

  // ---- phase 2: dQ for queries 16 (U w + u) .. +15 (query on lanes)
  if (16 * U * w >= a.Lq) return;
  f32x4 dq[U][T::DT];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int i = 0; i < T::DT; ++i) dq[u][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) {
    if (32 * s2 >= klim) break;
    short8_t dsf[U];
#pragma unroll
    for (int u = 0; u < U; ++u) dsf[u] = TS::frag_tr(ldsS, s2, U * w + u, lane);
#pragma unroll
    for (int dt = 0; dt < T::DT; ++dt) {
      const short8_t ktr = T::frag_tr(ldsK, s2, dt, lane);
#pragma unroll
      for (int u = 0; u < U; ++u) dq[u][dt] = mfma16(ktr, dsf[u], dq[u][dt]);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int qrow = 16 * (U * w + u) + cl;
    bf16_t* dqp = a.dq + b * a.dq_sb + (long long)qrow * a.dq_sl + h * a.dq_sh;
    uint32_t lo[T::DT], hi[T::DT];
#pragma unroll
    for (int dt = 0; dt < T::DT; ++dt) pack_acc(dq[u][dt], sc, lo[dt], hi[dt]);
    store_row16<T::DT>(dqp, lo, hi, g, qrow < a.Lq);
  }
#ifdef TDG_STAMPS
  TDG_STAMP(3);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  TDG_STAMP(4);
#endif
}

// ============================================================================ backward, e4m3 / e5m2
// BASELINE config 5's fp8 attention backward (reference: the autograd of
// transformer_model.py:73-109). Operands: the e4m3 Q / K / V the forward ran
// on (scales sq, sk, sv), the e5m2 dO (sdo8), P as e4m3(448 P) and dS as
// e5m2(dS * sds8) -- five products on v_mfma_f32_16x16x32_{fp8,bf8}_{fp8,bf8}:
//   S^T = K Q^T, dP^T = V dO^T, dV^T += dO^T P, dK^T += Q^T dS, dQ = dS K,
// softmax recomputed in f32 from the forward's log2-domain LSE.
// One workgroup per (batch, head) holds ALL of its <= 512 keys -- the e4m3
// K image is 32 KiB and a wave's K / V fragments 32 registers, half the bf16
// footprint -- so P and dS are computed once (the bf16 path recomputes them
// in a dQ kernel and a dK/dV kernel) and dQ needs no sum across workgroups.
// NW waves; wave w owns the 16-key subtiles s = w + NW u (u < U = 32 / NW:
// interleaved, so causal work stays balanced) with their dK^T / dV^T in
// accumulators. Per step of 32 queries (Q / dO tiles register-prefetched into
// a 2-slot LDS ring):
//  * S^T, dP^T with the key on the lane: lane cl of query half j reads the
//    Q / dO image row 8 (cl >> 2) + 4 j + (cl & 3), so accumulator register r
//    of lane group g is query 8 g + 4 j + r and the two halves' P / dS pack
//    into the e4m3 / e5m2 B operand of dV^T / dK^T as they stand (queries
//    8 g .. 8 g + 7 of the lane); dO^T / Q^T A operands by ds_read_b64_tr_b8;
//  * dS^T goes to a [key][32 queries] e5m2 image (double-buffered), and the
//    next step computes this step's dQ = dS K from it and the K image (both
//    operands transposing reads): one barrier per step.
// delta = rowsum(dO O) from the e5m2 dO actually used and the bf16 O
// (consistent with dP) in the prologue, with lse, for all queries in LDS.
// Swizzles (8-byte chunk c of row r): K image c ^ 2 ((r >> 2) & 3); Q / dO
// images c ^ 2 (((r >> 2) ^ (r >> 4)) & 3) (conflict-free for both the
// permuted row reads and the transposing reads); dS image c ^ 2 ((r >> 3) & 1).
__device__ __forceinline__ int f8k_off(int r, int c) { return r * 64 + 8 * (c ^ (2 * ((r >> 2) & 3))); }
__device__ __forceinline__ int f8q_off(int r, int c) {
  return r * 64 + 8 * (c ^ (2 * (((r >> 2) ^ (r >> 4)) & 3)));
}
__device__ __forceinline__ int f8s_off(int r, int c) { return r * 32 + 8 * (c ^ (2 * ((r >> 3) & 1))); }

template <int NW>
__global__ __launch_bounds__(NW * 64) void attn_bwd_f8_kernel(AttnArgs a) {
  constexpr int LMAX = 512, QT = 32, U = 32 / NW, NT = NW * 64;
  constexpr int KIMG = LMAX * 64, QIMG = QT * 64, SIMG = LMAX * QT;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ldsK = smem;
  char* ldsV = smem + KIMG;          // (the same layout; its row fragments only)
  char* ldsQ = ldsV + KIMG;          // slot i: Q at 2 i QIMG, dO at (2 i + 1) QIMG
  char* ldsS = ldsQ + 4 * QIMG;      // dS^T images, 2 x SIMG
  float* ldsL = reinterpret_cast<float*>(ldsS + 2 * SIMG);  // lse - log2(448)
  float* ldsD = ldsL + LMAX;                                 // delta * sds / 448
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, cl = lane & 15;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  int xb, h, b;
  attn_coords(a, xb, h, b);
  int klim;
  float scl;
  bool causal;
  key_window(a, b, klim, scl, causal);
  const uint8_t* qb = reinterpret_cast<const uint8_t*>(a.q) + b * a.q_sb + h * a.q_sh;
  const uint8_t* kb = reinterpret_cast<const uint8_t*>(a.k) + b * a.k_sb + h * a.k_sh;
  const uint8_t* vb = reinterpret_cast<const uint8_t*>(a.v) + b * a.v_sb + h * a.v_sh;
  const uint8_t* db = reinterpret_cast<const uint8_t*>(a.dout) + b * a.do_sb + h * a.do_sh;
  const bf16_t* ob = a.o + b * a.o_sb + h * a.o_sh;
  const float sq = a.sq8[0], sk = a.sk8[0], sv = a.sv8[0], sdo = a.sdo8[0], sds = a.sds8[0];
  const float c8 = scl * LOG2E / (sq * sk);     // log2-domain logit per raw S product
  const float k1 = sds / 448.f;                 // e5m2 dS = P448 (dP - delta) * k1
  const float cdp = k1 / (sdo * sv);            // raw dP product -> dP * k1
  const int nq = (a.Lq + QT - 1) / QT;

  // ---- prologue: K image, Q / dO tile 0, lse / delta of every query, V fragments
#pragma unroll
  for (int i = 0; i < 2 * KIMG / 16 / NT; ++i) {  // K, then V
    const int id = tid + i * NT, r = (id >> 2) & (LMAX - 1), p = id & 3;
    const bool isv = id >= KIMG / 16;
    const uint8_t* src = (isv ? vb + (long long)min(r, a.Lk - 1) * a.v_sl
                              : kb + (long long)min(r, a.Lk - 1) * a.k_sl) + 16 * p;
    uint4 v = *reinterpret_cast<const uint4*>(src);
    if (r >= a.Lk) v = make_uint4(0u, 0u, 0u, 0u);
    *reinterpret_cast<uint4*>((isv ? ldsV : ldsK) + r * 64 + 16 * (p ^ ((r >> 2) & 3))) = v;
  }
  // Q / dO tile t, piece tid (< 256): tensor tid >> 7, row (tid >> 2) & 31, 16-byte piece tid & 3
  const int pr = (tid >> 2) & 31, pp = tid & 3;
  const bool pdo = (tid >> 7) & 1;
  // (the load's zero-select is applied at the LDS write, so that the
  // prefetch of the next tile is not waited for where it is issued)
  auto tile_load = [&](int t) {
    const int q = min(t * QT + pr, a.Lq - 1);
    const uint8_t* src = (pdo ? db + (long long)q * a.do_sl : qb + (long long)q * a.q_sl) + 16 * pp;
    return *reinterpret_cast<const uint4*>(src);
  };
  auto tile_put = [&](int t, uint4 v) {
    if (t * QT + pr >= a.Lq) v = make_uint4(0u, 0u, 0u, 0u);
    char* dst = ldsQ + (2 * (t & 1) + (pdo ? 1 : 0)) * QIMG;
    *reinterpret_cast<uint4*>(dst + pr * 64 + 16 * (pp ^ (((pr >> 2) ^ (pr >> 4)) & 3))) = v;
  };
  if (tid < 256) tile_put(0, tile_load(0));
  for (int q = tid; q < LMAX; q += NT) {
    float l = INFINITY, d = 0.f;
    if (q < a.Lq) {
      l = a.lse[((long long)b * a.H + h) * a.Lq + q] - LOG2_448;
      const uint8_t* dr = db + (long long)q * a.do_sl;
      const bf16_t* orow = ob + (long long)q * a.o_sl;
#pragma unroll
      for (int c = 0; c < 8; ++c) {  // 8 elements per chunk
        const uint2 d8 = *reinterpret_cast<const uint2*>(dr + 8 * c);
        const short8_t o8 = *reinterpret_cast<const short8_t*>(orow + 8 * c);
        const auto x0 = __builtin_amdgcn_cvt_pk_f32_bf8(d8.x, false);
        const auto x1 = __builtin_amdgcn_cvt_pk_f32_bf8(d8.x, true);
        const auto x2 = __builtin_amdgcn_cvt_pk_f32_bf8(d8.y, false);
        const auto x3 = __builtin_amdgcn_cvt_pk_f32_bf8(d8.y, true);
        const float dv8[8] = {x0[0], x0[1], x1[0], x1[1], x2[0], x2[1], x3[0], x3[1]};
#pragma unroll
        for (int e = 0; e < 8; ++e) d += dv8[e] * bf2f((bf16_t)o8[e]);
      }
      d *= k1 / sdo;
    }
    ldsL[q] = l;
    ldsD[q] = d;
  }
  __syncthreads();

  f32x4 dk[U][4], dv[U][4];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int i = 0; i < 4; ++i) dk[u][i] = dv[u][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float amx = 0.f;  // max |dS| * sds
  // LDS addresses: every image row base below is a multiple of 16 (32 for the
  // dS image), so each swizzle term is the lane's own and a fragment address
  // is a per-lane offset plus a wave-uniform base plus a compile-time
  // immediate (no address arithmetic per read; all reads are the untracked
  // asm forms, waited for by count -- the compiler had merged tracked K / V
  // and Q / dO reads into ds_read2st64, whose 32-bank rule made them conflict)
  const uint32_t lK = (uint32_t)(uintptr_t)ldsK, lQ = (uint32_t)(uintptr_t)ldsQ;
  const uint32_t lS = (uint32_t)(uintptr_t)ldsS, lL = (uint32_t)(uintptr_t)ldsL;
  // K / V row fragments of subtile u: lK + 1024 w + kvo[ks] + 8192 u (+ KIMG for V)
  const uint32_t kvb0 = lK + 1024 * w + cl * 64 + 8 * ((0 + g) ^ (2 * ((cl >> 2) & 3)));
  const uint32_t kvb1 = lK + 1024 * w + cl * 64 + 8 * ((4 + g) ^ (2 * ((cl >> 2) & 3)));
  // Q / dO row fragments (row 8 (cl >> 2) + 4 j + (cl & 3)) and transposed ones
  uint32_t qo[2][2], to[4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) qo[j][ks] = f8q_off(8 * (cl >> 2) + 4 * j + (cl & 3), 4 * ks + g);
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) to[dt] = f8q_off(8 * g + (cl >> 1), 2 * dt + (cl & 1));
  // dS^T image row of subtile u: lS + 512 w + so + 4096 u (+ SIMG for odd steps)
  const uint32_t sob = lS + 512 * w + f8s_off(cl, g);
  // lse / delta of the lane's queries q0 + 8 g .. +7
  const uint32_t lgb = lL + 32 * g;

  // dQ: 8 output blocks of 16 queries x 16 head dims per step, blocks w + NW i;
  // the column sums of the bf16-rounded dQ (bias gradient) over every step
  const float gq = a.scale / (sds * sk), s8 = a.sg8 ? a.sg8[0] : 0.f;
  float csq[4] = {0.f, 0.f, 0.f, 0.f}, amq = 0.f;
  const long long dq_base = b * a.dq_sb + h * a.dq_sh;
  const int drow = 8 * g + (cl >> 1);
  auto dq_step = [&](int t) {
    const int q0 = t * QT;
    const int nkc = min(causal ? t + 1 : LMAX / 32, (klim + 31) / 32);
#pragma unroll
    for (int i = 0; i < 8 / NW; ++i) {
      const int blk = w + NW * i, qbk = blk >> 2, dt = blk & 3;
      // chunk kc: K^T at lK + dko + 2048 kc, dS at the step's image + dso + 1024 kc
      uint32_t ka = lK + f8k_off(drow, 2 * dt + (cl & 1));
      uint32_t sa = lS + (t & 1) * SIMG + f8s_off(drow, 2 * qbk + (cl & 1));
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      // batches of 4 chunks; a partial last batch reads clamped chunks and
      // zeroes their dS operand
      for (int kc0 = 0; kc0 < nkc; kc0 += 4) {
        long kt[4], st[4];
        static_for<4>([&](auto cc) {
          constexpr int c = decltype(cc)::value;
          kt[c] = lds_read_tr8_at<2048 * c>(ka);
          st[c] = lds_read_tr8_at<1024 * c>(sa);
        });
        lgkm_wait<0>();
        const int nv = nkc - kc0;  // valid chunks of this batch (wave-uniform)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          tie(kt[c]);
          tie(st[c]);
          if (c > 0 && nv <= c) st[c] = 0;
          acc = __builtin_amdgcn_mfma_f32_16x16x32_fp8_bf8(kt[c], st[c], acc, 0, 0, 0);
        }
        ka += 4 * 2048;
        sa += 4 * 1024;
      }
      const int q = q0 + 16 * qbk + cl;
      const bool ok = q < a.Lq;
      // (uniform base + 32-bit lane offset: a 64-bit per-lane address kept
      // across the loop was spilled)
      const long long off = dq_base + (q * (int)a.dq_sl + 16 * dt + 4 * g);
      float v[4];
      bf16_t e[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        e[r] = f2bf(acc[r] * gq);
        v[r] = ok ? bf2f(e[r]) : 0.f;
        csq[r] += v[r];
        amq = fmaxf(amq, fabsf(v[r]));
      }
      if (ok && a.dq)
        *reinterpret_cast<uint2*>(a.dq + off) = make_uint2((uint32_t)e[0] | ((uint32_t)e[1] << 16),
                                                           (uint32_t)e[2] | ((uint32_t)e[3] << 16));
      if (ok && a.dq8) {
        int w8 = pack2_e5m2c<false>(v[0] * s8, v[1] * s8, 0);
        w8 = pack2_e5m2c<true>(v[2] * s8, v[3] * s8, w8);
        *reinterpret_cast<int*>(a.dq8 + off) = w8;
      }
    }
  };
  // Q / dO tile t by LDS-DMA (waves 0-3, one 1 KiB piece each: wave wq
  // fills tensor wq >> 1, rows 16 (wq & 1) .. +15, lane l the 16-byte
  // position l & 3 of row l >> 2 -- the source piece is swizzled instead of
  // the destination). Rows past Lq repeat row Lq - 1 (finite; their P and dS
  // are masked to 0). No destination registers: nothing for a later register
  // reuse to wait on.
  auto tile_dma = [&](int t) {
    if (w < 4) {
      const int r = 16 * (w & 1) + (lane >> 2);
      const int q = min(t * QT + r, a.Lq - 1);
      const int pc = (lane & 3) ^ (((r >> 2) ^ (r >> 4)) & 3);
      const uint8_t* src = ((w >> 1) ? db + (long long)q * a.do_sl : qb + (long long)q * a.q_sl) + 16 * pc;
      char* dst = ldsQ + (2 * (t & 1) + (w >> 1)) * QIMG + 16 * (w & 1) * 64;
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst,
                                       16, 0, 0);
    }
  };
  for (int it = 0; it < nq; ++it) {
    if (it > 0) {
      if (w < 4) wait_vmcnt<0>();  // this tile's DMA (issued a whole step ago by waves 0-3)
      lds_barrier();
    }
    const int q0 = it * QT;
    // dQ of the previous tile first, then the next tile's DMA
    if (it > 0) dq_step(it - 1);
    if (it + 1 < nq) tile_dma(it + 1);
    const uint32_t sQa = lQ + 2 * (it & 1) * QIMG;
    long qf[2][2], of[2][2], qT[4], oT[4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        qf[j][ks] = lds_read_b64_at<0>(sQa + qo[j][ks]);
        of[j][ks] = lds_read_b64_at<QIMG>(sQa + qo[j][ks]);
      }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      qT[dt] = lds_read_tr8_at<0>(sQa + to[dt]);
      oT[dt] = lds_read_tr8_at<QIMG>(sQa + to[dt]);
    }
    lgkm_wait<0>();
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        tie(qf[j][ks]);
        tie(of[j][ks]);
      }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      tie(qT[dt]);
      tie(oT[dt]);
    }
    const uint32_t sw0 = sob + (it & 1) * SIMG;
    const uint32_t lgq = lgb + 4 * q0;
    // subtile u: S^T / dP^T, P and dS (e4m3 / e5m2 packed as they stand), the
    // dV^T / dK^T updates and dS^T into the image. (A branch-free copy of this
    // body for the all-active, unmasked case made the compiler spill 262
    // registers: one uniform branch per subtile instead.)
    static_for<U>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      const int s16 = 16 * (w + NW * u);  // the subtile's first key (wave-uniform)
      const bool act = s16 < klim && (!causal || s16 <= q0 + QT - 1);
      long pS = 0;
      if (act) {
        // the subtile's K / V row fragments (key on the lane) and the lse /
        // delta of the lane's 8 queries
        long kf[2], vf[2];
        kf[0] = lds_read_b64_at<8192 * u>(kvb0);
        kf[1] = lds_read_b64_at<8192 * u>(kvb1);
        vf[0] = lds_read_b64_at<KIMG + 8192 * u>(kvb0);
        vf[1] = lds_read_b64_at<KIMG + 8192 * u>(kvb1);
        f32x4 L4[2], D4[2];
        L4[0] = __builtin_bit_cast(f32x4, lds_read_b128_at<0>(lgq));
        L4[1] = __builtin_bit_cast(f32x4, lds_read_b128_at<16>(lgq));
        D4[0] = __builtin_bit_cast(f32x4, lds_read_b128_at<4 * LMAX>(lgq));
        D4[1] = __builtin_bit_cast(f32x4, lds_read_b128_at<4 * LMAX + 16>(lgq));
        lgkm_wait<4>();
        tie(kf[0]);
        tie(kf[1]);
        tie(vf[0]);
        tie(vf[1]);
        f32x4 s[2], dp[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          s[j] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(qf[j][0], kf[0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          s[j] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(qf[j][1], kf[1], s[j], 0, 0, 0);
          dp[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf8_fp8(of[j][0], vf[0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          dp[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf8_fp8(of[j][1], vf[1], dp[j], 0, 0, 0);
        }
        lgkm_wait<0>();
        tie(L4[0]);
        tie(L4[1]);
        tie(D4[0]);
        tie(D4[1]);
        const bool full = s16 + 15 < klim && q0 + QT <= a.Lq && (!causal || s16 + 15 <= q0);
        float x[2][4];
        if (full) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) x[j][r] = fmaf(s[j][r], c8, -L4[j][r]);
        } else {
          const int key = s16 + cl;
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int q = q0 + 8 * g + 4 * j + r;
              const bool ok = (key < klim) & (q < a.Lq) & (!causal | (key <= q));  // (no short circuit)
              const float xv = fmaf(s[j][r], c8, -L4[j][r]);
              x[j][r] = ok ? xv : -INFINITY;
            }
        }
        int pw[2], sw[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          // 448 P = exp2(x): x <= 0 up to rounding (the forward's LSE over the
          // same e4m3 products), so 448 P rounds to at most e4m3's 448
          float p[4], ds[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            p[r] = fast_exp2(x[j][r]);
            ds[r] = p[r] * fmaf(dp[j][r], cdp, -D4[j][r]);
          }
          amx = fmaxf(amx, fmaxf(fmaxf(fabsf(ds[0]), fabsf(ds[1])), fmaxf(fabsf(ds[2]), fabsf(ds[3]))));
#pragma unroll
          for (int r = 0; r < 4; ++r) ds[r] = __builtin_amdgcn_fmed3f(ds[r], -E5M2_MAX_F, E5M2_MAX_F);
          // (the first convert's old operand: any register -- the second one
          // overwrites its other half)
          const int pv = __builtin_amdgcn_cvt_pk_fp8_f32(p[0], p[1], __float_as_int(p[2]), false);
          pw[j] = __builtin_amdgcn_cvt_pk_fp8_f32(p[2], p[3], pv, true);
          const int sv2 = __builtin_amdgcn_cvt_pk_bf8_f32(ds[0], ds[1], __float_as_int(ds[2]), false);
          sw[j] = __builtin_amdgcn_cvt_pk_bf8_f32(ds[2], ds[3], sv2, true);
        }
        const long pP = (long)(uint32_t)pw[0] | ((long)pw[1] << 32);
        pS = (long)(uint32_t)sw[0] | ((long)sw[1] << 32);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          dv[u][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf8_fp8(oT[dt], pP, dv[u][dt], 0, 0, 0);
          dk[u][dt] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_bf8(qT[dt], pS, dk[u][dt], 0, 0, 0);
        }
      }
      lds_write_b64_at<4096 * u>(sw0, pS);
    });
  }
  wait_vmcnt<0>();
  lds_barrier();
  dq_step(nq - 1);

  // ---- epilogue: dK / dV (key rows on lanes) bf16 and / or e5m2, amax and
  // the bias-gradient column sums (dQ's, dK's, dV's) of this (b, h)
  const float gk = a.scale / (sds * sq), gv = 1.f / (448.f * sdo);
  const float s8kv = a.sgkv8 ? a.sgkv8[0] : s8;  // dK / dV e5m2 scale
  float csk[4][4], csv[4][4], amk = 0.f;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int r = 0; r < 4; ++r) csk[dt][r] = csv[dt][r] = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int key = 16 * (w + NW * u) + cl;
    const bool ok = key < a.Lk;
    const long long offk = b * a.dk_sb + (long long)key * a.dk_sl + h * a.dk_sh;
    const long long offv = b * a.dv_sb + (long long)key * a.dv_sl + h * a.dv_sh;
    uint32_t klo[4], khi[4], vlo[4], vhi[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      pack_acc(dk[u][dt], gk, klo[dt], khi[dt]);
      pack_acc(dv[u][dt], gv, vlo[dt], vhi[dt]);
    }
    if (a.dk) store_row16<4>(a.dk + offk, klo, khi, g, ok);
    if (a.dv) store_row16<4>(a.dv + offv, vlo, vhi, g, ok);
    if (a.dk8) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const float k4[4] = {__uint_as_float(klo[dt] << 16), __uint_as_float(klo[dt] & 0xffff0000u),
                             __uint_as_float(khi[dt] << 16), __uint_as_float(khi[dt] & 0xffff0000u)};
        const float v4[4] = {__uint_as_float(vlo[dt] << 16), __uint_as_float(vlo[dt] & 0xffff0000u),
                             __uint_as_float(vhi[dt] << 16), __uint_as_float(vhi[dt] & 0xffff0000u)};
        int wk = pack2_e5m2c<false>(k4[0] * s8kv, k4[1] * s8kv, 0);
        wk = pack2_e5m2c<true>(k4[2] * s8kv, k4[3] * s8kv, wk);
        int wv = pack2_e5m2c<false>(v4[0] * s8kv, v4[1] * s8kv, 0);
        wv = pack2_e5m2c<true>(v4[2] * s8kv, v4[3] * s8kv, wv);
        if (ok) {
          *reinterpret_cast<int*>(a.dk8 + offk + 16 * dt + 4 * g) = wk;
          *reinterpret_cast<int*>(a.dv8 + offv + 16 * dt + 4 * g) = wv;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          csk[dt][r] += ok ? k4[r] : 0.f;
          csv[dt][r] += ok ? v4[r] : 0.f;
          amk = fmaxf(amk, ok ? fmaxf(fabsf(k4[r]), fabsf(v4[r])) : 0.f);
        }
      }
    }
  }
  // amax: dS (its own slot), the gradients (the projection's e5m2 slot)
  amx = wave_max(amx);
  if (lane == 0 && a.amaxds8) atomic_amax(amax_word(a.amaxds8, b * 7 + h * 13 + w), amx / sds);
  if (a.amaxgkv8) {  // dK / dV in their own slot
    const float amq_w = wave_max(amq), amk_w = wave_max(amk);
    if (lane == 0 && a.amaxg8 && a.dq8) atomic_amax(amax_word(a.amaxg8, b * 5 + h * 11 + w), amq_w);
    if (lane == 0 && a.dk8) atomic_amax(amax_word(a.amaxgkv8, b * 5 + h * 11 + w), amk_w);
  } else {
    const float amg = wave_max(fmaxf(amq, amk));
    if (lane == 0 && a.amaxg8 && (a.dq8 || a.dk8)) atomic_amax(amax_word(a.amaxg8, b * 5 + h * 11 + w), amg);
  }
  if (!a.cs_part) return;
  // column sums: over the wave's 16 rows per lane group (shuffles), then the
  // waves through LDS (the Q / dO ring is free: every read of it is behind the
  // last barrier)
  float* red = reinterpret_cast<float*>(ldsQ);  // [3][NW][64]
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int sh = 1; sh < 16; sh <<= 1) csq[r] += __shfl_xor(csq[r], sh, 64);
  if (a.dk8) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int sh = 1; sh < 16; sh <<= 1) {
          csk[dt][r] += __shfl_xor(csk[dt][r], sh, 64);
          csv[dt][r] += __shfl_xor(csv[dt][r], sh, 64);
        }
  }
  if (cl == 0) {
    const int dtq = w & 3;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = 16 * dt + 4 * g + r;
        red[w * 64 + col] = dt == dtq ? csq[r] : 0.f;
        red[(NW + w) * 64 + col] = csk[dt][r];
        red[(2 * NW + w) * 64 + col] = csv[dt][r];
      }
  }
  __syncthreads();
  float* prow = a.cs_part + ((long long)b * a.cs_np) * a.cs_ld + h * 64;
  float* prow2 = a.cs_part2 ? a.cs_part2 + (long long)b * a.cs_ld2 + h * 64 : prow;
  if (tid < 64 * (a.dk8 ? 3 : 1)) {
    const int m = tid >> 6, col = tid & 63;
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < NW; ++i) sum += red[(m * NW + i) * 64 + col];
    if (m == 0) prow[a.cs_q + col] = sum;
    else prow2[(m == 1 ? a.cs_k : a.cs_v) + col] = sum;
  }
}

// ============================================================================ probabilities (inference maps)
// One wave per (b, h, q) row: emits the full softmax row [Lk] in f32, the
// attention_weights the reference returns (transformer_model.py:104-109,
// tester.py:51-53). Not on the training path.
template <int HD>
__global__ void attn_probs_kernel(AttnArgs a, float* __restrict__ probs) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  const long long total = (long long)a.B * a.H * a.Lq;
  if (row >= total) return;
  const int q = (int)(row % a.Lq);
  const int h = (int)((row / a.Lq) % a.H);
  const int b = (int)(row / ((long long)a.Lq * a.H));
  int klim;
  float scl;
  bool causal;
  key_window(a, b, klim, scl, causal);
  if (causal) klim = min(klim, q + 1);
  const bf16_t* qp = a.q + b * a.q_sb + (long long)q * a.q_sl + h * a.q_sh;
  float qv[HD];
#pragma unroll
  for (int d = 0; d < HD; ++d) qv[d] = bf2f(qp[d]);
  float* out = probs + row * a.Lk;
  float mx = -INFINITY;
  for (int k = lane; k < klim; k += 64) {
    const bf16_t* kp = a.k + b * a.k_sb + (long long)k * a.k_sl + h * a.k_sh;
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < HD; ++d) s += qv[d] * bf2f(kp[d]);
    s *= scl;
    out[k] = s;
    mx = fmaxf(mx, s);
  }
  mx = wave_max(mx);
  float sum = 0.f;
  for (int k = lane; k < klim; k += 64) {
    const float e = __expf(out[k] - mx);
    out[k] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
  for (int k = lane; k < a.Lk; k += 64) out[k] = k < klim ? out[k] * inv : 0.f;
}

// ============================================================================ fused Q|K|V projection + attention forward
// Self-attention of sequences of <= 128 tokens at head dim 64: one workgroup
// per (batch, head) computes the head's Q|K|V = X_b W_h^T + b_h (128 x 192,
// K = d_model; the GEMM main loop of gemm_impl.h: LDS-DMA K tiles, 8 waves as
// 2 x 4 of 64 x 48, MFMAs with swapped operands) and keeps them in LDS as the
// attention's K / V images and Q rows, writes them to the [M, 3d] projection
// output (the backward reads it), and runs the attention forward of
// attn_fwd_kernel on them (8 waves x 16 queries, one 128-key tile). The
// separate projection launch, its Q|K|V write and the attention's re-read of
// them (the attention forward at L = 128 is a load burst + a short compute
// phase) become one launch whose attention phase reads LDS.
// (reference: transformer_model.py:112-166 -- the Q / K / V Dense layers and
// scaled_dot_product_attention of MultiHeadAttention)
// CROSS (cross-attention): the GEMM is the head's Q projection only (128 x
// 64, 8 waves as 4 x 2 of 32 x 32) and K / V come from the batched K|V
// projection in memory (a.k / a.v), their loads issued before the GEMM.
// SB1: single-buffered fragments and a two-barrier K loop (the register
// budget of two workgroups per CU), STAGES = 2.
template <int STAGES, bool CROSS, bool SB1 = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(SB1 ? 4 : 2))) void qkv_attn_fwd_kernel(
    const QkvAttnArgs qa) {
  constexpr int NW = 8, WM = CROSS ? 4 : 2, WN = CROSS ? 2 : 4, BM = 128, BN = CROSS ? 64 : 192;
  constexpr int NPART = BN / 64;                      // projection parts computed here
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;  // 4 x 3 (2 x 2) subtiles per wave
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, SB = A_BYTES + B_BYTES;
  using GA = Glds<true, BM, NW>;
  using GB = Glds<true, BN, NW>;
  constexpr int PT = GA::P + GB::P;
  using T = ATile<64>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const AttnArgs& a = qa.a;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  // (head, batch): each XCD a contiguous run of batch elements, so a batch
  // element's X panel is read into one XCD's L2 for its heads
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int h = t % a.H, b = t / a.H;
  const int L = qa.L, d = qa.d, K = d;
  const bf16_t* X = reinterpret_cast<const bf16_t*>(qa.x) + (size_t)b * L * qa.ldx;
  // cross-attention K / V (128 keys each, two 64-row tiles): global loads now,
  // LDS after the GEMM
  using Ch = typename ATile<64>::template Chunks<512>;
  Ch ck[2], cv[2];
  if constexpr (CROSS) {
    const bf16_t* kb = a.k + b * a.k_sb + h * a.k_sh;
    const bf16_t* vb = a.v + b * a.v_sb + h * a.v_sh;
#pragma unroll
    for (int h64 = 0; h64 < 2; ++h64) {
      ATile<64>::template fetch<512>(ck[h64], kb, a.k_sl, 64 * h64, a.Lk, tid);
      ATile<64>::template fetch<512>(cv[h64], vb, a.v_sl, 64 * h64, a.Lk, tid);
    }
  }

  // ------------------------------------------------ Q|K|V GEMM (K = d_model)
  GA ga;
  GB gb;
  ga.init(wid, lane);
  gb.init(wid, lane);
  // B rows r of the tile: W row (r / 64) * d + 64 h + r % 64 (a 1 KiB piece
  // covers 8 rows of one 64-row block)
  int wrow[GB::P];
#pragma unroll
  for (int i = 0; i < GB::P; ++i) wrow[i] = (gb.row[i] >> 6) * d + 64 * h + (gb.row[i] & 63);
  auto issue_b = [&](int k0, char* lds) {
#pragma unroll
    for (int i = 0; i < GB::P; ++i) {
      const long long off = (long long)wrow[i] * qa.ldw + k0 + gb.col[i];
      __builtin_amdgcn_global_load_lds((const void*)(reinterpret_cast<const bf16_t*>(qa.w) + off),
                                       (__attribute__((address_space(3))) void*)(lds + (wid * GB::P + i) * 1024),
                                       16, 0, 0);
    }
  };
  const int nk = K / BK;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < STAGES; ++st) {
    if (st < nk) {
      ga.issue(X, qa.ldx, L, K, 0, st * BK, smem + st * SB, wid);
      issue_b(st * BK, smem + st * SB + A_BYTES);
    }
  }
  const int abase = wm * (BM / WM), bbase = wn * (BN / WN);
  if constexpr (SB1) {
    short8_t fa[TM], fb[TN];
    for (int kt = 0; kt < nk; ++kt) {
      // tile kt landed (the younger tile, if any, stays in flight)
      if (kt + 1 < nk) wait_vmcnt<PT>();
      else wait_vmcnt<0>();
      lds_barrier();
      const char* st = smem + (kt % STAGES) * SB;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = frag<true, BM>(st, abase + 16 * i, s2, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = frag<true, BN>(st + A_BYTES, bbase + 16 * j, s2, lane);
        lgkm_wait<0>();
        tie_all(fa);
        tie_all(fb);
        prio_hi();
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(fb[j], fa[i], acc[i][j]);
        prio_lo();
      }
      lds_barrier();  // everyone done with the stage: refill it
      if (kt + STAGES < nk) {
        char* ns = smem + (kt % STAGES) * SB;
        ga.issue(X, qa.ldx, L, K, 0, (kt + STAGES) * BK, ns, wid);
        issue_b((kt + STAGES) * BK, ns + A_BYTES);
      }
    }
  } else {
  short8_t fa0[TM], fb0[TN], fa1[TM], fb1[TN];
  if (nk >= STAGES)
    wait_vmcnt<(STAGES - 1) * PT>();
  else
    wait_vmcnt<0>();
  lds_barrier();
#pragma unroll
  for (int i = 0; i < TM; ++i) fa0[i] = frag<true, BM>(smem, abase + 16 * i, 0, lane);
#pragma unroll
  for (int j = 0; j < TN; ++j) fb0[j] = frag<true, BN>(smem + A_BYTES, bbase + 16 * j, 0, lane);
  constexpr int STEP_OPS = TM + TN;
  auto kstep = [&](int kt, auto modec) {
    constexpr int MODE = decltype(modec)::value;
    const char* st = smem + (kt % STAGES) * SB;
#pragma unroll
    for (int i = 0; i < TM; ++i) fa1[i] = frag<true, BM>(st, abase + 16 * i, 1, lane);
#pragma unroll
    for (int j = 0; j < TN; ++j) fb1[j] = frag<true, BN>(st + A_BYTES, bbase + 16 * j, 1, lane);
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
      if constexpr (MODE >= 2) wait_vmcnt<(STAGES - 2) * PT>();
      else wait_vmcnt<0>();
      lds_barrier();
      const char* nx = smem + ((kt + 1) % STAGES) * SB;
      if constexpr (MODE == 3) {
        char* ns = smem + (kt % STAGES) * SB;
        ga.issue(X, qa.ldx, L, K, 0, (kt + STAGES) * BK, ns, wid);
        issue_b((kt + STAGES) * BK, ns + A_BYTES);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) fa0[i] = frag<true, BM>(nx, abase + 16 * i, 0, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb0[j] = frag<true, BN>(nx + A_BYTES, bbase + 16 * j, 0, lane);
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
  }
  lds_barrier();  // the pipeline stages become the Q / K / V images

  // ------------------------------------------------ bias, bf16, LDS images
  // image p (0 Q, 1 K, 2 V): 128 rows x 64 head dims in the attention's
  // K-image layout (T::off over 128 rows = two 64-row tiles)
  char* img = smem;
  constexpr int IMG = 2 * T::BYTES;
  const int g = lane >> 4, cl = lane & 15;
  if constexpr (CROSS) {
#pragma unroll
    for (int h64 = 0; h64 < 2; ++h64) {
      ATile<64>::template put<512>(img + IMG + h64 * T::BYTES, ck[h64], tid);
      ATile<64>::template put<512>(img + 2 * IMG + h64 * T::BYTES, cv[h64], tid);
    }
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = bbase + 16 * j + 4 * g;  // 4 consecutive columns of one image
    const int part = n >> 6, hc = n & 63;
    const f32x4 bn = *reinterpret_cast<const f32x4*>(qa.bias + part * d + 64 * h + hc);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = abase + 16 * i + cl;
      short4_t o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(acc[i][j][r] + bn[r]);
      *reinterpret_cast<short4_t*>(img + part * IMG + T::off(m, hc * 2)) = o;
    }
  }
  __syncthreads();
  // the projection output for the backward ([M, NPART d]): rows < L,
  // 16-byte chunks
  {
    const WtBuf wt(qa.qkv, ((size_t)(b + 1) * L * NPART * d) * sizeof(bf16_t));
#pragma unroll
    for (int pass = 0; pass < NPART * 128 * 8 / 512; ++pass) {
      const int id = tid + 512 * pass;
      const int part = id >> 10, row = (id >> 3) & 127, c = id & 7;
      const short8_t v = *reinterpret_cast<const short8_t*>(img + part * IMG + T::off(row, c * 16));
      if (row < L)
        wt.st16(reinterpret_cast<bf16_t*>(qa.qkv) + ((size_t)b * L + row) * NPART * d + part * d + 64 * h + c * 8,
                v);
    }
  }

  // ------------------------------------------------ attention (attn_fwd_kernel, 8 x 16 queries)
  const char* ldsQ = img;
  const char* ldsK = img + IMG;
  const char* ldsV = img + 2 * IMG;
  const int w = wid;
  const int qrow = 16 * w + cl;
  int klim;
  float scl;
  bool causal;
  key_window(a, b, klim, scl, causal);
  if (causal) klim = min(klim, 128);
  const float c = scl * LOG2E;
  const int wq0 = 16 * w;
  short8_t qf[T::KS];
#pragma unroll
  for (int s2 = 0; s2 < T::KS; ++s2) qf[s2] = T::frag_row(ldsQ, 16 * w, s2, lane);
  f32x4 oacc[T::DT];
#pragma unroll
  for (int i = 0; i < T::DT; ++i) oacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  constexpr int NT16 = 8;
  if (klim > 0) {
    f32x4 sc[NT16];
#pragma unroll
    for (int tt = 0; tt < NT16; ++tt) {
      sc[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < T::KS; ++ks) sc[tt] = mfma16(T::frag_row(ldsK, 16 * tt, ks, lane), qf[ks], sc[tt]);
    }
    short8_t pf[NT16 / 2];
    softmax_tile<NT16, T::DT>(sc, m, l, oacc, pf, tile_masked(0, 128, klim, causal, wq0), 0, klim, causal,
                              qrow, g, c);
#pragma unroll
    for (int s2 = 0; s2 < NT16 / 2; ++s2)
#pragma unroll
      for (int dt = 0; dt < T::DT; ++dt) oacc[dt] = mfma16(T::frag_tr(ldsV, s2, dt, lane), pf[s2], oacc[dt]);
  }
  {
    float lu = rows_sum(l);
    const bool ok = qrow < a.Lq;
    const float inv = lu > 0.f ? 1.f / lu : 0.f;
    bf16_t* op = a.out + b * a.o_sb + (long long)qrow * a.o_sl + h * a.o_sh;
    uint32_t lo[T::DT], hi[T::DT];
#pragma unroll
    for (int dt = 0; dt < T::DT; ++dt) pack_acc(oacc[dt], inv, lo[dt], hi[dt]);
    store_row16<T::DT>(op, lo, hi, g, ok);
    if (ok && g == 0)
      a.lse[((long long)b * a.H + h) * a.Lq + qrow] = lu > 0.f ? m + log2f(lu) : INFINITY;
  }
}

}  // namespace tdg

using namespace tdg;

namespace {
template <int HD>
int fwd_hd(const AttnArgs& a, hipStream_t st) {
  // (64 queries per workgroup for Lq > 64 -- twice the workgroups, K / V
  // staged by both halves -- measured 17.2 vs 12.2 us at B 64, H 8, L 128:
  // csrc/lab/attn_lab.cpp, profiles/attn_lab/)
  // hd 64, > 128 queries: LDS-DMA pipelined kernel, 8 waves x 16 queries,
  // 3-slot ring (seq 512: 40.5 us vs 41-45 for 4 slots or 32 queries per
  // wave, 47 for the register-staged kernel; profiles/r3/attn_seq512_*)
  if constexpr (HD == 64) {
    if (a.Lq > 128) {
      constexpr int NWV = 8, U = 1, NS = 3;
      static bool attr = false;
      if (!attr) {
        hipFuncSetAttribute((const void*)attn_fwd_pipe_kernel<NWV, U, NS>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
      }
      hipLaunchKernelGGL((attn_fwd_pipe_kernel<NWV, U, NS>), dim3(cdiv(a.Lq, 16 * NWV * U), a.H, a.B),
                         dim3(NWV * 64), NS * 2 * ATile<64>::BYTES, st, a);
      return 0;
    }
  }
  if (a.Lq > 64) {
    dim3 grid(cdiv(a.Lq, 128), a.H, a.B);
    // 4 waves x 2 query subtiles (each K / V fragment read from LDS feeds two
    // MFMAs; 225 VGPRs, two 4-wave workgroups per CU): 9.6 vs 10.3 us (causal
    // 10.3 vs 11.7) for 8 waves x 1 subtile, whose 142 VGPRs fit only one
    // 8-wave workgroup per CU -- the 512 (batch, head) items ran in two
    // rounds (profiles/r3s2/attn_short_fwd_variants.txt); headline step
    // 5.04-5.06 vs 5.07-5.08 ms A/B (profiles/r3s2/attn_short_fwd_ab.txt)
    // (hd 128: 8 waves x 1 subtile, two subtiles per wave would spill)
    if constexpr (HD <= 64)
      hipLaunchKernelGGL((attn_fwd_kernel<HD, 4, 128, 2>), grid, dim3(256), 4 * ATile<HD>::BYTES, st, a);
    else
      hipLaunchKernelGGL((attn_fwd_kernel<HD, 8, 128, 1>), grid, dim3(512), 4 * ATile<HD>::BYTES, st, a);
  } else {
    dim3 grid(cdiv(a.Lq, 64), a.H, a.B);
    hipLaunchKernelGGL((attn_fwd_kernel<HD, 4, 64, 1>), grid, dim3(256), 2 * ATile<HD>::BYTES, st, a);
  }
  return 0;
}
template <int HD>
constexpr int fused_bwd_lds() {
  constexpr int TB = 128 * HD * 2, SB = 128 * 256;
  return (2 * TB >= SB ? 3 * TB : 3 * TB + SB) + 2 * 128 * 4;
}

template <int HD>
int bwd_hd(const AttnArgs& a, hipStream_t st);
}  // namespace

// Fused backward with the output-projection dgrad in-kernel (FDO): Lq, Lk <=
// 128, hd 64, d = 64 H. Returns -1 when not covered.
extern "C" int tdg_attn_bwd_fdo(const AttnArgs* ap, hipStream_t st) {
  const AttnArgs& a = *ap;
  if (a.Lq > 128 || a.Lk > 128 || a.fdo_d != 64 * a.H || a.fdo_d % BK || a.fdo_ldy % 8 ||
      a.fdo_ldw % 8 || !a.fdo_dy || !a.fdo_w)
    return -1;
  constexpr int lds = fused_bwd_lds<64>() > FDO_STAGES * FDO_SB ? fused_bwd_lds<64>() : FDO_STAGES * FDO_SB;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)attn_bwd_fused_kernel<64, 1, true>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((attn_bwd_fused_kernel<64, 1, true>), dim3(a.B * a.H), dim3(512), lds, st, a);
  return 0;
}

namespace {
template <int HD>
int bwd_hd(const AttnArgs& a, hipStream_t st) {
  if (a.Lq <= 128 && a.Lk <= 128) {
    constexpr int lds = fused_bwd_lds<HD>();
    // U = 1: 8 waves, 16 keys / queries each. U = 2 (4 waves, every fragment
    // read feeding two MFMAs, 231 VGPRs) measured slower: 22.7 vs 21.7 us per
    // call, step 5.15 vs 5.13 ms (profiles/r3s2/attn_bwd_u2.txt)
    constexpr int U = 1;
    static bool attr = false;
    if (!attr) {
      hipFuncSetAttribute((const void*)attn_bwd_fused_kernel<HD, U>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr = true;
    }
    hipLaunchKernelGGL((attn_bwd_fused_kernel<HD, U>), dim3(a.B * a.H), dim3(512 / U), lds, st, a);
    return 0;
  }
  // dQ first: it also writes delta = rowsum(dO * O), which dK/dV reads
  // hd 64: LDS-DMA pipelined kernels, 32 queries / keys per wave (seq 512:
  // 121 us vs 132-136 with 16 per wave in either, 147 register-staged)
  if constexpr (HD == 64) {
    constexpr int U = 2, NS = 4;
    constexpr int lds_dq = NS * 2 * ATile<64>::BYTES;
    constexpr int lds_kv = NS * (2 * ATile<64>::BYTES + 768);
    static bool attr = false;
    if (!attr) {
      hipFuncSetAttribute((const void*)attn_bwd_dq_pipe_kernel<U, NS>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      hipFuncSetAttribute((const void*)attn_bwd_dkdv_pipe_kernel<U, NS>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr = true;
    }
    hipLaunchKernelGGL((attn_bwd_dq_pipe_kernel<U, NS>), dim3(cdiv(a.Lq, 64 * U), a.H, a.B),
                       dim3(256), lds_dq, st, a);
    hipLaunchKernelGGL((attn_bwd_dkdv_pipe_kernel<U, NS>), dim3(cdiv(a.Lk, 64 * U), a.H, a.B),
                       dim3(256), lds_kv, st, a);
    return 0;
  }
  hipLaunchKernelGGL((attn_bwd_dq_kernel<HD, 1>), dim3(cdiv(a.Lq, QB), a.H, a.B), dim3(256),
                     2 * ATile<HD>::BYTES, st, a);
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<HD, 1>), dim3(cdiv(a.Lk, KB), a.H, a.B), dim3(256),
                     2 * ATile<HD>::BYTES + 2 * QB * 4, st, a);
  return 0;
}
template <int HD>
int probs_hd(const AttnArgs& a, float* probs, hipStream_t st) {
  const long long rows = (long long)a.B * a.H * a.Lq;
  hipLaunchKernelGGL(attn_probs_kernel<HD>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, a,
                     probs);
  return 0;
}
}  // namespace

#define TDG_HD_CASES(F, ...)           \
  switch (hd) {                        \
    case 16: return F<16>(__VA_ARGS__);   \
    case 32: return F<32>(__VA_ARGS__);   \
    case 64: return F<64>(__VA_ARGS__);   \
    case 128: return F<128>(__VA_ARGS__); \
    default: return -1;                \
  }

extern "C" int tdg_attn_fwd(const AttnArgs* a, int hd, hipStream_t st) {
  TDG_HD_CASES(fwd_hd, *a, st)
}
extern "C" int tdg_attn_bwd(const AttnArgs* a, int hd, hipStream_t st) {
  TDG_HD_CASES(bwd_hd, *a, st)
}
namespace {
template <int NS, int U>
int fwd_fp8_u(const AttnArgs& a, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)attn_fwd_fp8_kernel<NS, U>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((attn_fwd_fp8_kernel<NS, U>), dim3(cdiv(a.Lq, 128 * U), a.H, a.B), dim3(512),
                     NS * 2 * 64 * 64, st, a);
  return 0;
}
int fwd_fp8_ns() {
  static const int v = [] {
    const char* e = getenv("TDG_ATTN_FWD8_NS");
    return e ? atoi(e) : 3;
  }();
  return v;
}
}  // namespace
// ring depth NS from TDG_ATTN_FWD8_NS (3, 4 or 6: measured equal, 3 kept).
// (32 queries per wave, U = 2, measured 3-5 % slower at seq 512 and is not
// instantiated: profiles/r5/attn_fwd8_u_rows.txt)
extern "C" int tdg_attn_fwd_fp8(const AttnArgs* a, int hd, hipStream_t st) {
  if (hd != 64) return -1;
  switch (fwd_fp8_ns()) {
    case 4: return fwd_fp8_u<4, 1>(*a, st);
    case 6: return fwd_fp8_u<6, 1>(*a, st);
    default: return fwd_fp8_u<3, 1>(*a, st);
  }
}
namespace {
template <int NW>
int bwd_f8_nw(const AttnArgs& a, hipStream_t st) {
  constexpr int lds = 2 * 512 * 64 + 4 * 32 * 64 + 2 * 512 * 32 + 2 * 512 * 4;  // 108 KiB
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)attn_bwd_f8_kernel<NW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        lds);
    attr = true;
  }
  hipLaunchKernelGGL(attn_bwd_f8_kernel<NW>, dim3(1, a.H, a.B), dim3(NW * 64), lds, st, a);
  return 0;
}
}  // namespace
// hd 64, Lq, Lk <= 512: one 8-wave workgroup per (batch, head) (4 waves of
// 8 subtiles each -- one wave per SIMD -- spilled 155 registers at -O3)
extern "C" int tdg_attn_bwd_f8(const AttnArgs* a, int hd, hipStream_t st) {
  if (hd != 64 || a->Lq < 1 || a->Lk < 1 || a->Lq > 512 || a->Lk > 512) return -1;
  return bwd_f8_nw<8>(*a, st);
}
extern "C" int tdg_attn_probs(const AttnArgs* a, int hd, float* probs, hipStream_t st) {
  TDG_HD_CASES(probs_hd, *a, probs, st)
}

// Fused Q|K|V projection + attention forward (qkv_attn_fwd_kernel): L <= 128,
// hd 64, d % 64 == 0. Self-attention: 2 stages, single-buffered fragments,
// two workgroups per CU (116 VGPRs): 21.5 us per call at B 64, L 128, H 8
// against 25.7 for 3 stages with double-buffered fragments at one workgroup
// per CU (144 VGPRs; with 2 stages and double buffering it spilled, 32.1 us;
// profiles/r6/attn_fused_projections.txt). qa->cross:
// the cross-attention form (Q projection only, K / V from a.k / a.v, Lk <=
// 128). Returns -1 when the shape is not covered.
namespace {
template <int STAGES, bool CROSS, bool SB1>
void qkv_attn_launch(const QkvAttnArgs& qa, hipStream_t st) {
  constexpr int SB = (128 + (CROSS ? 64 : 192)) * BK * 2;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)qkv_attn_fwd_kernel<STAGES, CROSS, SB1>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((qkv_attn_fwd_kernel<STAGES, CROSS, SB1>), dim3(qa.a.B * qa.a.H), dim3(512),
                     STAGES * SB, st, qa);
}

}  // namespace
extern "C" int tdg_qkv_attn_fwd(const QkvAttnArgs* qa, hipStream_t st) {
  const AttnArgs& a = qa->a;
  if (qa->L > 128 || qa->L <= 0 || a.Lq != qa->L || a.Lk > 128 || a.Lk <= 0 || qa->d % 64 ||
      qa->d != 64 * a.H || qa->ldx % 8 || qa->ldw % 8 || (!qa->cross && a.Lk != qa->L))
    return -1;
  if (qa->cross)
    qkv_attn_launch<3, true, false>(*qa, st);
  else
    qkv_attn_launch<2, false, true>(*qa, st);
  return 0;
}
