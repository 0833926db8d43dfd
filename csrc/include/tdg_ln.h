// Row helpers of the fused residual + dropout + LayerNorm kernels (norm.hip):
// one wave per D-wide row, VEC = D/64 elements per lane (RowMap), and the
// per-element Philox dropout keep bits (the same mask in forward and
// backward, regenerated instead of stored).
#pragma once
#include "tdg_common.h"

namespace tdg {

// Lane -> column map of a D = 64*VEC row: lanes own W = min(VEC, 8)
// consecutive elements per chunk and the CH = VEC/W chunks sit 64*W apart, so
// every wave-wide load / store instruction covers one contiguous 64*W*2-byte
// span (D = 1024: two fully used 1 KiB accesses instead of two 32-byte-strided
// half-used ones).
template <int VEC>
struct RowMap {
  static constexpr int W = VEC < 8 ? VEC : 8;
  static constexpr int CH = VEC / W;
  __device__ static __forceinline__ int col(int lane, int i) {
    return (i / W) * (64 * W) + lane * W + (i % W);
  }
};

template <int VEC>
struct RowVec {
  using Map = RowMap<VEC>;
  float v[VEC];
  // row: the row's first element; lane's slots at Map::col(lane, i)
  __device__ __forceinline__ void load_row(const bf16_t* row, int lane) {
    const bf16_t* p = row + lane * Map::W;
    if constexpr (VEC == 2) {
      const uint32_t w = *reinterpret_cast<const uint32_t*>(p);
      v[0] = bf2f((bf16_t)(w & 0xffff));
      v[1] = bf2f((bf16_t)(w >> 16));
    } else if constexpr (VEC == 4) {
      const short4_t w = *reinterpret_cast<const short4_t*>(p);
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = bf2f((bf16_t)w[i]);
    } else {
#pragma unroll
      for (int c = 0; c < Map::CH; ++c) {
        const short8_t w = *reinterpret_cast<const short8_t*>(p + 512 * c);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[8 * c + i] = bf2f((bf16_t)w[i]);
      }
    }
  }
  // write-through variant (tdg_common.h WtBuf)
  __device__ __forceinline__ void store_row(bf16_t* row, int lane, const WtBuf& wt) const {
    bf16_t* p = row + lane * Map::W;
    if constexpr (VEC == 2) {
      wt.st4(p, pack2bf(v[0], v[1]));
    } else if constexpr (VEC == 4) {
      short4_t w;
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] = (short)f2bf(v[i]);
      wt.st8(p, w);
    } else {
#pragma unroll
      for (int c = 0; c < Map::CH; ++c) {
        short8_t w;
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = (short)f2bf(v[8 * c + i]);
        wt.st16(p + 512 * c, w);
      }
    }
  }
  __device__ __forceinline__ void store_row(bf16_t* row, int lane) const {
    bf16_t* p = row + lane * Map::W;
    if constexpr (VEC == 2) {
      *reinterpret_cast<uint32_t*>(p) = pack2bf(v[0], v[1]);
    } else if constexpr (VEC == 4) {
      short4_t w;
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] = (short)f2bf(v[i]);
      *reinterpret_cast<short4_t*>(p) = w;
    } else {
#pragma unroll
      for (int c = 0; c < Map::CH; ++c) {
        short8_t w;
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = (short)f2bf(v[8 * c + i]);
        *reinterpret_cast<short8_t*>(p + 512 * c) = w;
      }
    }
  }
};

// Keep bits of the lane's VEC slots (bit i = slot i, RowMap order) of the row
// starting at element e_row (a multiple of 8: D >= 128) of the flat [M, D]
// tensor: per element the same draw whatever the lane map (tdg_common.h
// dropout_keep); a lane's runs of W <= 8 elements never straddle an 8-block.
template <int VEC>
__device__ __forceinline__ uint32_t keep_bits(uint64_t seed, const long long* ctr, uint64_t site,
                                              uint64_t e_row, int lane, uint32_t thresh) {
  using Map = RowMap<VEC>;
  const uint64_t off = rng_offset(ctr, site);
  uint32_t m = 0;
#pragma unroll
  for (int c = 0; c < Map::CH; ++c)
    m |= dropout_keep_run<Map::W>(seed, off, e_row + Map::col(lane, Map::W * c), thresh)
         << (Map::W * c);
  return m;
}

// Forward of one row: h = x + dropout(t) (t = the sublayer output, already
// loaded; has_t false: h = x), h rounded to bf16 (and saved) so forward and
// backward see the same h, y = (h - mean) * rstd * gamma + beta. Stores y,
// hsave, mean/rstd; returns y (f32, pre-rounding) in o. Shared by the
// standalone LayerNorm and the GEMM+LayerNorm epilogue so both produce
// bitwise-identical results.
template <int D>
__device__ __forceinline__ void ln_row_fwd(RowVec<D / 64>& h, RowVec<D / 64>& t, bool has_t,
                                           size_t rbase, int row, int lane,
                                           const float* __restrict__ gamma,
                                           const float* __restrict__ beta, bf16_t* __restrict__ y,
                                           bf16_t* __restrict__ hsave, float* __restrict__ mean_out,
                                           float* __restrict__ rstd_out, float p, uint32_t thresh,
                                           uint64_t seed, const long long* ctr, uint64_t site,
                                           float eps, RowVec<D / 64>& o, size_t wt_bytes = 0,
                                           uint8_t* __restrict__ kbits = nullptr) {
  constexpr int VEC = D / 64;
  if (has_t) {
    if (p > 0.f) {
      const uint32_t km = keep_bits<VEC>(seed, ctr, site, rbase, lane, thresh);
      if constexpr (VEC >= 8) {
        // the keep bits as a row-major bitmap (bit c % 8 of byte c / 8 of the
        // row = column c): the LayerNorm backward reads them instead of
        // regenerating the mask (ln_bwd_kernel)
        if (kbits) {
#pragma unroll
          for (int c = 0; c < RowMap<VEC>::CH; ++c)
            kbits[rbase / 8 + 64 * c + lane] = (uint8_t)(km >> (8 * c));
        }
      }
      const float sc = 1.f / (1.f - p);
#pragma unroll
      for (int i = 0; i < VEC; ++i) t.v[i] = ((km >> i) & 1u) ? t.v[i] * sc : 0.f;
    }
#pragma unroll
    for (int i = 0; i < VEC; ++i) h.v[i] += t.v[i];
  }
  // wt_bytes > 0: y / hsave (that many bytes each) stored write-through
  if (hsave) {
    if (wt_bytes) h.store_row(hsave + rbase, lane, WtBuf(hsave, wt_bytes));
    else h.store_row(hsave + rbase, lane);
#pragma unroll
    for (int i = 0; i < VEC; ++i) h.v[i] = bf2f(f2bf(h.v[i]));
  }
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < VEC; ++i) sum += h.v[i];
  const float mean = wave_sum(sum) * (1.f / D);
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    const float d = h.v[i] - mean;
    sq += d * d;
  }
  const float var = wave_sum(sq) * (1.f / D);
  const float rstd = rsqrtf(var + eps);
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    const int col = RowMap<VEC>::col(lane, i);
    o.v[i] = (h.v[i] - mean) * rstd * gamma[col] + beta[col];
  }
  if (wt_bytes) o.store_row(y + rbase, lane, WtBuf(y, wt_bytes));
  else o.store_row(y + rbase, lane);
  if (lane == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
}

}  // namespace tdg
