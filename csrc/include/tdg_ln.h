// Row helpers of the fused residual + dropout + LayerNorm kernels (norm.hip,
// gemm_ln.hip): one wave per D-wide row, VEC = D/64 contiguous elements per
// lane, and the per-element Philox dropout keep bits (the same mask in
// forward and backward, regenerated instead of stored).
#pragma once
#include "tdg_common.h"

namespace tdg {

template <int VEC>
struct RowVec {
  float v[VEC];
  __device__ __forceinline__ void load_bf(const bf16_t* p) {
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
      for (int c = 0; c < VEC / 8; ++c) {
        const short8_t w = *reinterpret_cast<const short8_t*>(p + 8 * c);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[8 * c + i] = bf2f((bf16_t)w[i]);
      }
    }
  }
  // write-through variant (tdg_common.h WtBuf)
  __device__ __forceinline__ void store_bf(bf16_t* p, const WtBuf& wt) const {
    if constexpr (VEC == 2) {
      wt.st4(p, (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16));
    } else if constexpr (VEC == 4) {
      short4_t w;
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] = (short)f2bf(v[i]);
      wt.st8(p, w);
    } else {
#pragma unroll
      for (int c = 0; c < VEC / 8; ++c) {
        short8_t w;
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = (short)f2bf(v[8 * c + i]);
        wt.st16(p + 8 * c, w);
      }
    }
  }
  __device__ __forceinline__ void store_bf(bf16_t* p) const {
    if constexpr (VEC == 2) {
      *reinterpret_cast<uint32_t*>(p) = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    } else if constexpr (VEC == 4) {
      short4_t w;
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] = (short)f2bf(v[i]);
      *reinterpret_cast<short4_t*>(p) = w;
    } else {
#pragma unroll
      for (int c = 0; c < VEC / 8; ++c) {
        short8_t w;
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = (short)f2bf(v[8 * c + i]);
        *reinterpret_cast<short8_t*>(p + 8 * c) = w;
      }
    }
  }
};

// keep bits for VEC consecutive elements starting at e0 (e0 % min(VEC,4) == 0)
template <int VEC>
__device__ __forceinline__ uint32_t keep_bits(uint64_t seed, const long long* ctr, uint64_t site,
                                              uint64_t e0, uint32_t thresh) {
  const uint64_t off = rng_offset(ctr, site);
  uint32_t m = 0;
  if constexpr (VEC == 2) {
    uint32_t r[4];
    Philox::gen(seed, off, e0 >> 2, r);
    const int o = (int)(e0 & 3);
    m = (r[o] >= thresh ? 1u : 0u) | ((r[o + 1] >= thresh ? 1u : 0u) << 1);
  } else {
#pragma unroll
    for (int c = 0; c < VEC / 4; ++c) {
      uint32_t r[4];
      Philox::gen(seed, off, (e0 >> 2) + c, r);
#pragma unroll
      for (int i = 0; i < 4; ++i) m |= (r[i] >= thresh ? 1u : 0u) << (4 * c + i);
    }
  }
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
                                           size_t base, int row, int lane,
                                           const float* __restrict__ gamma,
                                           const float* __restrict__ beta, bf16_t* __restrict__ y,
                                           bf16_t* __restrict__ hsave, float* __restrict__ mean_out,
                                           float* __restrict__ rstd_out, float p, uint32_t thresh,
                                           uint64_t seed, const long long* ctr, uint64_t site,
                                           float eps, RowVec<D / 64>& o, size_t wt_bytes = 0) {
  constexpr int VEC = D / 64;
  if (has_t) {
    if (p > 0.f) {
      const uint32_t km = keep_bits<VEC>(seed, ctr, site, base, thresh);
      const float sc = 1.f / (1.f - p);
#pragma unroll
      for (int i = 0; i < VEC; ++i) t.v[i] = ((km >> i) & 1u) ? t.v[i] * sc : 0.f;
    }
#pragma unroll
    for (int i = 0; i < VEC; ++i) h.v[i] += t.v[i];
  }
  // wt_bytes > 0: y / hsave (that many bytes each) stored write-through
  if (hsave) {
    if (wt_bytes) h.store_bf(hsave + base, WtBuf(hsave, wt_bytes));
    else h.store_bf(hsave + base);
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
    const int col = lane * VEC + i;
    o.v[i] = (h.v[i] - mean) * rstd * gamma[col] + beta[col];
  }
  if (wt_bytes) o.store_bf(y + base, WtBuf(y, wt_bytes));
  else o.store_bf(y + base);
  if (lane == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
}

}  // namespace tdg
