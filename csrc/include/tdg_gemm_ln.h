// Post-LN block tails fused into the d_model-wide GEMM that produces them
// (the 128x128-tile, 2x4-wave gemm_kernel of gemm_impl.h):
//
//   EPI_LNF (forward, after the output projection / FFN2):
//     h = bf16(x + dropout(bf16(A W^T + bias)));  y = LN(h) * gamma + beta
//     -> y, h (saved for the backward), mean, rstd
//   EPI_LNB (backward, in the dgrad that produces the LayerNorm's input
//   gradient dy = A W (+ C, the residual gradient already accumulated)):
//     dh = rstd * (dy*gamma - mean(dy*gamma) - xhat * mean(dy*gamma*xhat))
//     ds = dropout_mask * dh / (1 - p)
//     -> dh, ds and per-tile column partials of dgamma / dbeta / the
//        sublayer bias gradient (folded later by reduce_partials_multi)
//
// A LayerNorm row (D = 512 columns) spans the 4 column tiles of one 128-row
// band. Each tile reduces its 128 columns (cross-lane shuffles, then LDS over
// the 4 column waves), publishes one pair of floats per row with write-through
// (sc1) stores, and the band's 4 workgroups meet at an arrival counter: one
// lane per workgroup adds 1 (agent scope) after every storing wave drained its
// stores and the workgroup passed a barrier, then polls the counter (sc1 loads)
// until the band's 4 arrivals of THIS launch are in; the partner pairs are
// read with sc1 loads after a workgroup barrier (MI355X_MICROARCH.md "Valid
// forms", first row of the hand-off table). Counters only grow: a launch's
// target is the next multiple of 4 above the value its add returned, so no
// reset is needed between launches or HIP-graph replays (all launches that
// share the counters run in stream order and add exactly 4 per band).
//
// Co-residency: the 4 tiles of a band are blocks b, b+8, b+16, b+24 of the
// XCD-remapped raster (tdg_common.h xcd_remap: one XCD, and dispatched within
// 25 consecutive block ids), so whatever the number of resident workgroups,
// the bands whose 4 blocks are all resident complete and free their CUs --
// progress does not depend on all 256 workgroups being resident at once. A
// spin is still bounded (it then records the failure in `err` and goes on
// with wrong values instead of hanging the GPU; ops/kernels.py ln_xch_check).
//
// Replaces the separate ln_fwd / ln_bwd launches after / before these GEMMs
// (norm.hip; reference: distributed_training_transformer/transformer_model.py
// 187-204, 219-248).
#pragma once
#include "tdg_common.h"
#include "tdg_gemm.h"

namespace tdg {

constexpr int EPI_LNF = 4;
constexpr int EPI_LNB = 5;
constexpr int LN_BAND_TILES = 4;  // D / 128 column tiles per band (D = 512)

struct LnEpiArgs {
  // forward
  const bf16_t* x;  // residual input [M][D]
  const float* gamma;
  const float* beta;
  bf16_t* y;
  bf16_t* hsave;
  float* mean;
  float* rstd;
  // backward
  const bf16_t* h_in;  // the forward's saved h [M][D]
  const float* mean_in;
  const float* rstd_in;
  bf16_t* dh;
  bf16_t* ds;   // nullptr: ds = dh (no dropout)
  float* part;  // [3][bands][D] column partials: dgamma, dbeta, sublayer bias
  int bands;
  // dropout keep bits as a row-major bitmap [M][D / 32] words (bit c % 32 of
  // word c / 32 = column c): written by the forward (LNF, or ln_fwd_kernel),
  // read by the backward instead of regenerating the Philox mask
  uint32_t* kbits;
  // exchange
  float2* xch;    // [bands * 128][LN_BAND_TILES] per-tile row pairs
  unsigned* ctr;  // [bands] arrival counters
  unsigned* err;  // bounded-spin failures
  // dropout / numerics
  float p;
  uint32_t thresh;
  uint64_t seed;
  const long long* rng_ctr;
  uint64_t site;
  float eps;
  // lab only (scripts/ln_fused_lab.py): bit 1 no dropout mask, 2 no band
  // exchange (tile-local statistics), 4 no h (fwd) / ds (bwd) store, 8 no
  // row reductions, 16 no y (fwd) / dh (bwd) store. 0 in training.
  int ablate;
};

__device__ __forceinline__ void st_sc1_f2(float2* p, float a, float b) {
  const uint64_t v = (uint64_t)__float_as_uint(a) | ((uint64_t)__float_as_uint(b) << 32);
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float2 ld_sc1_f2(const float2* p) {
  const uint64_t v = __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return make_float2(__uint_as_float((uint32_t)v), __uint_as_float((uint32_t)(v >> 32)));
}

// One lane of the workgroup, after every storing wave's vmcnt(0) and a
// workgroup barrier: arrive at the band counter; returns the count at which
// the band's tiles of this launch are all in.
__device__ __forceinline__ unsigned band_arrive(unsigned* ctr) {
  const unsigned old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return (old / LN_BAND_TILES + 1u) * LN_BAND_TILES;
}
// ... then (the same lane) wait for the band's other tiles (bounded).
__device__ __forceinline__ void band_wait(const unsigned* ctr, unsigned target, unsigned* err) {
  for (int it = 0;; ++it) {
    const unsigned v = __hip_atomic_load(const_cast<unsigned*>(ctr), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    if ((int)(v - target) >= 0) break;
    if (it > (1 << 22)) {
      atomicOr(err, 1u);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
__device__ __forceinline__ void band_arrive_wait(unsigned* ctr, unsigned* err) {
  band_wait(ctr, band_arrive(ctr), err);
}

// Column sums over the tile's valid rows of NQ quantities held in the
// accumulator layout (c[q][j][e]: column 16j + 4g + e of the wave's 32), as
// partial rows part[q0 + q][band][n0 + col] (two wave halves folded in LDS).
template <int NQ>
__device__ __forceinline__ void tile_col_partials(float (&c)[NQ][2][4], float* cred, int q0, int wm,
                                                  int wn, int lane, int band, int n0, int D,
                                                  const LnEpiArgs& a) {
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) c[q][j][e] += __shfl_xor(c[q][j][e], o, 64);
  const int g = lane >> 4;
  if ((lane & 15) == 0) {
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) cred[(wm * NQ + q) * 128 + wn * 32 + 16 * j + 4 * g + e] = c[q][j][e];
  }
  __syncthreads();
  for (int k = threadIdx.x; k < NQ * 128; k += 512) {
    const int q = k / 128, col = k % 128;
    a.part[((size_t)(q0 + q) * a.bands + band) * D + n0 + col] = cred[q * 128 + col] + cred[(NQ + q) * 128 + col];
  }
  __syncthreads();  // cred is reused
}

// Row sums over the tile's 128 columns, in the swapped-operand accumulator
// layout (lane l: rows 16i + (l & 15) of the wave's 64-row half, 8 columns
// per row in two 16-column sub-tiles). v[i] in: the lane's partial of row i;
// out: the tile total of that row (every lane of the row). NQ independent
// quantities share the barriers. red: 2 x 4 x 64 x NQ floats of LDS.
template <int NQ>
__device__ __forceinline__ void tile_row_sums(float (&v)[NQ][4], float* red, int wm, int wn, int lane) {
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[q][i] += __shfl_xor(v[q][i], 16, 64);
      v[q][i] += __shfl_xor(v[q][i], 32, 64);
    }
  if (lane < 16) {
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[((q * 2 + wm) * 4 + wn) * 64 + 16 * i + lane] = v[q][i];
  }
  __syncthreads();
  const int r = lane & 15;
#pragma unroll
  for (int q = 0; q < NQ; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float* b = red + (q * 2 + wm) * 4 * 64 + 16 * i + r;
      v[q][i] = (b[0] + b[64]) + (b[128] + b[192]);
    }
  __syncthreads();  // red is reused
}

using EpiLn = EpiLds<EPI_NONE, false, 4, 2, 64>;  // bf16 stores of a 64 x 32 wave tile

// Forward tail. acc: the sublayer output s = bf16(A W^T + bias) (rounded as
// the unfused GEMM stores it); xr: the residual x of the lane's elements
// (prefetched before the main loop).
__device__ __forceinline__ void ln_fwd_epilogue(char* smem, const f32x4 (&acc)[4][2], int lane,
                                                int wid, int wm, int wn, int m0, int n0, int band,
                                                int tn, int M, int D, const LnEpiArgs& a,
                                                const int2 (&xr)[4][2]) {
  const int g = lane >> 4, r16 = lane & 15;
  const int mw0 = m0 + wm * 64, nw0 = n0 + wn * 32;
  float* red = reinterpret_cast<float*>(smem + 64 * 1024);
  f32x4 gm[2], bt[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = nw0 + 16 * j + 4 * g;
    gm[j] = *reinterpret_cast<const f32x4*>(a.gamma + c);
    bt[j] = *reinterpret_cast<const f32x4*>(a.beta + c);
  }
  const uint64_t off = rng_offset(a.rng_ctr, a.site);
  const float sc = a.p > 0.f ? 1.f / (1.f - a.p) : 1.f;
  f32x4 h[4][2];
  float v[1][4];
  uint32_t kw[4];  // keep bits of the row's 32 wave columns (for the backward)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = mw0 + 16 * i + r16;
    v[0][i] = 0.f;
    kw[i] = 0u;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = nw0 + 16 * j + 4 * g;
      uint32_t km = 0xfu;
      if (a.p > 0.f && !(a.ablate & 1))
        km = dropout_keep_run<4>(a.seed, off, (uint64_t)row * D + col, a.thresh);
      kw[i] |= km << (16 * j + 4 * g);
      const short4_t xv = __builtin_bit_cast(short4_t, xr[i][j]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float t = ((km >> e) & 1u) ? acc[i][j][e] * sc : 0.f;
        h[i][j][e] = bf2f(f2bf(bf2f((bf16_t)xv[e]) + t));
        v[0][i] += h[i][j][e];
      }
    }
  }
  if (a.kbits && a.p > 0.f) {  // one word per row from the 4 lane groups
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      kw[i] |= __shfl_xor(kw[i], 16, 64);
      kw[i] |= __shfl_xor(kw[i], 32, 64);
      const int row = mw0 + 16 * i + r16;
      if (g == 0 && row < M) a.kbits[(size_t)row * (D / 32) + nw0 / 32] = kw[i];
    }
  }
  if (!(a.ablate & 8)) tile_row_sums<1>(v, red, wm, wn, lane);
  float mu[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    mu[i] = v[0][i] * (1.f / 128.f);
    float s2 = 0.f;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = h[i][j][e] - mu[i];
        s2 += d * d;
      }
    v[0][i] = s2;
  }
  if (!(a.ablate & 8)) tile_row_sums<1>(v, red, wm, wn, lane);
  // publish (tile sum, tile M2) of the rows this wave half owns
  float2* X = a.xch;
  const bool xchg = !(a.ablate & 2);
  if (xchg && wn == 0 && lane < 16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = mw0 + 16 * i + lane;
      st_sc1_f2(X + (size_t)row * LN_BAND_TILES + tn, mu[i] * 128.f, v[0][i]);
    }
  }
  if (xchg) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) band_arrive_wait(a.ctr + band, a.err);
    __syncthreads();
  }
  float mean[4], rstd[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = mw0 + 16 * i + r16;
    float2 pt[LN_BAND_TILES];
#pragma unroll
    for (int t = 0; t < LN_BAND_TILES; ++t)
      pt[t] = xchg ? ld_sc1_f2(X + (size_t)row * LN_BAND_TILES + t) : make_float2(mu[i] * 128.f, v[0][i]);
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < LN_BAND_TILES; ++t) s += pt[t].x;
    mean[i] = s / (float)D;
    float m2 = 0.f;
#pragma unroll
    for (int t = 0; t < LN_BAND_TILES; ++t) {
      const float dm = pt[t].x * (1.f / 128.f) - mean[i];
      m2 += pt[t].y + 128.f * dm * dm;
    }
    rstd[i] = rsqrtf(m2 / (float)D + a.eps);
  }
  f32x4 y[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) y[i][j][e] = (h[i][j][e] - mean[i]) * rstd[i] * gm[j][e] + bt[j][e];
  char* wimg = smem + wid * EpiLn::BYTES;
  if (!(a.ablate & 4)) EpiLn::run(wimg, h, lane, a.hsave, D, M, D, mw0, nw0, 1.f, 0.f, nullptr, nullptr, 0, true);
  if (!(a.ablate & 16)) EpiLn::run(wimg, y, lane, a.y, D, M, D, mw0, nw0, 1.f, 0.f, nullptr, nullptr, 0, true);
  if (tn == 0 && wn == 0 && lane < 16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = mw0 + 16 * i + lane;
      if (row < M) {
        a.mean[row] = mean[i];
        a.rstd[row] = rstd[i];
      }
    }
  }
}

// Backward tail. acc: A W (dgrad); cr: the residual gradient C of the lane's
// elements (prefetched; zero when the GEMM has no C), hr: the saved h, mr /
// rr: mean / rstd of the lane's 4 rows, kw: the lane's 32-column keep-bit
// words of its 4 rows (a.kbits; else the mask is regenerated from Philox).
// The dgamma / dbeta column partials need no row statistics, so they are
// reduced and stored while the band's partners arrive.
__device__ __forceinline__ void ln_bwd_epilogue(char* smem, const f32x4 (&acc)[4][2], int lane,
                                                int wid, int wm, int wn, int m0, int n0, int band,
                                                int tn, int M, int D, const LnEpiArgs& a,
                                                bool has_c, const int2 (&cr)[4][2],
                                                const int2 (&hr)[4][2], const float (&mr)[4],
                                                const float (&rr)[4], const uint32_t (&kw)[4]) {
  const int g = lane >> 4, r16 = lane & 15;
  const int mw0 = m0 + wm * 64, nw0 = n0 + wn * 32;
  float* red = reinterpret_cast<float*>(smem + 64 * 1024);
  f32x4 gm[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) gm[j] = *reinterpret_cast<const f32x4*>(a.gamma + nw0 + 16 * j + 4 * g);
  // dy exactly as the unfused path sees it: bf16(bf16(acc) + C)
  f32x4 dy[4][2], xh[4][2];
  float v[2][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[0][i] = v[1][i] = 0.f;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const short4_t cv = __builtin_bit_cast(short4_t, cr[i][j]);
      const short4_t hv = __builtin_bit_cast(short4_t, hr[i][j]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float d = bf2f(f2bf(acc[i][j][e]));
        if (has_c) d = bf2f(f2bf(d + bf2f((bf16_t)cv[e])));
        dy[i][j][e] = d;
        xh[i][j][e] = (bf2f((bf16_t)hv[e]) - mr[i]) * rr[i];
        const float gg = d * gm[j][e];
        v[0][i] += gg;
        v[1][i] += gg * xh[i][j][e];
      }
    }
  }
  if (!(a.ablate & 8)) tile_row_sums<2>(v, red, wm, wn, lane);
  float2* X = a.xch;
  const bool xchg = !(a.ablate & 2);
  if (xchg && wn == 0 && lane < 16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = mw0 + 16 * i + lane;
      st_sc1_f2(X + (size_t)row * LN_BAND_TILES + tn, v[0][i], v[1][i]);
    }
  }
  unsigned target = 0;
  if (xchg) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) target = band_arrive(a.ctr + band);
  }
  // meanwhile: dgamma = sum dy * xhat, dbeta = sum dy over the valid rows
  float* cred = red + 2 * 2 * 4 * 64;  // past tile_row_sums' area
  {
    float c2[2][2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) c2[0][j][e] = c2[1][j][e] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (mw0 + 16 * i + r16 >= M) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          c2[0][j][e] += dy[i][j][e] * xh[i][j][e];
          c2[1][j][e] += dy[i][j][e];
        }
    }
    tile_col_partials<2>(c2, cred, 0, wm, wn, lane, band, n0, D, a);
  }
  if (xchg) {
    if (threadIdx.x == 0) band_wait(a.ctr + band, target, a.err);
    __syncthreads();
  }
  const float invD = 1.f / (float)D;
  float sg[4], sgx[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = mw0 + 16 * i + r16;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int t = 0; t < LN_BAND_TILES; ++t) {
      const float2 pt = xchg ? ld_sc1_f2(X + (size_t)row * LN_BAND_TILES + t) : make_float2(v[0][i], v[1][i]);
      s1 += pt.x;
      s2 += pt.y;
    }
    sg[i] = s1 * invD;
    sgx[i] = s2 * invD;
  }
  const uint64_t off = rng_offset(a.rng_ctr, a.site);
  const float sc = a.p > 0.f ? 1.f / (1.f - a.p) : 1.f;
  f32x4 dh[4][2], ds[4][2];
  float c1[1][2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) c1[0][j][e] = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = mw0 + 16 * i + r16;
    const bool in = row < M;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = nw0 + 16 * j + 4 * g;
      uint32_t km = 0xfu;
      if (a.p > 0.f && !(a.ablate & 1)) {
        km = a.kbits ? (kw[i] >> (16 * j + 4 * g)) & 0xfu
                     : dropout_keep_run<4>(a.seed, off, (uint64_t)row * D + col, a.thresh);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = rr[i] * (dy[i][j][e] * gm[j][e] - sg[i] - xh[i][j][e] * sgx[i]);
        dh[i][j][e] = d;
        ds[i][j][e] = ((km >> e) & 1u) ? d * sc : 0.f;
        if (in) c1[0][j][e] += ds[i][j][e];
      }
    }
  }
  char* wimg = smem + wid * EpiLn::BYTES;
  if (!(a.ablate & 16)) EpiLn::run(wimg, dh, lane, a.dh, D, M, D, mw0, nw0, 1.f, 0.f, nullptr, nullptr, 0, true);
  if (a.ds && !(a.ablate & 4)) EpiLn::run(wimg, ds, lane, a.ds, D, M, D, mw0, nw0, 1.f, 0.f, nullptr, nullptr, 0, true);
  // the sublayer bias gradient: column sums of ds
  tile_col_partials<1>(c1, cred, 2, wm, wn, lane, band, n0, D, a);
}

}  // namespace tdg
