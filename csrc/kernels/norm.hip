// Fused post-LN residual block tail for gfx950:
//   h = x + dropout(s);  y = LayerNorm(h) * gamma + beta      (eps = 1e-6)
// Forward saves h (bf16) and per-row mean / rstd (f32); the dropout keep-mask
// is regenerated from Philox in backward instead of being stored.
// Backward computes dh (the residual gradient), ds = dh*mask/(1-p) (the
// sublayer gradient), and deterministic two-stage column sums for dgamma,
// dbeta and -- fused -- the bias gradient of the sublayer's output projection
// (sum of ds over rows), saving a separate pass over ds.
//
// Replaces the reference's `LayerNormalization(epsilon=1e-6)(x + Dropout(...))`
// (reference: distributed_training_transformer/transformer_model.py:187-204,
// 219-248). One wave per row; each lane owns D/64 elements in runs of up to
// 8 (tdg_ln.h RowMap: every access instruction is contiguous across the
// wave), so D in {128, 256, 512, 1024}.
#include "tdg_common.h"
#include "tdg_ln.h"
#include "tdg_reduce.h"

namespace tdg {

// e4m3 copy of one LayerNorm output row (delayed per-tensor scale s8) for an
// fp8 GEMM; the row's |y| max folded into am.
// FMT 0: e4m3 (a LayerNorm output for an fp8 forward GEMM), 1: e5m2 (the
// backward's sublayer gradient ds for an fp8 dgrad / weight gradient)
// (stored write-through: wt is y8's WtBuf)
template <int D, int FMT = 0>
__device__ __forceinline__ void ln_row_y8(const RowVec<D / 64>& o, float s8, uint8_t* __restrict__ y8,
                                          size_t rbase, int lane, float& am, const WtBuf& wt) {
  constexpr int VEC = D / 64;
  int w[(VEC + 3) / 4];
#pragma unroll
  for (int i = 0; i < (VEC + 3) / 4; ++i) w[i] = 0;
#pragma unroll
  for (int i = 0; i < VEC; i += 2) {
    const float a = bf2f(f2bf(o.v[i])), b = bf2f(f2bf(o.v[i + 1]));
    am = fmaxf(am, fmaxf(fabsf(a), fabsf(b)));
    if constexpr (FMT == 0) {
      if ((i & 2) == 0) w[i / 4] = pack2_e4m3<false>(a * s8, b * s8, w[i / 4]);
      else w[i / 4] = pack2_e4m3<true>(a * s8, b * s8, w[i / 4]);
    } else {
      if ((i & 2) == 0) w[i / 4] = pack2_e5m2c<false>(a * s8, b * s8, w[i / 4]);
      else w[i / 4] = pack2_e5m2c<true>(a * s8, b * s8, w[i / 4]);
    }
  }
  uint8_t* dst = y8 + rbase + lane * RowMap<VEC>::W;
  if constexpr (VEC == 2) {
    *reinterpret_cast<uint16_t*>(dst) = (uint16_t)(w[0] & 0xffff);
  } else if constexpr (VEC == 4) {
    wt.st4(dst, (uint32_t)w[0]);
  } else {
#pragma unroll
    for (int i = 0; i < VEC / 8; ++i) wt.st8(dst + 512 * i, make_int2(w[2 * i], w[2 * i + 1]));
  }
}

// block-wide |y| max of the e4m3 copy -> one atomic per block (spread slots)
__device__ __forceinline__ void ln_amax_flush(float am, float* red8, unsigned* amax8) {
  am = wave_max(am);
  if ((threadIdx.x & 63) == 0) red8[threadIdx.x >> 6] = am;
  __syncthreads();
  if (threadIdx.x == 0 && amax8)
    atomic_amax(amax_word(amax8, blockIdx.x), fmaxf(fmaxf(red8[0], red8[1]), fmaxf(red8[2], red8[3])));
}

// RPW rows per wave (4 waves per block): the loads of all of a wave's rows
// are issued before the first row is reduced, so a row's stores overlap the
// next rows' loads still in flight.
template <int D, int RPW>
__global__ __launch_bounds__(256) void ln_fwd_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ s, const float* __restrict__ gamma,
    const float* __restrict__ beta, bf16_t* __restrict__ y, bf16_t* __restrict__ hsave,
    float* __restrict__ mean_out, float* __restrict__ rstd_out, int M, float p, uint32_t thresh,
    uint64_t seed, const long long* ctr, uint64_t site, float eps, uint8_t* __restrict__ y8,
    const float* __restrict__ s8p, unsigned* __restrict__ amax8, uint8_t* __restrict__ kbits) {
  constexpr int VEC = D / 64;
  const int lane = threadIdx.x & 63;
  const int r0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  __shared__ float red8[4];
  RowVec<VEC> h[RPW], t[RPW];
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const size_t rbase = (size_t)min(r0 + k, M - 1) * D;
    h[k].load_row(x + rbase, lane);
    if (s) t[k].load_row(s + rbase, lane);
  }
  float am = 0.f;
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const int row = r0 + k;
    if (row >= M) break;
    const size_t rbase = (size_t)row * D;
    RowVec<VEC> o;
    ln_row_fwd<D>(h[k], t[k], s != nullptr, rbase, row, lane, gamma, beta, y, hsave, mean_out,
                  rstd_out, p, thresh, seed, ctr, site, eps, o, (size_t)M * D * sizeof(bf16_t), kbits);
    if (y8) ln_row_y8<D>(o, s8p[0], y8, rbase, lane, am, WtBuf(y8, (size_t)M * D));
  }
  if (y8) ln_amax_flush(am, red8, amax8);
}

// RPW rows per wave, 4 waves (4*RPW rows) per 256-thread block; all loads of
// a wave's rows are issued before any of them is used (one memory latency per
// wave instead of one per row). Partial column sums go to part_g / part_b /
// part_s [gridDim.x, D].
template <int D, int RPW, int NWV>
__global__ __launch_bounds__(NWV * 64) void ln_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ hsave,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const float* __restrict__ gamma, bf16_t* __restrict__ dh_out, bf16_t* __restrict__ ds_out,
    const bf16_t* __restrict__ dres_in, float* __restrict__ part_g, float* __restrict__ part_b,
    float* __restrict__ part_s, int M, float p, uint32_t thresh, uint64_t seed,
    const long long* ctr, uint64_t site, int iters, uint8_t* __restrict__ ds8,
    const float* __restrict__ s8p, unsigned* __restrict__ amax8,
    const uint8_t* __restrict__ kbits) {
  constexpr int VEC = D / 64;
  __shared__ float red[NWV][D];
  float am8 = 0.f;  // |ds| max of the e5m2 copy
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float ag[VEC], ab[VEC], as[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) ag[i] = ab[i] = as[i] = 0.f;
  float gm[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) gm[i] = gamma[RowMap<VEC>::col(lane, i)];
  const float sc = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const WtBuf wdh(dh_out, (size_t)M * D * sizeof(bf16_t));  // write-through outputs
  const WtBuf wds(ds_out ? ds_out : dh_out, (size_t)M * D * sizeof(bf16_t));
  // `iters` row groups per block, partial column sums accumulated across them
  // (fewer partial rows for the fold: D = 1024 uses 2)
#pragma unroll 1
  for (int it = 0; it < iters; ++it) {
  const int r0 = (blockIdx.x * iters + it) * (NWV * RPW) + w * RPW;
  if (r0 >= M) break;
  RowVec<VEC> g[RPW], h[RPW], e[RPW];
  float mean[RPW], rstd[RPW];
  // the forward's keep bits (tdg_ln.h ln_row_fwd kbits; VEC >= 8): one
  // byte per 8 columns, loaded with the rows instead of regenerating the
  // Philox mask
  uint32_t kb[RPW];
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const int row = min(r0 + k, M - 1);
    const size_t rbase = (size_t)row * D;
    g[k].load_row(dy + rbase, lane);
    h[k].load_row(hsave + rbase, lane);
    if (dres_in) e[k].load_row(dres_in + rbase, lane);
    mean[k] = mean_in[row];
    rstd[k] = rstd_in[row];
    kb[k] = 0u;
    if constexpr (VEC >= 8) {
      if (kbits) {
#pragma unroll
        for (int c = 0; c < RowMap<VEC>::CH; ++c) kb[k] |= (uint32_t)kbits[rbase / 8 + 64 * c + lane] << (8 * c);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const int row = r0 + k;
    if (row >= M) break;
    const size_t rbase = (size_t)row * D;
    float sg = 0.f, sgx = 0.f;
    float xh[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      xh[i] = (h[k].v[i] - mean[k]) * rstd[k];
      ag[i] += g[k].v[i] * xh[i];
      ab[i] += g[k].v[i];
      const float gg = g[k].v[i] * gm[i];
      sg += gg;
      sgx += gg * xh[i];
    }
    sg = wave_sum(sg) * (1.f / D);
    sgx = wave_sum(sgx) * (1.f / D);
    RowVec<VEC> dh;
#pragma unroll
    for (int i = 0; i < VEC; ++i) dh.v[i] = rstd[k] * (g[k].v[i] * gm[i] - sg - xh[i] * sgx);
    RowVec<VEC> ds = dh;
    if (p > 0.f) {
      const uint32_t km = (VEC >= 8 && kbits) ? kb[k] : keep_bits<VEC>(seed, ctr, site, rbase, lane, thresh);
#pragma unroll
      for (int i = 0; i < VEC; ++i) ds.v[i] = ((km >> i) & 1u) ? dh.v[i] * sc : 0.f;
    }
    if (ds_out || ds8) {
      if (ds_out) ds.store_row(ds_out + rbase, lane, wds);
      if (ds8) ln_row_y8<D, 1>(ds, s8p[0], ds8, rbase, lane, am8, WtBuf(ds8, (size_t)M * D));
#pragma unroll
      for (int i = 0; i < VEC; ++i) as[i] += ds.v[i];
    }
    if (dres_in) {  // fused accumulation of the residual branch's other gradient
#pragma unroll
      for (int i = 0; i < VEC; ++i) dh.v[i] += e[k].v[i];
    }
    dh.store_row(dh_out + rbase, lane, wdh);
  }
  }  // row groups
  // cross-wave fold, one quantity at a time (NWV x D floats of LDS: 8 waves
  // x D = 1024 stay at 32 KB)
  float* const parts[3] = {part_g, part_b, part_s};
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    if (q == 2 && !part_s) break;
#pragma unroll
    for (int i = 0; i < VEC; ++i) red[w][RowMap<VEC>::col(lane, i)] = q == 0 ? ag[i] : q == 1 ? ab[i] : as[i];
    __syncthreads();
    for (int col = threadIdx.x; col < D; col += NWV * 64) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < NWV; ++k) a += red[k][col];
      parts[q][(size_t)blockIdx.x * D + col] = a;
    }
    __syncthreads();
  }
  if (ds8) {  // one atomic per block (spread amax words)
    am8 = wave_max(am8);
    if (lane == 0) red[0][w] = am8;
    __syncthreads();
    if (threadIdx.x == 0 && amax8) {
      float m = 0.f;
#pragma unroll
      for (int k = 0; k < NWV; ++k) m = fmaxf(m, red[0][k]);
      atomic_amax(amax_word(amax8, blockIdx.x), m);
    }
  }
}

}  // namespace tdg

using namespace tdg;

namespace {
template <int D>
void ln_fwd_d(const void* x, const void* s, const float* gamma, const float* beta, void* y,
              void* hsave, float* mean, float* rstd, int M, float p, uint64_t seed,
              const long long* ctr, uint64_t site, float eps, void* y8, const float* s8,
              unsigned* amax8, void* kbits, hipStream_t st) {
  const uint32_t thresh = dropout_thresh(p);
  // one row per wave measured best with dropout (2 rows: 8.1 vs 8.2 us
  // without, 11.1 vs 9.3 us with, D = 1024 x 8192 rows); a grid-strided
  // variant (fewer waves, each loading its next row while it reduces and
  // stores the current one) lost 2-9 us per call (profiles/r3s2/ln_fwd_strided.txt)
  hipLaunchKernelGGL((ln_fwd_kernel<D, 1>), dim3(cdiv(M, 4)), dim3(256), 0, st, (const bf16_t*)x,
                     (const bf16_t*)s, gamma, beta, (bf16_t*)y, (bf16_t*)hsave, mean, rstd, M, p,
                     thresh, seed, ctr, site, eps, (uint8_t*)y8, s8, amax8, (uint8_t*)kbits);
}
template <int D>
void ln_bwd_d(const void* dy, const void* hsave, const float* mean, const float* rstd,
              const float* gamma, void* dh, void* ds, const void* dres, float* dgamma,
              float* dbeta, float* dbias, float* ws, int M, float p, uint64_t seed, const long long* ctr, uint64_t site,
              int accumulate, int skip_reduce, int rpb, void* ds8, const float* s8, unsigned* amax8,
              const void* kbits, hipStream_t st) {
  const uint32_t thresh = dropout_thresh(p);
  // rpb rows per block (kernels.py ln_bwd_nparts): 16 on 4 waves, 32 / 64 on
  // 8 waves (fewer partial rows for the fold); RPW rows per wave per pass
  constexpr int RPW = D >= 1024 ? 2 : 4;
  const int nb = cdiv(M, rpb);
  float* pg = ws;
  float* pb = ws + (size_t)nb * D;
  float* ps = dbias ? ws + 2 * (size_t)nb * D : nullptr;
  if (rpb <= 16)
    hipLaunchKernelGGL((ln_bwd_kernel<D, RPW, 4>), dim3(nb), dim3(256), 0, st, (const bf16_t*)dy,
                       (const bf16_t*)hsave, mean, rstd, gamma, (bf16_t*)dh, (bf16_t*)ds,
                       (const bf16_t*)dres, pg, pb, ps, M, p, thresh, seed, ctr, site,
                       max(1, rpb / (RPW * 4)), (uint8_t*)ds8, s8, amax8, (const uint8_t*)kbits);
  else
    hipLaunchKernelGGL((ln_bwd_kernel<D, RPW, 8>), dim3(nb), dim3(512), 0, st, (const bf16_t*)dy,
                       (const bf16_t*)hsave, mean, rstd, gamma, (bf16_t*)dh, (bf16_t*)ds,
                       (const bf16_t*)dres, pg, pb, ps, M, p, thresh, seed, ctr, site,
                       max(1, rpb / (RPW * 8)), (uint8_t*)ds8, s8, amax8, (const uint8_t*)kbits);
  if (skip_reduce) return;  // partials folded later by tdg_reduce_partials_multi
  const float beta = accumulate ? 1.f : 0.f;
  ReduceSet rs{{pg, pb, ps}, {dgamma, dbeta, dbias}};
  hipLaunchKernelGGL(reduce_partials3_kernel, dim3(cdiv(D, 16), dbias ? 3 : 2), dim3(256), 0, st,
                     rs, D, nb, beta);
}
}  // namespace

extern "C" int tdg_ln_fwd(const void* x, const void* s, const float* gamma, const float* beta,
                          void* y, void* hsave, float* mean, float* rstd, int M, int D, float p,
                          uint64_t seed, const long long* ctr, uint64_t site, float eps, void* y8,
                          const float* s8, unsigned* amax8, void* kbits, hipStream_t st) {
  if (kbits && D < 512) return -3;  // keep-bit bitmap: whole bytes per lane (D >= 512)
#define TDG_LN_F(DD) \
  ln_fwd_d<DD>(x, s, gamma, beta, y, hsave, mean, rstd, M, p, seed, ctr, site, eps, y8, s8, amax8, kbits, st); \
  return 0;
  switch (D) {
    case 128: TDG_LN_F(128)
    case 256: TDG_LN_F(256)
    case 512: TDG_LN_F(512)
    case 1024: TDG_LN_F(1024)
    default: return -1;
  }
#undef TDG_LN_F
}

// ws must hold 3 * ceil(M / rpb) * D floats.
extern "C" int tdg_ln_bwd(const void* dy, const void* hsave, const float* mean, const float* rstd,
                          const float* gamma, void* dh, void* ds, const void* dres, float* dgamma,
                          float* dbeta, float* dbias, float* ws, int M, int D, float p,
                          uint64_t seed, const long long* ctr, uint64_t site, int accumulate,
                          int skip_reduce, int rpb, void* ds8, const float* s8, unsigned* amax8,
                          const void* kbits, hipStream_t st) {
  if (rpb != 16 && rpb != 32 && rpb != 64) return -2;
  if (ds8 && !s8) return -2;
  if (kbits && D < 512) return -3;
#define TDG_LN_B(DD)                                                                              \
  ln_bwd_d<DD>(dy, hsave, mean, rstd, gamma, dh, ds, dres, dgamma, dbeta, dbias, ws, M, p, seed, \
               ctr, site, accumulate, skip_reduce, rpb, ds8, s8, amax8, kbits, st);              \
  return 0;
  switch (D) {
    case 128: TDG_LN_B(128)
    case 256: TDG_LN_B(256)
    case 512: TDG_LN_B(512)
    case 1024: TDG_LN_B(1024)
    default: return -1;
  }
#undef TDG_LN_B
}

// Deferred stage-2 folds of G (<= MAXR) independent column reductions
// out[g][n] (=|+=) sum_p part[g][p][n] (nparts[g] partial rows, N columns),
// one launch: the LayerNorm dgamma / dbeta / sublayer-bias partials of a whole
// backward, folded together when the deferred weight gradients flush
// instead of one small launch per LayerNorm.
namespace tdg {
constexpr int MAXR = 96;
struct MultiReduce {
  const float* part[MAXR];
  float* out[MAXR];
  int nparts[MAXR];
};
__global__ __launch_bounds__(256) void reduce_partials_multi_kernel(MultiReduce mr, int N,
                                                                    float beta) {
  __shared__ float red[16][17];
  const float* part = mr.part[blockIdx.y];
  float* out = mr.out[blockIdx.y];
  const int P = mr.nparts[blockIdx.y];
  const int c = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int col = blockIdx.x * 16 + c;
  float s = 0.f;
  if (col < N) {
#pragma unroll 8
    for (int q = g; q < P; q += 16) s += part[(size_t)q * N + col];
  }
  red[g][c] = s;
  __syncthreads();
  if (g == 0 && col < N) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][c];
    out[col] = (beta != 0.f ? beta * out[col] : 0.f) + t;
  }
}
// N % 4 == 0: 16-byte loads, a 64-column (256-byte) strip per block, 16 row
// groups; every partial row is read in whole 128-byte lines
__global__ __launch_bounds__(256) void reduce_partials_multi4_kernel(MultiReduce mr, int N,
                                                                     float beta) {
  __shared__ float4 red[16][17];
  const float* part = mr.part[blockIdx.y];
  float* out = mr.out[blockIdx.y];
  const int P = mr.nparts[blockIdx.y];
  const int c = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int col = blockIdx.x * 64 + c * 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (col < N) {
#pragma unroll 8
    for (int q = g; q < P; q += 16) {
      const float4 v = *reinterpret_cast<const float4*>(part + (size_t)q * N + col);
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
  }
  red[g][c] = s;
  __syncthreads();
  if (g == 0 && col < N) {
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      t.x += red[k][c].x;
      t.y += red[k][c].y;
      t.z += red[k][c].z;
      t.w += red[k][c].w;
    }
    float4* o = reinterpret_cast<float4*>(out + col);
    if (beta != 0.f) {
      const float4 b = *o;
      t.x += beta * b.x;
      t.y += beta * b.y;
      t.z += beta * b.z;
      t.w += beta * b.w;
    }
    *o = t;
  }
}
}  // namespace tdg

extern "C" int tdg_reduce_partials_multi(const float* const* parts, float* const* outs,
                                         const int* nparts, int G, int N, float beta,
                                         hipStream_t st) {
  if (G < 1 || G > MAXR) return -2;
  MultiReduce mr{};
  for (int i = 0; i < G; ++i) {
    mr.part[i] = parts[i];
    mr.out[i] = outs[i];
    mr.nparts[i] = nparts[i];
  }
  bool al = N % 4 == 0;  // float4 path: every base pointer 16-byte aligned
  for (int i = 0; i < G; ++i)
    al = al && (reinterpret_cast<uintptr_t>(parts[i]) % 16 == 0) &&
         (reinterpret_cast<uintptr_t>(outs[i]) % 16 == 0);
  if (al)
    hipLaunchKernelGGL(reduce_partials_multi4_kernel, dim3(cdiv(N, 64), G), dim3(256), 0, st, mr,
                       N, beta);
  else
    hipLaunchKernelGGL(reduce_partials_multi_kernel, dim3(cdiv(N, 16), G), dim3(256), 0, st, mr, N,
                       beta);
  return 0;
}
