// Fused token embedding + sqrt(d) scale + sinusoidal positional encoding +
// dropout (forward), and the embedding-table gradient (backward).
//
// Replaces reference: distributed_training_transformer/transformer_model.py:
// 29-53 (positional_encoding, interleaved sin/cos), 270-279 and 301-308
// (Embedding -> *sqrt(d) -> +PE[:L] -> Dropout). The PE table is computed once
// at model build (f32, [max_len, d], as the reference does) and read here; it
// stays L2-resident.
#include "tdg_common.h"
#include "tdg_ln.h"

#include <algorithm>

namespace tdg {

// out[row, :] = drop(table[tok[row]] * scale + pe[row % L])
// One wave per row, VEC = D/64 elements per lane (tdg_ln.h RowMap).
template <int D, typename TokT>
__global__ __launch_bounds__(256) void embed_fwd_kernel(
    const TokT* __restrict__ tok, const bf16_t* __restrict__ table, const float* __restrict__ pe,
    bf16_t* __restrict__ out, int M, int L, float scale, float p, uint32_t thresh, uint64_t seed,
    const long long* __restrict__ ctr, uint64_t site) {
  constexpr int VEC = D / 64;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int pos = row % L;
  const long long t = (long long)tok[row];
  const float* pr = pe + (size_t)pos * D;
  RowVec<VEC> v;
  v.load_row(table + t * D, lane);
#pragma unroll
  for (int i = 0; i < VEC; ++i) v.v[i] = v.v[i] * scale + pr[RowMap<VEC>::col(lane, i)];
  if (p > 0.f) {
    const float sc = 1.f / (1.f - p);
    const uint32_t km = keep_bits<VEC>(seed, ctr, site, (size_t)row * D, lane, thresh);
#pragma unroll
    for (int i = 0; i < VEC; ++i) v.v[i] = ((km >> i) & 1u) ? v.v[i] * sc : 0.f;
  }
  v.store_row(out + (size_t)row * D, lane);
}

// Keep bit of column lane + 64 c of a row for the backward kernels below, whose
// lanes own strided columns (coalesced atomics): each lane draws the 8-element
// run 8 lane + 512 s once (one Philox call per 8 elements instead of one per
// element) and the bits are fetched from the owning lane.
template <int D>
struct RowKeep {
  static constexpr int NS = (D + 511) / 512;
  uint32_t m[NS];
  __device__ __forceinline__ void draw(uint64_t seed, const long long* ctr, uint64_t site,
                                       size_t rbase, int lane, uint32_t thresh) {
    const uint64_t off = rng_offset(ctr, site);
#pragma unroll
    for (int s = 0; s < NS; ++s)
      m[s] = dropout_keep_run<8>(seed, off, rbase + 512 * s + 8 * lane, thresh);
  }
  // c: a constant after unrolling, so m[] stays in registers
  __device__ __forceinline__ bool keep(int c, int lane) const {
    const int col = c * 64 + lane;
    const uint32_t mm = (uint32_t)__shfl((int)m[c >> 3], (col >> 3) & 63, 64);
    return (mm >> (col & 7)) & 1u;
  }
};

// dtable[tok[row]] += drop_mask * dout[row] * scale  (f32 atomics into the
// f32 master-gradient buffer; rows of 2*D bytes per wave-instruction pair).
template <int D, typename TokT>
__global__ __launch_bounds__(256) void embed_bwd_kernel(
    const TokT* __restrict__ tok, const bf16_t* __restrict__ dout, float* __restrict__ dtable,
    int M, float scale, float p, uint32_t thresh, uint64_t seed, const long long* ctr, uint64_t site) {
  constexpr int VEC = D / 64;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const long long t = (long long)tok[row];
  const size_t rbase = (size_t)row * D;
  const float sc = p > 0.f ? scale / (1.f - p) : scale;
  RowKeep<D> rk;
  if (p > 0.f) rk.draw(seed, ctr, site, rbase, lane, thresh);
  // column c*64+lane: every atomic wave-instruction covers 256 contiguous bytes
#pragma unroll
  for (int c = 0; c < VEC; ++c) {
    const int col = c * 64 + lane;
    float g = bf2f(dout[rbase + col]) * sc;
    if (p > 0.f && !rk.keep(c, lane)) g = 0.f;
    atomicAdd(dtable + t * D + col, g);
  }
}

// Deterministic variant: contributions are added as 2^-32 fixed-point int64,
// so the sum is independent of the order the atomics land in (integer
// addition is associative); embed_acc_convert turns the accumulator into the
// f32 gradient and re-zeroes it. Resolution 2.3e-10, range +-2^31.
constexpr float FX_SCALE = 4294967296.f;  // 2^32

template <int D, typename TT>
__global__ __launch_bounds__(256) void embed_bwd_fx_kernel(
    const TT* __restrict__ tok, const bf16_t* __restrict__ dout, unsigned long long* __restrict__ acc,
    int M, float scale, float p, uint32_t thresh, uint64_t seed, const long long* ctr,
    uint64_t site) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const long long t = (long long)tok[row];
  const size_t rbase = (size_t)row * D;
  const float sc = p > 0.f ? scale / (1.f - p) : scale;
  RowKeep<D> rk;
  if (p > 0.f) rk.draw(seed, ctr, site, rbase, lane, thresh);
#pragma unroll
  for (int c = 0; c < D / 64; ++c) {
    const int col = c * 64 + lane;
    float g = bf2f(dout[rbase + col]) * sc;
    if (p > 0.f && !rk.keep(c, lane)) g = 0.f;
    const long long fx = (long long)rintf(g * FX_SCALE);
    if (fx != 0) atomicAdd(acc + t * D + col, (unsigned long long)fx);
  }
}

// 4 elements per thread and iteration: two 16-byte accumulator loads, one
// 16-byte write-through gradient store (the gradients are read by Adam on
// every XCD), the accumulator zeroed only where a row was touched.
// n % 4 == 0, out 16-byte aligned.
__global__ __launch_bounds__(256) void embed_acc_convert4_kernel(long long* __restrict__ acc,
                                                                 float* __restrict__ out,
                                                                 long long n, float beta) {
  const WtBuf wt(out, (size_t)n * sizeof(float));
  const long long stride = (long long)gridDim.x * blockDim.x * 4;
  for (long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
    longlong2* a2 = reinterpret_cast<longlong2*>(acc + i);
    const longlong2 x = a2[0], y = a2[1];
    float4 o = make_float4((float)x.x * (1.f / FX_SCALE), (float)x.y * (1.f / FX_SCALE),
                           (float)y.x * (1.f / FX_SCALE), (float)y.y * (1.f / FX_SCALE));
    if (beta != 0.f) {
      const float4 b = *reinterpret_cast<const float4*>(out + i);
      o.x += beta * b.x;
      o.y += beta * b.y;
      o.z += beta * b.z;
      o.w += beta * b.w;
    }
    wt.st16(out + i, o);
    if ((x.x | x.y | y.x | y.y) != 0) {
      a2[0] = make_longlong2(0, 0);
      a2[1] = make_longlong2(0, 0);
    }
  }
}

__global__ __launch_bounds__(256) void embed_acc_convert_kernel(long long* __restrict__ acc,
                                                                float* __restrict__ out,
                                                                long long n, float beta) {
  const long long i0 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 2;
  for (long long i = i0; i < n; i += (long long)gridDim.x * blockDim.x * 2) {
    if (i + 1 < n) {
      const long long a0 = acc[i], a1 = acc[i + 1];
      float2 o;
      if (beta != 0.f) {
        o = *reinterpret_cast<float2*>(out + i);
        o.x = beta * o.x + (float)a0 * (1.f / FX_SCALE);
        o.y = beta * o.y + (float)a1 * (1.f / FX_SCALE);
      } else {
        o = make_float2((float)a0 * (1.f / FX_SCALE), (float)a1 * (1.f / FX_SCALE));
      }
      *reinterpret_cast<float2*>(out + i) = o;
      if (a0 != 0 || a1 != 0) {
        acc[i] = 0;
        acc[i + 1] = 0;
      }
    } else {
      const float v = (float)acc[i] * (1.f / FX_SCALE);
      out[i] = beta != 0.f ? beta * out[i] + v : v;
      acc[i] = 0;
    }
  }
}

}  // namespace tdg

using namespace tdg;

namespace {
template <int D, typename TT>
void fwd_d(const void* tok, const void* table, const float* pe, void* out, int M, int L,
           float scale, float p, uint64_t seed, const long long* ctr, uint64_t site, hipStream_t st) {
  const uint32_t thresh = dropout_thresh(p);
  hipLaunchKernelGGL((embed_fwd_kernel<D, TT>), dim3(cdiv(M, 4)), dim3(256), 0, st,
                     (const TT*)tok, (const bf16_t*)table, pe, (bf16_t*)out, M, L, scale, p,
                     thresh, seed, ctr, site);
}
template <int D, typename TT>
void bwd_d(const void* tok, const void* dout, float* dtable, int M, float scale, float p,
           uint64_t seed, const long long* ctr, uint64_t site, hipStream_t st) {
  const uint32_t thresh = dropout_thresh(p);
  hipLaunchKernelGGL((embed_bwd_kernel<D, TT>), dim3(cdiv(M, 4)), dim3(256), 0, st,
                     (const TT*)tok, (const bf16_t*)dout, dtable, M, scale, p, thresh, seed, ctr, site);
}
template <int D, typename TT>
void bwd_fx_d(const void* tok, const void* dout, unsigned long long* acc, int M, float scale, float p,
              uint64_t seed, const long long* ctr, uint64_t site, hipStream_t st) {
  const uint32_t thresh = dropout_thresh(p);
  hipLaunchKernelGGL((embed_bwd_fx_kernel<D, TT>), dim3(cdiv(M, 4)), dim3(256), 0, st,
                     (const TT*)tok, (const bf16_t*)dout, acc, M, scale, p, thresh, seed, ctr, site);
}
}  // namespace

#define TDG_D_SWITCH(F, TT, ...)                  \
  switch (D) {                                    \
    case 128: F<128, TT>(__VA_ARGS__); return 0;  \
    case 256: F<256, TT>(__VA_ARGS__); return 0;  \
    case 512: F<512, TT>(__VA_ARGS__); return 0;  \
    case 1024: F<1024, TT>(__VA_ARGS__); return 0; \
    default: return -1;                           \
  }

extern "C" int tdg_embed_fwd(const void* tok, int tok64, const void* table, const float* pe,
                             void* out, int M, int L, int D, float scale, float p, uint64_t seed,
                             const long long* ctr, uint64_t site, hipStream_t st) {
  if (tok64) {
    TDG_D_SWITCH(fwd_d, long long, tok, table, pe, out, M, L, scale, p, seed, ctr, site, st)
  } else {
    TDG_D_SWITCH(fwd_d, int, tok, table, pe, out, M, L, scale, p, seed, ctr, site, st)
  }
}

extern "C" int tdg_embed_bwd(const void* tok, int tok64, const void* dout, float* dtable, int M,
                             int D, float scale, float p, uint64_t seed, const long long* ctr, uint64_t site,
                             hipStream_t st) {
  if (tok64) {
    TDG_D_SWITCH(bwd_d, long long, tok, dout, dtable, M, scale, p, seed, ctr, site, st)
  } else {
    TDG_D_SWITCH(bwd_d, int, tok, dout, dtable, M, scale, p, seed, ctr, site, st)
  }
}

// Deterministic embedding backward: fixed-point accumulation into acc
// ([V, D] int64, all-zero on entry and on exit), then dtable = beta*dtable + acc.
extern "C" int tdg_embed_bwd_det(const void* tok, int tok64, const void* dout, float* dtable,
                                 long long* acc, int M, int D, long long V, float scale, float p,
                                 uint64_t seed, const long long* ctr, uint64_t site, float beta,
                                 hipStream_t st) {
  unsigned long long* a = reinterpret_cast<unsigned long long*>(acc);
  int rc = -1;
  if (tok64) {
    switch (D) {
      case 128: bwd_fx_d<128, long long>(tok, dout, a, M, scale, p, seed, ctr, site, st); rc = 0; break;
      case 256: bwd_fx_d<256, long long>(tok, dout, a, M, scale, p, seed, ctr, site, st); rc = 0; break;
      case 512: bwd_fx_d<512, long long>(tok, dout, a, M, scale, p, seed, ctr, site, st); rc = 0; break;
      case 1024: bwd_fx_d<1024, long long>(tok, dout, a, M, scale, p, seed, ctr, site, st); rc = 0; break;
    }
  } else {
    switch (D) {
      case 128: bwd_fx_d<128, int>(tok, dout, a, M, scale, p, seed, ctr, site, st); rc = 0; break;
      case 256: bwd_fx_d<256, int>(tok, dout, a, M, scale, p, seed, ctr, site, st); rc = 0; break;
      case 512: bwd_fx_d<512, int>(tok, dout, a, M, scale, p, seed, ctr, site, st); rc = 0; break;
      case 1024: bwd_fx_d<1024, int>(tok, dout, a, M, scale, p, seed, ctr, site, st); rc = 0; break;
    }
  }
  if (rc) return rc;
  const long long n = V * D;
  if (n % 4 == 0 && reinterpret_cast<uintptr_t>(dtable) % 16 == 0 &&
      reinterpret_cast<uintptr_t>(acc) % 16 == 0 && (size_t)n * sizeof(float) <= 0x7fffffffull) {
    const int blocks = (int)std::min<long long>(4096, (n / 4 + 255) / 256);
    hipLaunchKernelGGL(embed_acc_convert4_kernel, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st, acc,
                       dtable, n, beta);
    return 0;
  }
  const int blocks = (int)std::min<long long>(4096, (n / 2 + 255) / 256 + 1);
  hipLaunchKernelGGL(embed_acc_convert_kernel, dim3(blocks), dim3(256), 0, st, acc, dtable, n, beta);
  return 0;
}
