// Deterministic two-stage column reductions shared by several kernels
// (bias gradients, LayerNorm dgamma/dbeta): stage 1 writes per-row-chunk
// partial sums [P][N]; this stage-2 kernel folds them.
#pragma once
#include "tdg_common.h"

namespace tdg {

// out[col] = beta*out[col] + sum_p part[p*N + col]. 256 threads per block
// cover 64 columns x 4 partial-lanes; grid = ceil(N / 64).
static __global__ __launch_bounds__(256) void reduce_partials_kernel(const float* __restrict__ part,
                                                              float* __restrict__ out, int N, int P,
                                                              float beta) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + c;
  float s = 0.f;
  if (col < N) {
#pragma unroll 8
    for (int p = g; p < P; p += 4) s += part[(size_t)p * N + col];
  }
  red[g][c] = s;
  __syncthreads();
  if (g == 0 && col < N) {
    const float t = red[0][c] + red[1][c] + red[2][c] + red[3][c];
    out[col] = (beta != 0.f ? beta * out[col] : 0.f) + t;
  }
}

// Up to 3 independent (partials, out) reductions in one launch (blockIdx.y).
struct ReduceSet {
  const float* part[3];
  float* out[3];
};
// 16 columns x 16 partial-lanes per block: many blocks even for small N
// (a LayerNorm's D = 512 columns x 3 sets = 96 blocks instead of 24).
static __global__ __launch_bounds__(256) void reduce_partials3_kernel(ReduceSet rs, int N, int P,
                                                                      float beta) {
  __shared__ float red[16][17];
  const float* part = rs.part[blockIdx.y];
  float* out = rs.out[blockIdx.y];
  const int c = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int col = blockIdx.x * 16 + c;
  float s = 0.f;
  if (col < N) {
#pragma unroll 8
    for (int p = g; p < P; p += 16) s += part[(size_t)p * N + col];
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

static inline void launch_reduce_partials(const float* part, float* out, int N, int P, float beta,
                                   hipStream_t st) {
  hipLaunchKernelGGL(reduce_partials_kernel, dim3(cdiv(N, 64)), dim3(256), 0, st, part, out, N, P,
                     beta);
}

}  // namespace tdg
