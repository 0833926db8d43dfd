// MFMA bf16 GEMM: public C entry points (kernels and their instantiations:
// gemm_impl.h, gemm_<layout>.hip) plus the bias-gradient column sums.
//
// Replaces the reference's Keras Dense MatMul+BiasAdd(+Relu) ops
// (reference: distributed_training_transformer/transformer_model.py:119-122,
// 165, 172-174, 333) and their gradients.
#include "gemm_impl.h"

namespace tdg {
#define TDG_DECL(NAME)                                                                          \
  int gemm_##NAME(int epi, bool f32, int tile_cfg, const bf16_t* A, const bf16_t* B, void* C,    \
                  const float* bias, const bf16_t* aux, int M, int N, int K, int lda, int ldb,     \
                  int ldc, int ldaux, float alpha, float beta, int splits, float* ws,              \
                  hipStream_t st);                                                               \
  int gemm_grouped_##NAME(const GemmGroup& g, int G, int M, int N, int K, int lda, int ldb,       \
                          int ldc, bool f32, float alpha, float beta, int tile_cfg,              \
                          hipStream_t st);                                                       \
  int gemm_ragged_##NAME(const R256Args& args, int tiles, int K, bool f32, float alpha,         \
                         float beta, int impl, hipStream_t st);
TDG_DECL(nt)
TDG_DECL(nn)
TDG_DECL(tn)
TDG_DECL(tt)
#undef TDG_DECL

// Column sum of a bf16 [M, N] matrix (row stride ld) into f32 out[N]
// (out = beta*out + sum): the bias gradient. Deterministic two-stage:
// block (bx, by) sums columns [64bx, 64bx+64) over rows [by*RB, by*RB+RB)
// with 16-byte loads (8 columns per thread, 32 row lanes), then
// reduce_partials folds the row chunks.
__global__ __launch_bounds__(256) void colsum_partial_kernel(const bf16_t* __restrict__ X,
                                                             float* __restrict__ part, int M, int N,
                                                             int ld, int rows_per_block) {
  __shared__ float red[32][65];
  const int cg = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int col0 = blockIdx.x * 64 + cg * 8;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;
  const bool vec = (col0 + 8 <= N) && (ld % 8 == 0);
  for (int r = r0 + rl; r < r1; r += 32) {
    const bf16_t* p = X + (size_t)r * ld + col0;
    if (vec) {
      const short8_t v = *reinterpret_cast<const short8_t*>(p);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += bf2f((bf16_t)v[i]);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (col0 + i < N) acc[i] += bf2f(p[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[rl][cg * 8 + i] = acc[i];
  __syncthreads();
  if (threadIdx.x < 64) {
    float s = 0.f;
#pragma unroll 8
    for (int k = 0; k < 32; ++k) s += red[k][threadIdx.x];
    const int col = blockIdx.x * 64 + threadIdx.x;
    if (col < N) part[(size_t)blockIdx.y * N + col] = s;
  }
}

// Grouped column sums: up to 32 same-shape problems (blockIdx.z), partials
// [z][P][N] in one workspace, then one grouped stage-2 fold.
struct ColsumGroup {
  const bf16_t* X[32];
  float* out[32];
};

__global__ __launch_bounds__(256) void colsum_partial_grouped_kernel(ColsumGroup grp,
                                                                     float* __restrict__ part, int M,
                                                                     int N, int ld,
                                                                     int rows_per_block) {
  __shared__ float red[32][65];
  const bf16_t* X = grp.X[blockIdx.z];
  float* pz = part + (size_t)blockIdx.z * gridDim.y * N;
  const int cg = threadIdx.x & 7, rl = threadIdx.x >> 3;
  const int col0 = blockIdx.x * 64 + cg * 8;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.f;
  const bool vec = (col0 + 8 <= N) && (ld % 8 == 0);
  for (int r = r0 + rl; r < r1; r += 32) {
    const bf16_t* p = X + (size_t)r * ld + col0;
    if (vec) {
      const short8_t v = *reinterpret_cast<const short8_t*>(p);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += bf2f((bf16_t)v[i]);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (col0 + i < N) acc[i] += bf2f(p[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[rl][cg * 8 + i] = acc[i];
  __syncthreads();
  if (threadIdx.x < 64) {
    float s = 0.f;
#pragma unroll 8
    for (int k = 0; k < 32; ++k) s += red[k][threadIdx.x];
    const int col = blockIdx.x * 64 + threadIdx.x;
    if (col < N) pz[(size_t)blockIdx.y * N + col] = s;
  }
}

__global__ __launch_bounds__(256) void reduce_partials_grouped_kernel(ColsumGroup grp,
                                                                      const float* __restrict__ part,
                                                                      int N, int P, float beta) {
  __shared__ float red[4][64];
  const float* pz = part + (size_t)blockIdx.y * P * N;
  float* out = grp.out[blockIdx.y];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + c;
  float s = 0.f;
  if (col < N) {
#pragma unroll 8
    for (int p = g; p < P; p += 4) s += pz[(size_t)p * N + col];
  }
  red[g][c] = s;
  __syncthreads();
  if (g == 0 && col < N) {
    const float t = red[0][c] + red[1][c] + red[2][c] + red[3][c];
    out[col] = (beta != 0.f ? beta * out[col] : 0.f) + t;
  }
}

}  // namespace tdg

// Public launcher. a_kc/b_kc select operand layouts. Returns 0 on success.
extern "C" int tdg_gemm(const void* A, const void* B, void* C, const float* bias, const void* aux,
                        int M, int N, int K, int lda, int ldb, int ldc, int ldaux, int a_kc,
                        int b_kc, int epi, int out_f32, float alpha, float beta, int tile_cfg,
                        int splits, float* ws, hipStream_t st) {
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* b = (const bf16_t*)B;
  const bf16_t* x = (const bf16_t*)aux;
  auto fn = a_kc ? (b_kc ? gemm_nt : gemm_nn) : (b_kc ? gemm_tt : gemm_tn);
  return fn(epi, out_f32 != 0, tile_cfg, a, b, C, bias, x, M, N, K, lda, ldb, ldc, ldaux, alpha,
            beta, splits, ws, st);
}

// Grouped GEMM: G (<= 32) problems of one shape / layout, plain epilogue
// (alpha, beta), one launch. Returns 0 on success.
extern "C" int tdg_gemm_grouped(const void* const* A, const void* const* B, void* const* C, int G,
                                int M, int N, int K, int lda, int ldb, int ldc, int a_kc, int b_kc,
                                int out_f32, float alpha, float beta, int tile_cfg, hipStream_t st) {
  if (G < 1 || G > MAXG) return -2;
  GemmGroup g{};
  for (int i = 0; i < G; ++i) {
    g.A[i] = (const bf16_t*)A[i];
    g.B[i] = (const bf16_t*)B[i];
    g.C[i] = C[i];
  }
  auto fn = a_kc ? (b_kc ? gemm_grouped_nt : gemm_grouped_nn)
                 : (b_kc ? gemm_grouped_tt : gemm_grouped_tn);
  return fn(g, G, M, N, K, lda, ldb, ldc, out_f32 != 0, alpha, beta, tile_cfg, st);
}

// Ragged grouped GEMM: P (<= 64) problems sharing K and layout, in runs of
// equal shape (<= 8 runs), plain epilogue, ONE launch of 256x256 tiles.
// shapes[7*i..] = (M, N, lda, ldb, ldc, t_first, t_count) of problem i:
// tiles [t_first, t_first + t_count) of it (t_count < 0: all; a partial
// problem is a run of its own). Returns 0 on success.
extern "C" int tdg_gemm_ragged(const void* const* A, const void* const* B, void* const* C, int P,
                               const int* shapes, int K, int a_kc, int b_kc, int out_f32,
                               float alpha, float beta, float* const* bias_out, int impl,
                               hipStream_t st) {
  if (P < 1 || P > R256_MAXP) return -2;
  R256Args args{};
  int ncls = 0, tiles = 0;
  bool prev_partial = false;
  for (int i = 0; i < P; ++i) {
    const int* s = shapes + 7 * i;
    const int tpp = cdiv(s[0], 256) * cdiv(s[1], 256);
    const int first = s[5], count = s[6] < 0 ? tpp - s[5] : s[6];
    if (first < 0 || count <= 0 || first + count > tpp) return -8;
    const bool partial = count != tpp;
    const bool same = ncls > 0 && !partial && !prev_partial && args.cls[ncls - 1].M == s[0] &&
                      args.cls[ncls - 1].N == s[1] && args.cls[ncls - 1].lda == s[2] &&
                      args.cls[ncls - 1].ldb == s[3] && args.cls[ncls - 1].ldc == s[4];
    if (!same) {
      if (ncls == R256_MAXC) return -5;
      R256Class& c = args.cls[ncls++];
      c.M = s[0]; c.N = s[1]; c.lda = s[2]; c.ldb = s[3]; c.ldc = s[4];
      c.tiles_m = cdiv(s[0], 256); c.tiles_n = cdiv(s[1], 256);
      c.tile_start = tiles; c.prob_start = i; c.t_first = first;
      if ((!a_kc && s[2] % 8) || (!b_kc && s[3] % 8)) return -6;
    }
    prev_partial = partial;
    tiles += count;
    args.A[i] = (const bf16_t*)A[i];
    args.B[i] = (const bf16_t*)B[i];
    args.C[i] = C[i];
    args.bias_out[i] = bias_out ? bias_out[i] : nullptr;
    if (args.bias_out[i] && a_kc) return -7;  // row sums need the MN-contiguous A path
  }
  args.ncls = ncls;
  if (impl != 0 && (a_kc || b_kc)) return -4;  // (pipelined: TN weight gradients only)
  if (a_kc && b_kc) return gemm_ragged_nt(args, tiles, K, out_f32 != 0, alpha, beta, 0, st);
  if (a_kc && !b_kc) return out_f32 ? -4 : gemm_ragged_nn(args, tiles, K, false, alpha, beta, 0, st);
  if (!a_kc && !b_kc) return gemm_ragged_tn(args, tiles, K, out_f32 != 0, alpha, beta, impl, st);
  return -4;
}

extern "C" void tdg_colsum(const void* X, float* out, float* part, int M, int N, int ld,
                           int rows_per_block, float beta, hipStream_t st) {
  const int nparts = cdiv(M, rows_per_block);
  dim3 grid(cdiv(N, 64), nparts);
  hipLaunchKernelGGL(colsum_partial_kernel, grid, dim3(256), 0, st, (const bf16_t*)X, part, M, N,
                     ld, rows_per_block);
  launch_reduce_partials(part, out, N, nparts, beta, st);
}

// Grouped bias gradients: out[g][n] (=|+=) sum_m X[g][m][n], G <= 32 problems.
extern "C" int tdg_colsum_grouped(const void* const* X, float* const* out, int G, float* part,
                                  int M, int N, int ld, int rows_per_block, float beta,
                                  hipStream_t st) {
  if (G < 1 || G > 32) return -2;
  ColsumGroup g{};
  for (int i = 0; i < G; ++i) {
    g.X[i] = (const bf16_t*)X[i];
    g.out[i] = out[i];
  }
  const int nparts = cdiv(M, rows_per_block);
  hipLaunchKernelGGL(colsum_partial_grouped_kernel, dim3(cdiv(N, 64), nparts, G), dim3(256), 0, st,
                     g, part, M, N, ld, rows_per_block);
  hipLaunchKernelGGL(reduce_partials_grouped_kernel, dim3(cdiv(N, 64), G), dim3(256), 0, st, g,
                     part, N, nparts, beta);
  return 0;
}
