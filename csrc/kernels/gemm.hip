// MFMA bf16 GEMM for gfx950 with fused epilogues.
//
//   C[m,n] = alpha * sum_k A(m,k) * B(n,k)  (+ beta*C_old) (+ bias[n]) (act)
//
// A(m,k) is either "K-contiguous" (row-major [M][lda], the activation layout)
// or "M-contiguous" ([K][lda], i.e. a transposed view: wgrad's dY^T / X^T).
// B(n,k) likewise: K-contiguous ([N][ldb], torch [out,in] weights: forward)
// or N-contiguous ([K][ldb]: dgrad's W, wgrad's X).
//
// One kernel template covers forward (NT), dgrad (NN) and wgrad (TN): tiles
// are staged global->registers->LDS in their memory layout and the MFMA
// fragments are read with ds_read_b128 (K-contiguous images) or the gfx950
// transposing ds_read_b64_tr_b16 (M/N-contiguous images). Both LDS images are
// XOR-swizzled at 32-byte granularity so that either read is bank-conflict
// free (derivation in docs/KERNELS.md).
//
// MFMA: v_mfma_f32_16x16x32_bf16, 4 waves (2x2) per workgroup, 64-deep K tiles,
// double-buffered LDS with one barrier per K tile, register prefetch of the
// next tile issued before the MFMAs of the current one.
//
// Replaces the reference's Keras Dense MatMul+BiasAdd(+Relu) ops
// (reference: distributed_training_transformer/transformer_model.py:119-122,
// 165, 172-174, 333) and their gradients.
#include "tdg_common.h"

namespace tdg {

enum Epi : int {
  EPI_NONE = 0,       // alpha*acc (+beta*C)
  EPI_BIAS = 1,       // alpha*acc + bias[n]
  EPI_BIAS_RELU = 2,  // relu(alpha*acc + bias[n])
  EPI_DRELU = 3,      // alpha*acc * (aux[m,n] > 0)      (ReLU backward fused in dgrad)
};

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
  } else if constexpr (R == 128) {
    const int seg = (byte >> 5) ^ ((row & 3) | (((row >> 3) & 1) << 2));
    return row * 256 + (seg << 5) + (byte & 31);
  } else {
    static_assert(R == 64, "MN-contiguous tiles must be 64 or 128 wide");
    const int seg = (byte >> 5) ^ (((row >> 1) & 1) | (((row >> 3) & 1) << 1));
    return row * 128 + (seg << 5) + (byte & 31);
  }
}

// Staging of one operand tile (R = BM or BN rows/cols, BK deep).
template <bool KC, int R, int NT>
struct Stage {
  static constexpr int CHUNKS = R * BK * 2 / 16;  // 16-byte chunks per tile
  static constexpr int PER = CHUNKS / NT;
  static_assert(CHUNKS % NT == 0, "tile/thread mismatch");
  short8_t v[PER];

  // Global load of tile (mn0, k0). `len` = M or N, ld in elements.
  __device__ __forceinline__ void load(const bf16_t* __restrict__ X, int ld, int len, int K, int mn0,
                                       int k0, int tid) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int id = tid + i * NT;
      int mn, kk;
      if constexpr (KC) {
        const int row = id >> 3, c = id & 7;
        mn = mn0 + row;
        kk = k0 + c * 8;
        if (mn < len && kk + 8 <= K) {
          v[i] = *reinterpret_cast<const short8_t*>(X + (size_t)mn * ld + kk);
        } else {
          short8_t t = {0, 0, 0, 0, 0, 0, 0, 0};
          if (mn < len) {
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (kk + e < K) t[e] = (short)X[(size_t)mn * ld + kk + e];
          }
          v[i] = t;
        }
      } else {
        constexpr int CPR = R / 8;  // chunks per k-row
        const int row = id / CPR, c = id % CPR;
        kk = k0 + row;
        mn = mn0 + c * 8;
        if (kk < K && mn + 8 <= len) {
          v[i] = *reinterpret_cast<const short8_t*>(X + (size_t)kk * ld + mn);
        } else {
          short8_t t = {0, 0, 0, 0, 0, 0, 0, 0};
          if (kk < K) {
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if (mn + e < len) t[e] = (short)X[(size_t)kk * ld + mn + e];
          }
          v[i] = t;
        }
      }
    }
  }

  __device__ __forceinline__ void store(char* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int id = tid + i * NT;
      int row, byte;
      if constexpr (KC) {
        row = id >> 3;
        byte = (id & 7) * 16;
      } else {
        constexpr int CPR = R / 8;
        row = id / CPR;
        byte = (id % CPR) * 16;
      }
      *reinterpret_cast<short8_t*>(lds + lds_off<KC, R>(row, byte)) = v[i];
    }
  }
};

// MFMA operand fragment for 16 rows/cols starting at `base` within the tile,
// k-step s (32 deep). Lane l holds X(base + (l&15), 32s + 8(l>>4) + j), j<8.
template <bool KC, int R>
__device__ __forceinline__ short8_t frag(const char* lds, int base, int s, int lane) {
  if constexpr (KC) {
    const int row = base + (lane & 15);
    const int byte = (s * 4 + (lane >> 4)) * 16;
    return *reinterpret_cast<const short8_t*>(lds + lds_off<KC, R>(row, byte));
  } else {
    const int g = lane >> 4, w = lane & 15, q = w >> 2, p = w & 3;
    const int krow = s * 32 + 8 * g + q;
    const int byte = (base + 4 * p) * 2;
    const short4_t lo = lds_read_tr(lds + lds_off<KC, R>(krow, byte));
    const short4_t hi = lds_read_tr(lds + lds_off<KC, R>(krow + 4, byte));
    return cat4(lo, hi);
  }
}

template <int BM, int BN, int WM, int WN, bool A_KC, bool B_KC, int EPI, bool OUT_F32>
__global__ __launch_bounds__(WM* WN * 64) void gemm_kernel(
    const bf16_t* __restrict__ A, const bf16_t* __restrict__ B, void* __restrict__ Cv,
    const float* __restrict__ bias, const bf16_t* __restrict__ aux, int M, int N, int K, int lda,
    int ldb, int ldc, int ldaux, float alpha, float beta, int k_per_split, long long split_stride) {
  constexpr int NT = WM * WN * 64;
  constexpr int TM = BM / WM / 16;  // 16x16 subtiles per wave along M
  constexpr int TN = BN / WN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_m = cdiv(M, BM), tiles_n = cdiv(N, BN);
  const int nwg = tiles_m * tiles_n;
  const int t = xcd_remap(blockIdx.x, nwg);
  const int tm = t % tiles_m, tn = t / tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;

  // split-K range
  const int kb = blockIdx.z * k_per_split;
  const int ke = min(K, kb + k_per_split);
  const int nk = cdiv(ke - kb, BK);

  constexpr int BUF = A_BYTES + B_BYTES;  // one stage = A tile then B tile

  Stage<A_KC, BM, NT> sa;
  Stage<B_KC, BN, NT> sb;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    sa.load(A, lda, M, ke, m0, kb, tid);
    sb.load(B, ldb, N, ke, n0, kb, tid);
    sa.store(smem, tid);
    sb.store(smem + A_BYTES, tid);
    __syncthreads();
  }

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      sa.load(A, lda, M, ke, m0, kb + (kt + 1) * BK, tid);
      sb.load(B, ldb, N, ke, n0, kb + (kt + 1) * BK, tid);
    }
    const char* la = smem + cur * BUF;
    const char* lb = la + A_BYTES;
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
      short8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = frag<A_KC, BM>(la, wm * (BM / WM) + 16 * i, s, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = frag<B_KC, BN>(lb, wn * (BN / WN) + 16 * j, s, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    if (more) {
      sa.store(smem + (cur ^ 1) * BUF, tid);
      sb.store(smem + (cur ^ 1) * BUF + A_BYTES, tid);
    }
    __syncthreads();
  }

  // ---------------- epilogue: C/D layout col = lane&15, row = 4*(lane>>4) + r
  const int g = lane >> 4, cl = lane & 15;
  if (gridDim.z > 1) {
    // split-K partial: raw f32 slab, epilogue applied by the reduce kernel
    float* C = reinterpret_cast<float*>(Cv) + (size_t)blockIdx.z * split_stride;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * (BN / WN) + 16 * j + cl;
        if (n >= N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * (BM / WM) + 16 * i + 4 * g + r;
          if (m < M) C[(size_t)m * ldc + n] = acc[i][j][r];
        }
      }
    return;
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * (BN / WN) + 16 * j + cl;
    if (n >= N) continue;
    float bn = 0.f;
    if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU) bn = bias[n];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * (BM / WM) + 16 * i + 4 * g + r;
        if (m >= M) continue;
        float v = alpha * acc[i][j][r];
        if constexpr (EPI == EPI_BIAS) v += bn;
        if constexpr (EPI == EPI_BIAS_RELU) v = fmaxf(v + bn, 0.f);
        if constexpr (EPI == EPI_DRELU) {
          if (!(bf2f(aux[(size_t)m * ldaux + n]) > 0.f)) v = 0.f;
        }
        const size_t o = (size_t)m * ldc + n;
        if constexpr (OUT_F32) {
          float* C = reinterpret_cast<float*>(Cv);
          if (beta != 0.f) v += beta * C[o];
          C[o] = v;
        } else {
          bf16_t* C = reinterpret_cast<bf16_t*>(Cv);
          if (beta != 0.f) v += beta * bf2f(C[o]);
          C[o] = f2bf(v);
        }
      }
    }
  }
}

// Split-K reduction: C = sum_z slab[z] (+beta*C) with the epilogue.
template <int EPI, bool OUT_F32>
__global__ void splitk_reduce_kernel(const float* __restrict__ ws, void* __restrict__ Cv,
                                     const float* __restrict__ bias, const bf16_t* __restrict__ aux,
                                     int M, int N, int ldc, int ldaux, int splits,
                                     long long split_stride, float alpha, float beta) {
  const long long total = (long long)M * N;
  for (long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int m = (int)(idx / N), n = (int)(idx % N);
    const size_t o = (size_t)m * ldc + n;
    float v = 0.f;
    for (int z = 0; z < splits; ++z) v += ws[(size_t)z * split_stride + o];
    v *= alpha;
    if constexpr (EPI == EPI_BIAS) v += bias[n];
    if constexpr (EPI == EPI_BIAS_RELU) v = fmaxf(v + bias[n], 0.f);
    if constexpr (EPI == EPI_DRELU) {
      if (!(bf2f(aux[(size_t)m * ldaux + n]) > 0.f)) v = 0.f;
    }
    if constexpr (OUT_F32) {
      float* C = reinterpret_cast<float*>(Cv);
      if (beta != 0.f) v += beta * C[o];
      C[o] = v;
    } else {
      bf16_t* C = reinterpret_cast<bf16_t*>(Cv);
      if (beta != 0.f) v += beta * bf2f(C[o]);
      C[o] = f2bf(v);
    }
  }
}

// Column sum of a bf16 [M, N] matrix (row stride ld) into f32 out[N]
// (out = beta*out + sum): the bias gradient. Two-stage, deterministic.
// Stage 1: block (bx, by) sums rows [by*RB, ..) for 64*8 columns.
__global__ void colsum_partial_kernel(const bf16_t* __restrict__ X, float* __restrict__ part,
                                      int M, int N, int ld, int rows_per_block) {
  // 256 threads: 64 column-groups of 8 columns? keep simple: each thread owns 2 columns
  const int col = (blockIdx.x * blockDim.x + threadIdx.x) * 2;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  if (col >= N) return;
  float s0 = 0.f, s1 = 0.f;
  if (col + 1 < N && (ld % 2) == 0) {
    for (int r = r0; r < r1; ++r) {
      const uint32_t w = *reinterpret_cast<const uint32_t*>(X + (size_t)r * ld + col);
      s0 += bf2f((bf16_t)(w & 0xffff));
      s1 += bf2f((bf16_t)(w >> 16));
    }
  } else {
    for (int r = r0; r < r1; ++r) {
      s0 += bf2f(X[(size_t)r * ld + col]);
      if (col + 1 < N) s1 += bf2f(X[(size_t)r * ld + col + 1]);
    }
  }
  part[(size_t)blockIdx.y * N + col] = s0;
  if (col + 1 < N) part[(size_t)blockIdx.y * N + col + 1] = s1;
}

__global__ void colsum_final_kernel(const float* __restrict__ part, float* __restrict__ out, int N,
                                    int nparts, float beta) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int p = 0; p < nparts; ++p) s += part[(size_t)p * N + n];
  out[n] = (beta != 0.f ? beta * out[n] : 0.f) + s;
}

}  // namespace tdg

// ============================================================================ host
using namespace tdg;

namespace {

template <int BM, int BN, int WM, int WN, bool AK, bool BKc, int EPI, bool F32>
void launch_cfg(const bf16_t* A, const bf16_t* B, void* C, const float* bias, const bf16_t* aux,
                int M, int N, int K, int lda, int ldb, int ldc, int ldaux, float alpha, float beta,
                int splits, float* ws, hipStream_t st) {
  const int tiles = cdiv(M, BM) * cdiv(N, BN);
  const int lds = 2 * (BM + BN) * BK * 2;
  if (splits <= 1) {
    hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, AK, BKc, EPI, F32>), dim3(tiles, 1, 1),
                       dim3(WM * WN * 64), lds, st, A, B, C, bias, aux, M, N, K, lda, ldb, ldc,
                       ldaux, alpha, beta, K, 0LL);
  } else {
    int kps = cdiv(cdiv(K, splits), BK) * BK;
    splits = cdiv(K, kps);
    const long long stride = (long long)M * ldc;
    hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, AK, BKc, EPI_NONE, true>),
                       dim3(tiles, 1, splits), dim3(WM * WN * 64), lds, st, A, B, (void*)ws, bias,
                       aux, M, N, K, lda, ldb, ldc, ldaux, 1.f, 0.f, kps, stride);
    const long long total = (long long)M * N;
    const int blocks = (int)std::min<long long>(4096, (total + 255) / 256);
    hipLaunchKernelGGL((splitk_reduce_kernel<EPI, F32>), dim3(blocks), dim3(256), 0, st, ws, C,
                       bias, aux, M, N, ldc, ldaux, splits, stride, alpha, beta);
  }
}

template <bool AK, bool BKc, int EPI, bool F32>
void launch_tiles(int tile_cfg, const bf16_t* A, const bf16_t* B, void* C, const float* bias,
                  const bf16_t* aux, int M, int N, int K, int lda, int ldb, int ldc, int ldaux,
                  float alpha, float beta, int splits, float* ws, hipStream_t st) {
  switch (tile_cfg) {
    case 0:
      launch_cfg<128, 128, 2, 2, AK, BKc, EPI, F32>(A, B, C, bias, aux, M, N, K, lda, ldb, ldc,
                                                    ldaux, alpha, beta, splits, ws, st);
      break;
    case 1:
      launch_cfg<128, 64, 2, 2, AK, BKc, EPI, F32>(A, B, C, bias, aux, M, N, K, lda, ldb, ldc,
                                                   ldaux, alpha, beta, splits, ws, st);
      break;
    case 2:
      launch_cfg<64, 128, 2, 2, AK, BKc, EPI, F32>(A, B, C, bias, aux, M, N, K, lda, ldb, ldc,
                                                   ldaux, alpha, beta, splits, ws, st);
      break;
    default:
      launch_cfg<64, 64, 2, 2, AK, BKc, EPI, F32>(A, B, C, bias, aux, M, N, K, lda, ldb, ldc,
                                                  ldaux, alpha, beta, splits, ws, st);
      break;
  }
}

template <bool AK, bool BKc>
int dispatch_epi(int epi, bool f32, int tile_cfg, const bf16_t* A, const bf16_t* B, void* C,
                 const float* bias, const bf16_t* aux, int M, int N, int K, int lda, int ldb,
                 int ldc, int ldaux, float alpha, float beta, int splits, float* ws,
                 hipStream_t st) {
#define TDG_E(E, F)                                                                              \
  if (epi == E && f32 == F) {                                                                    \
    launch_tiles<AK, BKc, E, F>(tile_cfg, A, B, C, bias, aux, M, N, K, lda, ldb, ldc, ldaux,     \
                                alpha, beta, splits, ws, st);                                    \
    return 0;                                                                                    \
  }
  TDG_E(EPI_NONE, false)
  TDG_E(EPI_NONE, true)
  TDG_E(EPI_BIAS, false)
  TDG_E(EPI_BIAS, true)
  TDG_E(EPI_BIAS_RELU, false)
  TDG_E(EPI_DRELU, false)
#undef TDG_E
  return -1;
}

}  // namespace

// Public launcher. a_kc/b_kc select operand layouts. Returns 0 on success.
extern "C" int tdg_gemm(const void* A, const void* B, void* C, const float* bias, const void* aux,
                        int M, int N, int K, int lda, int ldb, int ldc, int ldaux, int a_kc,
                        int b_kc, int epi, int out_f32, float alpha, float beta, int tile_cfg,
                        int splits, float* ws, hipStream_t st) {
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* b = (const bf16_t*)B;
  const bf16_t* x = (const bf16_t*)aux;
  if (a_kc && b_kc)
    return dispatch_epi<true, true>(epi, out_f32, tile_cfg, a, b, C, bias, x, M, N, K, lda, ldb,
                                    ldc, ldaux, alpha, beta, splits, ws, st);
  if (a_kc && !b_kc)
    return dispatch_epi<true, false>(epi, out_f32, tile_cfg, a, b, C, bias, x, M, N, K, lda, ldb,
                                     ldc, ldaux, alpha, beta, splits, ws, st);
  if (!a_kc && !b_kc)
    return dispatch_epi<false, false>(epi, out_f32, tile_cfg, a, b, C, bias, x, M, N, K, lda, ldb,
                                      ldc, ldaux, alpha, beta, splits, ws, st);
  return dispatch_epi<false, true>(epi, out_f32, tile_cfg, a, b, C, bias, x, M, N, K, lda, ldb,
                                   ldc, ldaux, alpha, beta, splits, ws, st);
}

extern "C" void tdg_colsum(const void* X, float* out, float* part, int M, int N, int ld,
                           int rows_per_block, float beta, hipStream_t st) {
  const int nparts = cdiv(M, rows_per_block);
  dim3 grid(cdiv(cdiv(N, 2), 256), nparts);
  hipLaunchKernelGGL(colsum_partial_kernel, grid, dim3(256), 0, st, (const bf16_t*)X, part, M, N,
                     ld, rows_per_block);
  hipLaunchKernelGGL(colsum_final_kernel, dim3(cdiv(N, 256)), dim3(256), 0, st, part, out, N,
                     nparts, beta);
}
