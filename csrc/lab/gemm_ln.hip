// Sublayer output projection + bias + dropout + residual + LayerNorm in ONE
// kernel (gfx950), for the post-LN block tails of the Transformer:
//
//   s = A @ W^T + bias            (A [M,K] = attention output or FFN hidden)
//   h = x + dropout(s);  y = LayerNorm(h) * gamma + beta    (saves h, mean, rstd)
//
// Replaces, per block, the reference's `Dense` output projection followed by
// `LayerNormalization(x + Dropout(...))` (reference:
// distributed_training_transformer/transformer_model.py:165,174 and
// :187-188,198,204,219-221,233,240,246). Unfused, the GEMM writes s to HBM
// and a LayerNorm kernel reads s and x back: two launches and a round trip of
// an [M, D] tensor per block tail.
//
// Design: a workgroup owns FULL rows -- a 32 x D output tile (D = 512: 8
// waves x 64 columns, 256 workgroups for M = 8192), so the row statistics
// never leave the workgroup. Every workgroup streams all of W ([D, K],
// K-contiguous) from L2, which makes the main loop latency x bytes-in-flight
// bound: operands go straight into MFMA fragment registers, GEMM_LN_PIPE K
// tiles deep per wave (an LDS pipeline could hold only 2 x 64 KiB stages;
// measured 2.3 us per K tile with it). The epilogue stages s (bf16,
// bias added, exactly the tensor the unfused GEMM would write) through LDS
// and then runs the standalone LayerNorm's row code (tdg_ln.h ln_row_fwd:
// one wave per row, same lane layout and reduction order), so the outputs
// are bitwise identical to GEMM + ln_fwd.
#include "tdg_common.h"
#include "tdg_gemm.h"
#include "tdg_ln.h"

namespace tdg {

constexpr int GEMM_LN_PIPE = 4;  // K tiles (64 deep) in flight per wave

template <int D>
__global__ __launch_bounds__(512) void gemm_ln_kernel(
    const bf16_t* __restrict__ A, int lda, const bf16_t* __restrict__ W, int ldw,
    const float* __restrict__ bias, const bf16_t* __restrict__ X, int ldx,
    const float* __restrict__ gamma, const float* __restrict__ beta, bf16_t* __restrict__ Y,
    bf16_t* __restrict__ H, float* __restrict__ mean_out, float* __restrict__ rstd_out, int M,
    int K, float p, uint32_t thresh, uint64_t seed, const long long* ctr, uint64_t site,
    float eps) {
  constexpr int NW = 8, BM = 32, WTN = D / NW, TN = WTN / 16, TM = BM / 16;
  constexpr int PIPE = GEMM_LN_PIPE;
  static_assert(D == 512, "one wave per 64 columns, one lane per 8 row elements");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * BM;
  const int nk = K / BK;  // host guarantees K % (BK * PIPE) == 0
  const int bbase = wid * WTN;

  // Main loop without LDS: both operands are loaded straight into MFMA
  // fragment registers (lane l: row (l&15), k 8(l>>4).. of each 32-deep step).
  // With one workgroup per 32 rows every workgroup streams all of W, so the
  // loop is bound by L2 latency x bytes in flight, not by MFMA: registers
  // hold PIPE K tiles in flight per wave (PIPE x 12 KiB per wave, ~4x what
  // LDS stages could), and no barrier couples the waves.
  const bf16_t* arow[TM];
  const bf16_t* brow[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
    arow[i] = A + (size_t)min(m0 + 16 * i + (lane & 15), M - 1) * lda + 8 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < TN; ++j)
    brow[j] = W + (size_t)(bbase + 16 * j + (lane & 15)) * ldw + 8 * (lane >> 4);
  struct Frags {
    short8_t a[TM][2];
    short8_t b[TN][2];
  };
  auto load = [&](Frags& f, int k0) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int i = 0; i < TM; ++i) f.a[i][s] = *reinterpret_cast<const short8_t*>(arow[i] + k0 + 32 * s);
#pragma unroll
      for (int j = 0; j < TN; ++j) f.b[j][s] = *reinterpret_cast<const short8_t*>(brow[j] + k0 + 32 * s);
    }
  };
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const Frags& f) {
    prio_hi();
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(f.a[i][s], f.b[j][s], acc[i][j]);
    prio_lo();
  };

  Frags buf[PIPE];  // ring of K tiles; constant slot indices only (no scratch)
#pragma unroll
  for (int q = 0; q < PIPE; ++q) load(buf[q], q * BK);
  for (int kt = 0; kt + PIPE < nk; kt += PIPE) {
#pragma unroll
    for (int q = 0; q < PIPE; ++q) {
      mma(buf[q]);
      load(buf[q], (kt + q + PIPE) * BK);
    }
  }
#pragma unroll
  for (int q = 0; q < PIPE; ++q) mma(buf[q]);

  // ---------------- epilogue: s = bf16(acc + bias) -> LDS row image -> LayerNorm rows
  constexpr int SROW = D * 2 + 16;  // padded row (bytes)
  const int g = lane >> 4, cl = lane & 15;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = bbase + 16 * j + cl;
    const float bn = bias[n];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        *reinterpret_cast<bf16_t*>(smem + (16 * i + 4 * g + r) * SROW + n * 2) =
            f2bf(acc[i][j][r] + bn);
  }
  lds_barrier();
  constexpr int VEC = D / 64;
#pragma unroll
  for (int rr = 0; rr < BM / NW; ++rr) {
    const int row = wid * (BM / NW) + rr;
    const int m = m0 + row;
    if (m >= M) break;
    const size_t base = (size_t)m * D + lane * VEC;  // element index of the [M, D] view (Philox)
    RowVec<VEC> h, t, o;
    h.load_bf(X + (size_t)m * ldx + lane * VEC);
    t.load_bf(reinterpret_cast<const bf16_t*>(smem + row * SROW + lane * VEC * 2));
    ln_row_fwd<D>(h, t, true, base, m, lane, gamma, beta, Y, H, mean_out, rstd_out, p, thresh,
                  seed, ctr, site, eps, o);
  }
}

}  // namespace tdg

using namespace tdg;

// y, hsave [M, D] contiguous; x residual [M, ldx]; A [M, lda]; W [D, ldw].
// Returns 0 on success, <0 if the shape is not covered (caller falls back to
// GEMM + LayerNorm).
extern "C" int tdg_gemm_ln(const void* A, int lda, const void* W, int ldw, const float* bias,
                           const void* X, int ldx, const float* gamma, const float* beta, void* Y,
                           void* H, float* mean, float* rstd, int M, int K, int D, float p,
                           uint64_t seed, const long long* ctr, uint64_t site, float eps,
                           hipStream_t st) {
  if (D != 512) return -1;
  if (K % (BK * GEMM_LN_PIPE) != 0 || K <= 0 || M <= 0) return -2;
  if (lda % 8 || ldw % 8 || ldx % 8) return -3;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(W) |
       reinterpret_cast<uintptr_t>(X) | reinterpret_cast<uintptr_t>(Y) |
       reinterpret_cast<uintptr_t>(H)) & 15)
    return -4;
  constexpr int lds = 32 * (512 * 2 + 16);  // the epilogue's s image
  const uint32_t thresh = (uint32_t)fminf(4294967295.f, p * 4294967296.f);
  hipLaunchKernelGGL(gemm_ln_kernel<512>, dim3(cdiv(M, 32)), dim3(512), lds, st,
                     (const bf16_t*)A, lda, (const bf16_t*)W, ldw, bias, (const bf16_t*)X, ldx,
                     gamma, beta, (bf16_t*)Y, (bf16_t*)H, mean, rstd, M, K, p, thresh, seed, ctr,
                     site, eps);
  return 0;
}
