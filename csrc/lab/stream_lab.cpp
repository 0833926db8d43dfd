// Stream lab: per-CU global -> LDS (LDS-DMA) throughput of GEMM operand
// panels as a function of the bytes kept in flight.
//
// One workgroup per output tile (BM x BN) streams its A rows [m0, m0+BM) and
// B rows [n0, n0+BN) (both K-contiguous) through K in 64-deep slots of
// (BM + BN) x 128 B, held in a ring of NSLOT LDS slots with DEPTH slots in
// flight (counted vmcnt + raw barrier, no MFMA, no fragment reads). Answers:
// is ~75-90 GB/s per CU (docs/KERNELS.md) a bandwidth ceiling or a latency
// (bytes in flight) limit?
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Icsrc/include -x hip \
//         csrc/lab/stream_lab.cpp -o lab_bin/stream_lab
#include "tdg_common.h"
#include "tdg_gemm.h"
#include "lab_common.h"

using namespace tdg;

template <int N>
__device__ __forceinline__ void vmwait() {
  if constexpr (N > 63) {
    asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  }
}

template <int NW, int BM, int BN, int NSLOT, int DEPTH>
__global__ __launch_bounds__(NW * 64) void stream_kernel(const bf16_t* __restrict__ A,
                                                         const bf16_t* __restrict__ B, int M,
                                                         int N, int K, float* __restrict__ sink,
                                                         int same) {
  static_assert(NSLOT >= DEPTH + 1, "ring must hold the in-flight slots plus the one read");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int ROWS = BM + BN;            // rows of 128 B per slot
  constexpr int SLOT = ROWS * 128;         // bytes per slot
  constexpr int PIECES = ROWS / 8;         // 1 KiB pieces per slot
  static_assert(PIECES % NW == 0, "pieces split evenly over waves");
  constexpr int PPW = PIECES / NW;         // DMA instructions per wave per slot
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_n = N / BN, tiles_m = M / BM;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn;
  if (tiles_n <= tiles_m) {
    tn = t % tiles_n;
    tm = t / tiles_n;
  } else {
    tm = t % tiles_m;
    tn = t / tiles_m;
  }
  const int m0 = same ? 0 : tm * BM, n0 = same ? 0 : tn * BN;
  const int nk = K / 64;
  // this lane's row / 16-byte chunk inside each of its pieces
  const bf16_t* src[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int piece = wid * PPW + i;
    const int r = piece * 8 + lane / 8, c = lane % 8;
    src[i] = r < BM ? A + (size_t)(m0 + r) * K + c * 8 : B + (size_t)(n0 + r - BM) * K + c * 8;
  }
  auto issue = [&](int kt) {
    char* sl = smem + (kt % NSLOT) * SLOT;
#pragma unroll
    for (int i = 0; i < PPW; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(src[i] + kt * 64),
                                       (__attribute__((address_space(3))) void*)(
                                           sl + (wid * PPW + i) * 1024),
                                       16, 0, 0);
  };
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (d < nk) issue(d);
  float acc = 0.f;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + DEPTH <= nk) vmwait<(DEPTH - 1) * PPW>();
    else vmwait<0>();
    lds_barrier();
    const char* cur = smem + (kt % NSLOT) * SLOT;
    acc += bf2f((bf16_t)reinterpret_cast<const short*>(cur)[tid]);
    if (kt + DEPTH < nk) issue(kt + DEPTH);
  }
  if (acc == 12345.f) sink[blockIdx.x] = acc;
}

template <int NW, int BM, int BN, int NSLOT, int DEPTH>
void run(hipStream_t st, const bf16_t* A, const bf16_t* B, int M, int N, int K, float* sink,
         int same = 0) {
  auto kern = stream_kernel<NW, BM, BN, NSLOT, DEPTH>;
  CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                         160 * 1024));
  const int tiles = (M / BM) * (N / BN);
  const size_t lds = (size_t)NSLOT * (BM + BN) * 128;
  auto go = [&] {
    hipLaunchKernelGGL(kern, dim3(tiles), dim3(NW * 64), lds, st, A, B, M, N, K, sink, same);
  };
  go();
  CK(hipStreamSynchronize(st));
  const float us = lab::graph_us(st, go);
  const double bytes = (double)(BM + BN) * K * 2;  // per workgroup
  const double per_cu = bytes * tiles / std::min(tiles, 256) / us / 1e3;
  std::printf("M %5d N %5d K %5d tile %3dx%-3d waves %2d slots %d depth %d (%3d KiB in flight) "
              "%8.2f us %7.1f GB/s per CU %6.2f TB/s chip\n",
              M, N, K, BM, BN, NW, NSLOT, DEPTH, DEPTH * (BM + BN) * 128 / 1024, us, per_cu,
              bytes * tiles / us / 1e6);
  std::fflush(stdout);
}

int main() {
  hipStream_t st;
  CK(hipStreamCreate(&st));
  std::mt19937 rng(5);
  float* sink;
  CK(hipMalloc(&sink, 4096 * 4));
  const int M = 8192;
  for (int K : {2048, 8192}) {
    const int N = 512;
    auto* A = (const bf16_t*)lab::rand_bf16((size_t)M * K, rng);
    auto* B = (const bf16_t*)lab::rand_bf16((size_t)2048 * K, rng);
    // 128x128 tiles, 256 workgroups
    run<8, 128, 128, 4, 1>(st, A, B, M, N, K, sink);
    run<8, 128, 128, 4, 2>(st, A, B, M, N, K, sink);
    run<8, 128, 128, 4, 3>(st, A, B, M, N, K, sink);
    run<8, 128, 128, 5, 4>(st, A, B, M, N, K, sink);
    run<4, 128, 128, 4, 3>(st, A, B, M, N, K, sink);
    run<16, 128, 128, 4, 3>(st, A, B, M, N, K, sink);
    // 256x256 (N = 2048: 256 workgroups) and 256x128 (N = 1024)
    run<8, 256, 256, 2, 1>(st, A, B, M, 2048, K, sink);
    run<8, 256, 128, 3, 2>(st, A, B, M, 1024, K, sink);
    run<4, 256, 128, 3, 2>(st, A, B, M, 1024, K, sink);
    run<8, 128, 256, 3, 2>(st, A, B, M, 2048, K, sink);
    CK(hipFree((void*)A));
    CK(hipFree((void*)B));
  }
  // same panels re-read by every workgroup (L2-resident source): the per-CU
  // ceiling with no L2 misses
  {
    const int K = 8192;
    auto* A = (const bf16_t*)lab::rand_bf16((size_t)256 * K, rng);
    run<8, 128, 128, 4, 3>(st, A, A, 128 * 256, 128, K, sink, 1);
    run<8, 128, 128, 5, 4>(st, A, A, 128 * 256, 128, K, sink, 1);
  }
  return 0;
}
