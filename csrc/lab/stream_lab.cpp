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

// WORK: 0 = staging only; 1 = + the GEMM's fragment reads (ds_read_b128,
// a 64x32 wave tile: 6 per 32-deep step, 2 steps per slot); 2 = + the
// GEMM's MFMAs (16 per slot per wave, on register operands); 3 = both.
template <int NW, int BM, int BN, int NSLOT, int DEPTH, int WORK = 0>
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
  unsigned long long c0 = 0, r0 = 0;
  if (blockIdx.x == 0 && tid == 0) {
    c0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
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
  f32x4 c[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) c[i][0] = c[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  short8_t fa[4], fb[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) fa[i] = short8_t{(short)lane, 1, 2, 3, 4, 5, 6, (short)i};
  fb[0] = fb[1] = short8_t{1, 1, 1, 1, 1, 1, 1, 1};
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + DEPTH <= nk) vmwait<(DEPTH - 1) * PPW>();
    else vmwait<0>();
    lds_barrier();
    const char* cur = smem + (kt % NSLOT) * SLOT;
    acc += bf2f((bf16_t)reinterpret_cast<const short*>(cur)[tid]);
    if (kt + DEPTH < nk) issue(kt + DEPTH);
#pragma unroll
    for (int step = 0; step < 2; ++step) {
      if constexpr (WORK & 1) {
        // fragment reads over the slot's A rows (wave-row base) and B rows
        const int wm = wid / 4, wn = wid % 4;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          fa[i] = lds_read_b128_async(cur + lds_off<true, 128>(wm * 64 + 16 * i + (lane & 15),
                                                               (step * 4 + (lane >> 4)) * 16));
#pragma unroll
        for (int j = 0; j < 2; ++j)
          fb[j] = lds_read_b128_async(cur + BM * 128 +
                                      lds_off<true, 128>(wn * 32 + 16 * j + (lane & 15),
                                                         (step * 4 + (lane >> 4)) * 16));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        tie_all(fa);
        tie_all(fb);
      }
      if constexpr (WORK & 2) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) c[i][j] = mfma16(fb[j], fa[i], c[i][j]);
        __builtin_amdgcn_s_setprio(0);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) acc += c[i][0][0] + c[i][1][1] + bf2f((bf16_t)fa[i][0]);
  if (acc == 12345.f) sink[blockIdx.x] = acc;
  if (blockIdx.x == 0 && tid == 0) {
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    sink[1024] = (float)(c1 - c0);
    sink[1025] = (float)(r1 - r0);
  }
}

template <int NW, int BM, int BN, int NSLOT, int DEPTH, int WORK = 0>
void run(hipStream_t st, const bf16_t* A, const bf16_t* B, int M, int N, int K, float* sink,
         int same = 0) {
  auto kern = stream_kernel<NW, BM, BN, NSLOT, DEPTH, WORK>;
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
  float clk[2];
  CK(hipMemcpy(clk, sink + 1024, 8, hipMemcpyDeviceToHost));
  const double mhz = clk[1] > 0 ? clk[0] / (clk[1] * 0.01) : 0.0;  // memrealtime: 100 MHz
  const double bytes = (double)(BM + BN) * K * 2;  // per workgroup
  const double per_cu = bytes * tiles / std::min(tiles, 256) / us / 1e3;
  std::printf("M %5d N %5d K %5d tile %3dx%-3d waves %2d slots %d depth %d (%3d KiB in flight) "
              "work %d %8.2f us %7.1f GB/s per CU %6.2f TB/s chip  clock %4.0f MHz\n",
              M, N, K, BM, BN, NW, NSLOT, DEPTH, DEPTH * (BM + BN) * 128 / 1024, WORK, us, per_cu,
              bytes * tiles / us / 1e6, mhz);
  std::fflush(stdout);
}

int main(int argc, char** argv) {
  hipStream_t st;
  CK(hipStreamCreate(&st));
  std::mt19937 rng(5);
  float* sink;
  CK(hipMalloc(&sink, 4096 * 4));
  const int M = 8192;
  if (argc > 1) {  // the work-mode experiment: 128x128 tiles, 8 waves, 4 slots, depth 3
    for (int K : {2048, 8192}) {
      auto* A = (const bf16_t*)lab::rand_bf16((size_t)M * K, rng);
      auto* B = (const bf16_t*)lab::rand_bf16((size_t)512 * K, rng);
      for (int rep = 0; rep < 2; ++rep) {
        run<8, 128, 128, 4, 3, 0>(st, A, B, M, 512, K, sink);
        run<8, 128, 128, 4, 3, 1>(st, A, B, M, 512, K, sink);
        run<8, 128, 128, 4, 3, 2>(st, A, B, M, 512, K, sink);
        run<8, 128, 128, 4, 3, 3>(st, A, B, M, 512, K, sink);
        // L2-resident panels (every workgroup the same): no miss path
        run<8, 128, 128, 4, 3, 0>(st, A, A, 128 * 256, 128, K, sink, 1);
        run<8, 128, 128, 4, 3, 3>(st, A, A, 128 * 256, 128, K, sink, 1);
      }
      CK(hipFree((void*)A));
      CK(hipFree((void*)B));
    }
    return 0;
  }
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
