// Staging lab: how fast can one workgroup per CU move GEMM operand tiles
// global -> LDS on MI355X? The 128x128-tile GEMMs of the N = 512 outputs are
// bound by this (docs/KERNELS.md), so this isolates the transfer from the
// MFMAs and fragment reads.
//
// Each of 256 workgroups (512 threads) streams the A row block (128 rows) and
// B column block (128 rows of B [N][K]) of one 128x128 output tile through K
// in 64-deep tiles, 3 LDS stages, exactly like gemm_kernel<128,128,2,4,3>:
//   mode 0: both operands by LDS-DMA (global_load_lds_dwordx4)
//   mode 1: A by LDS-DMA, B by global_load_dwordx4 -> VGPR -> ds_write_b128
//   mode 2: both by register staging
// Reports us per launch and GB/s per CU of staged bytes.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Icsrc/include -x hip \
//         csrc/lab/staging_lab.cpp -o lab_bin/staging_lab
#include "tdg_common.h"
#include "tdg_gemm.h"
#include "lab_common.h"

using namespace tdg;

constexpr int NWS = 8, BMS = 128, STG = 3;

template <int MODE>
__global__ __launch_bounds__(512) void stage_kernel(const bf16_t* __restrict__ A,
                                                    const bf16_t* __restrict__ B, int M, int N,
                                                    int K, float* __restrict__ sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  using GA = Glds<true, BMS, NWS>;
  constexpr int TILE = BMS * BK * 2;  // 16 KiB per operand per stage
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_n = N / 128;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (t / tiles_n) * 128, n0 = (t % tiles_n) * 128;
  GA ga;
  ga.init(wid, lane);
  const int nk = K / BK;
  // register staging: 16 KiB per operand tile / 512 threads = 2 x 16 B each
  short8_t ra[2], rb[2];
  auto reg_load = [&](const bf16_t* X, int mn0, int k0, short8_t* r) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int id = tid + 512 * i;  // chunk id: row = id / 8, 16-byte chunk = id % 8
      const int row = id >> 3, ch = id & 7;
      r[i] = *reinterpret_cast<const short8_t*>(X + (size_t)(mn0 + row) * K + k0 + ch * 8);
    }
  };
  auto reg_store = [&](char* lds, const short8_t* r) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int id = tid + 512 * i;
      const int row = id >> 3, ch = id & 7;
      *reinterpret_cast<short8_t*>(lds + lds_off<true, BMS>(row, ch * 16)) = r[i];
    }
  };
  float acc = 0.f;
  // Schedule (as gemm_kernel): at iteration kt the slot of tile kt is read
  // and tile kt + 2 is requested into the slot freed by iteration kt - 1.
  // Register-staged parts of tile kt + 2 are loaded at iteration kt (before
  // that iteration's DMAs, so a counted vmcnt retires them first) and written
  // to LDS at the top of iteration kt + 1, before its barrier.
  constexpr int DMA = (MODE == 0 ? 2 * GA::P : MODE == 1 ? GA::P : 0);  // DMAs per iteration
  auto issue_tile = [&](int tt) {
    char* sl = smem + (tt % STG) * 2 * TILE;
    if (MODE == 2) reg_load(A, m0, tt * BK, ra);
    if (MODE != 0) reg_load(B, n0, tt * BK, rb);
    if (MODE != 2) ga.issue(A, K, M, K, m0, tt * BK, sl, wid);
    if (MODE == 0) ga.issue(B, K, N, K, n0, tt * BK, sl + TILE, wid);
  };
  auto write_regs = [&](int tt) {
    char* sl = smem + (tt % STG) * 2 * TILE;
    if (MODE == 2) reg_store(sl, ra);
    if (MODE != 0) reg_store(sl + TILE, rb);
  };
  // prologue: tiles 0 and 1 fully staged
  for (int s = 0; s < 2 && s < nk; ++s) {
    issue_tile(s);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    write_regs(s);
  }
  for (int kt = 0; kt < nk; ++kt) {
    // retires tile kt+1's DMA and register loads (issued at kt-1); tile kt+2's
    // DMA (issued last) may stay in flight
    if (DMA == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (DMA == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (kt >= 1 && kt + 1 < nk) write_regs(kt + 1);
    lds_barrier();
    const char* cur = smem + (kt % STG) * 2 * TILE;
    acc += bf2f((bf16_t)reinterpret_cast<const short*>(cur)[tid]) +
           bf2f((bf16_t)reinterpret_cast<const short*>(cur + TILE)[tid]);
    if (kt + 2 < nk) issue_tile(kt + 2);
  }
  if (acc == 12345.f) sink[blockIdx.x] = acc;
}

int main() {
  hipStream_t st;
  CK(hipStreamCreate(&st));
  std::mt19937 rng(5);
  float* sink;
  CK(hipMalloc(&sink, 4096 * 4));
  for (int K : {512, 2048, 8192}) {
    const int M = 8192, N = 512;
    uint16_t* A = lab::rand_bf16((size_t)M * K, rng);
    uint16_t* B = lab::rand_bf16((size_t)N * K, rng);
    const int tiles = (M / 128) * (N / 128);
    const size_t lds = STG * 2 * BMS * BK * 2;
    const double bytes_per_cu = (double)(128 + 128) * K * 2;  // per workgroup
    auto run = [&](auto kern, const char* name) {
      CK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                             160 * 1024));
      auto go = [&] {
        hipLaunchKernelGGL(kern, dim3(tiles), dim3(512), lds, st, (const bf16_t*)A,
                           (const bf16_t*)B, M, N, K, sink);
      };
      go();
      CK(hipStreamSynchronize(st));
      const float us = lab::graph_us(st, go);
      std::printf("M %d N %d K %5d %-22s %8.2f us  %6.1f GB/s per workgroup\n", M, N, K, name, us,
                  bytes_per_cu / us / 1e3);
      std::fflush(stdout);
    };
    run(stage_kernel<0>, "A dma, B dma");
    run(stage_kernel<1>, "A dma, B regs");
    run(stage_kernel<2>, "A regs, B regs");
    CK(hipFree(A));
    CK(hipFree(B));
  }
  return 0;
}
