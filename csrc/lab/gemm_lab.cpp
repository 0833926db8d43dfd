// GEMM lab: standalone (no torch) timing + per-workgroup phase timelines of
// the MFMA GEMM kernels on the model's shapes.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DTDG_STAMPS -Icsrc/include \
//         csrc/lab/gemm_lab.cpp -o build/gemm_lab
//   build/gemm_lab            (on an MI355X)
//
// For every case: correctness against a naive f32 reference GEMM on device,
// median time of 20 launches captured in a HIP graph (what the training step
// sees), and -- from one extra stamped launch -- the median per-workgroup
// phase durations: prologue (entry -> first K tile in LDS), main loop,
// epilogue store issue, store drain, plus the launch skew (spread of the
// workgroups' entry times) and the whole kernel span.
#include "../kernels/gemm_impl.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

__global__ void ref_gemm_nt(const bf16_t* A, const bf16_t* B, float* C, int M, int N, int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += bf2f(A[(size_t)m * K + k]) * bf2f(B[(size_t)n * K + k]);
  C[(size_t)m * N + n] = s;
}

static bf16_t host_bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (bf16_t)(u >> 16);
}
static float host_f(bf16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

struct Case {
  int M, N, K, cfg;
};

int main(int argc, char** argv) {
  std::vector<Case> cases;
  for (int cfg : {12}) {
    cases.push_back({2048, 2048, 512, cfg});
    cases.push_back({8192, 2048, 512, cfg});
    cases.push_back({8192, 1536, 512, cfg});
    cases.push_back({8192, 2048, 2048, cfg});
    cases.push_back({4096, 4096, 4096, cfg});
  }
  for (int cfg : {4, 7, 13}) {
    cases.push_back({8192, 512, 512, cfg});
    cases.push_back({8192, 512, 2048, cfg});
  }
  if (argc > 1) {  // M N K cfg
    cases = {{std::atoi(argv[1]), std::atoi(argv[2]), std::atoi(argv[3]), std::atoi(argv[4])}};
  }
  hipStream_t st;
  CK(hipStreamCreate(&st));
  unsigned long long* stamps;
  const size_t nst = 4096 * 512;
  CK(hipMalloc(&stamps, nst * sizeof(unsigned long long)));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(tdg::tdg_stamps), &stamps, sizeof(stamps)));
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> U(-1.f, 1.f);

  for (const Case& c : cases) {
    const int M = c.M, N = c.N, K = c.K;
    std::vector<bf16_t> hA((size_t)M * K), hB((size_t)N * K);
    for (auto& x : hA) x = host_bf(U(rng));
    for (auto& x : hB) x = host_bf(U(rng));
    bf16_t *A, *B, *C;
    float* R;
    CK(hipMalloc(&A, hA.size() * 2));
    CK(hipMalloc(&B, hB.size() * 2));
    CK(hipMalloc(&C, (size_t)M * N * 2));
    CK(hipMalloc(&R, (size_t)M * N * 4));
    CK(hipMemcpy(A, hA.data(), hA.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, hB.data(), hB.size() * 2, hipMemcpyHostToDevice));
    auto launch = [&]() {
      const int rc = tdg_gemm(A, B, C, nullptr, nullptr, M, N, K, K, K, N, 0, 1, 1, 0, 0, 1.f, 0.f,
                              c.cfg, 1, nullptr, st);
      if (rc != 0) {
        std::fprintf(stderr, "tdg_gemm rc %d\n", rc);
        std::exit(1);
      }
    };
    // correctness
    launch();
    hipLaunchKernelGGL(ref_gemm_nt, dim3((N + 255) / 256, M), dim3(256), 0, st, A, B, R, M, N, K);
    CK(hipStreamSynchronize(st));
    std::vector<bf16_t> hC((size_t)M * N);
    std::vector<float> hR((size_t)M * N);
    CK(hipMemcpy(hC.data(), C, hC.size() * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hR.data(), R, hR.size() * 4, hipMemcpyDeviceToHost));
    double err = 0, ref = 0;
    for (size_t i = 0; i < hC.size(); ++i) {
      const double d = host_f(hC[i]) - hR[i];
      err += d * d;
      ref += (double)hR[i] * hR[i];
    }
    const double rel = std::sqrt(err / std::max(ref, 1e-30));
    // stamped launch (also warms up)
    CK(hipMemsetAsync(stamps, 0, nst * sizeof(unsigned long long), st));
    launch();
    CK(hipStreamSynchronize(st));
    // timing: 20 launches in a graph, median of 7 replays
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int i = 0; i < 20; ++i) launch();
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> ts;
    for (int r = 0; r < 7; ++r) {
      CK(hipEventRecord(e0, st));
      CK(hipGraphLaunch(ge, st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms * 1000.f / 20.f);
    }
    std::sort(ts.begin(), ts.end());
    const float us = ts[ts.size() / 2];
    // stamps: the stamped launch happened before the graph replays; its
    // buffer was not overwritten since (graph launches also stamp, so read
    // after one more plain launch)
    CK(hipMemsetAsync(stamps, 0, nst * sizeof(unsigned long long), st));
    launch();
    CK(hipStreamSynchronize(st));
    const bool t256 = c.cfg == 12;
    int tm = t256 ? 256 : (c.cfg == 7 ? 64 : 128), tn = t256 ? 256 : 128;
    const int nwg = ((M + tm - 1) / tm) * ((N + tn - 1) / tn);
    std::vector<unsigned long long> hs((size_t)nwg * 512);
    CK(hipMemcpy(hs.data(), stamps, hs.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> ph[4];
    unsigned long long t0min = ~0ull, t0max = 0, t4max = 0;
    for (int b = 0; b < nwg; ++b) {
      unsigned long long t[5];
      for (int i = 0; i < 5; ++i) t[i] = hs[(size_t)b * 512 + i * 64];
      if (!t[0] || !t[4]) continue;
      for (int i = 0; i < 4; ++i) ph[i].push_back((double)(t[i + 1] - t[i]) * 0.01);  // us
      t0min = std::min(t0min, t[0]);
      t0max = std::max(t0max, t[0]);
      t4max = std::max(t4max, t[4]);
    }
    auto med = [](std::vector<double> v) {
      if (v.empty()) return 0.0;
      std::sort(v.begin(), v.end());
      return v[v.size() / 2];
    };
    auto mx = [](const std::vector<double>& v) {
      return v.empty() ? 0.0 : *std::max_element(v.begin(), v.end());
    };
    std::printf(
        "%5dx%5dx%5d cfg%-2d %8.2f us %6.0f TF rel %.1e | per-WG median (max) us: prologue %.2f "
        "(%.2f) main %.2f (%.2f) epi-issue %.2f (%.2f) drain %.2f (%.2f) | entry skew %.2f span "
        "%.2f\n",
        M, N, K, c.cfg, us, 2.0 * M * N * K / us / 1e6, rel, med(ph[0]), mx(ph[0]), med(ph[1]),
        mx(ph[1]), med(ph[2]), mx(ph[2]), med(ph[3]), mx(ph[3]), (t0max - t0min) * 0.01,
        (t4max - t0min) * 0.01);
    std::fflush(stdout);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipFree(A));
    CK(hipFree(B));
    CK(hipFree(C));
    CK(hipFree(R));
  }
  return 0;
}
