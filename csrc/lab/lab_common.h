// Shared helpers of the standalone kernel labs (no torch): error checks, bf16
// host conversion, HIP-graph timing and the per-workgroup phase stamps
// (tdg_common.h TDG_STAMP: slot (block * 8 + phase) * 64, s_memrealtime at
// 100 MHz) summarised as median / max phase durations.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <random>
#include <string>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

namespace lab {

inline uint16_t host_bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
inline float host_f(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

// device buffer of n random bf16 in [-scale, scale)
inline uint16_t* rand_bf16(size_t n, std::mt19937& rng, float scale = 1.f,
                           std::vector<uint16_t>* keep = nullptr) {
  std::uniform_real_distribution<float> U(-scale, scale);
  std::vector<uint16_t> h(n);
  for (auto& x : h) x = host_bf(U(rng));
  uint16_t* d;
  CK(hipMalloc(&d, n * 2));
  CK(hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice));
  if (keep) *keep = std::move(h);
  return d;
}

// median us per launch of `fn` over 20 launches captured in a HIP graph
inline float graph_us(hipStream_t st, const std::function<void()>& fn) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int i = 0; i < 20; ++i) fn();
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
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return ts[ts.size() / 2];
}

struct Stamps {
  unsigned long long* d = nullptr;
  size_t nblocks = 0;
  template <typename Sym>
  void init(const Sym& symbol, size_t max_blocks) {
    nblocks = max_blocks;
    CK(hipMalloc(&d, nblocks * 512 * 8));
    CK(hipMemcpyToSymbol(symbol, &d, sizeof(d)));
  }
  void clear(hipStream_t st) { CK(hipMemsetAsync(d, 0, nblocks * 512 * 8, st)); }
  // "name a b c d" phase summary for phases 0->1->2->3->4 of nwg blocks
  std::string summary(size_t nwg, const char* names[4]) const {
    std::vector<unsigned long long> hs(nwg * 512);
    CK(hipMemcpy(hs.data(), d, hs.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> ph[4];
    unsigned long long t0min = ~0ull, t0max = 0, t4max = 0;
    for (size_t b = 0; b < nwg; ++b) {
      unsigned long long t[5];
      for (int i = 0; i < 5; ++i) t[i] = hs[b * 512 + i * 64];
      if (!t[0] || !t[4]) continue;
      for (int i = 0; i < 4; ++i) ph[i].push_back((double)(t[i + 1] - t[i]) * 0.01);
      t0min = std::min(t0min, t[0]);
      t0max = std::max(t0max, t[0]);
      t4max = std::max(t4max, t[4]);
    }
    char buf[512];
    int o = std::snprintf(buf, sizeof(buf), "per-WG median (max) us:");
    for (int i = 0; i < 4; ++i) {
      std::vector<double> v = ph[i];
      std::sort(v.begin(), v.end());
      const double med = v.empty() ? 0 : v[v.size() / 2], mx = v.empty() ? 0 : v.back();
      o += std::snprintf(buf + o, sizeof(buf) - o, " %s %.2f (%.2f)", names[i], med, mx);
    }
    std::snprintf(buf + o, sizeof(buf) - o, " | entry skew %.2f span %.2f",
                  (t0max - t0min) * 0.01, (t4max - t0min) * 0.01);
    return buf;
  }
};

}  // namespace lab
