// Attention lab: standalone timing + per-workgroup phase stamps of the fused
// attention forward / backward on the Transformer-base shapes (B 64, H 8,
// head dim 64, L 128; self, causal self, cross).
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DTDG_STAMPS -Icsrc/include \
//         -x hip csrc/lab/attn_lab.cpp -o lab_bin/attn_lab
#include "../kernels/attention.hip"
#include "lab_common.h"

int main() {
  const int B = 64, H = 8, D = 64, L = 128;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  lab::Stamps stamps;
  stamps.init(HIP_SYMBOL(tdg::tdg_stamps), (size_t)B * H * 4);
  std::mt19937 rng(3);
  const size_t n = (size_t)B * L * H * D;
  std::vector<uint16_t> hq, hk, hv;
  uint16_t* q = lab::rand_bf16(n, rng, 1.f, &hq);
  uint16_t* k = lab::rand_bf16(n, rng, 1.f, &hk);
  uint16_t* v = lab::rand_bf16(n, rng, 1.f, &hv);
  uint16_t* dout = lab::rand_bf16(n, rng, 0.1f);
  uint16_t *o, *dq, *dk, *dv;
  float *lse, *delta;
  CK(hipMalloc(&o, n * 2));
  CK(hipMalloc(&dq, n * 2));
  CK(hipMalloc(&dk, n * 2));
  CK(hipMalloc(&dv, n * 2));
  CK(hipMalloc(&lse, (size_t)B * H * L * 4));
  CK(hipMalloc(&delta, (size_t)B * H * L * 4));
  for (int causal = 0; causal < 2; ++causal) {
    AttnArgs a{};
    a.q = q; a.k = k; a.v = v; a.o = o; a.dout = dout; a.out = o; a.lse = lse; a.delta = delta;
    a.dq = dq; a.dk = dk; a.dv = dv; a.kv_len = nullptr;
    const long long sb = (long long)L * H * D, sl = H * D;
    a.q_sb = a.k_sb = a.v_sb = a.o_sb = a.dq_sb = a.dk_sb = a.dv_sb = a.do_sb = sb;
    a.q_sl = a.k_sl = a.v_sl = a.o_sl = a.dq_sl = a.dk_sl = a.dv_sl = a.do_sl = sl;
    a.q_sh = a.k_sh = a.v_sh = a.o_sh = a.dq_sh = a.dk_sh = a.dv_sh = a.do_sh = D;
    a.B = B; a.H = H; a.Lq = L; a.Lk = L; a.scale = 0.125f; a.causal = causal;
    // forward: check one (b, h) against the host
    CK((hipError_t)tdg_attn_fwd(&a, D, st));
    CK(hipStreamSynchronize(st));
    std::vector<uint16_t> ho(n);
    CK(hipMemcpy(ho.data(), o, n * 2, hipMemcpyDeviceToHost));
    double err = 0, ref2 = 0;
    const int bb = 5, hh = 3;
    for (int i = 0; i < L; ++i) {
      std::vector<double> s(L);
      double mx = -1e300;
      for (int j = 0; j < L; ++j) {
        double acc = 0;
        for (int d = 0; d < D; ++d)
          acc += lab::host_f(hq[((size_t)bb * L + i) * H * D + hh * D + d]) *
                 lab::host_f(hk[((size_t)bb * L + j) * H * D + hh * D + d]);
        s[j] = (causal && j > i) ? -1e300 : acc * 0.125;
        mx = std::max(mx, s[j]);
      }
      double den = 0;
      for (int j = 0; j < L; ++j) den += (s[j] > -1e299) ? std::exp(s[j] - mx) : 0.0;
      for (int d = 0; d < D; ++d) {
        double r = 0;
        for (int j = 0; j < L; ++j)
          if (s[j] > -1e299)
            r += std::exp(s[j] - mx) / den * lab::host_f(hv[((size_t)bb * L + j) * H * D + hh * D + d]);
        const double g = lab::host_f(ho[((size_t)bb * L + i) * H * D + hh * D + d]);
        err += (g - r) * (g - r);
        ref2 += r * r;
      }
    }
    const char* fn[4] = {"load", "compute", "epi-issue", "drain"};
    stamps.clear(st);
    CK((hipError_t)tdg_attn_fwd(&a, D, st));
    CK(hipStreamSynchronize(st));
    const std::string sf = stamps.summary((size_t)B * H * 2, fn);
    const float tf = lab::graph_us(st, [&] { tdg_attn_fwd(&a, D, st); });
    std::printf("fwd causal=%d %8.2f us rel %.1e | %s\n", causal, tf, std::sqrt(err / ref2), sf.c_str());
    const char* bn[4] = {"load", "phase1", "phase2+stores", "drain"};
    stamps.clear(st);
    CK((hipError_t)tdg_attn_bwd(&a, D, st));
    CK(hipStreamSynchronize(st));
    const std::string sbw = stamps.summary((size_t)B * H, bn);
    const float tb = lab::graph_us(st, [&] { tdg_attn_bwd(&a, D, st); });
    std::printf("bwd causal=%d %8.2f us | %s\n", causal, tb, sbw.c_str());
    std::fflush(stdout);
  }
  return 0;
}
