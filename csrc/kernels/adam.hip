// Multi-tensor Adam over the single flat f32 master-parameter buffer (gfx950).
//
// Keras Adam semantics (reference: distributed_training_transformer/__main__.py:
// 56-73 -- Adam(beta_1=0.9, beta_2=0.98, epsilon=1e-9) driven by the Noam
// schedule d^-0.5 * min(step * warmup^-1.5, step^-0.5)):
//   lr    = schedule(iterations)            (iterations starts at 0 -> lr = 0)
//   t     = iterations + 1
//   lr_t  = lr * sqrt(1 - b2^t) / (1 - b1^t)
//   m    += (g - m) * (1 - b1);  v += (g*g - v) * (1 - b2)
//   p    -= lr_t * m / (sqrt(v) + eps)
// The schedule is evaluated on device from a device-resident step counter, so
// the optimizer step needs no host sync and can be captured in a HIP graph.
// Fused: bf16 shadow-weight refresh (the compute copy the GEMMs read) and
// zeroing of the consumed gradient (so backward can accumulate).
#include "tdg_common.h"

namespace tdg {

struct AdamCfg {
  float beta1, beta2, eps;
  float lr_const;     // used when sched == 0
  float d_model;      // Noam: d^-0.5
  float warmup;       // Noam warmup steps
  float grad_scale;   // multiply incoming gradient
  float weight_decay; // decoupled (0 in the reference)
  int sched;          // 0 const, 1 noam
  int zero_grad;
};

__device__ __forceinline__ float noam_lr(const AdamCfg& c, float step) {
  if (c.sched == 0) return c.lr_const;
  const float rise = step * powf(c.warmup, -1.5f);
  const float fall = step > 0.f ? rsqrtf(step) : INFINITY;
  return rsqrtf(c.d_model) * fminf(rise, fall);
}

__device__ __forceinline__ void adam4(float4& pp, const float4& gg, float4& mm, float4& vv,
                                      const AdamCfg& c, float lr, float lr_t, float ob1,
                                      float ob2) {
  float* P = &pp.x;
  const float* G = &gg.x;
  float* Mm = &mm.x;
  float* Vv = &vv.x;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float gk = G[k] * c.grad_scale;
    Mm[k] += (gk - Mm[k]) * ob1;
    Vv[k] += (gk * gk - Vv[k]) * ob2;
    P[k] -= lr_t * Mm[k] / (sqrtf(Vv[k]) + c.eps) + lr * c.weight_decay * P[k];
  }
}


// Write-through (sc1) stores of everything Adam writes: the master weights
// and moments are re-read by nothing until the next step and the bf16 shadow
// by the next forward's GEMMs on other XCDs, so none of it should sit dirty
// in an XCD's L2 for the end-of-kernel write-back (tdg_common.h WtBuf).
struct AdamOut {
  WtBuf p, m, v, s;
  __device__ __forceinline__ AdamOut(float* P, float* M, float* V, bf16_t* S, long long n)
      : p(P, (size_t)n * 4), m(M, (size_t)n * 4), v(V, (size_t)n * 4), s(S ? (const void*)S : (const void*)P, (size_t)n * 2) {}
};

__device__ __forceinline__ void adam_store(const AdamOut& o, float4* P4, float4* G4, float4* M4,
                                           float4* V4, uint2* S2, long long i, const float4& pp,
                                           const float4& mm, const float4& vv, int zero_grad) {
  o.p.st16(P4 + i, pp);
  o.m.st16(M4 + i, mm);
  o.v.st16(V4 + i, vv);
  if (zero_grad) G4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (S2) {
    const uint32_t lo = pack2bf(pp.x, pp.y);
    const uint32_t hi = pack2bf(pp.z, pp.w);
    o.s.st8(S2 + i, make_uint2(lo, hi));
  }
}

// Streaming Adam: 16 B/param read (p, g, m, v) + 12 B written + 2 B shadow.
// Two float4 groups per thread per iteration with all eight 16-byte loads
// issued before any math (more bytes in flight per wave for HBM3E).
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   bf16_t* __restrict__ shadow, long long n,
                                                   const long long* __restrict__ step_ptr,
                                                   AdamCfg c) {
  const float step = (float)step_ptr[0];
  const float t = step + 1.f;
  const float lr = noam_lr(c, step);
  const float lr_t = lr * sqrtf(1.f - powf(c.beta2, t)) / (1.f - powf(c.beta1, t));
  const float ob1 = 1.f - c.beta1, ob2 = 1.f - c.beta2;
  const long long n4 = n >> 2;
  float4* P4 = reinterpret_cast<float4*>(p);
  float4* G4 = reinterpret_cast<float4*>(g);
  float4* M4 = reinterpret_cast<float4*>(m);
  float4* V4 = reinterpret_cast<float4*>(v);
  uint2* S2 = shadow ? reinterpret_cast<uint2*>(shadow) : nullptr;
  const AdamOut o(p, m, v, shadow, n);
  const long long stride = (long long)gridDim.x * blockDim.x;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + stride < n4; i += 2 * stride) {
    const long long j = i + stride;
    float4 pa = P4[i], ga = G4[i], ma = M4[i], va = V4[i];
    float4 pb = P4[j], gb = G4[j], mb = M4[j], vb = V4[j];
    adam4(pa, ga, ma, va, c, lr, lr_t, ob1, ob2);
    adam4(pb, gb, mb, vb, c, lr, lr_t, ob1, ob2);
    adam_store(o, P4, G4, M4, V4, S2, i, pa, ma, va, c.zero_grad);
    adam_store(o, P4, G4, M4, V4, S2, j, pb, mb, vb, c.zero_grad);
  }
  if (i < n4) {
    float4 pa = P4[i], ga = G4[i], ma = M4[i], va = V4[i];
    adam4(pa, ga, ma, va, c, lr, lr_t, ob1, ob2);
    adam_store(o, P4, G4, M4, V4, S2, i, pa, ma, va, c.zero_grad);
  }
}

// Adam over a table of chunks (<= 4096 parameters each, none crossing a
// parameter that has an e4m3 copy): a chunk inside such a weight also writes
// y8 = e4m3(bf16(p_new) * scale8[slot]) -- the refreshed e4m3 copy the next
// forward reads -- and folds its |bf16(p_new)| max into the slot's amax
// (one atomic per chunk). Replaces the separate re-quantisation pass over
// the bf16 shadow (fp8_quant_multi) after the optimizer step.
struct AdamChunk {
  long long start;  // first parameter (multiple of 4)
  long long n;      // parameter count (multiple of 4, <= 4096)
  long long slot;   // fp8 scale / amax slot, or -1
  long long y8;     // address of the e4m3 byte of parameter `start`, or 0
};
constexpr int ADAM_CHUNK = 4096, ADAM_PER_THREAD = ADAM_CHUNK / 4 / 256;

__global__ __launch_bounds__(256) void adam_chunk_kernel(
    float* __restrict__ p, float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
    bf16_t* __restrict__ shadow, long long n, const AdamChunk* __restrict__ chunks,
    const long long* __restrict__ step_ptr, AdamCfg c, const float* __restrict__ scale8,
    unsigned* __restrict__ amax8) {
  const AdamChunk ch = chunks[blockIdx.x];
  const float step = (float)step_ptr[0];
  const float t = step + 1.f;
  const float lr = noam_lr(c, step);
  const float lr_t = lr * sqrtf(1.f - powf(c.beta2, t)) / (1.f - powf(c.beta1, t));
  const float ob1 = 1.f - c.beta1, ob2 = 1.f - c.beta2;
  float4* P4 = reinterpret_cast<float4*>(p);
  float4* G4 = reinterpret_cast<float4*>(g);
  float4* M4 = reinterpret_cast<float4*>(m);
  float4* V4 = reinterpret_cast<float4*>(v);
  uint2* S2 = shadow ? reinterpret_cast<uint2*>(shadow) : nullptr;
  const AdamOut o(p, m, v, shadow, n);
  const long long i0 = ch.start / 4, n4 = ch.n / 4;
  float4 pa[ADAM_PER_THREAD], ga[ADAM_PER_THREAD], ma[ADAM_PER_THREAD], va[ADAM_PER_THREAD];
#pragma unroll
  for (int k = 0; k < ADAM_PER_THREAD; ++k) {
    const long long j = threadIdx.x + 256 * k;
    if (j < n4) {
      pa[k] = P4[i0 + j];
      ga[k] = G4[i0 + j];
      ma[k] = M4[i0 + j];
      va[k] = V4[i0 + j];
    }
  }
  uint8_t* y8 = reinterpret_cast<uint8_t*>(ch.y8);
  const float s8 = y8 ? scale8[ch.slot] : 0.f;
  float am = 0.f;
#pragma unroll
  for (int k = 0; k < ADAM_PER_THREAD; ++k) {
    const long long j = threadIdx.x + 256 * k;
    if (j >= n4) continue;
    adam4(pa[k], ga[k], ma[k], va[k], c, lr, lr_t, ob1, ob2);
    adam_store(o, P4, G4, M4, V4, S2, i0 + j, pa[k], ma[k], va[k], c.zero_grad);
    if (y8) {
      const float f0 = bf2f(f2bf(pa[k].x)), f1 = bf2f(f2bf(pa[k].y));
      const float f2 = bf2f(f2bf(pa[k].z)), f3 = bf2f(f2bf(pa[k].w));
      am = fmaxf(am, fmaxf(fmaxf(fabsf(f0), fabsf(f1)), fmaxf(fabsf(f2), fabsf(f3))));
      int w8 = pack2_e4m3<false>(f0 * s8, f1 * s8, 0);
      w8 = pack2_e4m3<true>(f2 * s8, f3 * s8, w8);
      *reinterpret_cast<int*>(y8 + 4 * j) = w8;
    }
  }
  if (y8) {
    __shared__ float red[4];
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) am = fmaxf(am, __shfl_xor(am, sh, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = am;
    __syncthreads();
    if (threadIdx.x == 0)
      atomic_amax(amax_word(amax8 + ch.slot * AMAX_WORDS, blockIdx.x),
                  fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
  }
}

__global__ void step_inc_kernel(long long* step) { step[0] += 1; }

// p_bf16 = bf16(p_f32) for the whole flat buffer (init / checkpoint load).
__global__ void to_bf16_kernel(const float* __restrict__ p, bf16_t* __restrict__ o, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    o[i] = f2bf(p[i]);
}

// Grouped bf16 transpose: dst[g] [C, R] = src[g] [R, C]^T, G same-shape
// matrices in one launch (the K-contiguous weight copies the relu-backward
// dgrads read; refreshed after every optimizer update). 64x64 tiles through
// LDS (padded rows: conflict-free column reads), 16-byte global accesses.
constexpr int TR_MAXG = 64;
struct TransposeGroup {
  const bf16_t* src[TR_MAXG];
  bf16_t* dst[TR_MAXG];
};

__global__ __launch_bounds__(256) void transpose_grouped_kernel(TransposeGroup grp, int R, int C) {
  __shared__ bf16_t tile[64][64 + 8];
  const bf16_t* __restrict__ src = grp.src[blockIdx.y];
  bf16_t* __restrict__ dst = grp.dst[blockIdx.y];
  const int tiles_c = (C + 63) / 64;
  const int r0 = (blockIdx.x / tiles_c) * 64, c0 = (blockIdx.x % tiles_c) * 64;
  const int tid = threadIdx.x;
  // load 64 rows x 64 cols: each thread 2 x 8 elements
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int id = tid + 256 * k;
    const int r = id >> 3, c = (id & 7) * 8;
    short8_t v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r0 + r < R && c0 + c + 8 <= C)
      v = *reinterpret_cast<const short8_t*>(src + (size_t)(r0 + r) * C + c0 + c);
    else
      for (int e = 0; e < 8; ++e)
        if (r0 + r < R && c0 + c + e < C) v[e] = (short)src[(size_t)(r0 + r) * C + c0 + c + e];
#pragma unroll
    for (int e = 0; e < 8; ++e) tile[r][c + e] = (bf16_t)v[e];
  }
  __syncthreads();
  // store 64 (former) columns x 64 (former) rows
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int id = tid + 256 * k;
    const int c = id >> 3, r = (id & 7) * 8;
    short8_t v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (short)tile[r + e][c];
    if (c0 + c < C && r0 + r + 8 <= R)
      *reinterpret_cast<short8_t*>(dst + (size_t)(c0 + c) * R + r0 + r) = v;
    else
      for (int e = 0; e < 8; ++e)
        if (c0 + c < C && r0 + r + e < R) dst[(size_t)(c0 + c) * R + r0 + r + e] = (bf16_t)v[e];
  }
}

}  // namespace tdg

using namespace tdg;

extern "C" int tdg_transpose_grouped(const void* const* src, void* const* dst, int G, int R, int C,
                                     hipStream_t st) {
  if (G < 1 || G > TR_MAXG || R < 1 || C < 1) return -1;
  TransposeGroup g{};
  for (int i = 0; i < G; ++i) {
    g.src[i] = (const bf16_t*)src[i];
    g.dst[i] = (bf16_t*)dst[i];
  }
  const int tiles = ((R + 63) / 64) * ((C + 63) / 64);
  hipLaunchKernelGGL(transpose_grouped_kernel, dim3(tiles, G), dim3(256), 0, st, g, R, C);
  return 0;
}

extern "C" int tdg_adam(float* p, float* g, float* m, float* v, void* shadow, long long n,
                        long long* step, float beta1, float beta2, float eps, float lr_const,
                        float d_model, float warmup, float grad_scale, float weight_decay,
                        int sched, int zero_grad, int inc_step, hipStream_t st) {
  if (n % 4 != 0) return -1;
  AdamCfg c{beta1, beta2, eps, lr_const, d_model, warmup, grad_scale, weight_decay, sched,
            zero_grad};
  // launches over chunks of <= 2^28 parameters: the write-through stores
  // address each buffer through a descriptor with 31-bit byte offsets
  constexpr long long CHUNK = 1LL << 28;
  for (long long o = 0; o < n; o += CHUNK) {
    const long long cn = std::min(CHUNK, n - o);
    const long long n4 = cn / 4;
    const int blocks = (int)std::min<long long>(8192, (n4 + 255) / 256);
    hipLaunchKernelGGL(adam_kernel, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st, p + o, g + o,
                       m + o, v + o, shadow ? (bf16_t*)shadow + o : nullptr, cn, step, c);
  }
  // per-bucket updates (data parallel) share one step: only the last advances it
  if (inc_step) hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, st, step);
  return 0;
}

// The whole flat buffer through a chunk table built by the host (ops/fp8.py
// Fp8Weights.adam_chunks); n < 2^28 (the write-through descriptors' 31-bit
// offsets).
extern "C" int tdg_adam_chunks(float* p, float* g, float* m, float* v, void* shadow, long long n,
                               const void* chunks, int nchunks, long long* step, float beta1,
                               float beta2, float eps, float lr_const, float d_model, float warmup,
                               float grad_scale, float weight_decay, int sched, int zero_grad,
                               int inc_step, const float* scale8, unsigned* amax8,
                               hipStream_t st) {
  if (n % 4 != 0 || n >= (1LL << 28) || nchunks <= 0) return -1;
  AdamCfg c{beta1, beta2, eps, lr_const, d_model, warmup, grad_scale, weight_decay, sched,
            zero_grad};
  hipLaunchKernelGGL(adam_chunk_kernel, dim3(nchunks), dim3(256), 0, st, p, g, m, v,
                     (bf16_t*)shadow, n, (const AdamChunk*)chunks, step, c, scale8, amax8);
  if (inc_step) hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, st, step);
  return 0;
}

extern "C" int tdg_to_bf16(const float* p, void* o, long long n, hipStream_t st) {
  const int blocks = (int)std::min<long long>(8192, (n + 255) / 256);
  hipLaunchKernelGGL(to_bf16_kernel, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st, p,
                     (bf16_t*)o, n);
  return 0;
}
