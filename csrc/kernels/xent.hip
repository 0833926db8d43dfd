// Fused masked softmax cross-entropy + argmax accuracy, forward and backward
// in one pass over the logits (gfx950).
//
// Replaces reference: distributed_training_transformer/transformer_model.py:7-26
// (SparseCategoricalCrossentropy(from_logits, reduction='none') masked by
// target != 0, token mean, divided by workers_count; accuracy = argmax match
// over non-pad tokens). Optional label smoothing eps (reference: 0).
//
// Per row (one 256-thread workgroup): online max / sum-exp / first-argmax over
// the vocabulary, then a second pass (row is L2-resident) writes
//   dlogits = (softmax - onehot_smoothed) * scale   (scale = 1/(ntok*workers))
// in place, or 0 for pad rows. Columns in [V, ldl) are zeroed so the padded
// logits buffer can feed the dgrad / wgrad GEMMs directly.
#include "tdg_common.h"

namespace tdg {

__device__ __forceinline__ void merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == -INFINITY) return;
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

template <typename LabT>
__global__ __launch_bounds__(256) void xent_kernel(bf16_t* __restrict__ logits, int V, int ldl,
                                                   const LabT* __restrict__ labels,
                                                   const float* __restrict__ ntok,
                                                   float workers, float smoothing,
                                                   float* __restrict__ row_loss,
                                                   float* __restrict__ row_correct,
                                                   int write_grad) {
  __shared__ float sm[4], ss[4], sv[4];
  __shared__ int si[4];
  const int row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  bf16_t* x = logits + (size_t)row * ldl;
  const int lab = (int)labels[row];
  // pass 1: max, sum-exp (online), argmax (first max), sum of logits (for smoothing)
  float m = -INFINITY, s = 0.f, bv = -INFINITY, sumx = 0.f;
  int bi = 0x7fffffff;
  for (int c = tid * 2; c < V; c += 512) {
    float v0, v1;
    if (c + 1 < V) {
      const uint32_t w2 = *reinterpret_cast<const uint32_t*>(x + c);
      v0 = bf2f((bf16_t)(w2 & 0xffff));
      v1 = bf2f((bf16_t)(w2 >> 16));
    } else {
      v0 = bf2f(x[c]);
      v1 = -INFINITY;
    }
    const float mx = fmaxf(v0, v1);
    if (mx > m) {
      s = s * __expf(m - mx);
      m = mx;
    }
    s += __expf(v0 - m) + (c + 1 < V ? __expf(v1 - m) : 0.f);
    sumx += v0 + (c + 1 < V ? v1 : 0.f);
    if (v0 > bv) { bv = v0; bi = c; }
    if (c + 1 < V && v1 > bv) { bv = v1; bi = c + 1; }
  }
  // wave reduction
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    merge(m, s, m2, s2);
    sumx += __shfl_xor(sumx, o, 64);
    const float bv2 = __shfl_xor(bv, o, 64);
    const int bi2 = __shfl_xor(bi, o, 64);
    if (bv2 > bv || (bv2 == bv && bi2 < bi)) { bv = bv2; bi = bi2; }
  }
  if (lane == 0) { sm[w] = m; ss[w] = s; sv[w] = bv; si[w] = bi; }
  __shared__ float sx[4];
  if (lane == 0) sx[w] = sumx;
  __syncthreads();
  m = sm[0]; s = ss[0]; bv = sv[0]; bi = si[0]; sumx = sx[0];
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    merge(m, s, sm[k], ss[k]);
    sumx += sx[k];
    if (sv[k] > bv || (sv[k] == bv && si[k] < bi)) { bv = sv[k]; bi = si[k]; }
  }
  const float lse = m + __logf(s);
  const bool valid = lab != 0;
  if (tid == 0) {
    float loss = 0.f;
    if (valid) {
      const float xl = bf2f(x[lab]);
      loss = (1.f - smoothing) * (lse - xl) + smoothing * (lse - sumx / (float)V);
    }
    row_loss[row] = loss;
    row_correct[row] = (valid && bi == lab) ? 1.f : 0.f;
  }
  if (!write_grad) return;
  __syncthreads();  // everyone read x[lab] before it is overwritten
  const float scale = valid ? 1.f / (fmaxf(ntok[0], 1.f) * workers) : 0.f;
  const float off = smoothing / (float)V;
  for (int c = tid * 2; c < ldl; c += 512) {
    float g0 = 0.f, g1 = 0.f;
    if (c < V && valid) {
      const float v0 = bf2f(x[c]);
      g0 = (__expf(v0 - lse) - off - (c == lab ? 1.f - smoothing : 0.f)) * scale;
      if (c + 1 < V) {
        const float v1 = bf2f(x[c + 1]);
        g1 = (__expf(v1 - lse) - off - (c + 1 == lab ? 1.f - smoothing : 0.f)) * scale;
      }
    }
    if (c + 1 < ldl) {
      *reinterpret_cast<uint32_t*>(x + c) = pack2bf(g0, g1);
    } else {
      x[c] = f2bf(g0);
    }
  }
}

// Register-resident variant for padded rows of <= 256 * 8 * NCH columns
// (ldl % 8 == 0): every thread loads its NCH 16-byte chunks once, so max /
// argmax / sum-exp / dlogits are computed from registers (no second pass over
// the row, no per-element online-softmax dependency chain); two block
// reductions (max+argmax+sum, then sum-exp). Same results as xent_kernel up to
// the order of the f32 sums (deterministic).
template <typename LabT, int NCH>
__global__ __launch_bounds__(256) void xent_reg_kernel(bf16_t* __restrict__ logits, int V, int ldl,
                                                       const LabT* __restrict__ labels,
                                                       const float* __restrict__ ntok,
                                                       float workers, float smoothing,
                                                       float* __restrict__ row_loss,
                                                       float* __restrict__ row_correct,
                                                       int write_grad) {
  __shared__ float r_m[4], r_x[4], r_s[4];
  __shared__ int r_i[4];
  const int row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  bf16_t* x = logits + (size_t)row * ldl;
  const int lab = (int)labels[row];
  const int nch = ldl >> 3;
  short8_t raw[NCH];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int ch = tid + 256 * k;
    if (ch < nch) raw[k] = *reinterpret_cast<const short8_t*>(x + 8 * ch);
  }
  const float xl = bf2f(x[lab]);  // read before any thread overwrites the row
  float m = -INFINITY, sumx = 0.f;
  int bi = 0x7fffffff;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c0 = 8 * (tid + 256 * k);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (c0 + e < V) {
        const float v = bf2f((bf16_t)raw[k][e]);
        sumx += v;
        if (v > m) { m = v; bi = c0 + e; }
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64);
    const int i2 = __shfl_xor(bi, o, 64);
    if (m2 > m || (m2 == m && i2 < bi)) { m = m2; bi = i2; }
    sumx += __shfl_xor(sumx, o, 64);
  }
  if (lane == 0) { r_m[w] = m; r_i[w] = bi; r_x[w] = sumx; }
  __syncthreads();
  m = r_m[0]; bi = r_i[0]; sumx = r_x[0];
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    if (r_m[k] > m || (r_m[k] == m && r_i[k] < bi)) { m = r_m[k]; bi = r_i[k]; }
    sumx += r_x[k];
  }
  float se = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c0 = 8 * (tid + 256 * k);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (c0 + e < V) se += __expf(bf2f((bf16_t)raw[k][e]) - m);
  }
  se = wave_sum(se);
  if (lane == 0) r_s[w] = se;
  __syncthreads();
  const float lse = m + __logf(r_s[0] + r_s[1] + r_s[2] + r_s[3]);
  const bool valid = lab != 0;
  if (tid == 0) {
    row_loss[row] = valid ? (1.f - smoothing) * (lse - xl) + smoothing * (lse - sumx / (float)V) : 0.f;
    row_correct[row] = (valid && bi == lab) ? 1.f : 0.f;
  }
  if (!write_grad) return;
  const float scale = valid ? 1.f / (fmaxf(ntok[0], 1.f) * workers) : 0.f;
  const float off = smoothing / (float)V;
  const WtBuf wt(logits, (size_t)gridDim.x * ldl * sizeof(bf16_t));  // one row per block
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int ch = tid + 256 * k;
    if (ch >= nch) continue;
    const int c0 = 8 * ch;
    short8_t g;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = c0 + e;
      float gv = 0.f;
      if (c < V && valid)
        gv = (__expf(bf2f((bf16_t)raw[k][e]) - lse) - off - (c == lab ? 1.f - smoothing : 0.f)) * scale;
      g[e] = (short)f2bf(gv);
    }
    wt.st16(x + c0, g);  // write-through: 115 MB of dlogits at Transformer-base
  }
}

// ntok = number of non-pad labels
template <typename LabT>
__global__ void count_tokens_kernel(const LabT* __restrict__ labels, int M, float* __restrict__ out) {
  __shared__ float red[4];
  float c = 0.f;
  for (int i = threadIdx.x; i < M; i += blockDim.x) c += labels[i] != 0 ? 1.f : 0.f;
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = red[0] + red[1] + red[2] + red[3];
}

// Batch preparation in one launch (replaces ~10 small framework kernels at the
// head of every step): teacher forcing tgt_in = tgt[:, :-1], labels =
// tgt[:, 1:] (reference: __main__.py:106-107), non-PAD lengths of src and
// tgt_in (the padding masks, transformer_model.py:56-62, as key lengths), the
// non-PAD label count, and the dropout RNG step counter bump. One workgroup,
// one wave per row at a time.
template <typename LabT>
__global__ __launch_bounds__(64) void prep_batch_kernel(
    const LabT* __restrict__ src, int S, const LabT* __restrict__ tgt, int T1, int B,
    LabT* __restrict__ tgt_in, LabT* __restrict__ labels, int* __restrict__ src_len,
    int* __restrict__ tgt_len, float* __restrict__ ntok, long long* __restrict__ ctr,
    int* __restrict__ row_lab, unsigned* __restrict__ ticket, int* __restrict__ bad_rows) {
  // one wave per row; the last wave to finish folds the label counts
  const int lane = threadIdx.x, b = blockIdx.x, T = T1 - 1;
  // cs/ct: non-PAD counts (the key lengths); es/et: one past the last non-PAD
  // position. They differ only when a PAD sits inside a row: attention masks
  // keys by length (trailing padding), while the reference masks every PAD
  // position (transformer_model.py:56-62), so such rows are counted in
  // bad_rows for the host to reject
  int cs = 0, ct = 0, cl = 0, es = 0, et = 0;
  for (int j = lane; j < S; j += 64) {
    const bool nz = src[(long long)b * S + j] != 0;
    cs += nz;
    es = nz ? j + 1 : es;
  }
  for (int j = lane; j < T1; j += 64) {
    const LabT v = tgt[(long long)b * T1 + j];
    if (j < T) {
      tgt_in[(long long)b * T + j] = v;
      ct += v != 0;
      et = v != 0 ? j + 1 : et;
    }
    if (j > 0) {
      labels[(long long)b * T + j - 1] = v;
      cl += v != 0;
    }
  }
  const float fs = wave_sum((float)cs), ft = wave_sum((float)ct), fl = wave_sum((float)cl);
  const float ms = wave_max((float)es), mt = wave_max((float)et);
  __shared__ bool last;
  if (lane == 0) {
    src_len[b] = (int)fs;
    tgt_len[b] = (int)ft;
    if (bad_rows && ((int)ms != (int)fs || (int)mt != (int)ft)) atomicAdd(bad_rows, 1);
    row_lab[b] = (int)fl;
    __threadfence();
    last = atomicAdd(ticket, 1u) == (unsigned)(B - 1);
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  int n = 0;  // integer counts: exact and order-independent
  for (int i = lane; i < B; i += 64) n += __atomic_load_n(row_lab + i, __ATOMIC_RELAXED);
  const float tot = wave_sum((float)n);
  if (lane == 0) {
    ntok[0] = tot;
    if (ctr) ctr[0] += 1;
    *ticket = 0u;  // re-armed for the next launch (graph replay)
  }
}

// stats[0] += sum(row_loss)/(ntok*workers), stats[1] += correct/ntok (accuracy
// ratio), stats[2] += 1 (batches), stats[3] += ntok; single block of 1024
// threads, 16-byte loads when the rows allow (vec: M % 4 == 0, 16-byte
// aligned), every load of a thread issued before the sums (the 256-thread
// scalar loop was a chain of dependent load rounds: 11 us for 8192 rows)
__global__ __launch_bounds__(1024) void xent_stats_kernel(const float* __restrict__ row_loss,
                                                          const float* __restrict__ row_correct,
                                                          int M, int vec,
                                                          const float* __restrict__ ntok, float workers,
                                                          float* __restrict__ step_out,
                                                          float* __restrict__ accum) {
  __shared__ float r1[16], r2[16];
  float a = 0.f, b = 0.f;
  int i0 = 0;
  if (vec) {
    const float4* L4 = reinterpret_cast<const float4*>(row_loss);
    const float4* C4 = reinterpret_cast<const float4*>(row_correct);
    const int M4 = M / 4;
#pragma unroll 4
    for (int i = threadIdx.x; i < M4; i += 1024) {
      const float4 x = L4[i], y = C4[i];
      a += (x.x + x.y) + (x.z + x.w);
      b += (y.x + y.y) + (y.z + y.w);
    }
    i0 = 4 * M4;
  }
  for (int i = i0 + threadIdx.x; i < M; i += 1024) {
    a += row_loss[i];
    b += row_correct[i];
  }
  a = wave_sum(a);
  b = wave_sum(b);
  if ((threadIdx.x & 63) == 0) {
    r1[threadIdx.x >> 6] = a;
    r2[threadIdx.x >> 6] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int w = 0; w < 16; ++w) {
      sa += r1[w];
      sb += r2[w];
    }
    const float n = fmaxf(ntok[0], 1.f);
    const float loss = sa / n / workers;
    const float acc = sb / n;
    if (step_out) {
      step_out[0] = loss;
      step_out[1] = acc;
    }
    if (accum) {
      accum[0] += loss;
      accum[1] += acc;
      accum[2] += 1.f;
      accum[3] += ntok[0];
    }
  }
}

}  // namespace tdg

using namespace tdg;

extern "C" int tdg_count_tokens(const void* labels, int lab64, int M, float* out, hipStream_t st) {
  if (lab64)
    hipLaunchKernelGGL(count_tokens_kernel<long long>, dim3(1), dim3(256), 0, st,
                       (const long long*)labels, M, out);
  else
    hipLaunchKernelGGL(count_tokens_kernel<int>, dim3(1), dim3(256), 0, st, (const int*)labels, M,
                       out);
  return 0;
}

extern "C" int tdg_prep_batch(const void* src, int S, const void* tgt, int T1, int B, int lab64,
                               void* tgt_in, void* labels, int* src_len, int* tgt_len,
                               float* ntok, long long* ctr, int* row_lab, unsigned* ticket,
                               int* bad_rows, hipStream_t st) {
  if (S < 1 || T1 < 2 || B < 1) return -1;
  if (lab64)
    hipLaunchKernelGGL(prep_batch_kernel<long long>, dim3(B), dim3(64), 0, st,
                       (const long long*)src, S, (const long long*)tgt, T1, B, (long long*)tgt_in,
                       (long long*)labels, src_len, tgt_len, ntok, ctr, row_lab, ticket, bad_rows);
  else
    hipLaunchKernelGGL(prep_batch_kernel<int>, dim3(B), dim3(64), 0, st, (const int*)src, S,
                       (const int*)tgt, T1, B, (int*)tgt_in, (int*)labels, src_len, tgt_len, ntok,
                       ctr, row_lab, ticket, bad_rows);
  return 0;
}

extern "C" int tdg_xent(void* logits, int M, int V, int ldl, const void* labels, int lab64,
                        const float* ntok, float workers, float smoothing, float* row_loss,
                        float* row_correct, int write_grad, hipStream_t st) {
  const bool aligned = (ldl % 8 == 0) && ((reinterpret_cast<uintptr_t>(logits) & 15) == 0);
  if (aligned && ldl <= 256 * 8 * 4) {
#define TDG_XR(NCH)                                                                              \
  if (lab64)                                                                                    \
    hipLaunchKernelGGL((xent_reg_kernel<long long, NCH>), dim3(M), dim3(256), 0, st,           \
                       (bf16_t*)logits, V, ldl, (const long long*)labels, ntok, workers,        \
                       smoothing, row_loss, row_correct, write_grad);                           \
  else                                                                                          \
    hipLaunchKernelGGL((xent_reg_kernel<int, NCH>), dim3(M), dim3(256), 0, st, (bf16_t*)logits, \
                       V, ldl, (const int*)labels, ntok, workers, smoothing, row_loss,          \
                       row_correct, write_grad);                                                \
  return 0;
    const int nch = cdiv(ldl / 8, 256);
    if (nch <= 1) { TDG_XR(1) }
    if (nch == 2) { TDG_XR(2) }
    if (nch == 3) { TDG_XR(3) }
    TDG_XR(4)
#undef TDG_XR
  }
  if (lab64)
    hipLaunchKernelGGL(xent_kernel<long long>, dim3(M), dim3(256), 0, st, (bf16_t*)logits, V, ldl,
                       (const long long*)labels, ntok, workers, smoothing, row_loss, row_correct,
                       write_grad);
  else
    hipLaunchKernelGGL(xent_kernel<int>, dim3(M), dim3(256), 0, st, (bf16_t*)logits, V, ldl,
                       (const int*)labels, ntok, workers, smoothing, row_loss, row_correct,
                       write_grad);
  return 0;
}

extern "C" int tdg_xent_stats(const float* row_loss, const float* row_correct, int M,
                              const float* ntok, float workers, float* step_out, float* accum,
                              hipStream_t st) {
  const int vec = M % 4 == 0 && reinterpret_cast<uintptr_t>(row_loss) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(row_correct) % 16 == 0;
  hipLaunchKernelGGL(xent_stats_kernel, dim3(1), dim3(1024), 0, st, row_loss, row_correct, M, vec,
                     ntok, workers, step_out, accum);
  return 0;
}
