// Fused token embedding + sqrt(d) scale + sinusoidal positional encoding +
// dropout (forward), and the embedding-table gradient (backward).
//
// Replaces reference: distributed_training_transformer/transformer_model.py:
// 29-53 (positional_encoding, interleaved sin/cos), 270-279 and 301-308
// (Embedding -> *sqrt(d) -> +PE[:L] -> Dropout). The PE table is computed once
// at model build (f32, [max_len, d], as the reference does) and read here; it
// stays L2-resident.
#include "tdg_common.h"
#include "tdg_ln.h"

#include <algorithm>

namespace tdg {

// out[row, :] = drop(table[tok[row]] * scale + pe[row % L])
// One wave per row, VEC = D/64 elements per lane (tdg_ln.h RowMap).
template <int D, typename TokT>
__global__ __launch_bounds__(256) void embed_fwd_kernel(
    const TokT* __restrict__ tok, const bf16_t* __restrict__ table, const float* __restrict__ pe,
    bf16_t* __restrict__ out, int M, int L, float scale, float p, uint32_t thresh, uint64_t seed,
    const long long* __restrict__ ctr, uint64_t site, uint8_t* __restrict__ kbits) {
  constexpr int VEC = D / 64;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int pos = row % L;
  const long long t = (long long)tok[row];
  const float* pr = pe + (size_t)pos * D;
  RowVec<VEC> v;
  v.load_row(table + t * D, lane);
#pragma unroll
  for (int i = 0; i < VEC; ++i) v.v[i] = v.v[i] * scale + pr[RowMap<VEC>::col(lane, i)];
  if (p > 0.f) {
    const float sc = 1.f / (1.f - p);
    const uint32_t km = keep_bits<VEC>(seed, ctr, site, (size_t)row * D, lane, thresh);
#pragma unroll
    for (int i = 0; i < VEC; ++i) v.v[i] = ((km >> i) & 1u) ? v.v[i] * sc : 0.f;
    if constexpr (VEC >= 8) {
      // the keep bits as a row-major bitmap (byte c / 8 of the row = columns
      // c..c+7) for the CSR backward, which then draws no Philox
      if (kbits) {
#pragma unroll
        for (int c = 0; c < RowMap<VEC>::CH; ++c)
          kbits[(size_t)row * (D / 8) + 64 * c + lane] = (uint8_t)(km >> (8 * c));
      }
    }
  }
  v.store_row(out + (size_t)row * D, lane);
}

// Keep bit of column lane + 64 c of a row for the backward kernels below, whose
// lanes own strided columns (coalesced atomics): each lane draws the 8-element
// run 8 lane + 512 s once (one Philox call per 8 elements instead of one per
// element) and the bits are fetched from the owning lane.
template <int D>
struct RowKeep {
  static constexpr int NS = (D + 511) / 512;
  uint32_t m[NS];
  __device__ __forceinline__ void draw(uint64_t seed, const long long* ctr, uint64_t site,
                                       size_t rbase, int lane, uint32_t thresh) {
    const uint64_t off = rng_offset(ctr, site);
#pragma unroll
    for (int s = 0; s < NS; ++s)
      m[s] = dropout_keep_run<8>(seed, off, rbase + 512 * s + 8 * lane, thresh);
  }
  // c: a constant after unrolling, so m[] stays in registers
  __device__ __forceinline__ bool keep(int c, int lane) const {
    const int col = c * 64 + lane;
    const uint32_t mm = (uint32_t)__shfl((int)m[c >> 3], (col >> 3) & 63, 64);
    return (mm >> (col & 7)) & 1u;
  }
};

// dtable[tok[row]] += drop_mask * dout[row] * scale  (f32 atomics into the
// f32 master-gradient buffer; rows of 2*D bytes per wave-instruction pair).
template <int D, typename TokT>
__global__ __launch_bounds__(256) void embed_bwd_kernel(
    const TokT* __restrict__ tok, const bf16_t* __restrict__ dout, float* __restrict__ dtable,
    int M, float scale, float p, uint32_t thresh, uint64_t seed, const long long* ctr, uint64_t site) {
  constexpr int VEC = D / 64;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const long long t = (long long)tok[row];
  const size_t rbase = (size_t)row * D;
  const float sc = p > 0.f ? scale / (1.f - p) : scale;
  RowKeep<D> rk;
  if (p > 0.f) rk.draw(seed, ctr, site, rbase, lane, thresh);
  // column c*64+lane: every atomic wave-instruction covers 256 contiguous bytes
#pragma unroll
  for (int c = 0; c < VEC; ++c) {
    const int col = c * 64 + lane;
    float g = bf2f(dout[rbase + col]) * sc;
    if (p > 0.f && !rk.keep(c, lane)) g = 0.f;
    atomicAdd(dtable + t * D + col, g);
  }
}

// Deterministic variant: contributions are added as 2^-32 fixed-point int64,
// so the sum is independent of the order the atomics land in (integer
// addition is associative); embed_acc_convert turns the accumulator into the
// f32 gradient and re-zeroes it. Resolution 2.3e-10, range +-2^31.
constexpr float FX_SCALE = 4294967296.f;  // 2^32

template <int D, typename TT>
__global__ __launch_bounds__(256) void embed_bwd_fx_kernel(
    const TT* __restrict__ tok, const bf16_t* __restrict__ dout, unsigned long long* __restrict__ acc,
    int M, float scale, float p, uint32_t thresh, uint64_t seed, const long long* ctr,
    uint64_t site) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const long long t = (long long)tok[row];
  const size_t rbase = (size_t)row * D;
  const float sc = p > 0.f ? scale / (1.f - p) : scale;
  RowKeep<D> rk;
  if (p > 0.f) rk.draw(seed, ctr, site, rbase, lane, thresh);
#pragma unroll
  for (int c = 0; c < D / 64; ++c) {
    const int col = c * 64 + lane;
    float g = bf2f(dout[rbase + col]) * sc;
    if (p > 0.f && !rk.keep(c, lane)) g = 0.f;
    const long long fx = (long long)rintf(g * FX_SCALE);
    if (fx != 0) atomicAdd(acc + t * D + col, (unsigned long long)fx);
  }
}

// 4 elements per thread and iteration: two 16-byte accumulator loads, one
// 16-byte write-through gradient store (the gradients are read by Adam on
// every XCD), the accumulator zeroed only where a row was touched.
// n % 4 == 0, out 16-byte aligned.
__global__ __launch_bounds__(256) void embed_acc_convert4_kernel(long long* __restrict__ acc,
                                                                 float* __restrict__ out,
                                                                 long long n, float beta) {
  const WtBuf wt(out, (size_t)n * sizeof(float));
  const long long stride = (long long)gridDim.x * blockDim.x * 4;
  for (long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
    longlong2* a2 = reinterpret_cast<longlong2*>(acc + i);
    const longlong2 x = a2[0], y = a2[1];
    float4 o = make_float4((float)x.x * (1.f / FX_SCALE), (float)x.y * (1.f / FX_SCALE),
                           (float)y.x * (1.f / FX_SCALE), (float)y.y * (1.f / FX_SCALE));
    if (beta != 0.f) {
      const float4 b = *reinterpret_cast<const float4*>(out + i);
      o.x += beta * b.x;
      o.y += beta * b.y;
      o.z += beta * b.z;
      o.w += beta * b.w;
    }
    wt.st16(out + i, o);
    if ((x.x | x.y | y.x | y.y) != 0) {
      a2[0] = make_longlong2(0, 0);
      a2[1] = make_longlong2(0, 0);
    }
  }
}

__global__ __launch_bounds__(256) void embed_acc_convert_kernel(long long* __restrict__ acc,
                                                                float* __restrict__ out,
                                                                long long n, float beta) {
  const long long i0 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 2;
  for (long long i = i0; i < n; i += (long long)gridDim.x * blockDim.x * 2) {
    if (i + 1 < n) {
      const long long a0 = acc[i], a1 = acc[i + 1];
      float2 o;
      if (beta != 0.f) {
        o = *reinterpret_cast<float2*>(out + i);
        o.x = beta * o.x + (float)a0 * (1.f / FX_SCALE);
        o.y = beta * o.y + (float)a1 * (1.f / FX_SCALE);
      } else {
        o = make_float2((float)a0 * (1.f / FX_SCALE), (float)a1 * (1.f / FX_SCALE));
      }
      *reinterpret_cast<float2*>(out + i) = o;
      if (a0 != 0 || a1 != 0) {
        acc[i] = 0;
        acc[i + 1] = 0;
      }
    } else {
      const float v = (float)acc[i] * (1.f / FX_SCALE);
      out[i] = beta != 0.f ? beta * out[i] + v : v;
      acc[i] = 0;
    }
  }
}

// ---------------------------------------------------------------- CSR backward
// Deterministic and free of global atomics (the fixed-point kernel above spends
// its time on 4 M int64 atomics per table: ~28 us + 12 us conversion at 8192 x
// 512). (1) One workgroup counting-sorts the token ids (LDS histogram, scan,
// scatter) and cuts every vocabulary row into work items of at most ET
// occurrences, each holding its token positions; (2) one wave per item adds
// its rows' dropout-masked, scaled gradients as 2^-32 fixed-point int64 in
// registers -- integer addition, so the order of the rows does not matter and
// the sum is bitwise the fixed-point atomic kernel's -- and writes the f32
// gradient row, or for a row cut into several items an int64 partial; (3) one
// workgroup per such row adds its partials. Every table row is written
// (untouched rows: 0, or beta * old).
constexpr int ET = 8;         // occurrences per work item (their loads in flight together)
constexpr int EVMAX = 8192;   // vocabulary rows of the LDS histogram
constexpr int EPMAX = 16;     // token positions per sort thread (M <= 16384)

struct EmbItem {
  int v, slot, n, pad;  // row, partial slot (-1: the row's only item), occurrences
  int pos[ET];          // token positions
};
struct EmbCsr {
  EmbItem* items;   // [V + M / ET + 1]
  int4* heavy;      // [M / ET + 1]: (row, first slot, slots, 0)
  int* counts;      // [2]: items, cut rows
  long long* slab;  // [2 M / ET + 2, D] int64 partials
};
// one table of a (one or two table) sort launch
struct EmbSortTab {
  const void* tok;
  int tok64, M, V;
  EmbCsr cs;
};
struct EmbSortArgs {
  EmbSortTab t[2];
  long long* stamps;  // lab only (null): s_memrealtime at the phase ends, [2][8][64]
};

__host__ __device__ inline int csr_ub_items(int M, int V) { return V + M / ET + 1; }
__host__ __device__ inline int csr_ub_heavy(int M) { return M / ET + 1; }
__host__ __device__ inline int csr_ub_slots(int M) { return 2 * (M / ET) + 2; }

// Workgroup barrier for LDS data only: __syncthreads() also waits for every
// outstanding global store of the wave (vmcnt(0)), which made each of the
// sort's per-round barriers wait for the item stores of that round (~2 us per
// round of 1024 vocabulary rows).
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// One 1024-thread workgroup per table. LDS: the histogram (then the scatter
// cursors), each row's packed (first item << 15 | first sorted position), the
// sorted token positions and the cut rows. One block scan over per-thread
// contiguous runs of rows gives every offset; the items are then written with
// rows dealt to lanes in rounds of 1024, so consecutive lanes write
// consecutive items (coalesced), and the cut rows' items one per thread.
__global__ __launch_bounds__(1024) void embed_sort_kernel(const EmbSortArgs a) {
  __shared__ int cnt[EVMAX];
  __shared__ int ibst[EVMAX];
  __shared__ int perm[1024 * EPMAX];
  __shared__ int hrow[1024 * EPMAX / ET + 1], hslot[1024 * EPMAX / ET + 1];  // cut rows
  __shared__ int4 wtot[16];
  const EmbSortTab tb = blockIdx.x ? a.t[1] : a.t[0];
  const int M = tb.M, V = tb.V;
  const EmbCsr cs = tb.cs;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // (lab stamps: wave 0 stores the clock, one slot per lane -- vector stores)
  auto stamp = [&](int k) {
    if (a.stamps && wid == 0)
      a.stamps[(blockIdx.x * 8 + k) * 64 + lane] = (long long)__builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  for (int v = tid; v < V; v += 1024) cnt[v] = 0;
  // each thread a contiguous run of <= EPMAX positions, all loads in flight
  // at once; equal consecutive ids are counted as one run (right padding:
  // one LDS atomic per thread instead of one per position on a single bin)
  const int P = (M + 1023) / 1024;
  const int i0 = min(M, tid * P), i1 = min(M, i0 + P);
  long long tl[EPMAX];
  if (tb.tok64) {
    const long long* t = static_cast<const long long*>(tb.tok);
#pragma unroll
    for (int u = 0; u < EPMAX; ++u) tl[u] = i0 + u < i1 ? t[i0 + u] : -1;
  } else {
    const int* t = static_cast<const int*>(tb.tok);
#pragma unroll
    for (int u = 0; u < EPMAX; ++u) tl[u] = i0 + u < i1 ? (long long)t[i0 + u] : -1;
  }
  int tk[EPMAX];
#pragma unroll
  for (int u = 0; u < EPMAX; ++u) tk[u] = (tl[u] >= 0 && tl[u] < V) ? (int)tl[u] : -1;
  lds_sync();
  {
    int cur = -1, len = 0;
#pragma unroll
    for (int u = 0; u < EPMAX; ++u) {
      if (tk[u] != cur) {
        if (cur >= 0) atomicAdd(&cnt[cur], len);
        cur = tk[u];
        len = 0;
      }
      ++len;
    }
    if (cur >= 0) atomicAdd(&cnt[cur], len);
  }
  lds_sync();
  stamp(1);
  // offsets: each thread a contiguous run of rows, one block scan of
  // (positions, items, partial slots, cut rows)
  const int C = (V + 1023) / 1024;
  const int v0 = min(V, tid * C), v1 = min(V, v0 + C);
  int4 loc = make_int4(0, 0, 0, 0);
  for (int v = v0; v < v1; ++v) {
    const int c = cnt[v];
    const int n = c > ET ? (c + ET - 1) / ET : 1;
    loc.x += c;
    loc.y += n;
    if (c > ET) {
      loc.z += n;
      loc.w += 1;
    }
  }
  int4 inc = loc;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int q0 = __shfl_up(inc.x, d, 64), q1 = __shfl_up(inc.y, d, 64);
    const int q2 = __shfl_up(inc.z, d, 64), q3 = __shfl_up(inc.w, d, 64);
    if (lane >= d) {
      inc.x += q0;
      inc.y += q1;
      inc.z += q2;
      inc.w += q3;
    }
  }
  if (lane == 63) wtot[wid] = inc;
  lds_sync();
  int4 o = make_int4(inc.x - loc.x, inc.y - loc.y, inc.z - loc.z, inc.w - loc.w);
  int4 tot = make_int4(0, 0, 0, 0);
#pragma unroll
  for (int w = 0; w < 16; ++w) {
    const int4 t = wtot[w];
    if (w < wid) {
      o.x += t.x;
      o.y += t.y;
      o.z += t.z;
      o.w += t.w;
    }
    tot.x += t.x;
    tot.y += t.y;
    tot.z += t.z;
    tot.w += t.w;
  }
  for (int v = v0; v < v1; ++v) {
    const int c = cnt[v];
    const bool cut = c > ET;
    const int n = cut ? (c + ET - 1) / ET : 1;
    ibst[v] = (o.y << 15) | o.x;
    cnt[v] = o.x;  // scatter cursor
    if (cut) {
      cs.heavy[o.w] = make_int4(v, o.z, n, 0);
      hrow[o.w] = v;
      hslot[o.w] = o.z;
      o.z += n;
      o.w += 1;
    }
    o.x += c;
    o.y += n;
  }
  if (tid == 0) {
    cs.counts[0] = tot.y;
    cs.counts[1] = tot.w;
  }
  lds_sync();
  stamp(2);
  {  // sorted positions into LDS
    int cur = -1, len = 0, r0 = i0;
#pragma unroll
    for (int u = 0; u < EPMAX; ++u) {
      if (tk[u] != cur) {
        if (cur >= 0) {
          const int b = atomicAdd(&cnt[cur], len);
          for (int k = 0; k < len; ++k) perm[b + k] = r0 + k;
        }
        cur = tk[u];
        len = 0;
        r0 = i0 + u;
      }
      ++len;
    }
    if (cur >= 0) {
      const int b = atomicAdd(&cnt[cur], len);
      for (int k = 0; k < len; ++k) perm[b + k] = r0 + k;
    }
  }
  lds_sync();
  stamp(3);
  // single-item rows (<= ET occurrences; untouched rows included): head and
  // positions, rows dealt to lanes in rounds of 1024
  for (int v = tid; v < V; v += 1024) {
    const int ib = ibst[v] >> 15, st = ibst[v] & 0x7fff;
    const int c = cnt[v] - st;
    if (c > ET) continue;
    int q[ET];
#pragma unroll
    for (int j = 0; j < ET; ++j) q[j] = j < c ? perm[st + j] : 0;
    int4* it = reinterpret_cast<int4*>(cs.items + ib);
    it[0] = make_int4(v, -1, c, 0);
    if (c > 0) {
      it[1] = make_int4(q[0], q[1], q[2], q[3]);
      it[2] = make_int4(q[4], q[5], q[6], q[7]);
    }
  }
  stamp(4);
  // the cut rows' items, one thread per item: item s of the tot.z cut items
  // belongs to the cut row h whose slot range holds it (binary search of the
  // ascending slot bases) -- a padding id's hundreds of items, or hundreds of
  // cut rows, are nobody's serial loop
  for (int sidx = tid; sidx < tot.z; sidx += 1024) {
    int lo = 0, hi = tot.w - 1;
    while (lo < hi) {  // last h with hslot[h] <= sidx
      const int mid = (lo + hi + 1) >> 1;
      if (hslot[mid] <= sidx) lo = mid;
      else hi = mid - 1;
    }
    const int v = hrow[lo], ib = ibst[v] >> 15, st = ibst[v] & 0x7fff;
    const int c = cnt[v] - st, k = sidx - hslot[lo];
    int q[ET];
#pragma unroll
    for (int j = 0; j < ET; ++j) q[j] = k * ET + j < c ? perm[st + k * ET + j] : 0;
    int4* it = reinterpret_cast<int4*>(cs.items + ib + k);
    it[0] = make_int4(v, sidx, min(c, (k + 1) * ET) - k * ET, 0);
    it[1] = make_int4(q[0], q[1], q[2], q[3]);
    it[2] = make_int4(q[4], q[5], q[6], q[7]);
  }
  stamp(5);
}

// f32 gradient row (fixed-point sums in RowMap slots) -> dtable row, beta * old
template <int VEC>
__device__ __forceinline__ void emb_store_row(float* __restrict__ row, const long long (&acc)[VEC],
                                              int lane, float beta, const WtBuf& wt) {
  using Map = RowMap<VEC>;
#pragma unroll
  for (int c = 0; c < Map::CH; ++c) {
    float* p = row + c * 64 * Map::W + lane * Map::W;
#pragma unroll
    for (int q = 0; q < Map::W; q += 4 > Map::W ? Map::W : 4) {
      if constexpr (Map::W >= 4) {
        float4 o = make_float4((float)acc[c * Map::W + q] * (1.f / FX_SCALE),
                               (float)acc[c * Map::W + q + 1] * (1.f / FX_SCALE),
                               (float)acc[c * Map::W + q + 2] * (1.f / FX_SCALE),
                               (float)acc[c * Map::W + q + 3] * (1.f / FX_SCALE));
        if (beta != 0.f) {
          const float4 b = *reinterpret_cast<const float4*>(p + q);
          o.x += beta * b.x;
          o.y += beta * b.y;
          o.z += beta * b.z;
          o.w += beta * b.w;
        }
        wt.st16(p + q, o);
      } else {
#pragma unroll
        for (int e = 0; e < Map::W; ++e) {
          float o = (float)acc[c * Map::W + e] * (1.f / FX_SCALE);
          if (beta != 0.f) o += beta * p[e];
          p[e] = o;
        }
      }
    }
  }
}

template <int D>
__global__ __launch_bounds__(256) void embed_gather_kernel(const bf16_t* __restrict__ dout,
                                                           const uint8_t* __restrict__ kbits,
                                                           float* __restrict__ dtable, EmbCsr cs,
                                                           int V, int nub, float sc, float p,
                                                           uint32_t thresh, uint64_t seed,
                                                           const long long* ctr, uint64_t site,
                                                           float beta) {
  constexpr int VEC = D / 64;
  using Map = RowMap<VEC>;
  const int lane = threadIdx.x & 63;
  const int it = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (it >= nub) return;
  // the item (row, slot, count and its positions) and the item count in
  // flight together; then all its rows (and keep bytes)
  const EmbItem* ip = cs.items + it;
  const int4 w = *reinterpret_cast<const int4*>(ip);
  const int4 pa = *reinterpret_cast<const int4*>(ip->pos);
  const int4 pb = *reinterpret_cast<const int4*>(ip->pos + 4);
  if (it >= cs.counts[0]) return;
  const int n = w.z;
  const int r[ET] = {pa.x, pa.y, pa.z, pa.w, pb.x, pb.y, pb.z, pb.w};
  static_assert(ET == 8, "positions as two int4");
  RowVec<VEC> g[ET];
  uint32_t km[ET];
#pragma unroll
  for (int u = 0; u < ET; ++u) {
    if (u < n) {
      g[u].load_row(dout + (size_t)r[u] * D, lane);
      km[u] = 0xffffffffu;
      if constexpr (VEC >= 8) {
        if (p > 0.f && kbits) {
          uint32_t b = 0;
#pragma unroll
          for (int c = 0; c < Map::CH; ++c)
            b |= (uint32_t)kbits[(size_t)r[u] * (D / 8) + 64 * c + lane] << (8 * c);
          km[u] = b;
        }
      }
    }
  }
  long long acc[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) acc[i] = 0;
#pragma unroll
  for (int u = 0; u < ET; ++u) {
    if (u >= n) break;
    uint32_t m = km[u];
    if (p > 0.f && !(VEC >= 8 && kbits))
      m = keep_bits<VEC>(seed, ctr, site, (size_t)r[u] * D, lane, thresh);
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      float x = g[u].v[i] * sc;  // (the fixed-point atomic kernel's arithmetic)
      if (!((m >> i) & 1u)) x = 0.f;
      acc[i] += (long long)rintf(x * FX_SCALE);
    }
  }
  if (w.y < 0) {
    emb_store_row<VEC>(dtable + (size_t)w.x * D, acc, lane, beta,
                       WtBuf(dtable, (size_t)V * D * sizeof(float)));
  } else {
    long long* sl = cs.slab + (size_t)w.y * D;
#pragma unroll
    for (int i = 0; i < VEC; ++i) sl[Map::col(lane, i)] = acc[i];
  }
}

// one 16-wave workgroup per cut row: wave w adds the row's partial slots
// w, w + 16, ...; the 16 sums are added through LDS (integers: any order)
template <int D>
__global__ __launch_bounds__(1024) void embed_combine_kernel(float* __restrict__ dtable, EmbCsr cs,
                                                             int V, int nub, float beta) {
  constexpr int VEC = D / 64;
  using Map = RowMap<VEC>;
  __shared__ long long red[16][D];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int hb = blockIdx.x;
  if (hb >= nub || hb >= cs.counts[1]) return;
  const int4 h = cs.heavy[hb];
  long long acc[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) acc[i] = 0;
  for (int k = wid; k < h.z; k += 16) {
    const long long* sl = cs.slab + (size_t)(h.y + k) * D;
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[i] += sl[Map::col(lane, i)];
  }
#pragma unroll
  for (int i = 0; i < VEC; ++i) red[wid][Map::col(lane, i)] = acc[i];
  __syncthreads();
  float* row = dtable + (size_t)h.x * D;
  for (int c = threadIdx.x; c < D; c += 1024) {
    long long t = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += red[q][c];
    float o = (float)t * (1.f / FX_SCALE);
    if (beta != 0.f) o += beta * row[c];
    row[c] = o;
  }
}

}  // namespace tdg

using namespace tdg;

namespace {
template <int D, typename TT>
void fwd_d(const void* tok, const void* table, const float* pe, void* out, int M, int L,
           float scale, float p, uint64_t seed, const long long* ctr, uint64_t site,
           void* kbits, hipStream_t st) {
  const uint32_t thresh = dropout_thresh(p);
  hipLaunchKernelGGL((embed_fwd_kernel<D, TT>), dim3(cdiv(M, 4)), dim3(256), 0, st,
                     (const TT*)tok, (const bf16_t*)table, pe, (bf16_t*)out, M, L, scale, p,
                     thresh, seed, ctr, site, (uint8_t*)kbits);
}
template <int D, typename TT>
void bwd_d(const void* tok, const void* dout, float* dtable, int M, float scale, float p,
           uint64_t seed, const long long* ctr, uint64_t site, hipStream_t st) {
  const uint32_t thresh = dropout_thresh(p);
  hipLaunchKernelGGL((embed_bwd_kernel<D, TT>), dim3(cdiv(M, 4)), dim3(256), 0, st,
                     (const TT*)tok, (const bf16_t*)dout, dtable, M, scale, p, thresh, seed, ctr, site);
}
template <int D, typename TT>
void bwd_fx_d(const void* tok, const void* dout, unsigned long long* acc, int M, float scale, float p,
              uint64_t seed, const long long* ctr, uint64_t site, hipStream_t st) {
  const uint32_t thresh = dropout_thresh(p);
  hipLaunchKernelGGL((embed_bwd_fx_kernel<D, TT>), dim3(cdiv(M, 4)), dim3(256), 0, st,
                     (const TT*)tok, (const bf16_t*)dout, acc, M, scale, p, thresh, seed, ctr, site);
}
}  // namespace

#define TDG_D_SWITCH(F, TT, ...)                  \
  switch (D) {                                    \
    case 128: F<128, TT>(__VA_ARGS__); return 0;  \
    case 256: F<256, TT>(__VA_ARGS__); return 0;  \
    case 512: F<512, TT>(__VA_ARGS__); return 0;  \
    case 1024: F<1024, TT>(__VA_ARGS__); return 0; \
    default: return -1;                           \
  }

// kbits (may be null; D >= 512): the dropout keep bits, uint8 [M, D / 8]
extern "C" int tdg_embed_fwd(const void* tok, int tok64, const void* table, const float* pe,
                             void* out, int M, int L, int D, float scale, float p, uint64_t seed,
                             const long long* ctr, uint64_t site, void* kbits, hipStream_t st) {
  if (kbits && D < 512) return -3;
  if (tok64) {
    TDG_D_SWITCH(fwd_d, long long, tok, table, pe, out, M, L, scale, p, seed, ctr, site, kbits, st)
  } else {
    TDG_D_SWITCH(fwd_d, int, tok, table, pe, out, M, L, scale, p, seed, ctr, site, kbits, st)
  }
}

extern "C" int tdg_embed_bwd(const void* tok, int tok64, const void* dout, float* dtable, int M,
                             int D, float scale, float p, uint64_t seed, const long long* ctr, uint64_t site,
                             hipStream_t st) {
  if (tok64) {
    TDG_D_SWITCH(bwd_d, long long, tok, dout, dtable, M, scale, p, seed, ctr, site, st)
  } else {
    TDG_D_SWITCH(bwd_d, int, tok, dout, dtable, M, scale, p, seed, ctr, site, st)
  }
}

// Deterministic embedding backward: fixed-point accumulation into acc
// ([V, D] int64, all-zero on entry and on exit), then dtable = beta*dtable + acc.
extern "C" int tdg_embed_bwd_det(const void* tok, int tok64, const void* dout, float* dtable,
                                 long long* acc, int M, int D, long long V, float scale, float p,
                                 uint64_t seed, const long long* ctr, uint64_t site, float beta,
                                 hipStream_t st) {
  unsigned long long* a = reinterpret_cast<unsigned long long*>(acc);
  int rc = -1;
  if (tok64) {
    switch (D) {
      case 128: bwd_fx_d<128, long long>(tok, dout, a, M, scale, p, seed, ctr, site, st); rc = 0; break;
      case 256: bwd_fx_d<256, long long>(tok, dout, a, M, scale, p, seed, ctr, site, st); rc = 0; break;
      case 512: bwd_fx_d<512, long long>(tok, dout, a, M, scale, p, seed, ctr, site, st); rc = 0; break;
      case 1024: bwd_fx_d<1024, long long>(tok, dout, a, M, scale, p, seed, ctr, site, st); rc = 0; break;
    }
  } else {
    switch (D) {
      case 128: bwd_fx_d<128, int>(tok, dout, a, M, scale, p, seed, ctr, site, st); rc = 0; break;
      case 256: bwd_fx_d<256, int>(tok, dout, a, M, scale, p, seed, ctr, site, st); rc = 0; break;
      case 512: bwd_fx_d<512, int>(tok, dout, a, M, scale, p, seed, ctr, site, st); rc = 0; break;
      case 1024: bwd_fx_d<1024, int>(tok, dout, a, M, scale, p, seed, ctr, site, st); rc = 0; break;
    }
  }
  if (rc) return rc;
  const long long n = V * D;
  if (n % 4 == 0 && reinterpret_cast<uintptr_t>(dtable) % 16 == 0 &&
      reinterpret_cast<uintptr_t>(acc) % 16 == 0 && (size_t)n * sizeof(float) <= 0x7fffffffull) {
    const int blocks = (int)std::min<long long>(4096, (n / 4 + 255) / 256);
    hipLaunchKernelGGL(embed_acc_convert4_kernel, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st, acc,
                       dtable, n, beta);
    return 0;
  }
  const int blocks = (int)std::min<long long>(4096, (n / 2 + 255) / 256 + 1);
  hipLaunchKernelGGL(embed_acc_convert_kernel, dim3(blocks), dim3(256), 0, st, acc, dtable, n, beta);
  return 0;
}

// Workspace of the CSR backward: int32 words (16-byte aligned pieces) and
// int64 partial words.
extern "C" void tdg_embed_csr_ws(int M, int V, int D, long long* n32, long long* n64) {
  *n32 = (long long)(sizeof(EmbItem) / 4) * csr_ub_items(M, V) + 4LL * csr_ub_heavy(M) + 4;
  *n64 = (long long)csr_ub_slots(M) * D;
}

namespace {
EmbCsr csr_view(int* ws32, long long* ws64, int M, int V) {
  EmbCsr cs;
  int* w = ws32;
  cs.items = reinterpret_cast<EmbItem*>(w);
  w += (long long)(sizeof(EmbItem) / 4) * csr_ub_items(M, V);
  cs.heavy = reinterpret_cast<int4*>(w);
  w += 4LL * csr_ub_heavy(M);
  cs.counts = w;
  cs.slab = ws64;
  return cs;
}
}  // namespace

// Supported by the CSR path: V <= EVMAX, M <= 1024 * EPMAX (else the
// fixed-point atomic path).
extern "C" int tdg_embed_csr_ok(int M, int V) {
  return V > 0 && V <= EVMAX && M > 0 && M <= 1024 * EPMAX;
}

// The token sort of one or two tables (one workgroup each, one launch): the
// work items of the CSR backward in ws32[i] (tdg_embed_csr_ws words).
extern "C" int tdg_embed_csr_sort(int ntab, const void* const* tok, const int* tok64, const int* M,
                                  const int* V, int* const* ws32, long long* stamps,
                                  hipStream_t st) {
  if (ntab < 1 || ntab > 2) return -2;
  EmbSortArgs a{};
  a.stamps = stamps;
  for (int i = 0; i < ntab; ++i) {
    if (!tdg_embed_csr_ok(M[i], V[i])) return -2;
    a.t[i].tok = tok[i];
    a.t[i].tok64 = tok64[i];
    a.t[i].M = M[i];
    a.t[i].V = V[i];
    a.t[i].cs = csr_view(ws32[i], nullptr, M[i], V[i]);
  }
  hipLaunchKernelGGL(embed_sort_kernel, dim3(ntab), dim3(1024), 0, st, a);
  return 0;
}

// The gradient from sorted work items (tdg_embed_csr_sort): dtable = beta *
// dtable + sum over the rows of each token of drop(dout) * scale; gather and
// cut-row combine launches. kbits: the forward's keep bits (or null: the
// Philox mask is regenerated).
extern "C" int tdg_embed_csr_apply(const void* dout, const void* kbits, float* dtable, int* ws32,
                                   long long* ws64, int M, int D, int V, float scale, float p,
                                   uint64_t seed, const long long* ctr, uint64_t site, float beta,
                                   hipStream_t st) {
  if (!tdg_embed_csr_ok(M, V)) return -2;
  const EmbCsr cs = csr_view(ws32, ws64, M, V);
  const uint32_t thresh = dropout_thresh(p);
  const float sc = p > 0.f ? scale / (1.f - p) : scale;
  const int ni = csr_ub_items(M, V), nh = csr_ub_heavy(M);
#define TDG_CSR(DD)                                                                               \
  hipLaunchKernelGGL(embed_gather_kernel<DD>, dim3(cdiv(ni, 4)), dim3(256), 0, st,                \
                     (const bf16_t*)dout, (const uint8_t*)kbits, dtable, cs, V, ni, sc, p, thresh, \
                     seed, ctr, site, beta);                                                      \
  hipLaunchKernelGGL(embed_combine_kernel<DD>, dim3(nh), dim3(1024), 0, st, dtable, cs, V, nh,    \
                     beta);                                                                       \
  return 0;
  switch (D) {
    case 128: TDG_CSR(128)
    case 256: TDG_CSR(256)
    case 512: TDG_CSR(512)
    case 1024: TDG_CSR(1024)
  }
#undef TDG_CSR
  return -1;
}
