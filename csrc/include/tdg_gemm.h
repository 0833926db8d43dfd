// Shared pieces of the MFMA GEMM kernels (gemm.hip, gemm_ln.hip): LDS tile
// image layout (XOR-swizzled), the LDS-DMA operand stager, counted waits and
// MFMA fragment reads.
#pragma once
#include "tdg_common.h"

namespace tdg {

constexpr int BK = 64;

// Byte offset inside an LDS tile image.
//  KC (K-contiguous): [R rows][BK] -> 128-B rows; 32-B segment ^= (row>>1)&3
//  MC (MN-contiguous): [BK rows][R] -> R*2-B rows
//     R=128 (256-B rows): seg ^= (row&3) | ((row>>3)&1)<<2
//     R=64  (128-B rows): seg ^= ((row>>1)&1) | ((row>>3)&1)<<1
template <bool KC, int R>
__device__ __forceinline__ int lds_off(int row, int byte) {
  if constexpr (KC) {
    const int seg = (byte >> 5) ^ ((row >> 1) & 3);
    return row * (BK * 2) + (seg << 5) + (byte & 31);
  } else if constexpr (R >= 128) {
    const int seg = (byte >> 5) ^ ((row & 3) | (((row >> 3) & 1) << 2));
    return row * (R * 2) + (seg << 5) + (byte & 31);
  } else {
    static_assert(R == 64, "MN-contiguous tiles must be 64 or 128 wide");
    const int seg = (byte >> 5) ^ (((row >> 1) & 1) | (((row >> 3) & 1) << 1));
    return row * 128 + (seg << 5) + (byte & 31);
  }
}

// Direct global->LDS staging (global_load_lds_dwordx4) of one operand tile.
// One wave instruction writes 1 KiB of LDS linearly (wave-uniform base +
// 16*lane), so the XOR swizzle of the image is applied to the per-lane SOURCE
// address: lane l fetches the logical 16-byte chunk that belongs at physical
// position l of the piece. Out-of-range rows/columns are clamped to valid
// addresses (their outputs are never stored); the K tail of the last tile is
// zeroed in LDS after it lands (zero_ktail).
template <bool KC, int R, int NW>
struct Glds {
  static constexpr int BYTES = R * BK * 2;
  static constexpr int P = BYTES / (NW * 1024);  // pieces per wave per tile
  static_assert(BYTES % (NW * 1024) == 0, "tile must split into 1 KiB pieces per wave");
  static constexpr int RPP = KC ? 8 : 1024 / (R * 2);  // tile rows per piece
  static constexpr int CPR = KC ? 8 : R / 8;           // 16-byte chunks per tile row
  // per piece: element offset of this lane's chunk relative to (mn0, k0)
  int row[P];   // KC: mn row within tile; MC: k row within tile
  int col[P];   // KC: k element offset (chunk*8); MC: mn element offset
  __device__ __forceinline__ void init(int wid, int lane) {
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const int j = wid * P + i;
      const int r = j * RPP + lane / CPR;
      const int pc = lane % CPR;
      int c;
      if constexpr (KC) {
        c = (((pc >> 1) ^ ((r >> 1) & 3)) << 1) | (pc & 1);
      } else if constexpr (R >= 128) {
        c = (((pc >> 1) ^ ((r & 3) | (((r >> 3) & 1) << 2))) << 1) | (pc & 1);
      } else {
        c = (((pc >> 1) ^ (((r >> 1) & 1) | (((r >> 3) & 1) << 1))) << 1) | (pc & 1);
      }
      row[i] = r;
      col[i] = c * 8;
    }
  }
  // Issue the tile at (mn0, k0). len = M or N; kend = K bound; ld elements.
  __device__ __forceinline__ void issue(const bf16_t* __restrict__ X, int ld, int len, int kend,
                                        int mn0, int k0, char* lds, int wid) const {
#pragma unroll
    for (int i = 0; i < P; ++i) {
      long long off;
      if constexpr (KC) {
        int mn = mn0 + row[i];
        mn = mn < len ? mn : len - 1;
        int k = k0 + col[i];
        k = k < kend ? k : 0;  // fully past K: any valid chunk (zeroed later)
        off = (long long)mn * ld + k;
      } else {
        int k = k0 + row[i];
        k = k < kend ? k : kend - 1;  // zeroed later
        int mn = mn0 + col[i];
        mn = mn < len ? mn : 0;  // fully past len: never stored
        off = (long long)k * ld + mn;
      }
      __builtin_amdgcn_global_load_lds(
          (const void*)(X + off),
          (__attribute__((address_space(3))) void*)(lds + (wid * P + i) * 1024), 16, 0, 0);
    }
  }
  // Zero the k >= kend part of the tile image at k0 (last, partial tile).
  __device__ __forceinline__ static void zero_ktail(char* lds, int k0, int kend, int tid, int nt) {
    if constexpr (KC) {
      for (int id = tid; id < R * 8; id += nt) {
        const int r = id >> 3, c = id & 7;
        const int kk = k0 + c * 8;
        if (kk + 8 <= kend) continue;
        short8_t* p = reinterpret_cast<short8_t*>(lds + lds_off<KC, R>(r, c * 16));
        short8_t v = *p;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (kk + e >= kend) v[e] = 0;
        *p = v;
      }
    } else {
      for (int id = tid; id < BK * (R / 8); id += nt) {
        const int r = id / (R / 8), c = id % (R / 8);
        if (k0 + r < kend) continue;
        *reinterpret_cast<short8_t*>(lds + lds_off<KC, R>(r, c * 16)) =
            short8_t{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
  }
};

#ifndef TDG_GEMM_PRIO
#define TDG_GEMM_PRIO 1
#endif
__device__ __forceinline__ void prio_hi() {
  if (TDG_GEMM_PRIO) __builtin_amdgcn_s_setprio(1);
}
__device__ __forceinline__ void prio_lo() {
  if (TDG_GEMM_PRIO) __builtin_amdgcn_s_setprio(0);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// Workgroup barrier that does NOT drain in-flight LDS-DMA (no vmcnt(0)).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// MFMA operand fragment for 16 rows/cols starting at `base` within the tile,
// k-step s (32 deep). Lane l holds X(base + (l&15), 32s + 8(l>>4) + j), j<8.
template <bool KC, int R>
__device__ __forceinline__ short8_t frag(const char* lds, int base, int s, int lane) {
  if constexpr (KC) {
    const int row = base + (lane & 15);
    const int byte = (s * 4 + (lane >> 4)) * 16;
    return lds_read_b128_async(lds + lds_off<KC, R>(row, byte));
  } else {
    const int g = lane >> 4, w = lane & 15, q = w >> 2, p = w & 3;
    const int krow = s * 32 + 8 * g + q;
    const int byte = (base + 4 * p) * 2;
    const short4_t lo = lds_read_tr_async(lds + lds_off<KC, R>(krow, byte));
    const short4_t hi = lds_read_tr_async(lds + lds_off<KC, R>(krow + 4, byte));
    return cat4(lo, hi);
  }
}

// LDS instructions one frag<KC>() issues (MN-contiguous: two transposing reads)
template <bool KC>
constexpr int frag_ops() {
  return KC ? 1 : 2;
}

// Fragments read with lds_read_tr_async are not tracked by the compiler:
// make every later use wait for them (see tdg_common.h).
template <int N>
__device__ __forceinline__ void tie_all(short8_t (&f)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) tie(f[i]);
}

}  // namespace tdg
