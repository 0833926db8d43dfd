// Probe: semantics of gfx950 ds_read_b64_tr_b8 (transposing 8-byte LDS read
// of 8-bit elements). Hypothesis by analogy with ds_read_b64_tr_b16: per
// group of 16 lanes, lane 2q+p supplies the address of row q (0..7), bytes
// 8p..8p+7 of a 16-byte-wide block; lane i of the group receives column i of
// the 8 rows, row q in byte q. Exact byte data; prints the first group's bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k(uint64_t* out, int mode) {
  __shared__ uint8_t t[64][64];
  const int l = threadIdx.x;
  for (int i = l; i < 64 * 64; i += 64) t[i / 64][i % 64] = (uint8_t)((i / 64) * 16 + (i % 64)) ;
  __syncthreads();
  const int g = l >> 4, w = l & 15;
  int row, col;
  if (mode == 0) { row = 8 * g + (w >> 1); col = 8 * (w & 1); }   // hypothesis
  else { row = l; col = 0; }                                       // plain row addresses
  uint64_t r;
  const uint32_t a = (uint32_t)(uintptr_t)&t[row][col];
  asm volatile("ds_read_b64_tr_b8 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a) : "memory");
  out[l] = r;
}

int main() {
  uint64_t* d;
  hipMalloc(&d, 64 * 8);
  uint64_t h[64];
  int bad = 0;
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, 0);
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) {
    const int g = l >> 4, i = l & 15;
    for (int q = 0; q < 8; ++q) {
      const int row = 8 * g + q, col = i;
      const uint8_t want = (uint8_t)(row * 16 + col);
      const uint8_t got = (uint8_t)(h[l] >> (8 * q));
      if (got != want) ++bad;
    }
  }
  printf("tr_b8 hypothesis (lane 2q+p -> row q bytes 8p..; lane i <- column i): %s (%d bad bytes)\n",
         bad ? "WRONG" : "OK", bad);
  for (int l = 0; l < 16; ++l) {
    printf("lane %2d:", l);
    for (int q = 0; q < 8; ++q) printf(" %3d", (int)(uint8_t)(h[l] >> (8 * q)));
    printf("\n");
  }
  return bad ? 1 : 0;
}
