// Probe: operand lane layout of v_mfma_scale_f32_16x16x128_f8f6f4 (fp8 e4m3,
// unit scales) against the hypothesis A[row l&15][k 32(l>>4)+j],
// B[k 32(l>>4)+j][col l&15], C/D col l&15 row 4(l>>4)+r. Exact integer data.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k(const i32x8* a, const i32x8* b, f32x4* c) {
  int l = threadIdx.x;
  f32x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, 0, 0, 0, 127, 0, 127);
  c[l] = acc;
}
static uint8_t enc(int v) {  // small integers -> OCP e4m3
  static const uint8_t t[9] = {0x00, 0x38, 0x40, 0x44, 0x48, 0x4A, 0x4C, 0x4E, 0x50};
  return v < 0 ? (uint8_t)(0x80 | t[-v]) : t[v];
}
int main() {
  int A[16][128], B[128][16];
  srand(1);
  for (int i = 0; i < 16; ++i) for (int kk = 0; kk < 128; ++kk) A[i][kk] = rand() % 9 - 4;
  for (int kk = 0; kk < 128; ++kk) for (int j = 0; j < 16; ++j) B[kk][j] = rand() % 9 - 4;
  uint8_t ha[64][32], hb[64][32];
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < 32; ++j) {
      ha[l][j] = enc(A[l & 15][32 * (l >> 4) + j]);
      hb[l][j] = enc(B[32 * (l >> 4) + j][l & 15]);
    }
  void *da, *db, *dc;
  hipMalloc(&da, sizeof ha); hipMalloc(&db, sizeof hb); hipMalloc(&dc, 64 * 16);
  hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
  hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, (const i32x8*)da, (const i32x8*)db, (f32x4*)dc);
  float hc[64][4];
  hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      int row = 4 * (l >> 4) + r, col = l & 15;
      long ref = 0;
      for (int kk = 0; kk < 128; ++kk) ref += (long)A[row][kk] * B[kk][col];
      if ((long)hc[l][r] != ref) ++bad;
    }
  printf("fp8 16x16x128 layout hypothesis: %s (%d mismatches of 1024)\n", bad ? "WRONG" : "OK", bad);
  return bad ? 1 : 0;
}
