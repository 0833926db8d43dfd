// Probe for the e4m3 attention kernels: (1) operand lane layout of
// v_mfma_f32_16x16x32_fp8_fp8 against A[row l&15][k 8(l>>4)+j],
// B[k 8(l>>4)+j][col l&15], C/D col l&15 row 4(l>>4)+r (exact integer data);
// (2) what ds_read_b64_tr_b8 returns: each lane passes the address of 8 bytes
// of a [rows][16-byte] LDS image; printed as (lane, byte j) -> source (row, col).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));

__global__ void kmfma(const long* a, const long* b, f32x4* c) {
  int l = threadIdx.x;
  f32x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a[l], b[l], acc, 0, 0, 0);
  c[l] = acc;
}
// LDS image: 16 rows x 16 bytes, byte (r, c) = r * 16 + c. Lane l reads at
// row (l & 15) >> 1, byte 8 * (l & 1) of its 16-lane group's 8-row block
// (group g = l >> 4 -> rows 8 * (g & 1) + ...), the hypothesis for tr_b8.
__global__ void ktr(int* out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[256];
  int l = threadIdx.x;
  for (int i = l; i < 256; i += 64) img[i] = (uint8_t)i;
  __syncthreads();
  typedef __attribute__((address_space(3))) i32x2 lds2;
  const int g = l >> 4, w = l & 15;
  const int row = 8 * (g & 1) + (w >> 1), col = 8 * (w & 1);
  i32x2 t = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds2*)(img + row * 16 + col));
  out[2 * l] = t[0];
  out[2 * l + 1] = t[1];
}
static uint8_t enc(int v) {  // small integers -> OCP e4m3
  static const uint8_t t[9] = {0x00, 0x38, 0x40, 0x44, 0x48, 0x4A, 0x4C, 0x4E, 0x50};
  return v < 0 ? (uint8_t)(0x80 | t[-v]) : t[v];
}
int main() {
  int A[16][32], B[32][16];
  srand(1);
  for (int i = 0; i < 16; ++i) for (int kk = 0; kk < 32; ++kk) A[i][kk] = rand() % 9 - 4;
  for (int kk = 0; kk < 32; ++kk) for (int j = 0; j < 16; ++j) B[kk][j] = rand() % 9 - 4;
  uint8_t ha[64][8], hb[64][8];
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < 8; ++j) {
      ha[l][j] = enc(A[l & 15][8 * (l >> 4) + j]);
      hb[l][j] = enc(B[8 * (l >> 4) + j][l & 15]);
    }
  void *da, *db, *dc, *dt;
  hipMalloc(&da, sizeof ha); hipMalloc(&db, sizeof hb); hipMalloc(&dc, 64 * 16); hipMalloc(&dt, 64 * 8);
  hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice);
  hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(kmfma, dim3(1), dim3(64), 0, 0, (const long*)da, (const long*)db, (f32x4*)dc);
  hipLaunchKernelGGL(ktr, dim3(1), dim3(64), 0, 0, (int*)dt);
  float hc[64][4];
  hipMemcpy(hc, dc, sizeof hc, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * (l >> 4) + r, col = l & 15;
      int ref = 0;
      for (int kk = 0; kk < 32; ++kk) ref += A[row][kk] * B[kk][col];
      if ((int)hc[l][r] != ref) ++bad;
    }
  printf("mfma_f32_16x16x32_fp8_fp8 layout: %s (%d mismatches)\n", bad ? "MISMATCH" : "ok", bad);
  uint8_t ht[64][8];
  hipMemcpy(ht, dt, sizeof ht, hipMemcpyDeviceToHost);
  printf("ds_read_b64_tr_b8: lane -> 8 bytes as (row,col) of the 16x16 image\n");
  for (int l = 0; l < 64; l += 1) {
    printf("lane %2d:", l);
    for (int j = 0; j < 8; ++j) printf(" (%d,%d)", ht[l][j] / 16, ht[l][j] % 16);
    printf("\n");
  }
  return bad ? 1 : 0;
}
