// Shared argument block for the attention kernels (host <-> device).
#pragma once
#include <stdint.h>

namespace tdg {
struct AttnArgs {
  const uint16_t* q;
  const uint16_t* k;
  const uint16_t* v;
  const uint16_t* o;
  const uint16_t* dout;
  uint16_t* out;   // forward O
  float* lse;    // [B, H, Lq] log2-domain LSE
  float* delta;  // [B, H, Lq]
  uint16_t* dq;
  uint16_t* dk;
  uint16_t* dv;
  const int* kv_len;  // [B] valid key count, or null
  long long q_sb, q_sl, k_sb, k_sl, v_sb, v_sl, o_sb, o_sl;
  long long dq_sb, dq_sl, dk_sb, dk_sl, dv_sb, dv_sl, do_sb, do_sl;
  int q_sh, k_sh, v_sh, o_sh, dq_sh, dk_sh, dv_sh, do_sh;
  int B, H, Lq, Lk;
  float scale;  // softmax scale (1/sqrt(dk))
  int causal;
  // e4m3 forward (attn_fwd_fp8): q / k / v point at e4m3 copies x8 =
  // e4m3(x * s) (strides in elements = bytes), with these per-tensor scales
  const float* sq8;
  const float* sk8;
  const float* sv8;
  // optional e4m3 copy of O (attn_fwd_fp8): out8 = e4m3(bf16(O) * so8[0]),
  // same element strides as out, amax recorded into the slot amax8
  uint8_t* out8;
  const float* so8;
  unsigned* amax8;
  // optional e5m2 copies of dQ / dK / dV (attention backward, hd-64 pipelined
  // kernels; same element strides as dq / dk / dv): x8 = e5m2(bf16(x) * sg8[0]),
  // amax into the slot amaxg8, and the column sums of the bf16-rounded values
  // (the fused projection's bias gradient) as partial rows
  // cs_part[(b * cs_np + block) * cs_ld + cs_{q,k,v} + h * 64 + col].
  // skip_bf16: the bf16 dq / dk / dv are not written (strides still used).
  uint8_t* dq8;
  uint8_t* dk8;
  uint8_t* dv8;
  const float* sg8;
  unsigned* amaxg8;
  float* cs_part;
  int cs_np, cs_ld, cs_q, cs_k, cs_v;
  int skip_bf16;
  // fp8 backward (attn_bwd_f8_kernel): dout points at the e5m2 dO = e5m2(dO *
  // sdo8[0]); dS is quantised e5m2(dS * sds8[0]) with its |max| recorded into
  // the slot amaxds8 (delayed scaling: the next step's sds8). The bf16 dq / dk
  // / dv and the e5m2 dq8 / dk8 / dv8 are each written when non-null.
  const float* sdo8;
  const float* sds8;
  unsigned* amaxds8;
  // fp8 backward, separate e5m2 format of dK / dV (the batched cross K|V
  // gradient of the decoder layers): scale / amax slot of dk8 / dv8 when
  // non-null (else sg8 / amaxg8), and their bias-gradient column sums into
  // cs_part2[b * cs_ld2 + cs_k / cs_v + h * 64 + col] when non-null
  const float* sgkv8;
  unsigned* amaxgkv8;
  float* cs_part2;
  int cs_ld2;
  // workgroup -> (block, head, batch) order: 1 = XCD-grouped by batch (each
  // XCD takes a contiguous run of batch elements, as the projection GEMMs'
  // xcd_remap'd tiles do: their Q/K/V / dO tiles are then in that XCD's L2),
  // 0 = the plain grid order (one head per XCD)
  int xcd;
  // fused backward with the output-projection dgrad (attn_bwd_fused_kernel
  // FDO): dO_bh = dY_b [Lq rows, d] @ Wo[:, 64 h ..] computed in-kernel
  // (dout unused); dY rows b * Lq + r (row stride fdo_ldy), Wo [d][d]
  const uint16_t* fdo_dy;
  const uint16_t* fdo_w;
  int fdo_d, fdo_ldy, fdo_ldw;
};

// Fused self-attention input projection + attention forward
// (attention.hip qkv_attn_fwd_kernel): a's out / lse / kv_len / o strides /
// B / H / Lq / Lk / scale / causal, plus the projection's operands
struct QkvAttnArgs {
  AttnArgs a;
  const uint16_t* x;  // [B * L, d] bf16 (row stride ldx)
  const uint16_t* w;  // [3d, d] bf16: Q rows, then K, then V (row stride ldw)
  const float* bias;  // [3d]
  uint16_t* qkv;      // [B * L, 3d] bf16 projection output (for the backward)
  int d, ldx, ldw, L;
  // cross-attention: w / bias / qkv are the Q projection's ([d, d], [d],
  // [B * L, d]); K / V are a.k / a.v (the batched K|V projection), Lk = a.Lk
  int cross;
};
}  // namespace tdg
