#include <atomic>
#include <chrono>
#include <thread>
#include <vector>
// Python bindings for the gfx950 kernels (module `_C`).
// Every op launches on the current HIP stream of the tensors' device, takes
// caller-allocated outputs (no allocation inside an op: HIP-graph capturable)
// and validates dtypes / shapes / strides on the host before launching, so a
// kernel never sees operands its grid does not assume.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include "tdg_attn.h"

using at::Tensor;
using c10::optional;

extern "C" {
int tdg_gemm(const void* A, const void* B, void* C, const float* bias, const void* aux, int M,
             int N, int K, int lda, int ldb, int ldc, int ldaux, int a_kc, int b_kc, int epi,
             int out_f32, float alpha, float beta, int tile_cfg, int splits, float* ws,
             hipStream_t st);
void tdg_colsum(const void* X, float* out, float* part, int M, int N, int ld, int rows_per_block,
                float beta, hipStream_t st);
int tdg_attn_fwd(const tdg::AttnArgs* a, int hd, hipStream_t st);
int tdg_qkv_attn_fwd(const tdg::QkvAttnArgs* qa, hipStream_t st);
int tdg_attn_bwd_fdo(const tdg::AttnArgs* a, hipStream_t st);
int tdg_attn_bwd(const tdg::AttnArgs* a, int hd, hipStream_t st);
int tdg_attn_probs(const tdg::AttnArgs* a, int hd, float* probs, hipStream_t st);
int tdg_attn_fwd_fp8(const tdg::AttnArgs* a, int hd, hipStream_t st);
int tdg_fp8_set_persist(int on);
int tdg_attn_bwd_f8(const tdg::AttnArgs* a, int hd, hipStream_t st);
int tdg_ln_fwd(const void* x, const void* s, const float* gamma, const float* beta, void* y,
               void* hsave, float* mean, float* rstd, int M, int D, float p, uint64_t seed,
               const long long* ctr, uint64_t site, float eps, void* y8, const float* s8,
               unsigned* amax8, void* kbits, hipStream_t st);
int tdg_ln_bwd(const void* dy, const void* hsave, const float* mean, const float* rstd,
               const float* gamma, void* dh, void* ds, const void* dres, float* dgamma,
               float* dbeta, float* dbias, float* ws, int M, int D, float p, uint64_t seed,
               const long long* ctr, uint64_t site, int accumulate, int skip_reduce,
               int rpb, void* ds8, const float* s8, unsigned* amax8, const void* kbits,
               hipStream_t st);
int tdg_reduce_partials_multi(const float* const* parts, float* const* outs, const int* nparts,
                              int G, int N, float beta, hipStream_t st);
int tdg_embed_fwd(const void* tok, int tok64, const void* table, const float* pe, void* out, int M,
                  int L, int D, float scale, float p, uint64_t seed, const long long* ctr,
                  uint64_t site, void* kbits, hipStream_t st);
int tdg_embed_bwd(const void* tok, int tok64, const void* dout, float* dtable, int M, int D,
                  float scale, float p, uint64_t seed, const long long* ctr, uint64_t site,
                  hipStream_t st);
void tdg_embed_csr_ws(int M, int V, int D, long long* n32, long long* n64);
int tdg_embed_csr_ok(int M, int V);
int tdg_embed_csr_sort(int ntab, const void* const* tok, const int* tok64, const int* M,
                       const int* V, int* const* ws32, long long* stamps, hipStream_t st);
int tdg_embed_csr_apply(const void* dout, const void* kbits, float* dtable, int* ws32,
                        long long* ws64, int M, int D, int V, float scale, float p, uint64_t seed,
                        const long long* ctr, uint64_t site, float beta, hipStream_t st);
int tdg_embed_bwd_det(const void* tok, int tok64, const void* dout, float* dtable, long long* acc,
                      int M, int D, long long V, float scale, float p, uint64_t seed,
                      const long long* ctr, uint64_t site, float beta, hipStream_t st);
int tdg_count_tokens(const void* labels, int lab64, int M, float* out, hipStream_t st);
int tdg_prep_batch(const void* src, int S, const void* tgt, int T1, int B, int lab64, void* tgt_in,
                   void* labels, int* src_len, int* tgt_len, float* ntok, long long* ctr,
                   int* row_lab, unsigned* ticket, int* bad_rows, hipStream_t st);
int tdg_colsum_grouped(const void* const* X, float* const* out, int G, float* part, int M, int N,
                       int ld, int rows_per_block, float beta, hipStream_t st);
int tdg_gemm_grouped(const void* const* A, const void* const* B, void* const* C, int G, int M,
                     int N, int K, int lda, int ldb, int ldc, int a_kc, int b_kc, int out_f32,
                     float alpha, float beta, int tile_cfg, hipStream_t st);
int tdg_gemm_ragged(const void* const* A, const void* const* B, void* const* C, int P,
                    const int* shapes, int K, int a_kc, int b_kc, int out_f32, float alpha,
                    float beta, float* const* bias_out, int impl, hipStream_t st);
int tdg_wgrad_fp8(const void* const* A, const void* const* B, float* const* C,
                  const float* const* sa, const float* const* sb, int P, const int* shapes, int T,
                  float beta, hipStream_t st);
int tdg_fp8_quant_colsum(const void* x, int ld, void* y8, int M, int N, const float* scale,
                         unsigned* amax, float* part, int fmt, hipStream_t st);
int tdg_fp8_quant_t(const void* const* src, void* const* dst, const int* slot, int G, int R, int C,
                    const float* scale, unsigned* amax, hipStream_t st);
int tdg_gemm_fp8(const void* A, const void* B, void* C, const float* bias, const float* sa,
                 const float* sb, void* C8, const float* sc8, unsigned* amax, int M, int N, int K,
                 int lda, int ldb, int ldc, int ldc8, int epi, int cfg, int afmt, int cfmt,
                 const void* aux, int ldaux, float beta, const void* aux8, float* colsum_out,
                 float colsum_beta, float* ws, hipStream_t st);
int tdg_fp8_quant_multi(const void* const* x, void* const* y, const long long* n, const int* slot,
                        int nseg, const float* scale, unsigned* amax, hipStream_t st);
int tdg_fp8_quant(const void* x, void* y8, long long n, const float* scale, unsigned* amax,
                  int fmt, hipStream_t st);
int tdg_fp8_scale_update(float* scale, unsigned* amax, int n, float margin_pow2, float fmax,
                         hipStream_t st);
int tdg_fp8_dequant(const void* x8, float* y, long long n, float inv_scale, hipStream_t st);
int tdg_xent(void* logits, int M, int V, int ldl, const void* labels, int lab64, const float* ntok,
             float workers, float smoothing, float* row_loss, float* row_correct, int write_grad,
             hipStream_t st);
int tdg_xent_stats(const float* row_loss, const float* row_correct, int M, const float* ntok,
                   float workers, float* step_out, float* accum, hipStream_t st);
int tdg_adam(float* p, float* g, float* m, float* v, void* shadow, long long n, long long* step,
             float beta1, float beta2, float eps, float lr_const, float d_model, float warmup,
             float grad_scale, float weight_decay, int sched, int zero_grad, int inc_step,
             hipStream_t st);
int tdg_adam_chunks(float* p, float* g, float* m, float* v, void* shadow, long long n,
                    const void* chunks, int nchunks, long long* step, float beta1, float beta2,
                    float eps, float lr_const, float d_model, float warmup, float grad_scale,
                    float weight_decay, int sched, int zero_grad, int inc_step,
                    const float* scale8, unsigned* amax8, hipStream_t st);
int tdg_to_bf16(const float* p, void* o, long long n, hipStream_t st);
int tdg_transpose_grouped(const void* const* src, void* const* dst, int G, int R, int C,
                          hipStream_t st);
int tdg_signal_create(unsigned long long** host, unsigned long long** dhost,
                      unsigned long long** cnt);
int tdg_signal_emit(unsigned long long* cnt, unsigned long long* dhost, hipStream_t st);
}

namespace {

hipStream_t stream_of(const Tensor& t) {
  TORCH_CHECK(t.is_cuda(), "tdg op: tensor must be on the GPU");
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

void check_bf16(const Tensor& t, const char* n) {
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, n, " must be bfloat16");
  TORCH_CHECK(t.is_cuda(), n, " must be a GPU tensor");
}
void check_f8_fmt(const Tensor& t, int64_t fmt, const char* n);
unsigned* amax_ptr(const optional<Tensor>& t);
void check_f32(const Tensor& t, const char* n) {
  TORCH_CHECK(t.scalar_type() == at::kFloat, n, " must be float32");
  TORCH_CHECK(t.is_cuda(), n, " must be a GPU tensor");
}
void check_contig(const Tensor& t, const char* n) {
  TORCH_CHECK(t.is_contiguous(), n, " must be contiguous");
}
// The extent [0, rows*ld) (minus trailing) must lie inside the storage.
void check_extent(const Tensor& t, long long rows, long long ld, long long cols, const char* n) {
  const long long need = rows > 0 ? (rows - 1) * ld + cols : 0;
  const long long have = (long long)(t.storage().nbytes() / t.element_size()) - t.storage_offset();
  TORCH_CHECK(need <= have, n, ": operand extent ", need, " exceeds storage ", have);
}
void check_err(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, ": unsupported configuration (rc=", rc, ")");
  const hipError_t e = hipGetLastError();
  TORCH_CHECK(e == hipSuccess, what, ": launch failed: ", hipGetErrorString(e));
}

// ---------------------------------------------------------------- GEMM
void gemm(const Tensor& A, const Tensor& B, const Tensor& C, const optional<Tensor>& bias,
          const optional<Tensor>& aux, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb,
          int64_t ldc, int64_t ldaux, bool a_kc, bool b_kc, int64_t epi, double alpha,
          double beta, int64_t tile_cfg, int64_t splits, const optional<Tensor>& ws) {
  check_bf16(A, "A");
  check_bf16(B, "B");
  TORCH_CHECK(C.is_cuda(), "C must be a GPU tensor");
  const bool f32 = C.scalar_type() == at::kFloat;
  TORCH_CHECK(f32 || C.scalar_type() == at::kBFloat16, "C must be f32 or bf16");
  TORCH_CHECK(M > 0 && N > 0 && K > 0, "gemm: empty problem");
  TORCH_CHECK(lda % 8 == 0 && ldb % 8 == 0, "gemm: lda/ldb must be multiples of 8");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(A.data_ptr()) % 16) == 0 &&
                  (reinterpret_cast<uintptr_t>(B.data_ptr()) % 16) == 0,
              "gemm: A/B must be 16-byte aligned");
  // A(m,k): KC -> [M][lda] ; MC -> [K][lda]. The kernel reads whole 16-byte
  // chunks, so the contiguous dimension must be readable up to a multiple of 8.
  auto r8 = [](int64_t v) { return (v + 7) / 8 * 8; };
  if (a_kc) {
    TORCH_CHECK(lda >= r8(K), "gemm: lda < round8(K)");
    check_extent(A, M, lda, r8(K), "A");
  } else {
    TORCH_CHECK(lda >= r8(M), "gemm: lda < round8(M)");
    check_extent(A, K, lda, r8(M), "A");
  }
  if (b_kc) {
    TORCH_CHECK(ldb >= r8(K), "gemm: ldb < round8(K)");
    check_extent(B, N, ldb, r8(K), "B");
  } else {
    TORCH_CHECK(ldb >= r8(N), "gemm: ldb < round8(N)");
    check_extent(B, K, ldb, r8(N), "B");
  }
  TORCH_CHECK(ldc >= N, "gemm: ldc < N");
  check_extent(C, M, ldc, N, "C");
  const float* bptr = nullptr;
  if (epi == 1 || epi == 2) {
    TORCH_CHECK(bias.has_value(), "gemm: bias epilogue needs bias");
    check_f32(*bias, "bias");
    TORCH_CHECK(bias->numel() >= N, "gemm: bias too short");
    bptr = bias->data_ptr<float>();
  }
  const void* xptr = nullptr;
  if (epi == 3) {
    TORCH_CHECK(aux.has_value(), "gemm: DRELU epilogue needs aux");
    check_bf16(*aux, "aux");
    check_extent(*aux, M, ldaux, N, "aux");
    xptr = aux->data_ptr();
  }
  float* wptr = nullptr;
  if (splits > 1) {
    TORCH_CHECK(ws.has_value(), "gemm: split-K needs a workspace");
    check_f32(*ws, "ws");
    TORCH_CHECK(ws->numel() >= splits * M * ldc, "gemm: workspace too small");
    wptr = ws->data_ptr<float>();
  }
  c10::DeviceGuard g(A.device());
  const int rc = tdg_gemm(A.data_ptr(), B.data_ptr(), C.data_ptr(), bptr, xptr, (int)M, (int)N,
                          (int)K, (int)lda, (int)ldb, (int)ldc, (int)ldaux, a_kc, b_kc, (int)epi,
                          f32, (float)alpha, (float)beta, (int)tile_cfg, (int)splits, wptr,
                          stream_of(A));
  check_err(rc, "tdg gemm");
}

// ---------------------------------------------------------------- LayerNorm helpers
// dropout keep-bit bitmap of a [M, D] LayerNorm: uint8 [M, D / 8]
void check_kbits(const optional<Tensor>& kbits, int64_t M, int64_t D) {
  if (!kbits.has_value()) return;
  TORCH_CHECK(kbits->is_cuda() && kbits->scalar_type() == at::kByte && kbits->is_contiguous() &&
                  kbits->numel() == M * D / 8 &&
                  (reinterpret_cast<uintptr_t>(kbits->data_ptr()) % 4) == 0,
              "kbits: uint8 [M, D / 8], 4-byte aligned");
}

void colsum(const Tensor& X, const Tensor& out, const Tensor& part, int64_t M, int64_t N,
            int64_t ld, int64_t rows_per_block, double beta) {
  check_bf16(X, "X");
  check_f32(out, "out");
  check_f32(part, "part");
  check_extent(X, M, ld, N, "X");
  TORCH_CHECK(out.numel() >= N, "colsum: out too short");
  TORCH_CHECK(part.numel() >= ((M + rows_per_block - 1) / rows_per_block) * N,
              "colsum: partial buffer too small");
  c10::DeviceGuard g(X.device());
  tdg_colsum(X.data_ptr(), out.data_ptr<float>(), part.data_ptr<float>(), (int)M, (int)N, (int)ld,
             (int)rows_per_block, (float)beta, stream_of(X));
  check_err(0, "tdg colsum");
}

// ---------------------------------------------------------------- attention
// XCD-grouped workgroup order of the attention kernels (tdg_attn.h xcd):
// TDG_ATTN_XCD=0 restores the plain grid order
static int attn_xcd() {
  static const int v = [] {
    const char* e = getenv("TDG_ATTN_XCD");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return v;
}
// q/k/v/o/do/dq/dk/dv are 4-D [B, L, H, hd] views (any strides, hd contiguous).
void fill_qkv(tdg::AttnArgs& a, const Tensor& q, const Tensor& k, const Tensor& v) {
  for (auto* t : {&q, &k, &v}) {
    check_bf16(*t, "q/k/v");
    TORCH_CHECK(t->dim() == 4 && t->stride(3) == 1, "q/k/v must be [B,L,H,hd] with hd contiguous");
  }
  a.B = (int)q.size(0);
  a.Lq = (int)q.size(1);
  a.H = (int)q.size(2);
  a.Lk = (int)k.size(1);
  TORCH_CHECK(k.size(0) == a.B && v.size(0) == a.B && k.size(2) == a.H && v.size(2) == a.H &&
                  v.size(1) == a.Lk && k.size(3) == q.size(3) && v.size(3) == q.size(3),
              "attention: q/k/v shape mismatch");
  a.q = (const uint16_t*)q.data_ptr();
  a.k = (const uint16_t*)k.data_ptr();
  a.v = (const uint16_t*)v.data_ptr();
  a.q_sb = q.stride(0); a.q_sl = q.stride(1); a.q_sh = (int)q.stride(2);
  a.k_sb = k.stride(0); a.k_sl = k.stride(1); a.k_sh = (int)k.stride(2);
  a.v_sb = v.stride(0); a.v_sl = v.stride(1); a.v_sh = (int)v.stride(2);
  for (auto* t : {&q, &k, &v}) {
    TORCH_CHECK((reinterpret_cast<uintptr_t>(t->data_ptr()) % 16) == 0 &&
                    t->stride(1) % 8 == 0 && t->stride(2) % 8 == 0 && t->stride(0) % 8 == 0,
                "attention: q/k/v rows must be 16-byte aligned");
  }
}
void check_like(const Tensor& t, const tdg::AttnArgs& a, int L, const char* n) {
  check_bf16(t, n);
  TORCH_CHECK(t.dim() == 4 && t.stride(3) == 1 && t.size(0) == a.B && t.size(1) == L &&
                  t.size(2) == a.H,
              n, ": bad shape/stride");
  // (16 bytes: the kernels store whole 16-byte row chunks, attention.hip store_row16)
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) % 16) == 0 && t.stride(0) % 8 == 0 &&
                  t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0,
              n, ": rows must be 16-byte aligned");
}

void attn_fwd(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& out,
              const Tensor& lse, const optional<Tensor>& kv_len, double scale, bool causal) {
  tdg::AttnArgs a{};
  a.xcd = attn_xcd();
  fill_qkv(a, q, k, v);
  check_like(out, a, a.Lq, "out");
  check_f32(lse, "lse");
  check_contig(lse, "lse");
  TORCH_CHECK(lse.numel() == (int64_t)a.B * a.H * a.Lq, "lse must be [B,H,Lq]");
  a.out = (uint16_t*)out.data_ptr();
  a.o_sb = out.stride(0); a.o_sl = out.stride(1); a.o_sh = (int)out.stride(2);
  a.lse = lse.data_ptr<float>();
  if (kv_len.has_value()) {
    TORCH_CHECK(kv_len->scalar_type() == at::kInt && kv_len->numel() == a.B, "kv_len: int32 [B]");
    a.kv_len = kv_len->data_ptr<int>();
  }
  a.scale = (float)scale;
  a.causal = causal;
  c10::DeviceGuard g(q.device());
  check_err(tdg_attn_fwd(&a, (int)q.size(3), stream_of(q)), "tdg attn_fwd");
}

// Fused self-attention input projection + attention forward (L <= 128, hd
// 64): qkv[M, 3d] = x2 @ w^T + bias (written for the backward) and out / lse
// of the attention over it, in one launch. Returns false (nothing launched)
// when the shape is not covered.
bool qkv_attn_fwd(const Tensor& x2, const Tensor& w, const Tensor& bias, const Tensor& qkv,
                  const Tensor& out, const Tensor& lse, const optional<Tensor>& kv_len,
                  double scale, bool causal, int64_t B, int64_t heads,
                  const optional<Tensor>& k, const optional<Tensor>& v) {
  // k / v given: the cross-attention form (w / bias / qkv = the Q
  // projection's; k / v the [B, Lk, H, 64] views of the batched K|V)
  const bool cross = k.has_value();
  TORCH_CHECK(cross == v.has_value(), "qkv_attn_fwd: k and v together");
  const int np = cross ? 1 : 3;
  check_bf16(x2, "x2");
  check_bf16(w, "w");
  check_bf16(qkv, "qkv");
  check_contig(qkv, "qkv");
  check_f32(bias, "bias");
  TORCH_CHECK(x2.dim() == 2 && w.dim() == 2 && x2.stride(1) == 1 && w.stride(1) == 1, "x2 / w rows");
  const int64_t M = x2.size(0), d = x2.size(1);
  TORCH_CHECK(M % B == 0 && w.size(0) == np * d && w.size(1) == d && bias.numel() >= np * d &&
                  qkv.numel() == M * np * d,
              "qkv_attn_fwd: shapes");
  const int64_t L = M / B;
  if (L > 128 || d != 64 * heads || d % 64 || x2.stride(0) % 8 || w.stride(0) % 8) return false;
  for (const Tensor* t : {&x2, &w, &qkv})
    TORCH_CHECK((reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0, "qkv_attn_fwd: 16-byte aligned");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(bias.data_ptr()) & 15) == 0, "bias 16-byte aligned");
  tdg::QkvAttnArgs qa{};
  tdg::AttnArgs& a = qa.a;
  if (cross) {
    for (const Tensor* t : {&*k, &*v}) {
      check_bf16(*t, "k/v");
      TORCH_CHECK(t->dim() == 4 && t->stride(3) == 1 && t->size(0) == B && t->size(2) == heads &&
                      t->size(3) == 64 && t->size(1) == k->size(1),
                  "qkv_attn_fwd: k / v [B, Lk, H, 64], head dim contiguous");
      TORCH_CHECK((reinterpret_cast<uintptr_t>(t->data_ptr()) % 16) == 0 && t->stride(0) % 8 == 0 &&
                      t->stride(1) % 8 == 0 && t->stride(2) % 8 == 0,
                  "qkv_attn_fwd: k / v rows 16-byte aligned");
    }
    a.B = (int)B;
    a.H = (int)heads;
    a.Lk = (int)k->size(1);
    a.k = (const uint16_t*)k->data_ptr();
    a.v = (const uint16_t*)v->data_ptr();
    a.k_sb = k->stride(0); a.k_sl = k->stride(1); a.k_sh = (int)k->stride(2);
    a.v_sb = v->stride(0); a.v_sl = v->stride(1); a.v_sh = (int)v->stride(2);
    if (a.Lk > 128) return false;
  } else {
    a.B = (int)B;
    a.H = (int)heads;
    a.Lk = (int)L;
  }
  a.xcd = 0;
  a.Lq = (int)L;
  check_like(out, a, a.Lq, "out");
  check_f32(lse, "lse");
  check_contig(lse, "lse");
  TORCH_CHECK(lse.numel() == (int64_t)a.B * a.H * a.Lq, "lse must be [B,H,Lq]");
  a.out = (uint16_t*)out.data_ptr();
  a.o_sb = out.stride(0); a.o_sl = out.stride(1); a.o_sh = (int)out.stride(2);
  a.lse = lse.data_ptr<float>();
  if (kv_len.has_value()) {
    TORCH_CHECK(kv_len->scalar_type() == at::kInt && kv_len->numel() == a.B, "kv_len: int32 [B]");
    a.kv_len = kv_len->data_ptr<int>();
  }
  a.scale = (float)scale;
  a.causal = causal;
  qa.x = (const uint16_t*)x2.data_ptr();
  qa.w = (const uint16_t*)w.data_ptr();
  qa.bias = bias.data_ptr<float>();
  qa.qkv = (uint16_t*)qkv.data_ptr();
  qa.d = (int)d;
  qa.ldx = (int)x2.stride(0);
  qa.ldw = (int)w.stride(0);
  qa.L = (int)L;
  qa.cross = cross;
  c10::DeviceGuard g(x2.device());
  const int rc = tdg_qkv_attn_fwd(&qa, stream_of(x2));
  if (rc == -1) return false;
  check_err(rc, "tdg qkv_attn_fwd");
  return true;
}

// e4m3 forward: q8/k8/v8 are [B, L, H, 64] float8_e4m3fn views (hd
// contiguous; K / V rows 16-byte aligned for the LDS-DMA staging), with
// per-tensor scales (x8 = e4m3(x * s), one-element f32 device tensors)
void attn_fwd_fp8(const Tensor& q8, const Tensor& k8, const Tensor& v8, const Tensor& out,
                  const Tensor& lse, const optional<Tensor>& kv_len, const Tensor& sq,
                  const Tensor& sk, const Tensor& sv, double scale, bool causal,
                  const optional<Tensor>& out8, const optional<Tensor>& so8,
                  const optional<Tensor>& amax8) {
  for (auto* t : {&q8, &k8, &v8}) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat8_e4m3fn, "attn_fwd_fp8: e4m3 q/k/v");
    TORCH_CHECK(t->dim() == 4 && t->stride(3) == 1 && t->size(3) == 64,
                "attn_fwd_fp8: [B,L,H,64] with hd contiguous");
  }
  for (auto* t : {&k8, &v8})
    TORCH_CHECK((reinterpret_cast<uintptr_t>(t->data_ptr()) % 16) == 0 && t->stride(0) % 16 == 0 &&
                    t->stride(1) % 16 == 0 && t->stride(2) % 16 == 0,
                "attn_fwd_fp8: K / V rows must be 16-byte aligned");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(q8.data_ptr()) % 8) == 0 && q8.stride(0) % 8 == 0 &&
                  q8.stride(1) % 8 == 0 && q8.stride(2) % 8 == 0,
              "attn_fwd_fp8: Q rows must be 8-byte aligned");
  tdg::AttnArgs a{};
  a.xcd = attn_xcd();
  a.B = (int)q8.size(0);
  a.Lq = (int)q8.size(1);
  a.H = (int)q8.size(2);
  a.Lk = (int)k8.size(1);
  TORCH_CHECK(k8.size(0) == a.B && v8.size(0) == a.B && k8.size(2) == a.H && v8.size(2) == a.H &&
                  v8.size(1) == a.Lk,
              "attn_fwd_fp8: q/k/v shape mismatch");
  a.q = (const uint16_t*)q8.data_ptr();
  a.k = (const uint16_t*)k8.data_ptr();
  a.v = (const uint16_t*)v8.data_ptr();
  a.q_sb = q8.stride(0); a.q_sl = q8.stride(1); a.q_sh = (int)q8.stride(2);
  a.k_sb = k8.stride(0); a.k_sl = k8.stride(1); a.k_sh = (int)k8.stride(2);
  a.v_sb = v8.stride(0); a.v_sl = v8.stride(1); a.v_sh = (int)v8.stride(2);
  check_like(out, a, a.Lq, "out");
  check_f32(lse, "lse");
  check_contig(lse, "lse");
  TORCH_CHECK(lse.numel() == (int64_t)a.B * a.H * a.Lq, "lse must be [B,H,Lq]");
  for (auto* t : {&sq, &sk, &sv}) check_f32(*t, "fp8 scale");
  a.out = (uint16_t*)out.data_ptr();
  a.o_sb = out.stride(0); a.o_sl = out.stride(1); a.o_sh = (int)out.stride(2);
  a.lse = lse.data_ptr<float>();
  if (kv_len.has_value()) {
    TORCH_CHECK(kv_len->scalar_type() == at::kInt && kv_len->numel() == a.B, "kv_len: int32 [B]");
    a.kv_len = kv_len->data_ptr<int>();
  }
  if (out8.has_value()) {
    check_f8_fmt(*out8, 0, "out8");
    TORCH_CHECK(out8->sizes() == out.sizes() && out8->strides() == out.strides() && so8.has_value() &&
                    amax8.has_value(),
                "attn_fwd_fp8: out8 has out's shape / strides, with so8 and amax8");
    check_f32(*so8, "so8");
    a.out8 = (uint8_t*)out8->data_ptr();
    a.so8 = so8->data_ptr<float>();
    a.amax8 = amax_ptr(amax8);
  }
  a.sq8 = sq.data_ptr<float>();
  a.sk8 = sk.data_ptr<float>();
  a.sv8 = sv.data_ptr<float>();
  a.scale = (float)scale;
  a.causal = causal;
  c10::DeviceGuard g(q8.device());
  check_err(tdg_attn_fwd_fp8(&a, 64, stream_of(q8)), "tdg attn_fwd_fp8");
}

static tdg::AttnArgs attn_bwd_args(const Tensor& q, const Tensor& k, const Tensor& v,
                                   const Tensor& o, const Tensor& dout, const Tensor& lse,
                                   const Tensor& delta, const Tensor& dq, const Tensor& dk,
                                   const Tensor& dv, const optional<Tensor>& kv_len, double scale,
                                   bool causal) {
  tdg::AttnArgs a{};
  a.xcd = attn_xcd();
  fill_qkv(a, q, k, v);
  check_like(o, a, a.Lq, "o");
  check_like(dout, a, a.Lq, "dout");
  check_like(dq, a, a.Lq, "dq");
  check_like(dk, a, a.Lk, "dk");
  check_like(dv, a, a.Lk, "dv");
  TORCH_CHECK(dout.stride(1) % 8 == 0 && o.stride(1) % 8 == 0 &&
                  (reinterpret_cast<uintptr_t>(dout.data_ptr()) % 16) == 0 &&
                  (reinterpret_cast<uintptr_t>(o.data_ptr()) % 16) == 0,
              "attn_bwd: o/dout rows must be 16-byte aligned");
  check_f32(lse, "lse");
  check_f32(delta, "delta");
  TORCH_CHECK(lse.numel() == (int64_t)a.B * a.H * a.Lq && delta.numel() == lse.numel(),
              "lse/delta must be [B,H,Lq]");
  a.o = (const uint16_t*)o.data_ptr();
  a.o_sb = o.stride(0); a.o_sl = o.stride(1); a.o_sh = (int)o.stride(2);
  a.dout = (const uint16_t*)dout.data_ptr();
  a.do_sb = dout.stride(0); a.do_sl = dout.stride(1); a.do_sh = (int)dout.stride(2);
  a.dq = (uint16_t*)dq.data_ptr();
  a.dq_sb = dq.stride(0); a.dq_sl = dq.stride(1); a.dq_sh = (int)dq.stride(2);
  a.dk = (uint16_t*)dk.data_ptr();
  a.dk_sb = dk.stride(0); a.dk_sl = dk.stride(1); a.dk_sh = (int)dk.stride(2);
  a.dv = (uint16_t*)dv.data_ptr();
  a.dv_sb = dv.stride(0); a.dv_sl = dv.stride(1); a.dv_sh = (int)dv.stride(2);
  a.lse = lse.data_ptr<float>();
  a.delta = delta.data_ptr<float>();
  if (kv_len.has_value()) {
    TORCH_CHECK(kv_len->scalar_type() == at::kInt && kv_len->numel() == a.B, "kv_len: int32 [B]");
    a.kv_len = kv_len->data_ptr<int>();
  }
  a.scale = (float)scale;
  a.causal = causal;
  return a;
}

void attn_bwd(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o,
              const Tensor& dout, const Tensor& lse, const Tensor& delta, const Tensor& dq,
              const Tensor& dk, const Tensor& dv, const optional<Tensor>& kv_len, double scale,
              bool causal) {
  tdg::AttnArgs a = attn_bwd_args(q, k, v, o, dout, lse, delta, dq, dk, dv, kv_len, scale, causal);
  c10::DeviceGuard g(q.device());
  check_err(tdg_attn_bwd(&a, (int)q.size(3), stream_of(q)), "tdg attn_bwd");
}

// attn_bwd with the output-projection dgrad in-kernel: dO = dy2 @ wo[:, head
// columns] per (batch, head) (dy2 [B * Lq, d], wo [d, d] bf16), never
// written to memory. Returns false (nothing launched) when not covered
// (Lq / Lk > 128, hd != 64).
bool attn_bwd_fdo(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o,
                  const Tensor& dy2, const Tensor& wo, const Tensor& lse, const Tensor& delta,
                  const Tensor& dq, const Tensor& dk, const Tensor& dv,
                  const optional<Tensor>& kv_len, double scale, bool causal) {
  // (o stands in for dout in the checks: the kernel computes dO itself)
  tdg::AttnArgs a = attn_bwd_args(q, k, v, o, o, lse, delta, dq, dk, dv, kv_len, scale, causal);
  a.dout = nullptr;
  check_bf16(dy2, "dy2");
  check_bf16(wo, "wo");
  const int64_t d = wo.size(1);
  TORCH_CHECK(dy2.dim() == 2 && wo.dim() == 2 && dy2.stride(1) == 1 && wo.stride(1) == 1 &&
                  dy2.size(0) == (int64_t)a.B * a.Lq && dy2.size(1) == d && wo.size(0) == d,
              "attn_bwd_fdo: dy2 [B * Lq, d], wo [d, d]");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(dy2.data_ptr()) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(wo.data_ptr()) & 15) == 0,
              "attn_bwd_fdo: 16-byte aligned operands");
  if (q.size(3) != 64 || a.Lq > 128 || a.Lk > 128 || d != 64 * a.H) return false;
  a.fdo_dy = (const uint16_t*)dy2.data_ptr();
  a.fdo_w = (const uint16_t*)wo.data_ptr();
  a.fdo_d = (int)d;
  a.fdo_ldy = (int)dy2.stride(0);
  a.fdo_ldw = (int)wo.stride(0);
  c10::DeviceGuard g(q.device());
  const int rc = tdg_attn_bwd_fdo(&a, stream_of(q));
  if (rc == -1) return false;
  check_err(rc, "tdg attn_bwd_fdo");
  return true;
}

// attn_bwd that also emits e5m2 copies of dQ (and of dK / dV when given),
// their amax, and the bias-gradient column-sum partials (tdg_attn.h); the
// hd-64 pipelined kernels (Lq or Lk > 128) only.
void attn_bwd_g8(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o,
                 const Tensor& dout, const Tensor& lse, const Tensor& delta, const Tensor& dq,
                 const Tensor& dk, const Tensor& dv, const optional<Tensor>& kv_len, double scale,
                 bool causal, const Tensor& dq8, const optional<Tensor>& dk8,
                 const optional<Tensor>& dv8, const Tensor& sg8, const optional<Tensor>& amax8,
                 const optional<Tensor>& cs_part, int64_t cs_np, int64_t cs_ld, int64_t cs_q,
                 int64_t cs_k, int64_t cs_v, bool skip_bf16) {
  tdg::AttnArgs a = attn_bwd_args(q, k, v, o, dout, lse, delta, dq, dk, dv, kv_len, scale, causal);
  TORCH_CHECK(q.size(3) == 64 && (a.Lq > 128 || a.Lk > 128),
              "attn_bwd_g8: the pipelined hd-64 kernels (Lq or Lk > 128) only");
  TORCH_CHECK(dk8.has_value() == dv8.has_value(), "attn_bwd_g8: dk8 and dv8 together");
  // skip_bf16 leaves the bf16 dK / dV unwritten: only legal when their e5m2
  // copies are the output (else the gradients would stay uninitialised)
  TORCH_CHECK(!skip_bf16 || dk8.has_value(), "attn_bwd_g8: skip_bf16 needs dk8/dv8");
  auto same = [](const Tensor& x8, const Tensor& x, const char* n) {
    check_f8_fmt(x8, 1, n);
    TORCH_CHECK(x8.sizes() == x.sizes() && x8.strides() == x.strides(), n,
                " must have the bf16 gradient's shape and strides");
  };
  same(dq8, dq, "dq8");
  a.dq8 = (uint8_t*)dq8.data_ptr();
  if (dk8.has_value()) {
    same(*dk8, dk, "dk8");
    same(*dv8, dv, "dv8");
    a.dk8 = (uint8_t*)dk8->data_ptr();
    a.dv8 = (uint8_t*)dv8->data_ptr();
  }
  check_f32(sg8, "sg8");
  a.sg8 = sg8.data_ptr<float>();
  a.amaxg8 = amax_ptr(amax8);
  TORCH_CHECK(a.amaxg8 != nullptr, "attn_bwd_g8: amax8 slot");
  if (cs_part.has_value()) {
    check_f32(*cs_part, "cs_part");
    const int64_t nqb = (a.Lq + 127) / 128, nkb = (a.Lk + 127) / 128;
    TORCH_CHECK(cs_np == nqb && (!dk8.has_value() || nkb == nqb),
                "attn_bwd_g8: cs_np must equal the query (and key) 128-row block count");
    TORCH_CHECK(cs_part->numel() >= (int64_t)a.B * cs_np * cs_ld &&
                    cs_q + a.H * 64 <= cs_ld && (!dk8.has_value() || (cs_k + a.H * 64 <= cs_ld &&
                                                                       cs_v + a.H * 64 <= cs_ld)),
                "attn_bwd_g8: column-sum partial extent");
    a.cs_part = cs_part->data_ptr<float>();
    a.cs_np = (int)cs_np;
    a.cs_ld = (int)cs_ld;
    a.cs_q = (int)cs_q;
    a.cs_k = (int)cs_k;
    a.cs_v = (int)cs_v;
  }
  a.skip_bf16 = skip_bf16 ? 1 : 0;
  c10::DeviceGuard g(q.device());
  check_err(tdg_attn_bwd(&a, 64, stream_of(q)), "tdg attn_bwd_g8");
}

// fp8 attention backward (attention.hip attn_bwd_f8_kernel): e4m3 q8/k8/v8
// (the forward's operands, scales sq/sk/sv), e5m2 do8 (scale sdo), bf16 o,
// the forward's lse; dS quantised with sds (amax into amaxds). Outputs, each
// written when given: bf16 dq/dk/dv, e5m2 dq8/dk8/dv8 (scale sg8, amax into
// amaxg8), and one row per batch of bias-gradient column sums of the e5m2
// outputs in cs_part[b * cs_ld + cs_{q,k,v} + h * 64 + col] (cs_np = 1).
void attn_bwd_f8(const Tensor& q8, const Tensor& k8, const Tensor& v8, const Tensor& sq,
                 const Tensor& sk, const Tensor& sv, const Tensor& o, const Tensor& do8,
                 const Tensor& sdo, const Tensor& lse, const optional<Tensor>& kv_len, double scale,
                 bool causal, const Tensor& sds, const Tensor& amaxds, const optional<Tensor>& dq,
                 const optional<Tensor>& dk, const optional<Tensor>& dv, const optional<Tensor>& dq8,
                 const optional<Tensor>& dk8, const optional<Tensor>& dv8,
                 const optional<Tensor>& sg8, const optional<Tensor>& amaxg8,
                 const optional<Tensor>& cs_part, int64_t cs_ld, int64_t cs_q, int64_t cs_k,
                 int64_t cs_v, const optional<Tensor>& sgkv8, const optional<Tensor>& amaxgkv8,
                 const optional<Tensor>& cs_part2, int64_t cs_ld2) {
  auto rows16 = [](const Tensor& t, const char* n) {
    TORCH_CHECK(t.dim() == 4 && t.stride(3) == 1 && t.size(3) == 64, n, ": [B,L,H,64] with hd contiguous");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) % 16) == 0 && t.stride(0) % 16 == 0 &&
                    t.stride(1) % 16 == 0 && t.stride(2) % 16 == 0,
                n, ": rows must be 16-byte aligned");
  };
  for (auto* t : {&q8, &k8, &v8}) {
    check_f8_fmt(*t, 0, "attn_bwd_f8 q8/k8/v8");
    rows16(*t, "attn_bwd_f8 q8/k8/v8");
  }
  check_f8_fmt(do8, 1, "attn_bwd_f8 do8");
  rows16(do8, "attn_bwd_f8 do8");
  tdg::AttnArgs a{};
  a.xcd = attn_xcd();
  a.B = (int)q8.size(0);
  a.Lq = (int)q8.size(1);
  a.H = (int)q8.size(2);
  a.Lk = (int)k8.size(1);
  TORCH_CHECK(k8.size(0) == a.B && v8.size(0) == a.B && k8.size(2) == a.H && v8.size(2) == a.H &&
                  v8.size(1) == a.Lk && do8.sizes() == q8.sizes(),
              "attn_bwd_f8: q/k/v/do shape mismatch");
  TORCH_CHECK(a.Lq <= 512 && a.Lk <= 512, "attn_bwd_f8: Lq, Lk <= 512 (all keys in one workgroup)");
  a.q = (const uint16_t*)q8.data_ptr();
  a.k = (const uint16_t*)k8.data_ptr();
  a.v = (const uint16_t*)v8.data_ptr();
  a.q_sb = q8.stride(0); a.q_sl = q8.stride(1); a.q_sh = (int)q8.stride(2);
  a.k_sb = k8.stride(0); a.k_sl = k8.stride(1); a.k_sh = (int)k8.stride(2);
  a.v_sb = v8.stride(0); a.v_sl = v8.stride(1); a.v_sh = (int)v8.stride(2);
  a.dout = (const uint16_t*)do8.data_ptr();
  a.do_sb = do8.stride(0); a.do_sl = do8.stride(1); a.do_sh = (int)do8.stride(2);
  check_like(o, a, a.Lq, "o");
  a.o = (const uint16_t*)o.data_ptr();
  a.o_sb = o.stride(0); a.o_sl = o.stride(1); a.o_sh = (int)o.stride(2);
  check_f32(lse, "lse");
  check_contig(lse, "lse");
  TORCH_CHECK(lse.numel() == (int64_t)a.B * a.H * a.Lq, "lse must be [B,H,Lq]");
  a.lse = lse.data_ptr<float>();
  for (auto* t : {&sq, &sk, &sv, &sdo, &sds}) check_f32(*t, "fp8 scale");
  a.sq8 = sq.data_ptr<float>();
  a.sk8 = sk.data_ptr<float>();
  a.sv8 = sv.data_ptr<float>();
  a.sdo8 = sdo.data_ptr<float>();
  a.sds8 = sds.data_ptr<float>();
  a.amaxds8 = amax_ptr(amaxds);
  if (kv_len.has_value()) {
    TORCH_CHECK(kv_len->scalar_type() == at::kInt && kv_len->numel() == a.B, "kv_len: int32 [B]");
    a.kv_len = kv_len->data_ptr<int>();
  }
  a.scale = (float)scale;
  a.causal = causal;
  // outputs: a bf16 / e5m2 pair shares its strides (one set per gradient)
  auto out = [&](const optional<Tensor>& x, const optional<Tensor>& x8, int L, const char* n,
                 uint16_t*& p, uint8_t*& p8, long long& sb, long long& sl, int& sh) {
    TORCH_CHECK(x.has_value() || x8.has_value(), "attn_bwd_f8: no output for ", n);
    const Tensor& ref = x.has_value() ? *x : *x8;
    if (x.has_value()) {
      check_like(*x, a, L, n);
      p = (uint16_t*)x->data_ptr();
    }
    if (x8.has_value()) {
      check_f8_fmt(*x8, 1, n);
      TORCH_CHECK(x8->dim() == 4 && x8->size(0) == a.B && x8->size(1) == L && x8->size(2) == a.H &&
                      x8->size(3) == 64 && x8->stride(3) == 1 &&
                      (reinterpret_cast<uintptr_t>(x8->data_ptr()) % 4) == 0 &&
                      x8->stride(1) % 4 == 0 && x8->stride(2) % 4 == 0 && x8->stride(0) % 4 == 0,
                  n, ": e5m2 copy [B,L,H,64], 4-byte aligned rows");
      TORCH_CHECK(!x.has_value() || x8->strides() == x->strides(), n, ": bf16 and e5m2 strides differ");
      p8 = (uint8_t*)x8->data_ptr();
    }
    sb = ref.stride(0); sl = ref.stride(1); sh = (int)ref.stride(2);
  };
  out(dq, dq8, a.Lq, "dq", a.dq, a.dq8, a.dq_sb, a.dq_sl, a.dq_sh);
  out(dk, dk8, a.Lk, "dk", a.dk, a.dk8, a.dk_sb, a.dk_sl, a.dk_sh);
  out(dv, dv8, a.Lk, "dv", a.dv, a.dv8, a.dv_sb, a.dv_sl, a.dv_sh);
  TORCH_CHECK(dk8.has_value() == dv8.has_value(), "attn_bwd_f8: dk8 and dv8 together");
  TORCH_CHECK(!dk8.has_value() || dq8.has_value(), "attn_bwd_f8: dk8 / dv8 need dq8");
  if (dq8.has_value()) {
    TORCH_CHECK(sg8.has_value() && amaxg8.has_value(), "attn_bwd_f8: e5m2 outputs need sg8 and amaxg8");
    check_f32(*sg8, "sg8");
    a.sg8 = sg8->data_ptr<float>();
    a.amaxg8 = amax_ptr(amaxg8);
  }
  // dK / dV e5m2 in a slot of their own (scale + amax together)
  TORCH_CHECK(sgkv8.has_value() == amaxgkv8.has_value(), "attn_bwd_f8: sgkv8 with amaxgkv8");
  if (sgkv8.has_value()) {
    TORCH_CHECK(dk8.has_value(), "attn_bwd_f8: sgkv8 needs dk8 / dv8");
    check_f32(*sgkv8, "sgkv8");
    a.sgkv8 = sgkv8->data_ptr<float>();
    a.amaxgkv8 = amax_ptr(amaxgkv8);
  }
  const int64_t ld2 = cs_part2.has_value() ? cs_ld2 : cs_ld;
  if (cs_part2.has_value()) {
    TORCH_CHECK(cs_part.has_value() && dk8.has_value(), "attn_bwd_f8: cs_part2 needs cs_part and dk8");
    check_f32(*cs_part2, "cs_part2");
    TORCH_CHECK(cs_part2->numel() >= (int64_t)a.B * cs_ld2, "attn_bwd_f8: cs_part2 extent");
    a.cs_part2 = cs_part2->data_ptr<float>();
    a.cs_ld2 = (int)cs_ld2;
  }
  if (cs_part.has_value()) {
    TORCH_CHECK(dq8.has_value(), "attn_bwd_f8: column sums come with the e5m2 outputs");
    check_f32(*cs_part, "cs_part");
    TORCH_CHECK(cs_part->numel() >= (int64_t)a.B * cs_ld && cs_q >= 0 && cs_q + a.H * 64 <= cs_ld &&
                    (!dk8.has_value() || (cs_k >= 0 && cs_v >= 0 && cs_k + a.H * 64 <= ld2 &&
                                          cs_v + a.H * 64 <= ld2)),
                "attn_bwd_f8: column-sum partial extent");
    a.cs_part = cs_part->data_ptr<float>();
    a.cs_np = 1;
    a.cs_ld = (int)cs_ld;
    a.cs_q = (int)cs_q;
    a.cs_k = (int)cs_k;
    a.cs_v = (int)cs_v;
  }
  c10::DeviceGuard g(q8.device());
  check_err(tdg_attn_bwd_f8(&a, 64, stream_of(q8)), "tdg attn_bwd_f8");
}

void attn_probs(const Tensor& q, const Tensor& k, const Tensor& probs,
                const optional<Tensor>& kv_len, double scale, bool causal) {
  tdg::AttnArgs a{};
  a.xcd = attn_xcd();
  fill_qkv(a, q, k, k);
  check_f32(probs, "probs");
  check_contig(probs, "probs");
  TORCH_CHECK(probs.numel() == (int64_t)a.B * a.H * a.Lq * a.Lk, "probs must be [B,H,Lq,Lk]");
  if (kv_len.has_value()) {
    TORCH_CHECK(kv_len->scalar_type() == at::kInt && kv_len->numel() == a.B, "kv_len: int32 [B]");
    a.kv_len = kv_len->data_ptr<int>();
  }
  a.scale = (float)scale;
  a.causal = causal;
  c10::DeviceGuard g(q.device());
  check_err(tdg_attn_probs(&a, (int)q.size(3), probs.data_ptr<float>(), stream_of(q)),
            "tdg attn_probs");
}

void check_f8(const Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.element_size() == 1, n, " must be a 1-byte (fp8 e4m3) GPU tensor");
}
// fmt 0: e4m3 (float8_e4m3fn), 1: e5m2 (float8_e5m2); raw uint8 buffers are
// accepted as untyped storage, a float8 dtype of the other format is not
void check_f8_fmt(const Tensor& t, int64_t fmt, const char* n) {
  check_f8(t, n);
  const auto st = t.scalar_type();
  TORCH_CHECK(st == at::kByte || st == (fmt ? at::kFloat8_e5m2 : at::kFloat8_e4m3fn), n,
              " has dtype ", st, " but the format argument says ", fmt ? "e5m2" : "e4m3");
}
unsigned* amax_ptr(const optional<Tensor>& t) {
  if (!t.has_value()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->element_size() == 4 && t->numel() >= 2048,
              "amax must be a 2048-word GPU tensor (one fp8 slot: 64 words, 32 apart)");
  return reinterpret_cast<unsigned*>(t->data_ptr());
}

// ---------------------------------------------------------------- layernorm
const long long* ctr_ptr(const optional<Tensor>& c) {
  if (!c.has_value()) return nullptr;
  TORCH_CHECK(c->scalar_type() == at::kLong && c->numel() >= 1 && c->is_cuda(),
              "rng counter must be an int64 GPU tensor");
  return reinterpret_cast<const long long*>(c->data_ptr<int64_t>());
}

void ln_fwd(const Tensor& x, const optional<Tensor>& s, const Tensor& gamma, const Tensor& beta,
            const Tensor& y, const optional<Tensor>& hsave, const optional<Tensor>& mean,
            const optional<Tensor>& rstd, double p, int64_t seed, const optional<Tensor>& ctr,
            int64_t site, double eps, const optional<Tensor>& y8, const optional<Tensor>& s8,
            const optional<Tensor>& amax8, const optional<Tensor>& kbits) {
  check_bf16(x, "x");
  check_contig(x, "x");
  const int64_t D = x.size(-1), M = x.numel() / D;
  check_bf16(y, "y");
  check_contig(y, "y");
  TORCH_CHECK(y.numel() == x.numel(), "ln: y shape");
  if (s.has_value()) {
    check_bf16(*s, "s");
    check_contig(*s, "s");
    TORCH_CHECK(s->numel() == x.numel(), "ln: s shape");
  }
  check_f32(gamma, "gamma");
  check_f32(beta, "beta");
  TORCH_CHECK(gamma.numel() == D && beta.numel() == D, "ln: gamma/beta shape");
  if (hsave.has_value()) {
    check_bf16(*hsave, "hsave");
    TORCH_CHECK(hsave->numel() == x.numel() && hsave->is_contiguous(), "ln: hsave shape");
  }
  for (auto* t : {&mean, &rstd})
    if (t->has_value()) {
      check_f32(**t, "mean/rstd");
      TORCH_CHECK((*t)->numel() == M, "ln: mean/rstd shape");
    }
  if (y8.has_value()) {
    check_f8_fmt(*y8, 0, "y8");
    TORCH_CHECK(y8->numel() == x.numel() && y8->is_contiguous() && s8.has_value(), "ln: y8");
    check_f32(*s8, "s8");
  }
  if (kbits.has_value()) {
    TORCH_CHECK(kbits->is_cuda() && kbits->scalar_type() == at::kByte && kbits->is_contiguous() &&
                    kbits->numel() == M * D / 8 && D >= 512 && s.has_value(),
                "ln: kbits uint8 [M, D / 8] (D >= 512, dropout on s)");
  }
  c10::DeviceGuard g(x.device());
  const int rc = tdg_ln_fwd(x.data_ptr(), s.has_value() ? s->data_ptr() : nullptr,
                            gamma.data_ptr<float>(), beta.data_ptr<float>(), y.data_ptr(),
                            hsave.has_value() ? hsave->data_ptr() : nullptr,
                            mean.has_value() ? mean->data_ptr<float>() : nullptr,
                            rstd.has_value() ? rstd->data_ptr<float>() : nullptr, (int)M, (int)D,
                            (float)p, (uint64_t)seed, ctr_ptr(ctr), (uint64_t)site, (float)eps,
                            y8 ? y8->data_ptr() : nullptr, s8 ? s8->data_ptr<float>() : nullptr,
                            amax_ptr(amax8), kbits.has_value() ? kbits->data_ptr() : nullptr,
                            stream_of(x));
  check_err(rc, "tdg ln_fwd");
}

// Fused output projection + bias + dropout + residual + LayerNorm:
// y = LN(x + dropout(a @ w^T + bias)). Returns 0, or a negative code when the
// shape is not covered (nothing launched; the caller runs GEMM + ln_fwd).
void ln_bwd(const Tensor& dy, const Tensor& hsave, const Tensor& mean, const Tensor& rstd,
            const Tensor& gamma, const Tensor& dh, const optional<Tensor>& ds,
            const optional<Tensor>& dres, const Tensor& dgamma, const Tensor& dbeta,
            const optional<Tensor>& dbias, const Tensor& ws, double p, int64_t seed,
            const optional<Tensor>& ctr, int64_t site, bool accumulate, bool skip_reduce,
            int64_t rpb, const optional<Tensor>& ds8, const optional<Tensor>& s8,
            const optional<Tensor>& amax8,
            const optional<Tensor>& kbits) {
  check_bf16(dy, "dy");
  check_contig(dy, "dy");
  const int64_t D = dy.size(-1), M = dy.numel() / D;
  for (auto* t : {&hsave, &dh}) {
    check_bf16(*t, "hsave/dh");
    TORCH_CHECK(t->numel() == dy.numel() && t->is_contiguous(), "ln_bwd: shape");
  }
  for (auto* t : {&ds, &dres})
    if (t->has_value()) {
      check_bf16(**t, "ds/dres");
      TORCH_CHECK((*t)->numel() == dy.numel() && (*t)->is_contiguous(), "ln_bwd: ds/dres shape");
    }
  check_f32(mean, "mean");
  check_f32(rstd, "rstd");
  check_f32(gamma, "gamma");
  check_f32(dgamma, "dgamma");
  check_f32(dbeta, "dbeta");
  TORCH_CHECK(mean.numel() == M && rstd.numel() == M, "ln_bwd: mean/rstd shape");
  TORCH_CHECK(gamma.numel() == D && dgamma.numel() == D && dbeta.numel() == D, "ln_bwd: D");
  if (dbias.has_value()) {
    check_f32(*dbias, "dbias");
    TORCH_CHECK(dbias->numel() == D && (ds.has_value() || ds8.has_value()), "ln_bwd: dbias needs ds");
  }
  if (ds8.has_value()) {
    check_f8_fmt(*ds8, 1, "ds8 (e5m2)");
    TORCH_CHECK(ds8->numel() == dy.numel() && ds8->is_contiguous() && s8.has_value(), "ln_bwd: ds8");
    check_f32(*s8, "s8");
  }
  check_f32(ws, "ws");
  TORCH_CHECK(rpb == 16 || rpb == 32 || rpb == 64, "ln_bwd: rows per block 16 / 32 / 64");
  TORCH_CHECK(ws.numel() >= 3 * ((M + rpb - 1) / rpb) * D, "ln_bwd: workspace too small");
  c10::DeviceGuard g(dy.device());
  if (kbits.has_value()) {
    const int64_t D = dy.size(-1), M = dy.numel() / D;
    TORCH_CHECK(kbits->is_cuda() && kbits->scalar_type() == at::kByte && kbits->is_contiguous() &&
                    kbits->numel() == M * D / 8 && D >= 512,
                "ln_bwd: kbits uint8 [M, D / 8] (D >= 512)");
  }
  const int rc = tdg_ln_bwd(
      dy.data_ptr(), hsave.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
      gamma.data_ptr<float>(), dh.data_ptr(), ds.has_value() ? ds->data_ptr() : nullptr,
      dres.has_value() ? dres->data_ptr() : nullptr, dgamma.data_ptr<float>(),
      dbeta.data_ptr<float>(), dbias.has_value() ? dbias->data_ptr<float>() : nullptr,
      ws.data_ptr<float>(), (int)M, (int)D, (float)p, (uint64_t)seed, ctr_ptr(ctr),
      (uint64_t)site, accumulate, skip_reduce, (int)rpb, ds8 ? ds8->data_ptr() : nullptr,
      s8 ? s8->data_ptr<float>() : nullptr, amax_ptr(amax8),
      kbits.has_value() ? kbits->data_ptr() : nullptr, stream_of(dy));
  check_err(rc, "tdg ln_bwd");
}

// Deferred LayerNorm partial folds: outs[g] (=|+=) column sums of parts[g]
// ([nparts[g], N] f32 each), one launch.
void reduce_partials_multi(const std::vector<Tensor>& parts, const std::vector<Tensor>& outs,
                           const std::vector<int64_t>& nparts, int64_t N, double beta) {
  const size_t G = parts.size();
  TORCH_CHECK(G >= 1 && G <= 96 && outs.size() == G && nparts.size() == G,
              "reduce_partials_multi: 1..96 problems");
  std::vector<const float*> pp(G);
  std::vector<float*> oo(G);
  std::vector<int> np(G);
  for (size_t i = 0; i < G; ++i) {
    check_f32(parts[i], "parts");
    check_f32(outs[i], "outs");
    check_contig(parts[i], "parts");
    TORCH_CHECK(outs[i].numel() == N && outs[i].is_contiguous(), "reduce_partials_multi: out");
    TORCH_CHECK(parts[i].numel() >= nparts[i] * N, "reduce_partials_multi: partials too small");
    TORCH_CHECK(parts[i].device() == parts[0].device() && outs[i].device() == parts[0].device(),
                "reduce_partials_multi: one device");
    pp[i] = parts[i].data_ptr<float>();
    oo[i] = outs[i].data_ptr<float>();
    np[i] = (int)nparts[i];
  }
  c10::DeviceGuard g(parts[0].device());
  check_err(tdg_reduce_partials_multi(pp.data(), oo.data(), np.data(), (int)G, (int)N, (float)beta,
                                      stream_of(parts[0])),
            "tdg reduce_partials_multi");
}

// ---------------------------------------------------------------- embedding
void embed_fwd(const Tensor& tok, const Tensor& table, const Tensor& pe, const Tensor& out,
               double scale, double p, int64_t seed, const optional<Tensor>& ctr, int64_t site,
               const optional<Tensor>& kbits) {
  TORCH_CHECK(tok.dim() == 2 && tok.is_contiguous() && tok.is_cuda(), "tok must be [B,L]");
  const bool t64 = tok.scalar_type() == at::kLong;
  TORCH_CHECK(t64 || tok.scalar_type() == at::kInt, "tok must be int32/int64");
  check_bf16(table, "table");
  check_contig(table, "table");
  check_f32(pe, "pe");
  check_contig(pe, "pe");
  check_bf16(out, "out");
  check_contig(out, "out");
  const int64_t D = table.size(1), L = tok.size(1), M = tok.numel();
  TORCH_CHECK(pe.dim() == 2 && pe.size(1) == D && pe.size(0) >= L, "pe table too short");
  TORCH_CHECK(out.numel() == M * D, "out shape");
  check_kbits(kbits, M, D);
  c10::DeviceGuard g(tok.device());
  const int rc = tdg_embed_fwd(tok.data_ptr(), t64, table.data_ptr(), pe.data_ptr<float>(),
                               out.data_ptr(), (int)M, (int)L, (int)D, (float)scale, (float)p,
                               (uint64_t)seed, ctr_ptr(ctr), (uint64_t)site,
                               kbits.has_value() ? kbits->data_ptr() : nullptr, stream_of(tok));
  check_err(rc, "tdg embed_fwd");
}

void embed_bwd(const Tensor& tok, const Tensor& dout, const Tensor& dtable, double scale,
               double p, int64_t seed, const optional<Tensor>& ctr, int64_t site) {
  TORCH_CHECK(tok.is_contiguous() && tok.is_cuda(), "tok");
  const bool t64 = tok.scalar_type() == at::kLong;
  TORCH_CHECK(t64 || tok.scalar_type() == at::kInt, "tok must be int32/int64");
  check_bf16(dout, "dout");
  check_contig(dout, "dout");
  check_f32(dtable, "dtable");
  check_contig(dtable, "dtable");
  const int64_t D = dtable.size(1), M = tok.numel();
  TORCH_CHECK(dout.numel() == M * D, "dout shape");
  c10::DeviceGuard g(tok.device());
  const int rc = tdg_embed_bwd(tok.data_ptr(), t64, dout.data_ptr(), dtable.data_ptr<float>(),
                               (int)M, (int)D, (float)scale, (float)p, (uint64_t)seed,
                               ctr_ptr(ctr), (uint64_t)site, stream_of(tok));
  check_err(rc, "tdg embed_bwd");
}

// Deterministic: acc is an all-zero int64 [V, D] scratch (left all-zero).
void embed_bwd_det(const Tensor& tok, const Tensor& dout, const Tensor& dtable, const Tensor& acc,
                   double scale, double p, int64_t seed, const optional<Tensor>& ctr, int64_t site,
                   bool accumulate) {
  TORCH_CHECK(tok.is_contiguous() && tok.is_cuda(), "tok");
  const bool t64 = tok.scalar_type() == at::kLong;
  TORCH_CHECK(t64 || tok.scalar_type() == at::kInt, "tok must be int32/int64");
  check_bf16(dout, "dout");
  check_contig(dout, "dout");
  check_f32(dtable, "dtable");
  check_contig(dtable, "dtable");
  TORCH_CHECK(acc.scalar_type() == at::kLong && acc.is_cuda() && acc.is_contiguous(), "acc int64");
  TORCH_CHECK(acc.numel() >= dtable.numel(), "acc too small");
  const int64_t D = dtable.size(1), M = tok.numel(), V = dtable.size(0);
  TORCH_CHECK(dout.numel() == M * D, "dout shape");
  c10::DeviceGuard g(tok.device());
  const int rc = tdg_embed_bwd_det(tok.data_ptr(), t64, dout.data_ptr(), dtable.data_ptr<float>(),
                                   reinterpret_cast<long long*>(acc.data_ptr<int64_t>()), (int)M, (int)D, (long long)V,
                                   (float)scale, (float)p, (uint64_t)seed, ctr_ptr(ctr),
                                   (uint64_t)site, accumulate ? 1.f : 0.f, stream_of(tok));
  check_err(rc, "tdg embed_bwd_det");
}

// (int32 words, int64 words) of the CSR embedding backward's workspace
std::vector<int64_t> embed_csr_ws(int64_t M, int64_t V, int64_t D) {
  long long n32 = 0, n64 = 0;
  tdg_embed_csr_ws((int)M, (int)V, (int)D, &n32, &n64);
  return {n32, n64};
}

bool embed_csr_ok(int64_t M, int64_t V) { return tdg_embed_csr_ok((int)M, (int)V) != 0; }

void check_csr_ws(const Tensor& ws32, int64_t M, int64_t V, int64_t D, const char* n) {
  long long n32 = 0, n64 = 0;
  tdg_embed_csr_ws((int)M, (int)V, (int)D, &n32, &n64);
  TORCH_CHECK(ws32.scalar_type() == at::kInt && ws32.is_cuda() && ws32.is_contiguous() &&
                  ws32.numel() >= n32 && (reinterpret_cast<uintptr_t>(ws32.data_ptr()) & 15) == 0,
              n, ": int32 workspace of ", n32, " words (16-byte aligned)");
}

// Token sort of the CSR embedding backward for one or two tables (one
// launch): toks[i] (int32/int64, any shape) over vocabularies V[i] into the
// int32 workspaces ws32[i] (embed_csr_ws words).
void embed_csr_sort(const std::vector<Tensor>& toks, const std::vector<int64_t>& V,
                    const std::vector<Tensor>& ws32, const optional<Tensor>& stamps) {
  const int n = (int)toks.size();
  TORCH_CHECK(n >= 1 && n <= 2 && (int)V.size() == n && (int)ws32.size() == n, "embed_csr_sort: 1-2 tables");
  const void* tp[2];
  int t64[2], M[2], VV[2];
  int* wp[2];
  for (int i = 0; i < n; ++i) {
    const Tensor& t = toks[i];
    TORCH_CHECK(t.is_contiguous() && t.is_cuda(), "tok");
    TORCH_CHECK(t.scalar_type() == at::kLong || t.scalar_type() == at::kInt, "tok must be int32/int64");
    TORCH_CHECK(tdg_embed_csr_ok((int)t.numel(), (int)V[i]), "embed_csr_sort: shape past the sort");
    check_csr_ws(ws32[i], t.numel(), V[i], 128, "embed_csr_sort");
    tp[i] = t.data_ptr();
    t64[i] = t.scalar_type() == at::kLong;
    M[i] = (int)t.numel();
    VV[i] = (int)V[i];
    wp[i] = ws32[i].data_ptr<int>();
  }
  c10::DeviceGuard g(toks[0].device());
  long long* sp = nullptr;
  if (stamps.has_value()) {  // lab: int64 [2 * 8 * 64]
    TORCH_CHECK(stamps->scalar_type() == at::kLong && stamps->is_cuda() && stamps->numel() >= 1024,
                "stamps");
    sp = reinterpret_cast<long long*>(stamps->data_ptr<int64_t>());
  }
  check_err(tdg_embed_csr_sort(n, tp, t64, M, VV, wp, sp, stream_of(toks[0])), "tdg embed_csr_sort");
}

// The embedding gradient from a sorted workspace (deterministic; bitwise the
// fixed-point atomic path's): dtable = beta * dtable + scatter of drop(dout) *
// scale; kbits: the forward's keep bits.
void embed_csr_apply(const Tensor& dout, const Tensor& dtable, const Tensor& ws32,
                     const Tensor& ws64, int64_t M, double scale, double p, int64_t seed,
                     const optional<Tensor>& ctr, int64_t site, bool accumulate,
                     const optional<Tensor>& kbits) {
  check_bf16(dout, "dout");
  check_contig(dout, "dout");
  check_f32(dtable, "dtable");
  check_contig(dtable, "dtable");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(dtable.data_ptr()) & 15) == 0, "dtable 16-byte aligned");
  const int64_t D = dtable.size(1), V = dtable.size(0);
  TORCH_CHECK(dout.numel() == M * D, "dout shape");
  TORCH_CHECK(tdg_embed_csr_ok((int)M, (int)V), "embed_csr_apply: shape past the sort");
  check_kbits(kbits, M, D);
  check_csr_ws(ws32, M, V, D, "embed_csr_apply");
  long long n32 = 0, n64 = 0;
  tdg_embed_csr_ws((int)M, (int)V, (int)D, &n32, &n64);
  TORCH_CHECK(ws64.scalar_type() == at::kLong && ws64.is_cuda() && ws64.is_contiguous() &&
                  ws64.numel() >= n64,
              "embed_csr_apply: int64 workspace of ", n64, " words");
  c10::DeviceGuard g(dout.device());
  check_err(tdg_embed_csr_apply(dout.data_ptr(), kbits.has_value() ? kbits->data_ptr() : nullptr,
                                dtable.data_ptr<float>(), ws32.data_ptr<int>(),
                                reinterpret_cast<long long*>(ws64.data_ptr<int64_t>()), (int)M,
                                (int)D, (int)V, (float)scale, (float)p, (uint64_t)seed,
                                ctr_ptr(ctr), (uint64_t)site, accumulate ? 1.f : 0.f,
                                stream_of(dout)),
            "tdg embed_csr_apply");
}

// ---------------------------------------------------------------- grouped GEMM
void gemm_grouped(const std::vector<Tensor>& As, const std::vector<Tensor>& Bs,
                  const std::vector<Tensor>& Cs, int64_t M, int64_t N, int64_t K, int64_t lda,
                  int64_t ldb, int64_t ldc, bool a_kc, bool b_kc, double alpha, double beta,
                  int64_t tile_cfg) {
  const size_t G = As.size();
  TORCH_CHECK(G >= 1 && G <= 32 && Bs.size() == G && Cs.size() == G, "gemm_grouped: 1..32 problems");
  TORCH_CHECK(M > 0 && N > 0 && K > 0 && lda % 8 == 0 && ldb % 8 == 0 && ldc >= N, "gemm_grouped: shape");
  auto r8 = [](int64_t v) { return (v + 7) / 8 * 8; };
  const bool f32 = Cs[0].scalar_type() == at::kFloat;
  std::vector<const void*> a(G), b(G);
  std::vector<void*> c(G);
  for (size_t i = 0; i < G; ++i) {
    check_bf16(As[i], "A");
    check_bf16(Bs[i], "B");
    TORCH_CHECK(Cs[i].is_cuda() && (Cs[i].scalar_type() == at::kFloat) == f32 &&
                    (f32 || Cs[i].scalar_type() == at::kBFloat16),
                "gemm_grouped: C dtypes must match (f32 or bf16)");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(As[i].data_ptr()) % 16) == 0 &&
                    (reinterpret_cast<uintptr_t>(Bs[i].data_ptr()) % 16) == 0,
                "gemm_grouped: A/B must be 16-byte aligned");
    if (a_kc) check_extent(As[i], M, lda, r8(K), "A");
    else check_extent(As[i], K, lda, r8(M), "A");
    if (b_kc) check_extent(Bs[i], N, ldb, r8(K), "B");
    else check_extent(Bs[i], K, ldb, r8(N), "B");
    check_extent(Cs[i], M, ldc, N, "C");
    a[i] = As[i].data_ptr();
    b[i] = Bs[i].data_ptr();
    c[i] = Cs[i].data_ptr();
  }
  c10::DeviceGuard g(As[0].device());
  const int rc = tdg_gemm_grouped(a.data(), b.data(), c.data(), (int)G, (int)M, (int)N, (int)K,
                                  (int)lda, (int)ldb, (int)ldc, a_kc, b_kc, f32, (float)alpha,
                                  (float)beta, (int)tile_cfg, stream_of(As[0]));
  check_err(rc, "tdg gemm_grouped");
}

// Ragged grouped GEMM (256x256 tiles): problems i = (As[i], Bs[i], Cs[i]) with
// shapes[i] = (M, N, lda, ldb, ldc), sharing K and the operand layouts.
void gemm_ragged(const std::vector<Tensor>& As, const std::vector<Tensor>& Bs,
                 const std::vector<Tensor>& Cs, const std::vector<int64_t>& shapes, int64_t K,
                 bool a_kc, bool b_kc, double alpha, double beta,
                 const std::vector<c10::optional<Tensor>>& bias_out, int64_t impl) {
  const size_t P = As.size();
  TORCH_CHECK(P >= 1 && P <= 64 && Bs.size() == P && Cs.size() == P && shapes.size() == 7 * P,
              "gemm_ragged: 1..64 problems, 7 shape values each (M, N, lda, ldb, ldc, t_first, "
              "t_count)");
  TORCH_CHECK(K > 0 && K % 64 == 0, "gemm_ragged: K must be a multiple of 64");
  auto r8 = [](int64_t v) { return (v + 7) / 8 * 8; };
  const bool f32 = Cs[0].scalar_type() == at::kFloat;
  std::vector<const void*> a(P), b(P);
  std::vector<void*> c(P);
  std::vector<int> sh(7 * P);
  for (size_t i = 0; i < P; ++i) {
    const int64_t M = shapes[7 * i], N = shapes[7 * i + 1], lda = shapes[7 * i + 2],
                  ldb = shapes[7 * i + 3], ldc = shapes[7 * i + 4];
    TORCH_CHECK(M > 0 && N > 0 && lda % 8 == 0 && ldb % 8 == 0 && ldc >= N, "gemm_ragged: shape");
    check_bf16(As[i], "A");
    check_bf16(Bs[i], "B");
    TORCH_CHECK(Cs[i].is_cuda() && (Cs[i].scalar_type() == at::kFloat) == f32 &&
                    (f32 || Cs[i].scalar_type() == at::kBFloat16),
                "gemm_ragged: C dtypes must match (f32 or bf16)");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(As[i].data_ptr()) % 16) == 0 &&
                    (reinterpret_cast<uintptr_t>(Bs[i].data_ptr()) % 16) == 0,
                "gemm_ragged: A/B must be 16-byte aligned");
    if (a_kc) check_extent(As[i], M, lda, r8(K), "A");
    else check_extent(As[i], K, lda, r8(M), "A");
    if (b_kc) check_extent(Bs[i], N, ldb, r8(K), "B");
    else check_extent(Bs[i], K, ldb, r8(N), "B");
    check_extent(Cs[i], M, ldc, N, "C");
    a[i] = As[i].data_ptr();
    b[i] = Bs[i].data_ptr();
    c[i] = Cs[i].data_ptr();
    for (int j = 0; j < 7; ++j) sh[7 * i + j] = (int)shapes[7 * i + j];
  }
  // optional fused bias gradients: bias_out[i][M_i] = alpha * row sums of A_i (+ beta * old)
  TORCH_CHECK(bias_out.empty() || bias_out.size() == P, "gemm_ragged: bias_out must be empty or P long");
  std::vector<float*> bo(P, nullptr);
  bool any_bias = false;
  for (size_t i = 0; i < bias_out.size(); ++i) {
    if (!bias_out[i].has_value()) continue;
    const Tensor& t = *bias_out[i];
    TORCH_CHECK(!a_kc, "gemm_ragged: fused bias sums need an MN-contiguous A");
    check_f32(t, "bias_out");
    TORCH_CHECK(t.is_contiguous() && t.numel() == shapes[7 * i], "gemm_ragged: bias_out[", i,
                "] must hold M floats");
    bo[i] = t.data_ptr<float>();
    any_bias = true;
  }
  c10::DeviceGuard g(As[0].device());
  const int rc = tdg_gemm_ragged(a.data(), b.data(), c.data(), (int)P, sh.data(), (int)K, a_kc,
                                 b_kc, f32, (float)alpha, (float)beta,
                                 any_bias ? bo.data() : nullptr, (int)impl, stream_of(As[0]));
  check_err(rc, "tdg gemm_ragged");
}

void colsum_grouped(const std::vector<Tensor>& Xs, const std::vector<Tensor>& outs,
                    const Tensor& part, int64_t M, int64_t N, int64_t ld, int64_t rows_per_block,
                    double beta) {
  const size_t G = Xs.size();
  TORCH_CHECK(G >= 1 && G <= 32 && outs.size() == G, "colsum_grouped: 1..32 problems");
  check_f32(part, "part");
  const int64_t nparts = (M + rows_per_block - 1) / rows_per_block;
  TORCH_CHECK(part.numel() >= (int64_t)G * nparts * N, "colsum_grouped: partials too small");
  std::vector<const void*> x(G);
  std::vector<float*> o(G);
  for (size_t i = 0; i < G; ++i) {
    check_bf16(Xs[i], "X");
    check_extent(Xs[i], M, ld, N, "X");
    check_f32(outs[i], "out");
    TORCH_CHECK(outs[i].numel() >= N, "colsum_grouped: out too short");
    x[i] = Xs[i].data_ptr();
    o[i] = outs[i].data_ptr<float>();
  }
  c10::DeviceGuard g(Xs[0].device());
  check_err(tdg_colsum_grouped(x.data(), o.data(), (int)G, part.data_ptr<float>(), (int)M, (int)N,
                               (int)ld, (int)rows_per_block, (float)beta, stream_of(Xs[0])),
            "tdg colsum_grouped");
}

// ---------------------------------------------------------------- fp8
void gemm_fp8(const Tensor& A, const Tensor& B, const optional<Tensor>& C, const optional<Tensor>& bias,
              const Tensor& sa, const Tensor& sb, const optional<Tensor>& C8,
              const optional<Tensor>& sc8, const optional<Tensor>& amax, int64_t M, int64_t N,
              int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int64_t ldc8, int64_t epi,
              int64_t cfg, int64_t afmt, int64_t cfmt, const optional<Tensor>& aux, int64_t ldaux,
              double beta, const optional<Tensor>& aux8, const optional<Tensor>& colsum_out,
              double colsum_beta, const optional<Tensor>& ws) {
  check_f8_fmt(A, afmt, "A8");
  check_f8_fmt(B, 0, "B8");
  TORCH_CHECK(C.has_value() || C8.has_value() || colsum_out.has_value(), "gemm_fp8: no output");
  if (C.has_value()) {
    check_bf16(*C, "C");
    TORCH_CHECK(C->numel() >= (M - 1) * ldc + N && ldc % 8 == 0, "gemm_fp8: C extent / ldc");
  } else {
    TORCH_CHECK(beta == 0.0 && !(epi & 16), "gemm_fp8: beta / C = dequant(C8) need C");
  }
  check_f32(sa, "sa");
  check_f32(sb, "sb");
  TORCH_CHECK(K % 128 == 0 && lda % 16 == 0 && ldb % 16 == 0, "gemm_fp8: K % 128, ld % 16");
  // flag 32: B is N-contiguous [K][ldb] (a plain weight as its dgrad's B operand)
  const bool bt = (epi & 32) != 0;
  TORCH_CHECK(A.numel() >= (M - 1) * lda + K &&
                  (bt ? B.numel() >= (K - 1) * ldb + N && ldb >= N && N % 16 == 0
                      : B.numel() >= (N - 1) * ldb + K),
              "gemm_fp8: A/B extent");
  TORCH_CHECK(!bt || ((cfg == 0 || cfg == 10) && afmt == 1 && cfmt == 1),
              "gemm_fp8: N-contiguous B runs the e5m2 backward 128x128 configs (cfg 0, 10) only");
  if (bias.has_value()) check_f32(*bias, "bias");
  const int64_t epi_id = epi & 15;  // (flag 16: C = dequant(C8))
  // (flag 64: the column-sum partials stay in ws, folded by the caller)
  TORCH_CHECK((epi & ~int64_t(127)) == 0 && epi_id <= 3, "gemm_fp8: epilogue id");
  TORCH_CHECK(!(epi & 64) || colsum_out.has_value(), "gemm_fp8: deferred column sums need colsum_out");
  TORCH_CHECK(!(epi & 16) || C8.has_value(), "gemm_fp8: C = dequant(C8) needs C8");
  TORCH_CHECK(epi_id == 0 || epi_id == 3 || bias.has_value(), "gemm_fp8: epilogue needs bias");
  TORCH_CHECK(epi_id != 3 || aux.has_value() != aux8.has_value(),
              "gemm_fp8: the ReLU-backward epilogue needs exactly one of aux (bf16) / aux8 (e4m3)");
  if (aux.has_value()) {
    check_bf16(*aux, "aux");
    TORCH_CHECK(aux->numel() >= (M - 1) * ldaux + N, "gemm_fp8: aux extent");
  }
  if (aux8.has_value()) {
    check_f8_fmt(*aux8, 0, "aux8");
    TORCH_CHECK(aux8->numel() >= (M - 1) * ldaux + N && ldaux % 8 == 0, "gemm_fp8: aux8 extent");
  }
  TORCH_CHECK((afmt == 0 || afmt == 1) && (cfmt == 0 || cfmt == 1), "gemm_fp8: formats are 0 / 1");
  if (C8.has_value()) {
    check_f8_fmt(*C8, cfmt, "C8");
    TORCH_CHECK(sc8.has_value() && C8->numel() >= (M - 1) * ldc8 + N && ldc8 % 8 == 0, "gemm_fp8: C8");
  }
  if (colsum_out.has_value()) {
    check_f32(*colsum_out, "colsum_out");
    TORCH_CHECK(colsum_out->is_contiguous() && colsum_out->numel() == N && (cfg == 0 || cfg == 10),
                "gemm_fp8: colsum_out is [N] f32 (128x128 tile configs 0, 10)");
    TORCH_CHECK(ws.has_value() && ws->scalar_type() == at::kFloat &&
                    ws->numel() >= ((M + 127) / 128) * 2 * N,
                "gemm_fp8: colsum workspace [ceil(M/128)*2, N] f32");
  }
  c10::DeviceGuard g(A.device());
  const int rc = tdg_gemm_fp8(A.data_ptr(), B.data_ptr(), C ? C->data_ptr() : nullptr,
                              bias ? bias->data_ptr<float>() : nullptr, sa.data_ptr<float>(),
                              sb.data_ptr<float>(), C8 ? C8->data_ptr() : nullptr,
                              sc8 ? sc8->data_ptr<float>() : nullptr, amax_ptr(amax), (int)M,
                              (int)N, (int)K, (int)lda, (int)ldb, (int)ldc, (int)ldc8, (int)epi,
                              (int)cfg, (int)afmt, (int)cfmt, aux ? aux->data_ptr() : nullptr,
                              (int)ldaux, (float)beta, aux8 ? aux8->data_ptr() : nullptr,
                              colsum_out ? colsum_out->data_ptr<float>() : nullptr,
                              (float)colsum_beta, ws ? ws->data_ptr<float>() : nullptr,
                              stream_of(A));
  check_err(rc, "tdg gemm_fp8");
}

// fp8 weight gradients: Cs[i][M,N] (f32, =|+= beta) = dequant(As[i][T,M]^T (e5m2)
// @ Bs[i][T,N] (e4m3)), token-major operands, one ragged launch.
void wgrad_fp8(const std::vector<Tensor>& As, const std::vector<Tensor>& Bs,
               const std::vector<Tensor>& Cs, const std::vector<Tensor>& sas,
               const std::vector<Tensor>& sbs, double beta) {
  const size_t P = As.size();
  TORCH_CHECK(P >= 1 && P <= 64 && Bs.size() == P && Cs.size() == P && sas.size() == P &&
                  sbs.size() == P,
              "wgrad_fp8: 1..64 problems");
  const int64_t T = As[0].size(0);
  std::vector<const void*> a(P), b(P);
  std::vector<float*> c(P);
  std::vector<const float*> sa(P), sb(P);
  std::vector<int> sh(5 * P);
  for (size_t i = 0; i < P; ++i) {
    check_f8_fmt(As[i], 1, "A8 (e5m2 gradient)");
    check_f8_fmt(Bs[i], 0, "B8 (e4m3 activation)");
    check_f32(Cs[i], "C");
    check_f32(sas[i], "sa");
    check_f32(sbs[i], "sb");
    TORCH_CHECK(As[i].dim() == 2 && Bs[i].dim() == 2 && Cs[i].dim() == 2, "wgrad_fp8: 2-D tensors");
    TORCH_CHECK(As[i].size(0) == T && Bs[i].size(0) == T, "wgrad_fp8: one token count");
    TORCH_CHECK(As[i].stride(1) == 1 && Bs[i].stride(1) == 1 && Cs[i].stride(1) == 1,
                "wgrad_fp8: unit inner stride");
    const int64_t M = Cs[i].size(0), N = Cs[i].size(1);
    TORCH_CHECK(As[i].size(1) == M && Bs[i].size(1) == N, "wgrad_fp8: shapes");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(As[i].data_ptr()) % 16) == 0 &&
                    (reinterpret_cast<uintptr_t>(Bs[i].data_ptr()) % 16) == 0,
                "wgrad_fp8: operands 16-byte aligned");
    a[i] = As[i].data_ptr();
    b[i] = Bs[i].data_ptr();
    c[i] = Cs[i].data_ptr<float>();
    sa[i] = sas[i].data_ptr<float>();
    sb[i] = sbs[i].data_ptr<float>();
    sh[5 * i] = (int)M;
    sh[5 * i + 1] = (int)N;
    sh[5 * i + 2] = (int)As[i].stride(0);
    sh[5 * i + 3] = (int)Bs[i].stride(0);
    sh[5 * i + 4] = (int)Cs[i].stride(0);
  }
  c10::DeviceGuard g(As[0].device());
  check_err(tdg_wgrad_fp8(a.data(), b.data(), c.data(), sa.data(), sb.data(), (int)P, sh.data(),
                          (int)T, (float)beta, stream_of(As[0])),
            "tdg wgrad_fp8");
}

void fp8_quant(const Tensor& x, const Tensor& y8, const Tensor& scale,
               const optional<Tensor>& amax, int64_t fmt) {
  check_bf16(x, "x");
  check_contig(x, "x");
  check_f8_fmt(y8, fmt, "y8");
  TORCH_CHECK(fmt == 0 || fmt == 1, "fp8_quant: format is 0 / 1");
  TORCH_CHECK(y8.numel() >= x.numel() && y8.is_contiguous(), "fp8_quant: y8");
  check_f32(scale, "scale");
  c10::DeviceGuard g(x.device());
  check_err(tdg_fp8_quant(x.data_ptr(), y8.data_ptr(), x.numel(), scale.data_ptr<float>(),
                          amax_ptr(amax), (int)fmt, stream_of(x)), "tdg fp8_quant");
}

// y8 = fp8(x) (amax recorded) + per-256-row-block column sums of x into part
void fp8_quant_colsum(const Tensor& x, const Tensor& y8, const Tensor& scale, const Tensor& amax,
                      const Tensor& part, int64_t fmt) {
  check_bf16(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "fp8_quant_colsum: x [M, N], unit inner stride");
  const int64_t M = x.size(0), N = x.size(1);
  check_f8_fmt(y8, fmt, "y8");
  TORCH_CHECK(y8.is_contiguous() && y8.numel() == M * N, "fp8_quant_colsum: y8 [M, N]");
  check_f32(scale, "scale");
  check_f32(part, "part");
  TORCH_CHECK(part.numel() >= ((M + 255) / 256) * N, "fp8_quant_colsum: part [ceil(M/256), N]");
  TORCH_CHECK(N % 8 == 0 && x.stride(0) % 8 == 0, "fp8_quant_colsum: N, ld % 8");
  c10::DeviceGuard g(x.device());
  check_err(tdg_fp8_quant_colsum(x.data_ptr(), (int)x.stride(0), y8.data_ptr(), (int)M, (int)N,
                                 scale.data_ptr<float>(), amax_ptr(amax), part.data_ptr<float>(),
                                 (int)fmt, stream_of(x)),
            "tdg fp8_quant_colsum");
}

// dsts[g] [C, R] e4m3 = transposed, quantised srcs[g] [R, C] bf16 (slot scales / amax)
void fp8_quant_t(const std::vector<Tensor>& srcs, const std::vector<Tensor>& dsts,
                 const std::vector<int64_t>& slots, const Tensor& scale, const Tensor& amax) {
  const int n = (int)srcs.size();
  TORCH_CHECK(n >= 1 && n <= 64 && (int)dsts.size() == n && (int)slots.size() == n,
              "fp8_quant_t: 1..64 weights");
  check_f32(scale, "scale");
  TORCH_CHECK(amax.numel() == 2048 * scale.numel(), "fp8_quant_t: amax is [slots, 2048]");
  const int64_t R = srcs[0].size(0), C = srcs[0].size(1);
  std::vector<const void*> sp(n);
  std::vector<void*> dp(n);
  std::vector<int> sl(n);
  for (int i = 0; i < n; ++i) {
    check_bf16(srcs[i], "src");
    check_contig(srcs[i], "src");
    check_f8_fmt(dsts[i], 0, "dst");
    TORCH_CHECK(srcs[i].dim() == 2 && srcs[i].size(0) == R && srcs[i].size(1) == C &&
                    dsts[i].is_contiguous() && dsts[i].numel() == R * C,
                "fp8_quant_t: same-shape [R, C] sources, [C, R] destinations");
    TORCH_CHECK(slots[i] >= 0 && slots[i] < scale.numel(), "fp8_quant_t: slot range");
    sp[i] = srcs[i].data_ptr();
    dp[i] = dsts[i].data_ptr();
    sl[i] = (int)slots[i];
  }
  c10::DeviceGuard g(scale.device());
  check_err(tdg_fp8_quant_t(sp.data(), dp.data(), sl.data(), n, (int)R, (int)C,
                            scale.data_ptr<float>(), amax_ptr(amax), stream_of(scale)),
            "tdg fp8_quant_t");
}

void fp8_quant_multi(const std::vector<Tensor>& xs, const std::vector<Tensor>& ys,
                     const std::vector<int64_t>& slots, const Tensor& scale, const Tensor& amax) {
  const int n = (int)xs.size();
  TORCH_CHECK(n >= 1 && n <= 64 && (int)ys.size() == n && (int)slots.size() == n,
              "fp8_quant_multi: 1..64 tensors, one output and slot each");
  check_f32(scale, "scale");
  TORCH_CHECK(amax.numel() == 2048 * scale.numel(), "fp8_quant_multi: amax is [slots, 2048]");
  std::vector<const void*> xp(n);
  std::vector<void*> yp(n);
  std::vector<long long> ne(n);
  std::vector<int> sl(n);
  for (int i = 0; i < n; ++i) {
    check_bf16(xs[i], "x");
    check_contig(xs[i], "x");
    check_f8_fmt(ys[i], 0, "y8");
    TORCH_CHECK(ys[i].numel() >= xs[i].numel() && ys[i].is_contiguous(), "fp8_quant_multi: y8");
    TORCH_CHECK(xs[i].device() == scale.device() && ys[i].device() == scale.device(),
                "fp8_quant_multi: one device");
    TORCH_CHECK(slots[i] >= 0 && slots[i] < scale.numel(), "fp8_quant_multi: slot range");
    xp[i] = xs[i].data_ptr();
    yp[i] = ys[i].data_ptr();
    ne[i] = xs[i].numel();
    sl[i] = (int)slots[i];
  }
  c10::DeviceGuard g(scale.device());
  check_err(tdg_fp8_quant_multi(xp.data(), yp.data(), ne.data(), sl.data(), n,
                                scale.data_ptr<float>(), amax_ptr(amax), stream_of(scale)),
            "tdg fp8_quant_multi");
}

void fp8_scale_update(const Tensor& scale, const Tensor& amax, double margin_pow2, double fmax) {
  check_f32(scale, "scale");
  TORCH_CHECK(amax.numel() == 2048 * scale.numel(), "fp8_scale_update: amax is [n, 2048]");
  c10::DeviceGuard g(scale.device());
  check_err(tdg_fp8_scale_update(scale.data_ptr<float>(), amax_ptr(amax), (int)scale.numel(),
                                 (float)margin_pow2, (float)fmax, stream_of(scale)), "tdg fp8_scale_update");
}

void fp8_dequant(const Tensor& x8, const Tensor& y, double inv_scale) {
  check_f8_fmt(x8, 0, "x8");
  check_f32(y, "y");
  TORCH_CHECK(y.numel() == x8.numel(), "fp8_dequant: sizes");
  c10::DeviceGuard g(x8.device());
  check_err(tdg_fp8_dequant(x8.data_ptr(), y.data_ptr<float>(), x8.numel(), (float)inv_scale,
                            stream_of(x8)), "tdg fp8_dequant");
}

// ---------------------------------------------------------------- loss
void count_tokens(const Tensor& labels, const Tensor& out) {
  TORCH_CHECK(labels.is_contiguous() && labels.is_cuda(), "labels");
  const bool l64 = labels.scalar_type() == at::kLong;
  check_f32(out, "out");
  c10::DeviceGuard g(labels.device());
  check_err(tdg_count_tokens(labels.data_ptr(), l64, (int)labels.numel(), out.data_ptr<float>(),
                             stream_of(labels)),
            "tdg count_tokens");
}

// tgt_in, labels [B, T] (token dtype), src_len, tgt_len [B] int32, ntok [1] f32,
// ctr (optional int64 [1], += 1)
void prep_batch(const Tensor& src, const Tensor& tgt, const Tensor& tgt_in, const Tensor& labels,
                const Tensor& src_len, const Tensor& tgt_len, const Tensor& ntok,
                const c10::optional<Tensor>& ctr, const Tensor& scratch) {
  TORCH_CHECK(src.is_cuda() && src.dim() == 2 && src.is_contiguous(), "prep_batch: src");
  TORCH_CHECK(tgt.is_cuda() && tgt.dim() == 2 && tgt.is_contiguous() && tgt.size(0) == src.size(0),
              "prep_batch: tgt");
  const auto dt = src.scalar_type();
  TORCH_CHECK((dt == at::kLong || dt == at::kInt) && tgt.scalar_type() == dt,
              "prep_batch: tokens must be int64 or int32 (both)");
  const int64_t B = src.size(0), S = src.size(1), T1 = tgt.size(1);
  TORCH_CHECK(T1 >= 2, "prep_batch: target needs >= 2 tokens");
  for (const Tensor* t : {&tgt_in, &labels})
    TORCH_CHECK(t->is_cuda() && t->is_contiguous() && t->scalar_type() == dt &&
                    t->numel() == B * (T1 - 1), "prep_batch: tgt_in / labels");
  for (const Tensor* t : {&src_len, &tgt_len})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kInt && t->numel() == B, "prep_batch: lengths");
  check_f32(ntok, "ntok");
  // scratch: int32 [B + 2] -- per-row label counts, a zero-initialised
  // ticket, and a sticky count of rows with a PAD before a non-PAD token
  TORCH_CHECK(scratch.is_cuda() && scratch.scalar_type() == at::kInt && scratch.numel() >= B + 2,
              "prep_batch: scratch must be int32 [B + 2], ticket word zero");
  long long* c = nullptr;
  if (ctr.has_value()) {
    TORCH_CHECK(ctr->is_cuda() && ctr->scalar_type() == at::kLong, "prep_batch: ctr");
    c = reinterpret_cast<long long*>(ctr->data_ptr<int64_t>());
  }
  c10::DeviceGuard g(src.device());
  check_err(tdg_prep_batch(src.data_ptr(), (int)S, tgt.data_ptr(), (int)T1, (int)B, dt == at::kLong,
                           tgt_in.data_ptr(), labels.data_ptr(), src_len.data_ptr<int>(),
                           tgt_len.data_ptr<int>(), ntok.data_ptr<float>(), c,
                           scratch.data_ptr<int>(),
                           reinterpret_cast<unsigned*>(scratch.data_ptr<int>() + B),
                           scratch.data_ptr<int>() + B + 1, stream_of(src)),
            "tdg prep_batch");
}

void xent(const Tensor& logits, int64_t V, const Tensor& labels, const Tensor& ntok,
          double workers, double smoothing, const Tensor& row_loss, const Tensor& row_correct,
          bool write_grad) {
  check_bf16(logits, "logits");
  check_contig(logits, "logits");
  const int64_t ldl = logits.size(-1), M = logits.numel() / ldl;
  TORCH_CHECK(ldl % 2 == 0 && V <= ldl && V > 0, "xent: logits row must be even-padded >= V");
  TORCH_CHECK(labels.numel() == M && labels.is_contiguous(), "xent: labels");
  const bool l64 = labels.scalar_type() == at::kLong;
  TORCH_CHECK(l64 || labels.scalar_type() == at::kInt, "labels int32/int64");
  check_f32(ntok, "ntok");
  check_f32(row_loss, "row_loss");
  check_f32(row_correct, "row_correct");
  TORCH_CHECK(row_loss.numel() == M && row_correct.numel() == M, "xent: row outputs");
  c10::DeviceGuard g(logits.device());
  check_err(tdg_xent(logits.data_ptr(), (int)M, (int)V, (int)ldl, labels.data_ptr(), l64,
                     ntok.data_ptr<float>(), (float)workers, (float)smoothing,
                     row_loss.data_ptr<float>(), row_correct.data_ptr<float>(), write_grad,
                     stream_of(logits)),
            "tdg xent");
}

void xent_stats(const Tensor& row_loss, const Tensor& row_correct, const Tensor& ntok,
                double workers, const optional<Tensor>& step_out,
                const optional<Tensor>& accum) {
  check_f32(row_loss, "row_loss");
  check_f32(row_correct, "row_correct");
  if (step_out.has_value()) check_f32(*step_out, "step_out");
  if (accum.has_value()) {
    check_f32(*accum, "accum");
    TORCH_CHECK(accum->numel() >= 4, "accum needs 4 slots");
  }
  c10::DeviceGuard g(row_loss.device());
  check_err(tdg_xent_stats(row_loss.data_ptr<float>(), row_correct.data_ptr<float>(),
                           (int)row_loss.numel(), ntok.data_ptr<float>(), (float)workers,
                           step_out.has_value() ? step_out->data_ptr<float>() : nullptr,
                           accum.has_value() ? accum->data_ptr<float>() : nullptr,
                           stream_of(row_loss)),
            "tdg xent_stats");
}

// ---------------------------------------------------------------- optimizer
void adam(const Tensor& p, const Tensor& g, const Tensor& m, const Tensor& v,
          const optional<Tensor>& shadow, const Tensor& step, double beta1, double beta2,
          double eps, double lr_const, double d_model, double warmup, double grad_scale,
          double weight_decay, int64_t sched, bool zero_grad, bool inc_step) {
  for (auto* t : {&p, &g, &m, &v}) {
    check_f32(*t, "adam buffers");
    check_contig(*t, "adam buffers");
    TORCH_CHECK(t->numel() == p.numel(), "adam: buffer sizes differ");
  }
  TORCH_CHECK(p.numel() % 4 == 0, "adam: flat buffer must be a multiple of 4");
  if (shadow.has_value()) {
    check_bf16(*shadow, "shadow");
    TORCH_CHECK(shadow->numel() == p.numel(), "adam: shadow size");
  }
  TORCH_CHECK(step.scalar_type() == at::kLong && step.is_cuda(), "adam: step int64 GPU");
  c10::DeviceGuard gd(p.device());
  check_err(tdg_adam(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(),
                     v.data_ptr<float>(), shadow.has_value() ? shadow->data_ptr() : nullptr,
                     p.numel(), reinterpret_cast<long long*>(step.data_ptr<int64_t>()), (float)beta1, (float)beta2, (float)eps,
                     (float)lr_const, (float)d_model, (float)warmup, (float)grad_scale,
                     (float)weight_decay, (int)sched, zero_grad, inc_step, stream_of(p)),
            "tdg adam");
}

// Adam over the chunk table [nchunks, 4] int64 (start, n, fp8 slot or -1,
// e4m3 address or 0) built by ops/fp8.py Fp8Weights.adam_chunks: the weights
// with e4m3 copies get them refreshed in the same pass.
void adam_chunks(const Tensor& p, const Tensor& g, const Tensor& m, const Tensor& v,
                 const Tensor& shadow, const Tensor& chunks, const Tensor& step, double beta1,
                 double beta2, double eps, double lr_const, double d_model, double warmup,
                 double grad_scale, double weight_decay, int64_t sched, bool zero_grad,
                 bool inc_step, const Tensor& scale8, const Tensor& amax8) {
  for (auto* t : {&p, &g, &m, &v}) {
    check_f32(*t, "adam buffers");
    check_contig(*t, "adam buffers");
    TORCH_CHECK(t->numel() == p.numel(), "adam: buffer sizes differ");
  }
  check_bf16(shadow, "shadow");
  TORCH_CHECK(shadow.numel() == p.numel() && p.numel() % 4 == 0 && p.numel() < (1LL << 28),
              "adam_chunks: shadow size / flat size");
  TORCH_CHECK(chunks.is_cuda() && chunks.scalar_type() == at::kLong && chunks.dim() == 2 &&
                  chunks.size(1) == 4 && chunks.is_contiguous(),
              "adam_chunks: chunk table [n, 4] int64 on the GPU");
  TORCH_CHECK(step.scalar_type() == at::kLong && step.is_cuda(), "adam: step int64 GPU");
  // The table's CONTENTS (start + n <= numel, n <= 4096, n % 4 == 0, slot <
  // scale8.numel(), live e4m3 addresses) are validated on the host where it
  // is built (ops/fp8.py validate_chunk_table: Fp8Weights.adam_chunks and
  // Adam.apply_range) -- reading it back here would be a device sync inside
  // the captured step. Here: its size against the buffer.
  TORCH_CHECK(chunks.size(0) >= 1 && chunks.size(0) <= (p.numel() + 3) / 4,
              "adam_chunks: chunk count out of range for the flat buffer");
  check_f32(scale8, "scale8");
  TORCH_CHECK(amax8.numel() >= 2048, "adam_chunks: amax slot table");
  c10::DeviceGuard gd(p.device());
  check_err(tdg_adam_chunks(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(),
                            v.data_ptr<float>(), shadow.data_ptr(), p.numel(), chunks.data_ptr(),
                            (int)chunks.size(0), reinterpret_cast<long long*>(step.data_ptr<int64_t>()),
                            (float)beta1, (float)beta2, (float)eps, (float)lr_const, (float)d_model,
                            (float)warmup, (float)grad_scale, (float)weight_decay, (int)sched,
                            zero_grad, inc_step, scale8.data_ptr<float>(),
                            reinterpret_cast<unsigned*>(amax8.data_ptr()), stream_of(p)),
            "tdg adam_chunks");
}

// dsts[g] [C, R] = srcs[g] [R, C]^T (bf16, same shape, <= 64 matrices, one launch)
void transpose_grouped(const std::vector<Tensor>& srcs, const std::vector<Tensor>& dsts) {
  const size_t G = srcs.size();
  TORCH_CHECK(G >= 1 && G <= 64 && dsts.size() == G, "transpose_grouped: 1..64 matrices");
  const int64_t R = srcs[0].size(0), C = srcs[0].size(1);
  TORCH_CHECK(R % 8 == 0 && C % 8 == 0, "transpose_grouped: rows and columns multiples of 8");
  std::vector<const void*> s(G);
  std::vector<void*> d(G);
  for (size_t i = 0; i < G; ++i) {
    check_bf16(srcs[i], "src");
    check_bf16(dsts[i], "dst");
    TORCH_CHECK(srcs[i].dim() == 2 && srcs[i].size(0) == R && srcs[i].size(1) == C &&
                    srcs[i].is_contiguous(), "transpose_grouped: same-shape contiguous sources");
    TORCH_CHECK(dsts[i].dim() == 2 && dsts[i].size(0) == C && dsts[i].size(1) == R &&
                    dsts[i].is_contiguous(), "transpose_grouped: dst must be [C, R]");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(srcs[i].data_ptr()) % 16) == 0 &&
                    (reinterpret_cast<uintptr_t>(dsts[i].data_ptr()) % 16) == 0,
                "transpose_grouped: 16-byte aligned");
    s[i] = srcs[i].data_ptr();
    d[i] = dsts[i].data_ptr();
  }
  c10::DeviceGuard g(srcs[0].device());
  check_err(tdg_transpose_grouped(s.data(), d.data(), (int)G, (int)R, (int)C, stream_of(srcs[0])),
            "tdg transpose_grouped");
}

// diagnostic: nblocks workgroups streaming 1 MiB each of buf, iters times
void to_bf16(const Tensor& p, const Tensor& o) {
  check_f32(p, "p");
  check_bf16(o, "o");
  TORCH_CHECK(p.numel() == o.numel() && p.is_contiguous() && o.is_contiguous(), "to_bf16 shape");
  c10::DeviceGuard g(p.device());
  check_err(tdg_to_bf16(p.data_ptr<float>(), o.data_ptr(), p.numel(), stream_of(p)),
            "tdg to_bf16");
}

// ---- stream-position signal (csrc/kernels/signal.hip, parallel/ddp.py)
// (host word, its device address, device counter) as integers
std::vector<int64_t> signal_create() {
  unsigned long long *h = nullptr, *d = nullptr, *c = nullptr;
  const int rc = tdg_signal_create(&h, &d, &c);
  TORCH_CHECK(rc == 0, "signal_create failed (rc=", rc, ")");
  return {reinterpret_cast<int64_t>(h), reinterpret_cast<int64_t>(d), reinterpret_cast<int64_t>(c)};
}

// launches the signal kernel on the current stream of `device` (captured
// into a graph when the stream is capturing)
void signal_emit(int64_t dhost, int64_t cnt, int64_t device) {
  hipStream_t st = c10::hip::getCurrentHIPStream(static_cast<c10::DeviceIndex>(device)).stream();
  const int rc = tdg_signal_emit(reinterpret_cast<unsigned long long*>(cnt),
                                 reinterpret_cast<unsigned long long*>(dhost), st);
  TORCH_CHECK(rc == 0, "signal_emit: launch failed");
}

// Spins (pause, then yield) until the host word reaches `expected`; false on
// timeout. Runs without the GIL: the comm thread waits here while the main
// thread keeps launching.
bool signal_wait(int64_t host, int64_t expected, double timeout_s) {
  py::gil_scoped_release nogil;
  const volatile unsigned long long* p = reinterpret_cast<const volatile unsigned long long*>(host);
  const unsigned long long want = static_cast<unsigned long long>(expected);
  const auto t0 = std::chrono::steady_clock::now();
  unsigned spins = 0;
  while (*p < want) {
    if (++spins < 4096) {
      __builtin_ia32_pause();
      continue;
    }
    spins = 0;
    std::this_thread::yield();
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
      return false;
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  return true;
}

int64_t signal_read(int64_t host) {
  return static_cast<int64_t>(*reinterpret_cast<const volatile unsigned long long*>(host));
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "gfx950 (MI355X) HIP kernels for tensorflow_distributed_on_gke_amd";
  m.def("gemm", &gemm);
  m.def("signal_create", &signal_create);
  m.def("signal_emit", &signal_emit);
  m.def("signal_wait", &signal_wait);
  m.def("signal_read", &signal_read);
  m.def("qkv_attn_fwd", &qkv_attn_fwd);
  m.def("attn_bwd_fdo", &attn_bwd_fdo);
  m.def("gemm_grouped", &gemm_grouped);
  m.def("gemm_ragged", &gemm_ragged, py::arg("As"), py::arg("Bs"), py::arg("Cs"), py::arg("shapes"),
        py::arg("K"), py::arg("a_kc"), py::arg("b_kc"), py::arg("alpha"), py::arg("beta"),
        py::arg("bias_out") = std::vector<c10::optional<Tensor>>{}, py::arg("impl") = 0);
  m.def("colsum_grouped", &colsum_grouped);
  m.def("gemm_fp8", &gemm_fp8, py::arg("A"), py::arg("B"), py::arg("C"), py::arg("bias"),
        py::arg("sa"), py::arg("sb"), py::arg("C8"), py::arg("sc8"), py::arg("amax"), py::arg("M"),
        py::arg("N"), py::arg("K"), py::arg("lda"), py::arg("ldb"), py::arg("ldc"), py::arg("ldc8"),
        py::arg("epi"), py::arg("cfg"), py::arg("afmt"), py::arg("cfmt"), py::arg("aux"),
        py::arg("ldaux"), py::arg("beta"), py::arg("aux8") = py::none(),
        py::arg("colsum_out") = py::none(), py::arg("colsum_beta") = 0.0, py::arg("ws") = py::none());
  m.def("wgrad_fp8", &wgrad_fp8);
  m.def("fp8_quant_colsum", &fp8_quant_colsum);
  m.def("fp8_quant_t", &fp8_quant_t);
  m.def("fp8_quant", &fp8_quant);
  m.def("fp8_quant_multi", &fp8_quant_multi);
  m.def("fp8_scale_update", &fp8_scale_update);
  m.def("fp8_dequant", &fp8_dequant);
  m.def("colsum", &colsum);
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_fwd_fp8", &attn_fwd_fp8);
  m.def("fp8_set_persist", [](int64_t on) { return (int64_t)tdg_fp8_set_persist((int)on); },
        "persistent 128x128 fp8 GEMM on (1) / off (0) / query (-1); returns the previous state");
  m.def("attn_bwd", &attn_bwd);
  m.def("attn_bwd_g8", &attn_bwd_g8);
  m.def("attn_bwd_f8", &attn_bwd_f8);
  m.def("attn_probs", &attn_probs);
  m.def("ln_fwd", &ln_fwd);
  m.def("ln_bwd", &ln_bwd);
  m.def("embed_fwd", &embed_fwd);
  m.def("embed_bwd", &embed_bwd);
  m.def("embed_bwd_det", &embed_bwd_det);
  m.def("embed_csr_ws", &embed_csr_ws);
  m.def("embed_csr_ok", &embed_csr_ok);
  m.def("embed_csr_sort", &embed_csr_sort);
  m.def("embed_csr_apply", &embed_csr_apply);
  m.def("count_tokens", &count_tokens);
  m.def("prep_batch", &prep_batch);
  m.def("transpose_grouped", &transpose_grouped);
  m.def("xent", &xent);
  m.def("xent_stats", &xent_stats);
  m.def("adam", &adam);
  m.def("adam_chunks", &adam_chunks);
  m.def("reduce_partials_multi", &reduce_partials_multi);
  m.def("to_bf16", &to_bf16);
  m.attr("ARCH") = "gfx950";
}
