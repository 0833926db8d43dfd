"""Thin, shape-checked launch wrappers over the gfx950 HIP kernels (`_C`).

All GPU compute of the model goes through here. Outputs are allocated from
the PyTorch caching allocator (stream-ordered, graph-capture safe); scratch
buffers (split-K slabs, column-sum partials) come from a grow-only per-device
workspace so a captured HIP graph sees stable addresses.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Tuple

import torch

from tensorflow_distributed_on_gke_amd.ops._ext import C

EPI_NONE, EPI_BIAS, EPI_BIAS_RELU, EPI_DRELU = 0, 1, 2, 3
NUM_CU = 256

# ------------------------------------------------------------------ workspace
_WS: Dict[Tuple[int, int, str], torch.Tensor] = {}
_WS_RETIRED: List[torch.Tensor] = []


def workspace(name: str, numel: int, device, dtype=torch.float32, zero: bool = False) -> torch.Tensor:
    """Named scratch buffer, one per (device, stream): a buffer is only ever
    used by kernels of one stream, so growing it (which frees the old one to
    the caching allocator, in that stream's pool) cannot race a kernel of
    another stream."""
    dev = torch.device(device)
    sid = torch.cuda.current_stream(dev).stream_id if dev.type == "cuda" else 0
    key = (dev.index or 0, sid, name)
    t = _WS.get(key)
    if t is None or t.numel() < numel or t.dtype != dtype:
        if t is not None:
            # a captured HIP graph may still address the smaller buffer (the
            # step cache keeps one graph per batch shape, train/step.py):
            # never hand its memory to another tensor
            _WS_RETIRED.append(t)
        t = (torch.zeros if zero else torch.empty)(max(numel, 1), dtype=dtype, device=dev)
        _WS[key] = t
    return t


def reset_workspace() -> None:
    _WS.clear()
    _WS_RETIRED.clear()


# ------------------------------------------------------------------ GEMM
# tile configs (see csrc/kernels/gemm.hip): 0=128x128, 1=128x64, 2=64x128, 3=64x64
_TILES = {0: (128, 128), 1: (128, 64), 2: (64, 128), 3: (64, 64), 4: (128, 128), 5: (256, 128),
          6: (128, 256), 7: (64, 128), 8: (64, 64), 9: (256, 128), 10: (128, 256), 11: (128, 128),
          12: (256, 256), 13: (128, 128), 14: (128, 128),
          20: (256, 256), 21: (256, 128), 22: (128, 256)}
_CFG_OVERRIDE: Dict[Tuple[int, int, int, bool, bool], Tuple[int, int]] = {}


def set_gemm_config(M: int, N: int, K: int, a_kc: bool, b_kc: bool, cfg: int, splits: int) -> None:
    _CFG_OVERRIDE[(M, N, K, a_kc, b_kc)] = (cfg, splits)


def choose_gemm(M: int, N: int, K: int, a_kc: bool = True, b_kc: bool = True) -> Tuple[int, int]:
    """Tile config (and split-K) for a shape with no tuned entry -- no timed
    search at run time. From the in-tree sweep on MI355X
    (scripts/gemm_vs_blas.py, profiles/gemm/r3_tile_sweep_*.txt): 256x256
    tiles once they fill the chip (>= 192 tiles, K % 64 == 0); for the
    d_model-wide dgrads (N = 1024) 128x256 tiles, 8 waves; otherwise 128x128
    tiles, 8 waves, 3-4 stages. Weight gradients (K = tokens, small output,
    normally the ragged launch) split K to fill 256 CUs."""
    o = _CFG_OVERRIDE.get((M, N, K, a_kc, b_kc))
    if o is not None:
        return o
    if not a_kc and not b_kc:  # weight gradient: split K (= tokens)
        t128 = math.ceil(M / 128) * math.ceil(N / 128)
        splits = 1
        while t128 * splits < NUM_CU and K // (splits * 2) >= 512:
            splits *= 2
        return 0, splits
    if K % 64 == 0 and math.ceil(M / 256) * math.ceil(N / 256) >= 192:
        return 12, 1
    if a_kc and not b_kc and N >= 1024 and math.ceil(M / 128) * math.ceil(N / 256) >= NUM_CU:
        return 6, 1
    return (13, 1) if not b_kc else (4, 1)


_TUNED: Dict[tuple, Tuple[int, int]] = {}
# Timed tile search for shapes missing from the tuned table: a tool
# (TDG_GEMM_AUTOTUNE=1, scripts/tune_in_model.py), never on in training runs,
# where results must not depend on the timing noise of the box
AUTOTUNE = os.environ.get("TDG_GEMM_AUTOTUNE", "0") == "1"
_CANDIDATES = [(0, 1), (4, 1), (5, 1), (6, 1), (9, 1), (10, 1), (12, 1), (13, 1), (14, 1),
               (20, 1), (21, 1), (22, 1)]


def _autotune(key, run) -> Tuple[int, int]:
    """Time the candidate tile configs once for this problem (HIP events on
    the current stream, two interleaved rounds, min) and keep the fastest."""
    M, N, K, a_kc, b_kc = key[:5]
    cands = list(_CANDIDATES)
    if not a_kc and not b_kc:
        cands = [(c, s) for c in (0, 7, 8) for s in (1, 2, 4, 8) if K // s >= 256] + [(12, 1)]
    times: Dict[Tuple[int, int], float] = {}
    for rnd in range(2):  # two interleaved rounds, min per config: robust to clock noise
        for cfg in cands:
            if rnd and cfg not in times:
                continue
            try:
                run(cfg)  # warm-up (also surfaces unsupported configs)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record()
                for _ in range(5):
                    run(cfg)
                ev[1].record()
                ev[1].synchronize()
                t = ev[0].elapsed_time(ev[1])
            except RuntimeError:
                continue
            times[cfg] = min(t, times.get(cfg, float("inf")))
    return min(times, key=times.get)


def _key_str(k: tuple) -> str:
    M, N, K, a_kc, b_kc, epi, dt, ld8, beta = k
    return f"{M},{N},{K},{int(a_kc)},{int(b_kc)},{epi},{str(dt).replace('torch.', '')},{int(ld8)},{int(beta)}"


def save_tuned(path: str) -> None:
    """Persist the autotuned GEMM choices (JSON) so later runs are
    deterministic and skip tuning."""
    import json

    with open(path, "w") as f:
        json.dump({_key_str(k): list(v[0]) for k, v in sorted(_TUNED.items(), key=lambda kv: str(kv[0]))},
                  f, indent=0)


def load_tuned(path: str) -> int:
    import json

    if not os.path.exists(path):
        return 0
    with open(path) as f:
        data = json.load(f)
    for ks, v in data.items():
        M, N, K, a, b, epi, dt, ld8, beta = ks.split(",")
        key = (int(M), int(N), int(K), bool(int(a)), bool(int(b)), int(epi), getattr(torch, dt),
               bool(int(ld8)), bool(int(beta)))
        cfg = (int(v[0]), int(v[1]))
        _TUNED[key] = (cfg, cfg)
    return len(data)


TUNED_FILE = os.environ.get("TDG_GEMM_TUNED_FILE") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "gemm_tuned_gfx950.json")
load_tuned(TUNED_FILE)


def _tok_bucket(v: int) -> int:
    return -(-v // 1024) * 1024


def gemm(A, B, Cout, M, N, K, lda, ldb, ldc, a_kc, b_kc, epi=EPI_NONE, bias=None, aux=None,
         ldaux=0, alpha=1.0, beta=0.0, cfg: Optional[Tuple[int, int]] = None) -> torch.Tensor:
    """Every GEMM of the model: the in-tree MFMA kernels (csrc/kernels/gemm.hip)
    with the tile config from the tuned table, else the heuristic."""

    def run(c, out=Cout):
        tile, splits = c
        ws = workspace("splitk", splits * M * ldc, A.device) if splits > 1 else None
        C().gemm(A, B, out, bias, aux, M, N, K, lda, ldb, ldc, ldaux, a_kc, b_kc, epi, alpha,
                 beta, tile, splits, ws)

    if cfg is None:
        # token-count dimensions (M of forward / dgrad, K of wgrad) are bucketed
        # to multiples of 1024 for the tuning key, so variable-length text
        # batches reuse a handful of tunings instead of re-tuning every length
        Mk, Kk = (M, _tok_bucket(K)) if (not a_kc and not b_kc) else (_tok_bucket(M), K)
        key = (Mk, N, Kk, a_kc, b_kc, epi, Cout.dtype, ldc % 8 == 0, beta != 0.0)
        ent = _TUNED.get(key)
        if ent is None:
            o = _CFG_OVERRIDE.get((M, N, K, a_kc, b_kc))
            if o is not None:
                ent = (o, o)
        if ent is None and AUTOTUNE and A.is_cuda and not torch.cuda.is_current_stream_capturing():
            if beta != 0.0:
                # accumulate into C: tune on a scratch copy so C is untouched
                scratch = workspace("tune_c", Cout.numel(), A.device, Cout.dtype)[: Cout.numel()]
                scratch = scratch.view_as(Cout)
                best = _autotune(key, lambda c: run(c, scratch))
            else:
                best = _autotune(key, run)
            ent = (best, best)
            _TUNED[key] = ent
        if ent is None:
            cfg = choose_gemm(M, N, K, a_kc, b_kc)
        else:
            cfg = ent[0]
    run(cfg)
    return Cout


def tuned_table() -> Dict[str, str]:
    return {f"{k[0]}x{k[1]}x{k[2]} a_kc={k[3]} b_kc={k[4]} epi={k[5]}": f"cfg{v[0]} split{v[1]}"
            for k, v in _TUNED.items()}


def linear_fwd(x2: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], relu: bool = False,
               out: Optional[torch.Tensor] = None, ldc: Optional[int] = None) -> torch.Tensor:
    """y[M,N] = x[M,K] @ w[N,K]^T + bias (bf16 out)."""
    M, K = x2.shape
    N = w.shape[0]
    ldc = ldc or N
    if out is None:
        out = torch.empty(M, ldc, dtype=torch.bfloat16, device=x2.device)
    epi = EPI_BIAS_RELU if relu else (EPI_BIAS if bias is not None else EPI_NONE)
    return gemm(x2, w, out, M, N, K, x2.stride(0), w.stride(0), ldc, True, True, epi, bias=bias)


def linear_dgrad(dy2: torch.Tensor, w: torch.Tensor, N: int, relu_aux: Optional[torch.Tensor] = None,
                 out: Optional[torch.Tensor] = None, beta: float = 0.0) -> torch.Tensor:
    """dx[M,K] = dy[M,N] @ w[N,K] (optionally * (relu_aux > 0))."""
    M = dy2.shape[0]
    K = w.shape[1]
    if out is None:
        out = torch.empty(M, K, dtype=torch.bfloat16, device=dy2.device)
    epi = EPI_DRELU if relu_aux is not None else EPI_NONE
    return gemm(dy2, w, out, M, K, N, dy2.stride(0), w.stride(0), out.stride(0), True, False, epi,
                aux=relu_aux, ldaux=(relu_aux.stride(0) if relu_aux is not None else 0), beta=beta)


def transpose_grouped(srcs, dsts) -> None:
    """dsts[g] = srcs[g].T for same-shape bf16 matrices, one launch per 64."""
    for c0 in range(0, len(srcs), 64):
        C().transpose_grouped(list(srcs[c0:c0 + 64]), list(dsts[c0:c0 + 64]))


def linear_dgrad_t(dy2: torch.Tensor, w_t: torch.Tensor, relu_aux: Optional[torch.Tensor] = None,
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dx[M,N] = dy[M,K] @ w[K,N] computed against the weight's transposed copy
    w_t [N, K] (K-contiguous): the forward (NT) operand layout, whose kernels
    are faster than the N-contiguous dgrad ones; optional ReLU-backward mask."""
    M, K = dy2.shape
    N = w_t.shape[0]
    if out is None:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dy2.device)
    epi = EPI_DRELU if relu_aux is not None else EPI_NONE
    return gemm(dy2, w_t, out, M, N, K, dy2.stride(0), w_t.stride(0), out.stride(0), True, True, epi,
                aux=relu_aux, ldaux=(relu_aux.stride(0) if relu_aux is not None else 0))


def linear_wgrad(dy2: torch.Tensor, x2: torch.Tensor, N: int, dw: torch.Tensor,
                 beta: float = 0.0) -> torch.Tensor:
    """dw[N,K] (f32) (+)= dy[M,N]^T @ x[M,K]."""
    M, K = x2.shape
    return gemm(dy2, x2, dw, N, K, M, dy2.stride(0), x2.stride(0), dw.stride(0), False, False,
                EPI_NONE, beta=beta)


_GROUP_TUNED: Dict[tuple, int] = {}
_GROUP_CANDS = (0, 4, 5, 6, 7, 8, 2, 12)


def wgrad_grouped(dys, xs, dws, beta: float = 0.0) -> None:
    """dws[i][N,K] (f32) (+)= dys[i][M,N]^T @ xs[i][M,K] for up to 32 same-shape
    problems in ONE launch (blockIdx.y = problem): whole-K tiles over the
    whole chip, no split-K slabs."""
    M, K = xs[0].shape
    N = dws[0].shape[0]
    lda, ldb, ldc = dys[0].stride(0), xs[0].stride(0), dws[0].stride(0)

    def run(c):
        C().gemm_grouped(dys, xs, dws, N, K, M, lda, ldb, ldc, False, False, 1.0, beta, c)

    key = (M, N, K, len(dys), lda, ldb, beta != 0.0)
    cfg = _GROUP_TUNED.get(key)
    if cfg is None:
        if AUTOTUNE and not torch.cuda.is_current_stream_capturing():
            scratch = [workspace(f"gw{i}", d.numel(), d.device)[: d.numel()].view_as(d)
                       for i, d in enumerate(dws)]

            def trial(c):
                C().gemm_grouped(dys, xs, scratch, N, K, M, lda, ldb, ldc, False, False, 1.0, 0.0, c)

            times: Dict[int, float] = {}
            for _ in range(2):
                for c in _GROUP_CANDS:
                    try:
                        trial(c)
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        for _ in range(3):
                            trial(c)
                        e1.record()
                        e1.synchronize()
                        times[c] = min(times.get(c, float("inf")), e0.elapsed_time(e1))
                    except RuntimeError:
                        continue
            if not times:
                run(0)  # surfaces the binding's error for this problem
            cfg = min(times, key=times.get)
        else:
            cfg = 0
        _GROUP_TUNED[key] = cfg
    run(cfg)


RAGGED_MAX_PROBLEMS, RAGGED_MAX_SHAPES = 64, 8
# main loop of the ragged weight-gradient launch: 0 = lock-step 256x256 tiles
# at 2 waves per SIMD (gemm256_kernel), 1 / 2 = the pipelined loop at one wave
# per SIMD with a 4 / 5-slot LDS ring (wgrad_pipe_kernel)
WGRAD_IMPL = int(os.environ.get("TDG_WGRAD_IMPL", "0") or 0)


def wgrad_ragged(dys, xs, dws, beta: float = 0.0, biases=None, ranges=None) -> None:
    """dws[i][N_i,K_i] (f32) (+)= dys[i][M,N_i]^T @ xs[i][M,K_i] for up to 64
    problems of up to 8 shapes sharing the token count M, as ONE launch of
    256x256 tiles (ragged grouping, csrc/kernels/gemm.hip gemm256_kernel).
    Problems of equal shape must be adjacent. biases[i] (f32 [N_i] or None):
    the bias gradient sum_m dys[i][m] (+ beta * old), summed inside the same
    launch from the dY fragments the MFMAs consume (no second pass over dY).
    ranges[i] = (t_first, t_count) or None: only those 256x256 tiles of
    problem i (in the kernel's enumeration of its tile grid); a cut problem
    gets a shape class of its own."""
    M = xs[0].shape[0]
    shapes = []
    for i, (dy, x, dw) in enumerate(zip(dys, xs, dws)):
        if x.shape[0] != M or dy.shape[0] != M:
            raise ValueError("wgrad_ragged: all problems must share the token count")
        r = ranges[i] if ranges is not None else None
        shapes += [dw.shape[0], x.shape[1], dy.stride(0), x.stride(0), dw.stride(0)]
        shapes += [0, -1] if r is None else [int(r[0]), int(r[1])]
    C().gemm_ragged(list(dys), list(xs), list(dws), shapes, M, False, False, 1.0, beta,
                    list(biases) if biases is not None else [], impl=WGRAD_IMPL)


def colsum_grouped(xs, outs, beta: float = 0.0) -> None:
    """outs[i][N] (+)= column sums of bf16 xs[i][M, N] (same shape), one
    partial pass + one fold for the whole group."""
    M, N = xs[0].shape[0], outs[0].numel()
    rpb = 256
    part = workspace("colsum_g", len(xs) * math.ceil(M / rpb) * N, xs[0].device)
    C().colsum_grouped(xs, outs, part, M, N, xs[0].stride(0), rpb, beta)


def colsum(x2: torch.Tensor, N: int, out: torch.Tensor, beta: float = 0.0) -> torch.Tensor:
    """out[N] (+)= sum over rows of bf16 x2[M, N]."""
    M = x2.shape[0]
    rpb = 128
    part = workspace("colsum", math.ceil(M / rpb) * N, x2.device)
    C().colsum(x2, out, part, M, N, x2.stride(0), rpb, beta)
    return out


# ------------------------------------------------------------------ attention
def attn_fwd(q, k, v, kv_len, scale: float, causal: bool):
    B, Lq, H, hd = q.shape
    out = torch.empty(B, Lq, H, hd, dtype=torch.bfloat16, device=q.device)
    lse = torch.empty(B, H, Lq, dtype=torch.float32, device=q.device)
    C().attn_fwd(q, k, v, out, lse, kv_len, scale, causal)
    return out, lse


# self-attention of <= 128 tokens: the Q|K|V projection and the attention
# forward in one launch (attention.hip qkv_attn_fwd_kernel)
QKV_ATTN = os.environ.get("TDG_QKV_ATTN", "1") != "0"


def qkv_attn_fwd(x2, w, bias, B: int, heads: int, kv_len, scale: float, causal: bool,
                 k=None, v=None):
    """(qkv [M, 3d], out [B, L, H, hd], lse [B, H, L]) of the self-attention
    over qkv = x2 @ w^T + bias, one launch; None when the shape is not covered
    (L > 128, hd != 64). k / v ([B, Lk, H, 64] views): the cross-attention
    form -- w / bias the Q projection's, the first result q [M, d]."""
    M, d = x2.shape
    L, hd = M // B, d // heads
    if not QKV_ATTN or L > 128 or hd != 64 or (k is not None and k.shape[1] > 128):
        return None
    np_ = 1 if k is not None else 3
    qkv = torch.empty(M, np_ * d, dtype=torch.bfloat16, device=x2.device)
    out = torch.empty(B, L, heads, hd, dtype=torch.bfloat16, device=x2.device)
    lse = torch.empty(B, heads, L, dtype=torch.float32, device=x2.device)
    if not C().qkv_attn_fwd(x2, w, bias, qkv, out, lse, kv_len, scale, causal, B, heads, k, v):
        return None
    return qkv, out, lse


def attn_fwd_fp8_ok(Lq: int, Lk: int, hd: int) -> bool:
    """Shapes the e4m3 attention forward covers (attention.hip
    attn_fwd_fp8_kernel): hd 64, the long-sequence path."""
    return hd == 64 and Lq > 128


def attn_fwd_fp8(q8, k8, v8, sq, sk, sv, kv_len, scale: float, causal: bool, o8=None, so8=None,
                 amax8=None):
    """Attention forward on e4m3 copies q8 = e4m3(q * sq) etc. (per-tensor
    scales, one-element device tensors): O (bf16) and the log2-domain LSE, as
    attn_fwd. o8 ([B, Lq, H, hd] e4m3, with its scale so8 and amax slot
    amax8): also O's e4m3 copy from the epilogue (= quantising the bf16 O)."""
    B, Lq, H, hd = q8.shape
    out = torch.empty(B, Lq, H, hd, dtype=torch.bfloat16, device=q8.device)
    lse = torch.empty(B, H, Lq, dtype=torch.float32, device=q8.device)
    C().attn_fwd_fp8(q8, k8, v8, out, lse, kv_len, sq, sk, sv, scale, causal, o8, so8, amax8)
    return out, lse


def attn_bwd(q, k, v, o, dout, lse, dq, dk, dv, kv_len, scale: float, causal: bool):
    delta = workspace("attn_delta", lse.numel(), q.device)[: lse.numel()]
    C().attn_bwd(q, k, v, o, dout, lse, delta, dq, dk, dv, kv_len, scale, causal)


# the fused backward of <= 128-token attention computes dO = dY @ Wo[:, head]
# itself (the output projection's dgrad, never written to memory)
ATTN_BWD_FDO = os.environ.get("TDG_ATTN_BWD_FDO", "1") != "0"


def attn_bwd_fdo(q, k, v, o, dy2, wo, lse, dq, dk, dv, kv_len, scale: float, causal: bool) -> bool:
    """attn_bwd with dout = (dy2 @ wo).view(q.shape) computed in-kernel; False
    (nothing launched) when not covered (Lq / Lk > 128, hd != 64)."""
    if not ATTN_BWD_FDO:
        return False
    delta = workspace("attn_delta", lse.numel(), q.device)[: lse.numel()]
    return C().attn_bwd_fdo(q, k, v, o, dy2, wo, lse, delta, dq, dk, dv, kv_len, scale, causal)


def attn_bwd_g8_ok(Lq: int, Lk: int, hd: int) -> bool:
    """Shapes whose attention backward can emit e5m2 gradients (the hd-64
    pipelined kernels, attention.hip attn_emit_g8)."""
    return hd == 64 and (Lq > 128 or Lk > 128)


def attn_bwd_g8(q, k, v, o, dout, lse, dq, dk, dv, kv_len, scale: float, causal: bool, dq8,
                dk8, dv8, sg8, amax8, cs_part, cs_ld: int, cs_q: int, cs_k: int, cs_v: int,
                skip_bf16: Optional[bool] = None) -> int:
    """attn_bwd that also writes e5m2 copies dq8 (dk8 / dv8 optional, same
    layout as dq / dk / dv) = e5m2(bf16(grad) * sg8), their amax into the
    slot amax8, and the bias-gradient column-sum partials cs_part[B *
    nblocks, cs_ld] (columns cs_q / cs_k / cs_v + head * 64 + j). skip_bf16:
    the bf16 dq / dk / dv are not written (default: when the e5m2 dk8 / dv8
    are requested -- without them the bf16 dK / dV are the output and must be
    written). Returns the partial row count."""
    if skip_bf16 is None:
        skip_bf16 = dk8 is not None
    B, Lq = q.shape[0], q.shape[1]
    np_ = -(-Lq // 128)
    delta = workspace("attn_delta", lse.numel(), q.device)[: lse.numel()]
    C().attn_bwd_g8(q, k, v, o, dout, lse, delta, dq, dk, dv, kv_len, scale, causal, dq8, dk8, dv8,
                    sg8, amax8, cs_part, np_, cs_ld, cs_q, cs_k, cs_v, skip_bf16)
    return B * np_


def attn_bwd_f8_ok(Lq: int, Lk: int, hd: int) -> bool:
    """Shapes the fp8 attention backward covers (attention.hip
    attn_bwd_f8_kernel: every key of a (batch, head) in one workgroup)."""
    return hd == 64 and 128 < Lq <= 512 and Lk <= 512


def attn_bwd_f8(q8, k8, v8, sq, sk, sv, o, do8, sdo, lse, kv_len, scale: float, causal: bool,
                sds, amaxds, dq=None, dk=None, dv=None, dq8=None, dk8=None, dv8=None, sg8=None,
                amaxg8=None, cs_part=None, cs_ld: int = 0, cs_q: int = 0, cs_k: int = 0,
                cs_v: int = 0, sgkv8=None, amaxgkv8=None, cs_part2=None, cs_ld2: int = 0) -> int:
    """Attention backward on fp8 MFMAs: the forward's e4m3 q8 / k8 / v8
    (scales sq / sk / sv), the e5m2 do8 (scale sdo), bf16 o and the forward's
    lse; dS in e5m2 with scale sds (its amax into the slot amaxds). Writes each
    given output: bf16 dq / dk / dv, e5m2 dq8 / dk8 / dv8 = e5m2(bf16(grad) *
    sg8) (amax into amaxg8) and the bias-gradient column sums of the e5m2
    outputs, one row per batch element: cs_part[b, cs_{q,k,v} + head * 64 + j].
    sgkv8 / amaxgkv8: dk8 / dv8 in their own e5m2 slot (the batched cross
    K|V gradient); cs_part2 / cs_ld2: their column sums in a buffer of their
    own. Returns the partial row count (B)."""
    C().attn_bwd_f8(q8, k8, v8, sq, sk, sv, o, do8, sdo, lse, kv_len, scale, causal, sds, amaxds,
                    dq, dk, dv, dq8, dk8, dv8, sg8, amaxg8, cs_part, cs_ld, cs_q, cs_k, cs_v, sgkv8,
                    amaxgkv8, cs_part2, cs_ld2)
    return q8.shape[0]


def attn_probs(q, k, kv_len, scale: float, causal: bool) -> torch.Tensor:
    B, Lq, H, hd = q.shape
    Lk = k.shape[1]
    probs = torch.empty(B, H, Lq, Lk, dtype=torch.float32, device=q.device)
    C().attn_probs(q, k, probs, kv_len, scale, causal)
    return probs


# ------------------------------------------------------------------ layernorm
def ln_fwd(x, s, gamma, beta, p, seed, ctr, site, eps=1e-6, save=True, y8=None, s8=None,
           amax8=None, kbits=None):
    """y = LN(x + dropout(s)); optionally also y8 = e4m3(y * s8) (fp8 copy,
    amax recorded into amax8) and kbits (uint8 [M, D / 8]): the dropout keep
    mask as a row-major bitmap for a fused backward (dgrad_ln_bwd)."""
    D = x.shape[-1]
    M = x.numel() // D
    y = torch.empty_like(x)
    h = torch.empty_like(x) if save else None
    mean = torch.empty(M, dtype=torch.float32, device=x.device) if save else None
    rstd = torch.empty(M, dtype=torch.float32, device=x.device) if save else None
    C().ln_fwd(x, s, gamma, beta, y, h, mean, rstd, p, seed, ctr, site, eps, y8, s8, amax8, kbits)
    return y, h, mean, rstd


# LayerNorm-backward rows per workgroup (norm.hip ln_bwd_d): 16 on 4 waves,
# 32 / 64 on 8 waves -- fewer dgamma / dbeta partial rows for the fold.
# Measured (profiles/r3s2/ln_rpb.txt): 32 for D <= 512 (base step 5.00-5.02 vs
# 5.02-5.05 ms, LN backward 308 vs 321 us + fold 10.6 vs 20.4 us), 16 for
# D = 1024 (big 13.14-13.19 vs 13.20-13.22 ms); 64 loses 3.5 % (two serial
# row passes). Non-zero LN_BWD_RPB forces one value (tests).
LN_BWD_RPB = int(os.environ.get("TDG_LN_BWD_RPB", "0") or 0)


def ln_bwd_rpb(D: int) -> int:
    return LN_BWD_RPB or (32 if D <= 512 else 16)


def ln_bwd_nparts(M: int, D: int) -> int:
    """Partial-sum rows ln_bwd writes (one per workgroup)."""
    return math.ceil(M / ln_bwd_rpb(D))


def ln_bwd(dy, h, mean, rstd, gamma, dgamma, dbeta, dbias, p, seed, ctr, site, want_ds=True,
           dres=None, accumulate=False, defer=None, ds8=None, s8=None, amax8=None, kbits=None):
    """`defer` (a list): leave the dgamma / dbeta / dbias partial sums in a
    per-site workspace and append their fold to `defer` (run later, all
    LayerNorms of a backward in one launch, by reduce_partials_multi).
    ds8 (e5m2, shape of dy) with scale s8 / amax slot amax8: also the e5m2
    copy of ds for an fp8 backward; with want_ds=False the bf16 ds is then
    not written at all (the bias column sums still come from ds). kbits
    (uint8 [M, D / 8], from ln_fwd): the dropout mask read instead of
    regenerated."""
    D = dy.shape[-1]
    M = dy.numel() // D
    dh = torch.empty_like(dy)
    need_ds = (want_ds and (p > 0 or dres is not None)) or (dbias is not None and ds8 is None)
    ds = torch.empty_like(dy) if need_ds else None
    if defer is None:
        ws = workspace("ln_bwd", 3 * ln_bwd_nparts(M, D) * D, dy.device)
    else:  # partials must survive until the fold: one workspace per site
        ws = workspace(f"ln_bwd_part_{site}", 3 * ln_bwd_nparts(M, D) * D, dy.device)
    C().ln_bwd(dy, h, mean, rstd, gamma, dh, ds, dres, dgamma, dbeta, dbias, ws, p, seed, ctr, site,
               accumulate, defer is not None, ln_bwd_rpb(D), ds8, s8, amax8, kbits)
    if defer is not None:
        nb = ln_bwd_nparts(M, D)
        outs = [dgamma, dbeta] + ([dbias] if dbias is not None else [])
        for i, o in enumerate(outs):
            defer.append((ws[i * nb * D:(i + 1) * nb * D], o, nb, D, 1.0 if accumulate else 0.0))
    if ds is None:
        ds = dh
    return dh, ds


def reduce_partials_multi(items) -> None:
    """Fold deferred (partials, out, nparts, N, beta) column reductions; one
    launch per (N, beta) group of up to 96."""
    groups = {}
    for part, out, nparts, N, beta in items:
        groups.setdefault((N, beta), []).append((part, out, nparts))
    for (N, beta), its in groups.items():
        for c0 in range(0, len(its), 96):
            ch = its[c0:c0 + 96]
            C().reduce_partials_multi([i[0] for i in ch], [i[1] for i in ch], [i[2] for i in ch],
                                      N, beta)


# ------------------------------------------------------------------ embedding / loss / optim
def embed_fwd(tok, table, pe, scale, p, seed, ctr, site, kbits=None):
    """dropout(table[tok] * scale + pe); kbits (uint8 [B * L, D / 8], D >=
    512): also the dropout keep bits, for the CSR backward."""
    B, L = tok.shape
    D = table.shape[1]
    out = torch.empty(B, L, D, dtype=torch.bfloat16, device=tok.device)
    C().embed_fwd(tok, table, pe, out, scale, p, seed, ctr, site, kbits)
    return out


DETERMINISTIC_EMBED = os.environ.get("TDG_DETERMINISTIC", "1") != "0"


# deterministic embedding backward without global atomics: token sort, one
# wave per vocabulary row (or cut of a frequent row), fixed-point sums in
# registers (embed.hip "CSR backward"); else the fixed-point atomic kernel
EMBED_CSR = os.environ.get("TDG_EMBED_CSR", "1") != "0"


class EmbCsr:
    """The token sort of one table's CSR embedding backward (its work items in
    an int32 workspace of its own, `name`)."""

    def __init__(self, tok: torch.Tensor, V: int, name: str):
        self.tok, self.V, self.M = tok, int(V), tok.numel()
        n32, _ = C().embed_csr_ws(self.M, self.V, 128)
        self.w32 = workspace("embed_csr32_" + name, n32, tok.device, torch.int32)


def embed_csr_ok(M: int, V: int) -> bool:
    return DETERMINISTIC_EMBED and EMBED_CSR and C().embed_csr_ok(M, V)


def embed_csr_sort(tables, stamps=None) -> list:
    """[(tok, V, name)] (one or two tables) -> [EmbCsr]: their token sorts in
    one launch (one workgroup per table). stamps: lab phase clocks."""
    cs = [EmbCsr(t.contiguous(), V, name) for t, V, name in tables]
    C().embed_csr_sort([c.tok for c in cs], [c.V for c in cs], [c.w32 for c in cs], stamps)
    return cs


def embed_csr_apply(cs: EmbCsr, dout, dtable, scale, p, seed, ctr, site, accumulate=False,
                    kbits=None) -> None:
    """dtable (=|+=) the embedding gradient from a sorted table (bitwise the
    fixed-point atomic path's)."""
    _, n64 = C().embed_csr_ws(cs.M, cs.V, dtable.shape[1])
    w64 = workspace("embed_csr64", n64, dtable.device, torch.int64)
    C().embed_csr_apply(dout, dtable, cs.w32, w64, cs.M, scale, p, seed, ctr, site, accumulate, kbits)


def embed_bwd(tok, dout, dtable, scale, p, seed, ctr, site, accumulate=False, kbits=None,
              csr: Optional[EmbCsr] = None):
    """dtable (=|+=) scatter-add of the embedding gradient. Default: the
    deterministic paths (bitwise reproducible and bitwise equal to each
    other): the CSR kernels (`csr`: the forward already sorted the tokens),
    else fixed-point int64 atomics; TDG_DETERMINISTIC=0 uses plain f32
    atomics (dtable must then be zero unless accumulating). kbits: the
    forward's keep bits (CSR path; else the Philox mask is regenerated)."""
    if csr is not None or embed_csr_ok(tok.numel(), dtable.shape[0]):
        if csr is None:
            csr = embed_csr_sort([(tok, dtable.shape[0], "bwd")])[0]
        embed_csr_apply(csr, dout.contiguous(), dtable, scale, p, seed, ctr, site, accumulate, kbits)
        return
    if DETERMINISTIC_EMBED:
        acc = workspace("embed_fx", dtable.numel(), dtable.device, torch.int64, zero=True)
        C().embed_bwd_det(tok, dout, dtable, acc, scale, p, seed, ctr, site, accumulate)
    else:
        C().embed_bwd(tok, dout, dtable, scale, p, seed, ctr, site)


def count_tokens(labels, out):
    C().count_tokens(labels, out)


_PREP_SCRATCH: Dict[tuple, torch.Tensor] = {}


def prep_batch(src, tgt, ctr=None):
    """One launch: (tgt_in, labels, src_len, tgt_len, ntok) of a teacher-forced
    batch -- tgt[:, :-1], tgt[:, 1:], int32 non-PAD lengths, f32 [1] non-PAD
    label count -- and ctr += 1 when given (the dropout RNG step)."""
    src = src.contiguous()
    tgt = tgt.contiguous()
    B, T1 = tgt.shape
    tgt_in = torch.empty(B, T1 - 1, dtype=tgt.dtype, device=tgt.device)
    labels = torch.empty(B, T1 - 1, dtype=tgt.dtype, device=tgt.device)
    lens = torch.empty(2, B, dtype=torch.int32, device=tgt.device)
    ntok = torch.empty(1, dtype=torch.float32, device=tgt.device)
    key = (tgt.device, B)
    scratch = _PREP_SCRATCH.get(key)
    if scratch is None:  # [B] label counts, ticket (zero; the kernel re-arms it), bad-row count
        scratch = _PREP_SCRATCH[key] = torch.zeros(B + 2, dtype=torch.int32, device=tgt.device)
    C().prep_batch(src, tgt, tgt_in, labels, lens[0], lens[1], ntok, ctr, scratch)
    return tgt_in, labels, lens[0], lens[1], ntok


def interior_pad_rows(reset: bool = False) -> int:
    """Rows seen by prep_batch (since the last reset) with a PAD token before
    a non-PAD one. Attention masks keys by length, i.e. assumes trailing
    padding; the reference masks each PAD position individually
    (transformer_model.py:56-62), so callers reject batches where this is
    non-zero. Reads a device counter (a host sync): call at log points."""
    n = 0
    for scratch in _PREP_SCRATCH.values():
        n += int(scratch[-1].item())
        if reset:
            scratch[-1].zero_()
    return n


def check_trailing_padding() -> None:
    """Raise if any batch prepared on the GPU had interior PAD tokens."""
    n = interior_pad_rows(reset=True)
    if n:
        raise ValueError(f"{n} batch rows had a PAD (id 0) token before a non-PAD token; sequences "
                         "must be right-padded (attention masks keys by length)")


def xent(logits, V, labels, ntok, workers, smoothing, row_loss, row_correct, write_grad=True):
    C().xent(logits, V, labels, ntok, workers, smoothing, row_loss, row_correct, write_grad)


def xent_stats(row_loss, row_correct, ntok, workers, step_out=None, accum=None):
    C().xent_stats(row_loss, row_correct, ntok, workers, step_out, accum)


def adam_chunks(p, g, m, v, shadow, chunks, step, beta1, beta2, eps, lr_const, d_model, warmup,
                grad_scale, weight_decay, sched, zero_grad, inc_step, scale8, amax8):
    """Adam over a chunk table that also refreshes e4m3 weight copies
    (adam.hip adam_chunk_kernel; table: ops.fp8.Fp8Weights.adam_chunks)."""
    C().adam_chunks(p, g, m, v, shadow, chunks, step, beta1, beta2, eps, lr_const, d_model, warmup,
                    grad_scale, weight_decay, sched, zero_grad, inc_step, scale8, amax8)


def adam(p, g, m, v, shadow, step, beta1, beta2, eps, lr_const, d_model, warmup, grad_scale=1.0,
         weight_decay=0.0, sched=1, zero_grad=True, inc_step=True):
    C().adam(p, g, m, v, shadow, step, beta1, beta2, eps, lr_const, d_model, warmup, grad_scale,
             weight_decay, sched, zero_grad, inc_step)


# ------------------------------------------------------------------ stream signal
class StreamSignal:
    """A host-visible position marker on a HIP stream (csrc/kernels/signal.hip):
    emit() enqueues a one-wave kernel that bumps a device counter and publishes
    it to a coherent pinned host word; wait(n) spins (GIL released) until the
    n-th emitted kernel has run. Captured into a HIP graph, each replay
    publishes again, so a host thread can follow a graph's progress without
    the graph being cut or an event recorded (parallel/ddp.py's comm thread)."""

    def __init__(self, device: torch.device):
        self.device = device.index if device.index is not None else torch.cuda.current_device()
        with torch.cuda.device(self.device):
            self._host, self._dhost, self._cnt = C().signal_create()
        # emits handed to the host side so far (the value the next wait expects)
        self.expected = 0

    def emit(self) -> None:
        C().signal_emit(self._dhost, self._cnt, self.device)

    def wait(self, n: int, timeout_s: float) -> bool:
        return C().signal_wait(self._host, n, timeout_s)

    def value(self) -> int:
        return C().signal_read(self._host)
