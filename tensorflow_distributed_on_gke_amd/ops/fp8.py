"""FP8 training path (BASELINE config 5: "Transformer-big seq_len=512 fp8 MFMA
attention+FFN"): e4m3 / e5m2 operands on gfx950's block-scaled MFMA
(`v_mfma_scale_f32_*_f8f6f4`, csrc/kernels/fp8.hip) with delayed
per-tensor scaling.

Every fp8 operand has a slot in a device-resident `Fp8Meta` (e4m3 for
activations and weights, a second e5m2 one for gradients): `scale[i]`
(x8 = fp8(x * scale)) and `amax[i]` (max |x| recorded by whoever quantised
slot i this step). Once per step `Fp8Meta.update()` turns the recorded amax
into the next step's power-of-two scale and clears amax -- on device, so the
step stays one HIP graph; the e4m3 weight copies are refreshed by the Adam
kernel itself (adam_chunk_kernel) with the scale the next forward uses.

What runs in which format is `precision_map()` (bench.py prints it in its
record for `--dtype fp8`): every projection GEMM of the encoder / decoder
layers -- forward, dgrad and weight gradient -- and the attention forward
and backward (sequences of 129-512) are fp8; the vocabulary projection,
LayerNorm, embeddings, cross-entropy and the fp32 Adam are not. Measured
(docs/PERF.md): Transformer-big seq 512 fp8 11.78 vs 13.59 ms/step bf16 on
one box (round 4, before the fp8 attention backward).
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Tuple

import torch

from tensorflow_distributed_on_gke_amd.ops._ext import C
from tensorflow_distributed_on_gke_amd.ops import kernels as K

FP8 = torch.float8_e4m3fn
BF8 = torch.float8_e5m2  # gradient format of the fp8 backward
E4M3_MAX = 448.0
E5M2_MAX = 57344.0
AMAX_WORDS = 64 * 32  # per slot (csrc/include/tdg_common.h AMAX_WORDS)
_CANDS = (0, 1, 2, 3, 4, 5, 8, 9, 10)
# FFN weight gradients in fp8 (wgrad_fp8) when the step runs the fp8 backward
WGRAD_FP8 = True
# attention projections in fp8 too (Fp8State(backward=True)): output
# projection forward, every projection dgrad and weight gradient
ATTN_PROJ_FP8 = True
# tile config of the e5m2 x e4m3 backward GEMMs (0: 128x128 / 4 waves; 9: 256x256 at one wave per SIMD;
# 10: 128x128 / 4 waves on a ring of 64-byte K half-stages)
BWD_CFG = 0
# ... of those reading the weight N-contiguous or producing column sums (0 or 10)
BWD_CFG_128 = 0
# fp8 dgrads read the forward's e4m3 weight copy N-contiguous (transposing LDS
# reads, 128x128 tiles) instead of a transposed copy: no fp8_quant_t pass
# over every weight per step
DGRAD_PLAIN_W = True
# the attention backward emits the e5m2 dQ|dK|dV (and the projection bias
# gradient partials) of the fp8 projection backward itself, instead of a
# quantise + column-sum pass over the bf16 gradient (long sequences)
ATTN_BWD_G8 = True
_TUNED: Dict[tuple, int] = {}


def precision_map() -> Dict[str, str]:
    """Per-op number formats of the `--dtype fp8` training step with the
    module flags as they are (the truthful record bench.py prints)."""
    proj_bwd = "e5m2 x e4m3" if ATTN_PROJ_FP8 else "bf16"
    return {
        "ffn_forward": "e4m3 x e4m3 (FFN1 bias+ReLU, FFN2)",
        "attention_input_projections_forward": "e4m3 x e4m3 (self Q|K|V, cross Q, batched cross K|V)",
        "attention_output_projection_forward": "e4m3 x e4m3" if ATTN_PROJ_FP8 else "bf16",
        "attention_forward": "e4m3 Q/K/V and P, fp32 softmax (hd 64, seq > 128; else bf16)",
        "attention_backward": _attn_bwd_precision(),
        "ffn_dgrads": "e5m2 x e4m3 (ReLU-backward epilogue)",
        "attention_projection_dgrads": proj_bwd,
        "ffn_weight_gradients": "e5m2 x e4m3" if WGRAD_FP8 else "bf16",
        "attention_projection_weight_gradients": proj_bwd if WGRAD_FP8 else "bf16",
        "vocab_projection": "bf16 (forward, dgrad, weight gradient)",
        "layernorm": "fp32 math on bf16 I/O (emits the e4m3 / e5m2 copies its fp8 consumers read)",
        "embedding": "bf16 gather, fp32 fixed-point gradient",
        "cross_entropy": "fp32 on bf16 logits",
        "optimizer": "fp32 Keras Adam (refreshes the bf16 and e4m3 weight copies)",
    }


# fp8 attention backward (attention.hip attn_bwd_f8_kernel, sequences of
# 129-512 at hd 64): the forward's e4m3 Q/K/V and e4m3 P, e5m2 dO and dS on
# the fp8 MFMAs, every key of a (batch, head) in one workgroup (P and dS once)
ATTN_BWD_F8 = os.environ.get("TDG_ATTN_BWD_F8", "1") != "0"
_ATTN_BWD_F8_STR = ("e4m3 Q/K/V/P x e5m2 dO/dS on fp8 MFMA (v_mfma_f32_16x16x32 fp8/bf8), f32 "
                    "softmax from the forward LSE (seq 129-512; longer: the bf16 backward below); "
                    "e5m2 dQ|dK|dV out -- cross-attention dK/dV as e5m2 straight into the batched "
                    "K|V gradient (its own scale slot) when every decoder layer runs this kernel, "
                    "else bf16 into it")
_ATTN_BWD_BF16_STR = "bf16 MFMA on the dequantised e4m3 Q/K/V, bf16 dO (e5m2 dQ|dK|dV out)"


def _attn_bwd_precision() -> str:
    return _ATTN_BWD_F8_STR if ATTN_BWD_F8 else _ATTN_BWD_BF16_STR


# the attention backward's format as configured at import (precision_map
# reads the flag when called)
ATTN_BWD_PRECISION = _attn_bwd_precision()


def precision_string() -> str:
    return "fp8: " + "; ".join(f"{k}={v}" for k, v in precision_map().items())


ADAM_CHUNK = 4096  # parameters per adam_chunk_kernel workgroup


def validate_chunk_table(rows, total: int, nslots: int, w8_extents=()) -> None:
    """Host-side check of an adam_chunk_kernel table (rows of (start, n,
    slot, e4m3 address)) before it is uploaded: every chunk inside the flat
    buffer, n in (0, 4096] and a multiple of 4, starts 4-aligned, chunks
    disjoint and in order, slots in range, and every e4m3 address inside one
    of the live copies w8_extents = [(address, bytes)] at the chunk's offset
    within it. The kernel trusts the table (it silently skips parameters past
    4096 in a chunk), so a malformed one must never reach it."""
    pos = 0
    ext = sorted(w8_extents)
    for start, n, slot, addr in rows:
        if not (0 < n <= ADAM_CHUNK and n % 4 == 0 and start % 4 == 0):
            raise ValueError(f"adam chunk ({start}, {n}): n must be in (0, {ADAM_CHUNK}] and 4-aligned")
        if start < pos or start + n > total:
            raise ValueError(f"adam chunk ({start}, {n}) overlaps or leaves the flat buffer [0, {total})")
        pos = start + n
        if slot >= 0:
            if slot >= nslots or not addr:
                raise ValueError(f"adam chunk ({start}, {n}): slot {slot} / address {addr:#x} invalid")
            if not any(a <= addr and addr + n <= a + nb for a, nb in ext):
                raise ValueError(f"adam chunk ({start}, {n}): e4m3 address {addr:#x} outside every copy")
        elif addr:
            raise ValueError(f"adam chunk ({start}, {n}): address without a slot")


class Fp8Meta:
    """fmt 0: e4m3 slots (activations, weights); fmt 1: e5m2 (gradients)."""

    def __init__(self, device, capacity: int = 256, margin: int = 0, fmt: int = 0):
        self.device = torch.device(device)
        self.fmt = fmt
        self.dtype = BF8 if fmt else FP8
        self.fmax = E5M2_MAX if fmt else E4M3_MAX
        self.scale = torch.ones(capacity, dtype=torch.float32, device=self.device)
        # [slot, 2048]: producers spread their atomics over 64 words, one per
        # 128-byte line (tdg_common.h AMAX_SPREAD / AMAX_STRIDE; the rest stay 0)
        self.amax = torch.zeros(capacity, AMAX_WORDS, dtype=torch.int32, device=self.device)
        self.margin = margin
        self.names: List[str] = []

    def slot(self, name: str) -> int:
        if len(self.names) >= self.scale.numel():
            raise RuntimeError("Fp8Meta capacity exhausted")
        self.names.append(name)
        return len(self.names) - 1

    def s(self, i: int) -> torch.Tensor:
        return self.scale[i:i + 1]

    def a(self, i: int) -> torch.Tensor:
        return self.amax[i]

    def update(self) -> None:
        n = len(self.names)
        if n:
            C().fp8_scale_update(self.scale[:n], self.amax[:n], float(2 ** self.margin), self.fmax)

    def amax_values(self) -> torch.Tensor:
        return self.amax[: len(self.names)].view(torch.float32).amax(dim=1)


def quantize(x: torch.Tensor, meta: Fp8Meta, i: int, out: Optional[torch.Tensor] = None,
             record: bool = True) -> torch.Tensor:
    if out is None:
        out = torch.empty(x.shape, dtype=meta.dtype, device=x.device)
    C().fp8_quant(x.contiguous(), out, meta.s(i), meta.a(i) if record else None, meta.fmt)
    return out


def quantize_colsum(x: torch.Tensor, meta: Fp8Meta, i: int, key: str):
    """(x8, part, nparts): fp8 copy of the 2-D bf16 x (amax recorded) and the
    per-256-row-block column sums of x in a per-`key` workspace [nparts, N] --
    fold them into a bias gradient (ops.kernels.reduce_partials_multi)."""
    M, N = x.shape
    nparts = math.ceil(M / 256)
    x8 = torch.empty(M, N, dtype=meta.dtype, device=x.device)
    part = K.workspace("qcs_" + key, nparts * N, x.device)[: nparts * N]
    C().fp8_quant_colsum(x, x8, meta.s(i), meta.a(i), part, meta.fmt)
    return x8, part, nparts


def dequantize(x8: torch.Tensor, scale: float) -> torch.Tensor:
    return x8.float() / scale


def gemm_fp8(a8, b8, bias, meta: Fp8Meta, ia: int, ib: int, relu: bool = False,
             out8_slot: Optional[int] = None, cfg: Optional[int] = None, c_deq: bool = False,
             want_y: bool = True) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
    """y[M,N] = dequant(a8[M,K] @ b8[N,K]^T) + bias (relu), bf16, on the
    block-scaled e4m3 MFMA (csrc/kernels/fp8.hip); with out8_slot also
    y8 = e4m3(y * scale[out8_slot]) (amax recorded). c_deq (needs out8_slot):
    y = y8 / scale instead, the exact values the e4m3 consumer of y8 sees
    (scales are powers of two), so a backward reading y is consistent with
    a forward that ran on y8. want_y = False (needs out8_slot): only y8 is
    written (y is None)."""
    M, Kd = a8.shape
    N = b8.shape[0]
    y8 = torch.empty(M, N, dtype=FP8, device=a8.device) if out8_slot is not None else None
    if c_deq and y8 is None:
        raise ValueError("gemm_fp8: c_deq needs out8_slot")
    if not want_y and (y8 is None or c_deq):
        raise ValueError("gemm_fp8: want_y=False needs out8_slot and no c_deq")
    epi = (2 if relu else (1 if bias is not None else 0)) | (16 if c_deq else 0)
    y = torch.empty(M, N, dtype=torch.bfloat16, device=a8.device) if want_y else None

    def run(c):
        C().gemm_fp8(a8, b8, y, bias, meta.s(ia), meta.s(ib), y8,
                     meta.s(out8_slot) if y8 is not None else None,
                     meta.a(out8_slot) if y8 is not None else None,
                     M, N, Kd, a8.stride(0), b8.stride(0), N, N, epi, c, 0, 0, None, 0, 0.0)

    if cfg is None:
        key = (M, N, Kd, epi, y8 is not None, want_y)
        cfg = _TUNED.get(key)
        if cfg is None:
            if K.AUTOTUNE and a8.is_cuda and not torch.cuda.is_current_stream_capturing():
                cfg = _autotune(run)
            else:
                cfg = choose_fp8(M, N, Kd)
            _TUNED[key] = cfg
    run(cfg)
    return y, y8


def gemm_bf8_dgrad(g8, gmeta: Fp8Meta, ig: int, w8, wmeta: Fp8Meta, iw: int,
                   out: Optional[torch.Tensor], relu_aux: Optional[torch.Tensor] = None,
                   beta: float = 0.0, out8_slot: Optional[int] = None, cfg: Optional[int] = None,
                   relu_aux8: Optional[torch.Tensor] = None, colsum_out: Optional[torch.Tensor] = None,
                   colsum_beta: float = 0.0, w_plain: bool = False,
                   defer: Optional[list] = None) -> Optional[torch.Tensor]:
    """Backward GEMM on the block-scaled MFMA: out[M,N] (=|+= beta) dequant(
    g8[M,K] (e5m2 gradient) @ W), bf16, where W[K,N] is the e4m3 weight:
    w_plain: w8 IS that weight ([out=K][in=N], the forward's copy; the kernel
    reads it N-contiguous through the transposing LDS path, 128x128 tiles),
    else w8 is its transposed copy [N,K]. relu_aux: zero where relu_aux <= 0
    (ReLU backward), or relu_aux8: zero where the e4m3 ReLU output is 0;
    out8_slot: also the e5m2 copy of out in gmeta's slot (returned, amax
    recorded); colsum_out[N] (=|+= colsum_beta): the column sums of the
    (bf16-rounded) output -- a bias gradient -- from the epilogue (128x128
    tiles). out may be None (nothing but the e5m2 copy and the sums is
    written). defer (a list): the column sums' partials stay in a workspace
    of colsum_out's own and their fold is appended to defer
    (kernels.reduce_partials_multi, with the other deferred reductions)."""
    M, Kd = g8.shape
    N = w8.shape[1] if w_plain else w8.shape[0]
    o8 = torch.empty(M, N, dtype=BF8, device=g8.device) if out8_slot is not None else None
    aux = relu_aux if relu_aux is not None else relu_aux8
    c = BWD_CFG if cfg is None else cfg
    ws = None
    if (colsum_out is not None or w_plain) and c not in (0, 10):
        c = BWD_CFG_128
    nparts = math.ceil(M / 128) * 2
    if colsum_out is not None:
        # (deferred: the partials must survive until the fold -- a workspace
        # per output)
        key = "fp8_colsum" if defer is None else f"fp8_colsum_{colsum_out.data_ptr()}"
        ws = K.workspace(key, nparts * N, g8.device)
    epi = (3 if aux is not None else 0) | (32 if w_plain else 0)
    if colsum_out is not None and defer is not None:
        epi |= 64
    C().gemm_fp8(g8, w8, out, None, gmeta.s(ig), wmeta.s(iw), o8,
                 gmeta.s(out8_slot) if o8 is not None else None,
                 gmeta.a(out8_slot) if o8 is not None else None,
                 M, N, Kd, g8.stride(0), w8.stride(0), out.stride(0) if out is not None else N, N,
                 epi, c, 1, 1, relu_aux,
                 aux.stride(0) if aux is not None else 0, beta, aux8=relu_aux8,
                 colsum_out=colsum_out, colsum_beta=colsum_beta, ws=ws)
    if colsum_out is not None and defer is not None:
        defer.append((ws[:nparts * N], colsum_out, nparts, N, colsum_beta))
    return o8


def wgrad_fp8(dy8s, sas, x8s, sbs, dws, beta: float = 0.0) -> None:
    """dws[i][M,N] (f32, =|+= beta) = dequant(dy8s[i][T,M]^T @ x8s[i][T,N]):
    weight gradients from the e5m2 gradient and the e4m3 activation copies
    the step already holds (token-major, read through the transposing LDS
    path: csrc/kernels/fp8.hip wgrad_fp8_kernel). sas / sbs: the one-element
    scale tensors of each operand. One launch per token count T, shape
    classes adjacent, at most 64 problems in 8 shape classes per launch (the
    kernel's argument block)."""
    def key(i):
        return (dy8s[i].shape[1], x8s[i].shape[1], dy8s[i].stride(0), x8s[i].stride(0),
                dws[i].stride(0))

    by_t = {}
    for i in range(len(dws)):
        by_t.setdefault(dy8s[i].shape[0], []).append(i)
    for idx in by_t.values():
        idx.sort(key=key)
        launch, classes = [], []
        for i in idx + [None]:
            if i is not None:
                k = key(i)
                new_cls = not classes or classes[-1] != k
                if len(launch) < 64 and (not new_cls or len(classes) < 8):
                    launch.append(i)
                    if new_cls:
                        classes.append(k)
                    continue
            C().wgrad_fp8([dy8s[j] for j in launch], [x8s[j] for j in launch],
                          [dws[j] for j in launch], [sas[j] for j in launch],
                          [sbs[j] for j in launch], float(beta))
            if i is not None:
                launch, classes = [i], [key(i)]


def wgrad_fp8_ok(T: int, M: int, N: int) -> bool:
    return T % 128 == 0 and M % 16 == 0 and N % 16 == 0


def choose_fp8(M: int, N: int, Kd: int) -> int:
    """fp8 tile config without a timed search (csrc/kernels/fp8.hip table):
    128x128 on 4 waves whenever that fills the CUs -- it beat 256x128 / 8
    waves on every Transformer-big forward shape, 3-14 % (qkv 42.7 vs 47.0 us,
    xkv6 160.6 vs 186.6; profiles/r3/fp8_gemm_sweep.jsonl)."""
    if -(-M // 128) * -(-N // 128) >= K.NUM_CU:
        return 0  # 128x128, 4 waves, 2 stages
    return 5


def _tkey_str(k: tuple) -> str:
    return ",".join(str(int(x)) for x in k)


def save_tuned(path: str) -> None:
    """Persist the fp8 forward GEMM tile choices (JSON: "M,N,K,epi,y8,y" ->
    cfg), e.g. from scripts/tune_fp8_in_model.py."""
    import json

    with open(path, "w") as f:
        json.dump({_tkey_str(k): v for k, v in sorted(_TUNED.items())}, f, indent=0)


def load_tuned(path: str) -> int:
    import json

    if not os.path.exists(path):
        return 0
    with open(path) as f:
        data = json.load(f)
    for ks, v in data.items():
        M, N, Kd, epi, y8, y = (int(x) for x in ks.split(","))
        _TUNED[(M, N, Kd, epi, bool(y8), bool(y))] = int(v)
    return len(data)


# in-model measured tiles of the Transformer-big fp8 forward GEMMs
# (scripts/tune_fp8_in_model.py); shapes not in it: choose_fp8
TUNED_FILE = os.environ.get("TDG_FP8_TUNED_FILE") or os.path.join(
    os.path.dirname(os.path.abspath(__file__)), "fp8_tuned_gfx950.json")


def _autotune(run) -> int:
    times = {}
    for rnd in range(2):
        for c in _CANDS:
            try:
                run(c)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    run(c)
                e1.record()
                e1.synchronize()
                times[c] = min(times.get(c, math.inf), e0.elapsed_time(e1))
            except RuntimeError:
                continue
    return min(times, key=times.get)


class Fp8Weights:
    """fp8 copies of selected weight matrices, refreshed from the bf16 shadow
    after every optimizer step (after the scale update)."""

    def __init__(self, meta: Fp8Meta):
        self.meta = meta
        self.items: List[Tuple[object, torch.Tensor, int]] = []
        self.by_param: Dict[int, Tuple[torch.Tensor, int]] = {}

    def add(self, param, transposed: bool = False) -> Tuple[torch.Tensor, int]:
        """transposed: an e4m3 copy of the weight transposed ([in, out], the
        layout a dgrad reads K-contiguous), quantised straight from the bf16
        compute copy by the transposing kernel (fp8_quant_t)."""
        shape = (param.shape[1], param.shape[0]) if transposed else param.shape
        w8 = torch.empty(shape, dtype=FP8, device=self.meta.device)
        slot = self.meta.slot(("wt:" if transposed else "w:") + param.name)
        self.items.append((param, w8, slot, transposed))
        self.by_param[(id(param), transposed)] = (w8, slot)
        return w8, slot

    def get(self, param, transposed: bool = False) -> Tuple[torch.Tensor, int]:
        return self.by_param[(id(param), transposed)]

    def has(self, param, transposed: bool = False) -> bool:
        return (id(param), transposed) in self.by_param

    def refresh(self) -> None:
        """All weight copies, each with its own scale and amax slot: the plain
        ones in one launch per 64 weights (fp8_quant_multi), the transposed
        ones one launch per weight shape (fp8_quant_t)."""
        plain = [it for it in self.items if not it[3]]
        for c0 in range(0, len(plain), 64):
            chunk = plain[c0:c0 + 64]
            C().fp8_quant_multi([p.compute for p, _, _, _ in chunk],
                                [w8 for _, w8, _, _ in chunk], [slot for _, _, slot, _ in chunk],
                                self.meta.scale, self.meta.amax)
        groups: Dict[tuple, list] = {}
        for it in self.items:
            if it[3]:
                groups.setdefault(tuple(it[0].shape), []).append(it)
        for its in groups.values():
            for c0 in range(0, len(its), 64):
                chunk = its[c0:c0 + 64]
                C().fp8_quant_t([p.compute for p, _, _, _ in chunk], [w8 for _, w8, _, _ in chunk],
                                [slot for _, _, slot, _ in chunk], self.meta.scale, self.meta.amax)

    def adam_chunks(self, store) -> Optional[torch.Tensor]:
        """Chunk table of the flat parameter buffer for the Adam kernel that
        also refreshes these e4m3 copies (adam_chunk_kernel): int64 [n, 4]
        rows (start, count <= 4096, slot or -1, e4m3 address or 0); chunks
        never cross into or out of a weight with an e4m3 copy. None when some
        copy is transposed or the buffer exceeds the kernel's 2^28 limit."""
        # the table bakes in the e4m3 copies' addresses and the buffer size:
        # rebuilt if either changed since it was built
        sig = (store.total, tuple((w8.data_ptr(), w8.numel()) for _, w8, _, _ in self.items))
        if getattr(self, "_chunks", None) is not None and self._chunk_sig == sig:
            return self._chunks
        if any(it[3] for it in self.items) or store.total >= (1 << 28):
            return None
        CH = ADAM_CHUNK
        segs = sorted(((p.offset, p.numel, w8, slot) for p, w8, slot, _ in self.items),
                      key=lambda t: t[0])
        rows, pos = [], 0

        def plain(a, b):
            for c0 in range(a, b, CH):
                rows.append((c0, min(CH, b - c0), -1, 0))

        for off, n, w8, slot in segs:
            if off % 4 or n % 4 or off < pos:
                return None
            plain(pos, off)
            base = w8.data_ptr()
            for c0 in range(0, n, CH):
                rows.append((off + c0, min(CH, n - c0), slot, base + c0))
            pos = off + n
        plain(pos, store.total)
        validate_chunk_table(rows, store.total, self.meta.scale.numel(),
                             [(w8.data_ptr(), w8.numel()) for _, w8, _, _ in self.items])
        self._chunks = torch.tensor(rows, dtype=torch.int64, device=self.meta.device)
        self._chunk_sig = sig
        return self._chunks

    def calibrate(self) -> None:
        """Initial weight scales from their actual amax."""
        self.refresh()
        self.meta.update()
        self.refresh()


class Fp8State:
    """Per-model fp8 bookkeeping: meta, weight copies and activation slots.

    fp8 forward GEMMs: both FFN projections of every layer, and the attention
    input projections -- self-attention Q|K|V, cross-attention Q and the
    batched cross-attention K|V of the encoder output. Each of their inputs is
    the output of a LayerNorm (which then emits the e4m3 copy, `ln_slots`),
    except the first layer's Q|K|V input (the embedding), quantised by its
    own kernel. With ATTN_PROJ_FP8 the attention output projections run e4m3
    too (the attention output is quantised once), and the backward of every
    attention projection -- dgrad and weight gradient -- runs on e5m2
    gradients."""

    def __init__(self, model, margin: int = 0, backward: bool = True):

        self.meta = Fp8Meta(model.device, margin=margin)
        self.weights = Fp8Weights(self.meta)
        # e5m2 gradients of the FFN backward (`backward`): ds (LayerNorm
        # backward output) and the ReLU-backward dgrad's output, per layer
        self.gmeta = Fp8Meta(model.device, margin=margin, fmt=1)
        # first-step scale of the gradient slots (delayed scaling takes over
        # after one step): 2^16 keeps |g| in [2^-32, 0.875] representable
        self.gmeta.scale.fill_(65536.0)
        self.ffn_bwd_slots: Dict[int, Tuple[int, int]] = {}
        self.ffn_slots: Dict[int, Tuple[int, int]] = {}
        # LayerNorms whose output is an fp8 GEMM input: they emit the e4m3 copy
        self.ln_slots: Dict[int, int] = {}
        # attention input projections: weight -> activation slot, output slot
        # (their e4m3 outputs feed the e4m3 attention, attention.hip
        # attn_fwd_fp8_kernel, on the sequences it covers)
        self.proj_slots: Dict[int, int] = {}
        self.out_slots: Dict[int, int] = {}
        # batched cross K|V (e4m3) of the CURRENT forward, with its scale slot:
        # set by CrossKVFn, cleared by Transformer.forward after the decoder
        self.kv8: Optional[Tuple[torch.Tensor, int]] = None
        self.stash: Dict[int, torch.Tensor] = {}
        for layer in list(model.enc_layers) + list(model.dec_layers):
            self.weights.add(layer.ff1.w)
            self.weights.add(layer.ff2.w)
            xs = self.meta.slot(f"x:{id(layer)}")
            hs = self.meta.slot(f"h:{id(layer)}")
            self.ffn_slots[id(layer.ff1.w)] = (xs, hs)
            feeder = layer.ln1 if hasattr(layer, "qkv") else layer.ln2  # encoder / decoder
            self.ln_slots[id(feeder.gamma)] = xs
            if backward:
                # every FFN backward now runs on the e4m3 weights: the bf16
                # W2^T copies (ParamStore.add_transposed) are not read, and the
                # optimizer stops re-transposing them (0.07 ms per big step)
                if getattr(model, "store", None) is not None:
                    model.store.transposed_paused = True
                if not DGRAD_PLAIN_W:
                    self.weights.add(layer.ff1.w, transposed=True)
                    self.weights.add(layer.ff2.w, transposed=True)
                self.ffn_bwd_slots[id(layer.ff1.w)] = (self.gmeta.slot(f"gs:{id(layer)}"),
                                                       self.gmeta.slot(f"gh:{id(layer)}"))

        def proj(w, feeder_ln) -> None:
            self.weights.add(w)
            xs = self.meta.slot("p:" + w.name)
            self.proj_slots[id(w)] = xs
            self.out_slots[id(w)] = self.meta.slot("y:" + w.name)
            if feeder_ln is not None:
                self.ln_slots[id(feeder_ln.gamma)] = xs

        enc, dec = list(model.enc_layers), list(model.dec_layers)
        for i, layer in enumerate(enc):
            proj(layer.qkv.w, enc[i - 1].ln2 if i else None)
        for i, layer in enumerate(dec):
            proj(layer.qkv1.w, dec[i - 1].ln3 if i else None)
            proj(layer.q2.w, layer.ln1)
        proj(model.cross_kv.w, enc[-1].ln2)

        # fp8 attention projections (ATTN_PROJ_FP8, with `backward`): the
        # output projection runs e4m3 in the forward (input: the attention
        # output, quantised once -- `attn_out`: weight -> (O slot, e5m2 slot
        # of its output gradient ds)) and its dgrad / weight gradient on the
        # e5m2 ds the LayerNorm backward emits; the input projections' dgrad
        # and weight gradient run on the e5m2 copy of the attention backward's
        # dQ|dK|dV (`proj_bwd`: weight -> e5m2 slot) against the e4m3 weights
        # (DGRAD_PLAIN_W: the forward's copies, read N-contiguous) and the
        # forward's e4m3 input
        self.attn_out: Dict[int, Tuple[int, int]] = {}
        self.attn_bwd8: Dict[int, Tuple[int, int]] = {}
        self.proj_bwd: Dict[int, int] = {}
        if backward and ATTN_PROJ_FP8:
            outs = [l.o.w for l in enc] + [w for l in dec for w in (l.o1.w, l.o2.w)]
            for w in outs:
                self.weights.add(w)
                if not DGRAD_PLAIN_W:
                    self.weights.add(w, transposed=True)
                self.attn_out[id(w)] = (self.meta.slot("o:" + w.name), self.gmeta.slot("go:" + w.name))
                # fp8 attention backward of this block: e5m2 dO and dS slots
                self.attn_bwd8[id(w)] = (self.gmeta.slot("gdo:" + w.name), self.gmeta.slot("gds:" + w.name))
            ins = [l.qkv.w for l in enc] + [w for l in dec for w in (l.qkv1.w, l.q2.w)] + [model.cross_kv.w]
            for w in ins:
                if not DGRAD_PLAIN_W:
                    self.weights.add(w, transposed=True)
                self.proj_bwd[id(w)] = self.gmeta.slot("gp:" + w.name)
        self.weights.calibrate()

    def linear(self, x2: torch.Tensor, w, b, want8: bool = False, keep_x8: Optional[list] = None,
               want_y: bool = True):
        """y = x2 @ w^T + b with e4m3 operands when `w` is an fp8 attention
        projection (the input's e4m3 copy comes from its LayerNorm, else it is
        quantised here); None otherwise. want8: also the e4m3 copy of y from
        the GEMM epilogue -- returns (y, y8, scale slot of y8); want_y = False
        (with want8): y is not written (None) -- its consumers all read y8.
        keep_x8 (a list): receives (x8, its scale slot) for the fp8 weight
        gradient."""
        xs = self.proj_slots.get(id(w))
        if xs is None:
            return None
        w8, ws = self.weights.get(w)
        x8 = self.stash.pop(xs, None)
        if x8 is None:
            x8 = quantize(x2, self.meta, xs)
        x8 = x8.view(x2.shape)
        if keep_x8 is not None:
            keep_x8[:] = [x8, xs]
        ys = self.out_slots[id(w)] if want8 else None
        # want8: y is the dequantised y8 (the attention backward reads y and
        # must see the operands the e4m3 attention forward used)
        if want8 and not want_y:
            y, y8 = gemm_fp8(x8, w8, b.master, self.meta, xs, ws, out8_slot=ys, want_y=False)
        else:
            y, y8 = gemm_fp8(x8, w8, b.master, self.meta, xs, ws, out8_slot=ys, c_deq=want8)
        return (y, y8, ys) if want8 else y

    def o8_for(self, w, shape, device):
        """(o8, scale, amax) for the e4m3 attention forward to emit the e4m3
        copy of its output straight into (the input of output projection w),
        or None when w's projection is not e4m3."""
        sl = self.attn_out.get(id(w))
        if sl is None:
            return None
        return (torch.empty(shape, dtype=FP8, device=device), self.meta.s(sl[0]), self.meta.a(sl[0]))

    def out_proj(self, o2: torch.Tensor, w, b, o8: Optional[torch.Tensor] = None):
        """Attention output projection in e4m3 (ATTN_PROJ_FP8): o2 quantised
        once (its e4m3 copy also feeds the weight gradient) unless the
        attention forward already emitted it (o8, see o8_for). Returns
        (s, o8) or None when w is not covered."""
        sl = self.attn_out.get(id(w))
        if sl is None:
            return None
        if o8 is None:
            o8 = quantize(o2.contiguous(), self.meta, sl[0]).view(o2.shape)
        else:
            o8 = o8.view(o2.shape)
        w8, ws = self.weights.get(w)
        s, _ = gemm_fp8(o8, w8, b.master, self.meta, sl[0], ws)
        return s, o8

    def after_step(self) -> None:
        self.meta.update()
        self.gmeta.update()
        self.weights.refresh()

    def before_fused_opt(self) -> None:
        """Scale update ahead of an optimizer step that refreshes the e4m3
        weight copies itself (Adam.apply(fp8w=...)): the same scales as
        after_step(), which runs the update after the optimizer (neither
        reads anything the optimizer writes)."""
        self.meta.update()
        self.gmeta.update()


load_tuned(TUNED_FILE)
