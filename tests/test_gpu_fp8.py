"""FP8 (OCP e4m3) path: quantisation vs torch's float8_e4m3fn, the block-scaled
MFMA GEMM vs an fp32 reference of the dequantised operands, the fused fp8
epilogue output, delayed scaling, and an fp8 training run vs bf16."""
import pytest
import torch

from tensorflow_distributed_on_gke_amd.ops import fp8 as F
from tensorflow_distributed_on_gke_amd.ops._ext import C

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_quantize_matches_torch_e4m3():
    meta = F.Fp8Meta(DEV)
    i = meta.slot("x")
    meta.scale[i] = 37.0
    x = (torch.randn(1000, 96, device=DEV) * 3).bfloat16()
    x[0, 0] = 100.0  # saturates at 448 after scaling
    x8 = F.quantize(x, meta, i)
    ref = (x.float() * 37.0).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert (x8.view(torch.uint8) == ref.view(torch.uint8)).float().mean().item() > 0.999
    assert abs(meta.amax_values()[i].item() - x.float().abs().max().item()) < 1e-6
    meta.update()
    assert abs(meta.scale[i].item() - 448.0 / x.float().abs().max().item()) < 1e-3
    assert meta.amax_values()[i].item() == 0.0


@pytest.mark.parametrize("M,N,K", [(512, 384, 256), (333, 1000, 512), (8192, 2048, 512), (64, 64, 128)])
@pytest.mark.parametrize("epi", [0, 1, 2])
def test_gemm_fp8(M, N, K, epi):
    torch.manual_seed(0)
    meta = F.Fp8Meta(DEV)
    ia, ib, io = meta.slot("a"), meta.slot("b"), meta.slot("o")
    meta.scale[ia], meta.scale[ib], meta.scale[io] = 60.0, 900.0, 4.0
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    bias = torch.randn(N, device=DEV) if epi else None
    a8, b8 = F.quantize(a, meta, ia), F.quantize(b, meta, ib)
    ref = (a8.float() / 60.0) @ (b8.float() / 900.0).t()
    if epi:
        ref = ref + bias
    if epi == 2:
        ref = ref.relu()
    for cfg in F._CANDS:
        y, y8 = F.gemm_fp8(a8, b8, bias, meta, ia, ib, relu=epi == 2, out8_slot=io, cfg=cfg)
        err = (y.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
        assert err < 1e-2, (cfg, err)
        want8 = (y.float() * 4.0).clamp(-448, 448).to(torch.float8_e4m3fn)
        assert (y8.view(torch.uint8) == want8.view(torch.uint8)).float().mean().item() > 0.999
    assert abs(meta.amax_values()[io].item() - y.float().abs().max().item()) <= 1e-3 * y.float().abs().max().item()


def test_fp8_training_tracks_bf16():
    from tensorflow_distributed_on_gke_amd.data.synthetic import SyntheticPairs
    from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config
    from tensorflow_distributed_on_gke_amd.train.optim import Adam
    from tensorflow_distributed_on_gke_amd.train.step import TrainStep

    cfg = model_config("tiny", src_vocab=64, tgt_vocab=64, dropout=0.0)
    data = SyntheticPairs(batch=32, src_len=16, tgt_len=17, src_vocab=64, tgt_vocab=64, copy_task=True, seed=0)
    finals = {}
    for mode in ("bf16", "fp8"):
        m = Transformer(cfg).build("cuda", seed=1)
        opt = Adam(m.store, cfg.d_model, lr=1e-3)
        st = F.Fp8State(m) if mode == "fp8" else None
        step = TrainStep(m, opt, None, workers=1.0, seed=3, fp8_state=st)
        losses = []
        for i in range(150):
            src, tgt = data.batch(i)
            losses.append(step(src.cuda(), tgt.cuda())[0].item())
        finals[mode] = (losses[0], sum(losses[-10:]) / 10)
    (b0, b1), (f0, f1) = finals["bf16"], finals["fp8"]
    assert b1 < 0.75 * b0 and f1 < 0.75 * f0, finals
    assert abs(f1 - b1) < 0.1 * b1 + 0.05, finals


@pytest.mark.parametrize("D", [128, 512, 1024])
def test_layernorm_fused_fp8_copy(D):
    from tensorflow_distributed_on_gke_amd.ops import kernels as kk
    meta = F.Fp8Meta(DEV)
    i = meta.slot("y")
    meta.scale[i] = 50.0
    x = torch.randn(777, D, device=DEV).bfloat16()
    s = torch.randn(777, D, device=DEV).bfloat16()
    g, b = torch.rand(D, device=DEV) + 0.5, torch.randn(D, device=DEV)
    y8 = torch.empty(777, D, dtype=F.FP8, device=DEV)
    y, *_ = kk.ln_fwd(x, s, g, b, 0.0, 0, None, 0, y8=y8, s8=meta.s(i), amax8=meta.a(i))
    want = (y.float() * 50.0).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert (y8.view(torch.uint8) == want.view(torch.uint8)).float().mean().item() > 0.999
    assert abs(meta.amax_values()[i].item() - y.float().abs().max().item()) < 1e-6 * D
