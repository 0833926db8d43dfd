"""Per-parameter relative gradient error GPU (bf16) vs CPU (f32) — diagnostic."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
from test_gpu_model import _batch, _rel
from tensorflow_distributed_on_gke_amd.models.layers import RunCtx
from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config

for preset, kw in (("reference", dict(src_vocab=7765, tgt_vocab=7010)), ("tiny", dict(src_vocab=300, tgt_vocab=250))):
    for dropout in (0.0, 0.1):
        cfg = model_config(preset, dropout=dropout, **kw)
        gpu = Transformer(cfg).build("cuda", seed=11)
        cpu = Transformer(cfg).build("cpu", seed=11)
        cpu.store.flat.copy_(gpu.store.flat_compute.float().cpu())
        src, tgt = _batch(6, 40, 33, cfg.src_vocab, cfg.tgt_vocab, seed=5)
        outs = []
        for m, dev in ((gpu, "cuda"), (cpu, "cpu")):
            rt = RunCtx(training=True, dropout=dropout, seed=99,
                        ctr=torch.tensor([2], dtype=torch.int64, device=dev), store=m.store)
            outs.append(m.loss_and_backward(src.to(dev), tgt.to(dev), rt, workers=1.0).cpu())
        print(f"== {preset} dropout={dropout} loss gpu {outs[0].tolist()} cpu {outs[1].tolist()}")
        errs = [(p_g.name, _rel(p_g.grad, p_c.grad), p_c.grad.norm().item()) for p_g, p_c in zip(gpu.store.params, cpu.store.params)]
        for n, e, g in errs:
            print(f"  {e:.4f} |g|={g:.3e} {n}")
