"""Embedding backward paths back to back at several (tokens, vocab, d)
shapes, for rocprofv3 kernel traces: the CSR kernels (sort / gather /
combine) against the fixed-point atomic kernels."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorflow_distributed_on_gke_amd.ops import kernels as kk  # noqa: E402

dev = "cuda"
for M, V, D, pad in [(1024, 1000, 512, 0.0), (8192, 1000, 512, 0.0), (8192, 7765, 512, 0.0),
                     (8192, 7765, 512, 0.35), (8192, 7765, 128, 0.35), (16384, 7765, 512, 0.35)]:
    g = torch.Generator().manual_seed(M + V)
    tok = torch.randint(1, V, (M,), generator=g)
    tok[: int(pad * M)] = 0
    tok = tok.view(-1, 128 if M >= 128 else M).to(dev)
    dout = (torch.randn(M, D, generator=g) * 0.1).to(torch.bfloat16).to(dev)
    ctr = torch.zeros(1, dtype=torch.int64, device=dev)
    dt = torch.zeros(V, D, device=dev)
    for csr in (True, False):
        kk.EMBED_CSR = csr
        for _ in range(20):
            kk.embed_bwd(tok, dout, dt, math.sqrt(D), 0.1, 1, ctr, 3)
        torch.cuda.synchronize()
    print(f"M={M} V={V} D={D} pad={pad} done", flush=True)

# phase clocks of the sort (s_memrealtime, 100 MHz): wave 0's view
for M, V, pad in [(8192, 1000, 0.0), (8192, 7765, 0.0), (8192, 7765, 0.35)]:
    g = torch.Generator().manual_seed(M + V)
    tok = torch.randint(1, V, (M,), generator=g)
    tok[: int(pad * M)] = 0
    tok = tok.to(dev)
    st = torch.zeros(1024, dtype=torch.int64, device=dev)
    for _ in range(3):
        kk.embed_csr_sort([(tok, V, "lab")], stamps=st)
    torch.cuda.synchronize()
    t = st.view(2, 8, 64)[0, :6, 0].cpu()
    print(f"sort M={M} V={V} pad={pad}: phases (us) " + " ".join(f"{(t[i + 1] - t[i]).item() / 100:.2f}" for i in range(5)), flush=True)
