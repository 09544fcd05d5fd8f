#!/usr/bin/env python3
"""Diagnostics: run the same fwd+bwd twice and list the parameter gradients that differ bitwise.
    python scripts/diag_determinism.py [points] [d] [experts]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnot-replication_amd")]
import torch  # noqa: E402

from gnot_amd import GNOT  # noqa: E402
from gnot_amd import train as gtrain  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
d = int(sys.argv[2]) if len(sys.argv) > 2 else 256
E = int(sys.argv[3]) if len(sys.argv) > 3 else 8
M = 805
dev = torch.device("cuda")
torch.manual_seed(1234)
model = GNOT(3, 1, 3, 1, 4, d, 4, d, d, E, 8, 1).to(dev)
g = torch.Generator(device="cpu").manual_seed(100)
x = torch.rand(N, 3, generator=g).to(dev)
theta = torch.rand(1, 1, generator=g).to(dev)
fns = [torch.rand(M, 3, generator=g).to(dev)]
y = torch.sin(3.0 * x.sum(1, keepdim=True))
loss_fn = gtrain.RelL2Loss()
names = [n for n, _ in model.named_parameters()]


def step():
    model.zero_grad(set_to_none=True)
    out = model.forward_packed(x, [0, N], theta, fns, [[0, M]])
    out.retain_grad()
    loss_fn([0, N], out, y).backward()
    torch.cuda.synchronize()
    eng = model.engine()
    dbg = {k: eng.debug_tensor(k, N, d) for k in ("dquery", "dsum0", "dsum1", "dres", "du0")}
    return [p.grad.detach().clone() for p in model.parameters()], out.grad.detach().clone(), dbg


ref, dref, bref = step()
for rep in range(2):
    g2, d2, b2 = step()
    same = [n for n, a, b in zip(names, ref, g2) if torch.equal(a, b)]
    bad = [(n, float((a - b).abs().max()), float(a.abs().max())) for n, a, b in zip(names, ref, g2) if not torch.equal(a, b)]
    print(f"rep {rep}: {len(bad)} of {len(names)} gradients differ; dpred equal: {torch.equal(dref, d2)}; "
          + ", ".join(f"{k} equal: {torch.equal(bref[k], b2[k])}" for k in bref), flush=True)
    print("   identical:", same)
    for n, dmax, amax in bad[-12:]:
        print(f"   {n}: max|diff| {dmax:.3e} (max|g| {amax:.3e})")
