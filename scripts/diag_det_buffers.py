#!/usr/bin/env python3
"""Diagnostics: which workspace buffers differ bitwise between two identical forward(+backward) runs.
    python scripts/diag_det_buffers.py [points]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnot-replication_amd")]
import torch  # noqa: E402

from gnot_amd import GNOT  # noqa: E402
from gnot_amd import train as gtrain  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
d, E, L, M = 256, 8, 4, 805
dev = torch.device("cuda")
torch.manual_seed(1234)
model = GNOT(3, 1, 3, 1, L, d, 4, d, d, E, 8, 1).to(dev)
g = torch.Generator(device="cpu").manual_seed(100)
x = torch.rand(N, 3, generator=g).to(dev)
theta = torch.rand(1, 1, generator=g).to(dev)
fns = [torch.rand(M, 3, generator=g).to(dev)]
y = torch.sin(3.0 * x.sum(1, keepdim=True))
loss_fn = gtrain.RelL2Loss()
names = ["x", "xin", "scores", "gate_save", "x_save", "out_save", "query0", "fn_save0", "fnenc0", "stage",
         "dscore", "dout", "dquery", "dsum0", "dsum1", "dres", "dqkv0", "dqkv1", "du0", "dden0", "dstate0", "dfn0",
         "dz0", "dz1", "dzf", "grads", "slab_wgrad", "slab_state"]
for l in range(L):
    names += [f"b{l}.{k}" for k in ("cq", "ckv0", "cstate0", "cres", "a", "m1save", "query1", "sq", "sstate", "sres",
                                    "bb", "m2save", "query2")]
    names += [f"dstate{l}_0", f"dkv{l}_0"]


def sig(eng):
    ws = eng.ws
    ptrs = []
    for n in names:
        try:
            ptrs.append((eng.debug_ptr(n)[0] - ws.data_ptr(), n))
        except Exception:
            pass
    ptrs.sort()
    out = {}
    for i, (o, n) in enumerate(ptrs):
        e = ptrs[i + 1][0] if i + 1 < len(ptrs) else o + 4096
        t = ws[o: o + ((e - o) // 8) * 8].view(torch.int64)
        out[n] = (int(t.sum()), int((t * 2654435761).sum()))
    return out


def run(bwd):
    model.zero_grad(set_to_none=True)
    out = model.forward_packed(x, [0, N], theta, fns, [[0, M]])
    if bwd:
        loss_fn([0, N], out, y).backward()
    torch.cuda.synchronize()
    return sig(model.engine())


if len(sys.argv) > 2:          # dump the signatures (compare two library builds across processes)
    import json
    json.dump({"fwd": run(False), "fwd+bwd": run(True)}, open(sys.argv[2], "w"))
    sys.exit(0)
for bwd in (False, True):
    a = run(bwd)
    b = run(bwd)
    diff = [n for n in a if a[n] != b[n]]
    print(f"{'fwd+bwd' if bwd else 'fwd'}: {len(diff)} of {len(a)} buffers differ: {diff}", flush=True)
