#!/usr/bin/env python3
"""Where the bf16 input-gradient error comes from (CPU diagnostic, no GPU).

tests/test_gpu_input_grads.py's d256_I1 case (the bf16-mode row), on the stock-torch port of the
reference (oracle/torch_port.py) under torch.autocast('cpu', bfloat16), against float64 autograd:
  * autocast      -- the reference's own bf16 arithmetic everywhere;
  * fp32 first    -- the same, but the encoders' FIRST Linear (x and each input function: the products whose
                     backward-data gives d x / d theta / d fn) in fp32 (autocast off for that Linear only).
If the second does not bring d theta / d fn under 1e-2, forming the first-Linear backward-data from fp32
operands does not either: their error is carried in by the bf16 gradient arriving at that Linear.

    python scripts/diag_bf16_input_grads.py
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnot-replication_amd"), os.path.join(ROOT, "tests")]

from golden_util import model_args  # noqa: E402
from oracle import torch_port  # noqa: E402

CFG = dict(input_dim=3, theta_dim=2, input_func_dim=3, out_dim=1, n_attn_layers=1, d=256,
           n_mlp_num_layers=4, n_expert=2, n_head=8, n_input_functions=1)


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def grads(sd64, data, mode):
    """d x, d theta, d fn per sample: mode 'fp64', 'autocast' or 'fp32first'"""
    dt = torch.float64 if mode == "fp64" else torch.float32
    sd = {k: v.to(dt) for k, v in sd64.items()}
    first = {"x.layers.0.weight"} | {f"input_func_mlps.{i}.layers.0.weight" for i in range(CFG["n_input_functions"])}
    lin = F.linear

    def linear(h, w, b=None):
        if mode == "fp32first" and any(w is sd[k] for k in first):
            with torch.autocast("cpu", enabled=False):
                return lin(h.float(), w, b)
        return lin(h, w, b)

    out = []
    F.linear = linear
    try:
        for x, th, fns, G in data:
            xt = torch.tensor(x, dtype=dt)[None].requires_grad_(True)
            tt = torch.tensor(th, dtype=dt)[None].requires_grad_(True)
            ft = [torch.tensor(f, dtype=dt)[None].requires_grad_(True) for f in fns]
            with torch.autocast("cpu", dtype=torch.bfloat16, enabled=mode != "fp64"):
                o = torch_port.gnot_forward(sd, CFG, xt, tt, ft)
            (o[0].to(dt) * torch.tensor(G, dtype=dt)).sum().backward()
            out.append((xt.grad[0].double().numpy(), tt.grad[0].double().numpy(),
                        [f.grad[0].double().numpy() for f in ft]))
    finally:
        F.linear = lin
    return out


if __name__ == "__main__":
    from gnot_amd import GNOT
    torch.manual_seed(5)
    m = GNOT(*model_args(CFG))
    sd64 = {k: v.detach().double() for k, v in m.state_dict().items()}
    rng = np.random.default_rng(3)
    Ns, Ms = [300, 173], [[120, 77]]
    xs = [rng.random((n, CFG["input_dim"])) for n in Ns]
    ths = [rng.random(CFG["theta_dim"]) for _ in Ns]
    fns = [[rng.random((Ms[0][b], CFG["input_func_dim"]))] for b in range(len(Ns))]
    Gs = [rng.standard_normal((n, CFG["out_dim"])) for n in Ns]
    data = list(zip(xs, ths, fns, Gs))
    ref = grads(sd64, data, "fp64")
    cat = lambda g, k: np.concatenate([np.ravel(s[k]) if k < 2 else np.ravel(s[2][0]) for s in g])
    for mode in ("autocast", "fp32first"):
        g = grads(sd64, data, mode)
        print(f"{mode:10s}: d x {rel(cat(g, 0), cat(ref, 0)):.2e}  d theta {rel(cat(g, 1), cat(ref, 1)):.2e}  "
              f"d fn {rel(cat(g, 2), cat(ref, 2)):.2e}", flush=True)
