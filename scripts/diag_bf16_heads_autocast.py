#!/usr/bin/env python3
"""The reference's own bf16 error at a given head width (CPU diagnostic, no GPU).

Runs the stock-torch port (oracle/torch_port.py, the reference's op sequence) under
torch.autocast('cpu', bfloat16) -- model.py run in bf16 autocast -- and in float64 on the same random
model / mesh, and prints the norm-wise relative error of the output and of all parameter gradients
concatenated (the measure tests/test_gpu_bf16.py applies to the engine's bf16 mode), per head count.

    python scripts/diag_bf16_heads_autocast.py [d] [H ...]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnot-replication_amd"), os.path.join(ROOT, "tests")]

from golden_util import model_args  # noqa: E402
from oracle import torch_port  # noqa: E402


def run(cfg, Ns, Ms, seed, autocast):
    from gnot_amd import GNOT
    torch.manual_seed(seed)
    ref = GNOT(*model_args(cfg))
    dt = torch.float32 if autocast else torch.float64
    sd = {k: v.detach().to(dt).clone().requires_grad_(True) for k, v in ref.state_dict().items()}
    # the data of tests/test_gpu_parity.py _random_case (same seed, same draws)
    rng = np.random.default_rng(seed)
    xa = rng.random((sum(Ns), cfg["input_dim"]))
    tha = rng.random((len(Ns), cfg["theta_dim"]))
    fa = [rng.random((sum(Ms[i]), cfg["input_func_dim"])) for i in range(cfg["n_input_functions"])]
    Ga = rng.standard_normal((sum(Ns), cfg["out_dim"]))
    xo = np.concatenate([[0], np.cumsum(Ns)])
    fo = [np.concatenate([[0], np.cumsum(Ms[i])]) for i in range(cfg["n_input_functions"])]
    outs = []
    loss = 0.0
    for b, n in enumerate(Ns):
        x = torch.tensor(xa[xo[b]:xo[b + 1]][None], dtype=dt)
        th = torch.tensor(tha[b:b + 1], dtype=dt)
        fs = [torch.tensor(fa[i][fo[i][b]:fo[i][b + 1]][None], dtype=dt) for i in range(cfg["n_input_functions"])]
        G = torch.tensor(Ga[xo[b]:xo[b + 1]][None], dtype=dt)
        with torch.autocast("cpu", dtype=torch.bfloat16, enabled=autocast):
            out = torch_port.gnot_forward(sd, cfg, x, th, fs)
        out = out.to(dt)
        outs.append(out.detach().double().numpy().ravel())
        loss = loss + (out * G).sum()
    loss.backward()
    return np.concatenate(outs), {k: sd[k].grad.double().numpy() for k in sd}


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


if __name__ == "__main__":
    d = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    Hs = [int(h) for h in sys.argv[2:]] or [8, 2, 1]
    for H in Hs:
        cfg = dict(input_dim=3, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=2, d=d,
                   n_mlp_num_layers=4, n_expert=3, n_head=H, n_input_functions=1)
        o64, g64 = run(cfg, [900, 300], [[200, 77]], 23, False)
        o16, g16 = run(cfg, [900, 300], [[200, 77]], 23, True)
        cat = lambda g: np.concatenate([g[k].ravel() for k in sorted(g)])
        print(f"d={d} H={H} dh={d // H}: autocast bf16 vs float64: output {rel(o16, o64):.2e}, "
              f"parameter gradients {rel(cat(g16), cat(g64)):.2e}", flush=True)
        tot = np.linalg.norm(cat(g64))
        share = sorted(((np.linalg.norm(g16[k] - g64[k]) / tot, rel(g16[k], g64[k]), np.linalg.norm(g64[k]) / tot, k)
                        for k in g64), reverse=True)
        for s_, r_, n_, k in share[:8]:
            print(f"  err/|g| {s_:.2e}  rel {r_:.2e}  |g_k|/|g| {n_:.2e}  {k}")
