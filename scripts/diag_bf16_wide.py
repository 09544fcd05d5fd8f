#!/usr/bin/env python3
"""Per-tensor errors of the bf16 mode against the float64 oracle at a given (d, H) (GPU diagnostic).

    python scripts/diag_bf16_wide.py <d> <H> [fp32|bf16]

Prints the output error and the 12 parameter gradients with the largest relative errors, on the
tests/test_gpu_bf16.py wide-head case (2 blocks, 3 experts, one input function, meshes 900 + 300).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnot-replication_amd"), os.path.join(ROOT, "tests")]

from test_gpu_configs import CFG_3D  # noqa: E402
from test_gpu_parity import _random_case, build_model, run_packed  # noqa: E402


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


if __name__ == "__main__":
    d, H = int(sys.argv[1]), int(sys.argv[2])
    prec = sys.argv[3] if len(sys.argv) > 3 else "bf16"
    cfg = dict(CFG_3D, d=d, n_head=H, n_attn_layers=2, n_expert=3)
    fx, G = _random_case(23, cfg, [900, 300], [[200, 77]])
    m = build_model(fx["params"], fx["cfg"])
    m.set_precision(prec)
    out, g = run_packed(m, fx, G)
    print(f"d={d} H={H} {prec}: output {rel(out, fx['out']):.2e}")
    ks = sorted(fx["grads"])
    cat = lambda g: np.concatenate([g[k].ravel() for k in ks])
    tot = np.linalg.norm(cat(fx["grads"]))
    print(f"  parameter gradients {rel(cat(g), cat(fx['grads'])):.2e}")
    share = sorted(((np.linalg.norm(g[k] - fx["grads"][k]) / tot, rel(g[k], fx["grads"][k]),
                     np.linalg.norm(fx["grads"][k]) / tot, k) for k in ks), reverse=True)
    for s_, r_, n_, k in share[:8]:
        print(f"  err/|g| {s_:.2e}  rel {r_:.2e}  |g_k|/|g| {n_:.2e}  {k}")
