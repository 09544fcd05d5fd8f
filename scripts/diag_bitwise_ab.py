#!/usr/bin/env python3
"""Bitwise A/B of two builds of libgnot_hip.so on the same inputs (a refactor must not change one bit).

    GNOT_LIB=<a.so> python scripts/diag_bitwise_ab.py dump gpurun_out/a.npz
    GNOT_LIB=<b.so> python scripts/diag_bitwise_ab.py dump gpurun_out/b.npz
    python scripts/diag_bitwise_ab.py compare gpurun_out/a.npz gpurun_out/b.npz

Each case runs one training forward + backward (sum(out * G)) and stores the output and the flat gradient
arena: d = 256 / E = 8 (configs[2]'s widths) in fp32, bf16 mode and with MoE recompute, d = 128 / E = 4 /
two input functions (configs[1]'s) in fp32 and bf16 mode, and d = 64 (chain.hip).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnot-replication_amd")]

CASES = [
    # name, (input, theta, fn, out, L, d, nl, E, H, I), P, precision, recompute
    ("d256_fp32", (3, 1, 3, 1, 2, 256, 4, 8, 8, 1), 20000, "fp32", False),
    ("d256_bf16", (3, 1, 3, 1, 2, 256, 4, 8, 8, 1), 20000, "bf16", False),
    ("d256_recompute", (3, 1, 3, 1, 2, 256, 4, 8, 8, 1), 20000, "fp32", True),
    ("d128_fp32", (2, 1, 3, 1, 2, 128, 4, 4, 8, 2), 10000, "fp32", False),
    ("d128_bf16", (2, 1, 3, 1, 2, 128, 4, 4, 8, 2), 10000, "bf16", False),
    ("d64_fp32", (2, 1, 3, 2, 2, 64, 3, 3, 4, 1), 3000, "fp32", False),
]


def dump(path):
    import torch
    from gnot_amd import GNOT
    dev = torch.device("cuda")
    res = {}
    for name, (i, t, f, o, L, d, nl, E, H, I), P, prec, rec in CASES:
        torch.manual_seed(5)
        m = GNOT(i, t, f, o, L, d, nl, d, d, E, H, I).to(dev)
        m.set_precision(prec)
        m.set_moe_recompute(rec)
        g = torch.Generator(device="cpu").manual_seed(6)
        x_off = [0, P // 3, P]
        x = torch.rand(P, i, generator=g).to(dev)
        th = torch.rand(2, t, generator=g).to(dev)
        fns = [torch.rand(500, f, generator=g).to(dev) for _ in range(I)]
        G = torch.randn(P, o, generator=g).to(dev)
        out = m.forward_packed(x, x_off, th, fns, [[0, 200, 500]] * I)
        (out * G).sum().backward()
        torch.cuda.synchronize()
        res[name + ".out"] = out.detach().cpu().numpy()
        res[name + ".grad"] = m.engine().grad_flat.detach().cpu().numpy()
        print(name, "done", flush=True)
    np.savez(path, **res)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in A.files:
        same = np.array_equal(A[k], B[k])
        print(f"{k:24s} {'bitwise equal' if same else 'DIFFERS max %.3e' % np.abs(A[k] - B[k]).max()}")
        bad += not same
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        compare(sys.argv[2], sys.argv[3])
