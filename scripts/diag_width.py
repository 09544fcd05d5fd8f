#!/usr/bin/env python3
"""Per-parameter relative gradient error of width cases against the float64 oracle (diagnostics for
tests/test_gpu_widths.py).  Args: case names of test_gpu_widths.CASES or d,H,E,I,L,nl tuples."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "gnot-replication_amd")]
import numpy as np  # noqa: E402

import test_gpu_widths as T  # noqa: E402
from test_gpu_parity import _random_case, build_model, run_packed  # noqa: E402

for name in sys.argv[1:]:
    if name in T.CASES:
        fx, G = T._case(name)
    else:
        d, H, E, I, L, nl = (int(v) for v in name.split(","))
        cfg = T._cfg(d, H, E, I, L=L, nl=nl)
        fx, G = _random_case(13, cfg, [300], [[120]] * I)
    m = build_model(fx["params"], fx["cfg"])
    out, grads = run_packed(m, fx, G)
    print(name, "out rel %.2e" % (np.linalg.norm(out - fx["out"]) / np.linalg.norm(fx["out"])))
    groups = {}
    for k in fx["grads"]:
        r = fx["grads"][k]
        e = np.linalg.norm(grads[k] - r) / max(np.linalg.norm(r), 1e-30)
        key = ".".join(k.split(".")[:3]) if k.startswith("blocks") else k.split(".")[0]
        groups[key] = max(groups.get(key, 0.0), e if np.linalg.norm(r) > 1e-8 else 0.0)
    print("   " + "  ".join(f"{k}={v:.1e}" for k, v in groups.items()))
