#!/usr/bin/env python3
"""Diagnostics: dump x_save / gate_save of one forward (training) to an .npy file.
    python scripts/diag_dump_save.py points out.npz"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnot-replication_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gnot_amd import GNOT  # noqa: E402

N = int(sys.argv[1])
d, E, L, M, NL = 256, 8, 4, 805, 5
dev = torch.device("cuda")
torch.manual_seed(1234)
model = GNOT(3, 1, 3, 1, L, d, 4, d, d, E, 8, 1).to(dev)
g = torch.Generator(device="cpu").manual_seed(100)
x = torch.rand(N, 3, generator=g).to(dev)
theta = torch.rand(1, 1, generator=g).to(dev)
fns = [torch.rand(M, 3, generator=g).to(dev)]
out = model.forward_packed(x, [0, N], theta, fns, [[0, M]])
torch.cuda.synchronize()
eng = model.engine()
np.savez(sys.argv[2], x_save=eng.debug_tensor("x_save", NL * N, d).cpu().numpy(),
         gate_save=eng.debug_tensor("gate_save", NL * N, d).cpu().numpy(), out=out.detach().cpu().numpy())
