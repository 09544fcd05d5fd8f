#!/usr/bin/env python3
"""Diagnostic (GPU box): is the cfg2 training step host-bound, and does a hipGraph of the whole step
(pack + forward + RelL2 + backward + fused AdamW) capture, replay correctly and run faster?"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnot-replication_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from gnot_amd import GNOT  # noqa: E402

dev = torch.device("cuda", 0)
w = bench.WORKLOADS["cfg2"]
m = w["model"]
args = [m[k] for k in ("input_dim", "theta_dim", "input_func_dim", "out_dim", "n_attn_layers", "n_attn_hidden_dim",
                       "n_mlp_num_layers", "n_mlp_hidden_dim", "n_input_hidden_dim", "n_expert", "n_head",
                       "n_input_functions")]


def setup(capturable):
    torch.manual_seed(1234)
    model = GNOT(*args).to(dev)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3, fused=True, capturable=capturable)
    x, x_off, theta, fns, fn_offs, y, seg = bench.make_batch(w, 100, dev)

    def step():
        out = model.forward_packed(x, x_off, theta, fns, fn_offs)
        loss = bench.rel_l2_loss(out, y, seg, w["B"])
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss
    return model, step


K = 30
model, step = setup(False)
for _ in range(5):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
host = []
for _ in range(K):
    h0 = time.perf_counter()
    step()
    host.append(time.perf_counter() - h0)
torch.cuda.synchronize()
eager = (time.perf_counter() - t0) / K
print(f"eager: {eager * 1e3:.3f} ms/step, host enqueue {sum(host) / K * 1e3:.3f} ms/step", flush=True)
l_eager = [float(step()) for _ in range(3)]

model, step = setup(True)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(5):
        step()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    static_loss = step()
torch.cuda.synchronize()
print("captured", flush=True)
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    g.replay()
torch.cuda.synchronize()
gt = (time.perf_counter() - t0) / K
print(f"graph: {gt * 1e3:.3f} ms/step -> {w['N'] / gt / 1e6:.3f} M pts/s (eager {w['N'] / eager / 1e6:.3f})", flush=True)

# correctness: graph replays vs eager steps from the same initial state follow the same loss curve
model_e, step_e = setup(True)
ref = [float(step_e()) for _ in range(8)]
model_g, step_g = setup(True)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    first = [float(step_g()) for _ in range(3)]
torch.cuda.current_stream().wait_stream(s)
g2 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g2):
    sl = step_g()
got = list(first)
for _ in range(5):
    g2.replay()
    got.append(float(sl))
print("eager loss:", [f"{v:.6f}" for v in ref])
print("graph loss:", [f"{v:.6f}" for v in got])
