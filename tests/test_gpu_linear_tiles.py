"""Projection-kernel tile variants (linear.hip, GNOT_LINEAR_OC): the default cfg2 choice is 4 output
tiles per workgroup; 1, 2 and 8 are the measured alternatives.  Each variant
runs GNOT forward + backward through the HIP engine in a child process (the knob is read once per
process) and must match the CPU oracle at the same bar as the main parity suite."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CFG = dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=2, n_attn_layers=1, d=128,
           n_mlp_num_layers=2, n_expert=2, n_head=8, n_input_functions=1)
NS, MS = [173, 90], [[41, 30]]


def _child(oc, q):
    os.environ["GNOT_LINEAR_OC"] = str(oc)
    sys.path[:0] = [ROOT, os.path.join(ROOT, "gnot-replication_amd"), os.path.join(ROOT, "tests")]
    try:
        from golden_util import check_parity, model_args
        from gnot_amd import GNOT
        from test_gpu_shard import _case
        fx = _case(CFG, NS, MS, seed=5)
        dev = torch.device("cuda", 0)
        m = GNOT(*model_args(CFG)).to(dev)
        m.load_state_dict({k: torch.from_numpy(v).float() for k, v in fx["params"].items()})
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).float().to(dev)
        out = m.forward_packed(t(fx["x"]), fx["x_off"].tolist(), t(fx["theta"]), [t(f) for f in fx["fns"]],
                               [o.tolist() for o in fx["fn_offs"]])
        (out * t(fx["G"])).sum().backward()
        torch.cuda.synchronize()
        grads = {k: p.grad.double().cpu().numpy() for k, p in m.named_parameters()}
        q.put(check_parity(out.detach().double().cpu().numpy(), grads, fx))
    except Exception as e:
        q.put([f"exception: {e!r}"])
        raise


@pytest.mark.parametrize("oc", [1, 2, 8])
def test_linear_tile_variant_matches_oracle(oc):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(oc, q))
    p.start()
    errs = q.get(timeout=100)
    p.join(timeout=30)
    assert p.exitcode == 0, p.exitcode
    assert not errs, errs
