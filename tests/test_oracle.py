"""The CPU oracle (oracle/gnot_oracle.py) against the reference's golden fixtures."""
import numpy as np
import pytest

from golden_util import check_parity, fixture_names, load
from oracle import gnot_oracle as O


@pytest.mark.parametrize("name", fixture_names())
def test_oracle_fp64_matches_reference(name):
    fx = load(name)
    out, grads = O.gnot_forward_backward(fx["params"], fx["cfg"], fx["x"], fx["x_off"], fx["theta"], fx["fns"],
                                         fx["fn_offs"], G=fx["G"], dtype=np.float64)
    assert np.abs(out - fx["out"]).max() <= 1e-12 * max(1.0, np.abs(fx["out"]).max())
    errs = check_parity(out, grads, fx, rtol=1e-9, slack=0.0)
    # cancellation-only tensors (see golden_util) are exempt at this tolerance, not the rest
    errs = [e for e in errs if not any(t in e for t in ("key", "query"))]
    assert not errs, errs


@pytest.mark.parametrize("name", ["cross1_sharp", "main_pad_h8"])
def test_oracle_fp32_within_reference_tolerance(name):
    fx = load(name)
    out, grads = O.gnot_forward_backward(fx["params"], fx["cfg"], fx["x"], fx["x_off"], fx["theta"], fx["fns"],
                                         fx["fn_offs"], G=fx["G"], dtype=np.float32)
    assert not check_parity(out, grads, fx)


def test_padded_equals_per_sample():
    """A zero-padded batch is per-sample computation on the padded rows."""
    fx = load("main_pad_h8")
    out, _ = O.gnot_forward_backward(fx["params"], fx["cfg"], fx["x"], fx["x_off"], fx["theta"], fx["fns"],
                                     fx["fn_offs"])
    outs = []
    for b in range(len(fx["x_off"]) - 1):
        s, e = fx["x_off"][b], fx["x_off"][b + 1]
        fs = [f[o[b]:o[b + 1]] for f, o in zip(fx["fns"], fx["fn_offs"])]
        fo = [np.array([0, o[b + 1] - o[b]]) for o in fx["fn_offs"]]
        ob, _ = O.gnot_forward_backward(fx["params"], fx["cfg"], fx["x"][s:e], np.array([0, e - s]),
                                        fx["theta"][b:b + 1], fs, fo)
        outs.append(ob)
    assert np.allclose(np.concatenate(outs), out, rtol=0, atol=1e-14)


def test_padding_changes_real_outputs():
    """The reference does not mask padding: real-point outputs depend on the pad rows."""
    fx = load("cross2_packed")
    b0 = slice(fx["x_off"][0], fx["x_off"][1])
    fs = [f[o[0]:o[1]] for f, o in zip(fx["fns"], fx["fn_offs"])]
    fo = [np.array([0, o[1] - o[0]]) for o in fx["fn_offs"]]
    n = fx["x_off"][1]
    out0, _ = O.gnot_forward_backward(fx["params"], fx["cfg"], fx["x"][b0], np.array([0, n]), fx["theta"][:1], fs, fo)
    xp = np.concatenate([fx["x"][b0], np.zeros((9, fx["x"].shape[1]))])
    outp, _ = O.gnot_forward_backward(fx["params"], fx["cfg"], xp, np.array([0, n + 9]), fx["theta"][:1], fs, fo)
    assert np.abs(outp[:n] - out0).max() > 1e-10


@pytest.mark.parametrize("name", ["cross1_sharp", "self_only_pad", "cross2_packed"])
def test_torch_port_matches_fixtures(name):
    """The stock-torch CPU port timed as bench.py's cpu_baseline computes the reference's numbers."""
    import torch
    from oracle import torch_port
    fx = load(name)
    cfg = fx["cfg"]
    p = {k: torch.from_numpy(v).clone().requires_grad_(True) for k, v in fx["params"].items()}
    outs = []
    for b in range(len(fx["x_off"]) - 1):
        s, e = fx["x_off"][b], fx["x_off"][b + 1]
        x = torch.from_numpy(fx["x"][s:e])[None]
        fns = [torch.from_numpy(f[o[b]:o[b + 1]])[None] for f, o in zip(fx["fns"], fx["fn_offs"])]
        o = torch_port.gnot_forward(p, cfg, x, torch.from_numpy(fx["theta"][b:b + 1]), fns)[0]
        (o * torch.from_numpy(fx["G"][s:e])).sum().backward()
        outs.append(o.detach().numpy())
    grads = {k: v.grad.numpy() for k, v in p.items()}
    errs = check_parity(np.concatenate(outs), grads, fx, rtol=1e-9, slack=0.0)
    errs = [e for e in errs if not any(t in e for t in ("key", "query"))]
    assert not errs, errs
