"""HIP path vs the CPU oracle at the BASELINE.json model configurations:
the widths, depths and expert counts of configs[0..4] at point counts the float64 oracle finishes in
seconds, plus configs[1]'s exact timed shape.  Tolerance: golden_util.check_parity (1e-4 relative,
fp32 vs the float64 oracle; per-tensor slack from the oracle's own fp32 error)."""
import numpy as np
import pytest
import torch

from golden_util import check_parity
from test_gpu_parity import _random_case, build_model, run_packed

pytestmark = pytest.mark.gpu

# main.py defaults (configs[0], configs[4]) and the 3-D configs[2] / configs[3] model
CFG_MAIN = dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=4, d=256,
                n_mlp_num_layers=4, n_expert=3, n_head=8, n_input_functions=1)
CFG_3D = dict(input_dim=3, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=4, d=256,
              n_mlp_num_layers=4, n_expert=8, n_head=8, n_input_functions=1)
CFG_CFG2 = dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=4, d=128,
                n_mlp_num_layers=4, n_expert=4, n_head=8, n_input_functions=2)


def _port_forward_backward(params, cfg, x, theta, f, G, dt):
    """The reference's padded call (x [B,N,in], theta [B,th], one input function [B,M,F]) through the
    stock-torch port on the CPU: output [B*N, out] and every parameter gradient of sum(out * G)."""
    from oracle import torch_port
    torch.set_num_threads(min(16, torch.get_num_threads()))
    p = {k: torch.tensor(v, dtype=dt).requires_grad_(True) for k, v in params.items()}
    c = dict(cfg, n_attn_hidden_dim=cfg["d"])
    out = torch_port.gnot_forward(p, c, torch.tensor(x, dtype=dt), torch.tensor(theta, dtype=dt),
                                  [torch.tensor(f, dtype=dt)])
    (out * torch.tensor(G, dtype=dt)).sum().backward()
    return (out.detach().double().numpy().reshape(-1, out.shape[-1]),
            {k: v.grad.double().numpy() for k, v in p.items()})


@pytest.mark.timeout(300)
@pytest.mark.parametrize("Ns,Ms", [
    ([431, 600, 377, 512], [101, 64, 88, 97]),
    # the bench's configs[0] shape (bench.py --workload cfg1: 4 x 4,096 padded points, 805-point input
    # functions): real sizes inside BASELINE's 1-4k, padded to 4,096 and to one common M = 805.  16,384
    # padded points is the kernel selection the bench times: weight gradients forked onto the side stream,
    # expert grid + moe_combine pass, MFMA attention apply / K-V backward (>= 8,192 points per launch)
    ([4096, 1731, 2950, 1207], [805, 612, 805, 700]),
], ids=["small", "bench_shape"])
def test_configs0_padded_batch_of_4(Ns, Ms):
    """configs[0] (main.py widths) through the reference calling convention: a batch of 4 meshes
    zero-padded to the batch max N and one common max M (main.py:60-82, utils.py:3-4).  The pad rows
    are computed and enter the attention sums exactly as in the reference; the loss gradient is zero
    on them (main.py:89 drops them before the loss)."""
    rng = np.random.default_rng(7)
    B, Nmax, Mmax = len(Ns), max(Ns), max(Ms)
    # the padded arrays ARE the samples the reference sees: equal-stride offsets over the pad rows
    from gnot_amd import GNOT
    from golden_util import model_args
    torch.manual_seed(11)
    params = {k: v.double().numpy() for k, v in GNOT(*model_args(CFG_MAIN)).state_dict().items()}
    x = rng.random((B, Nmax, CFG_MAIN["input_dim"]))
    f = rng.random((B, Mmax, CFG_MAIN["input_func_dim"]))
    theta = rng.random((B, CFG_MAIN["theta_dim"]))
    fx = dict(params=params, cfg=CFG_MAIN, theta=theta, x_off=np.arange(B + 1, dtype=np.int64) * Nmax,
              fn_offs=[np.arange(B + 1, dtype=np.int64) * Mmax])
    for b in range(B):
        x[b, Ns[b]:] = 0.0
        f[b, Ms[b]:] = 0.0
    G = rng.standard_normal((B, Nmax, 1))
    for b in range(B):
        G[b, Ns[b]:] = 0.0
    if B * Nmax <= 4096:
        from oracle import gnot_oracle as O
        args = (fx["params"], fx["cfg"], x.reshape(B * Nmax, -1), fx["x_off"], fx["theta"], [f.reshape(B * Mmax, -1)],
                fx["fn_offs"])
        out64, g64 = O.gnot_forward_backward(*args, G=G.reshape(B * Nmax, -1))
        _, g32 = O.gnot_forward_backward(*args, G=G.reshape(B * Nmax, -1), dtype=np.float32)
    else:
        # the numpy oracle takes minutes at 16,384 points; the stock-torch port (pinned to the same reference
        # fixtures at 1e-9, tests/test_oracle.py) runs the reference's padded call in float64 in seconds
        out64, g64 = _port_forward_backward(params, CFG_MAIN, x, theta, f, G, torch.float64)
        _, g32 = _port_forward_backward(params, CFG_MAIN, x, theta, f, G, torch.float32)
    ref = dict(out=out64, grads=g64, e32={k: float(np.linalg.norm(g32[k].astype(np.float64) - g64[k])) for k in g64})

    m = build_model(fx["params"], fx["cfg"])
    dev = torch.device("cuda")
    out = m(torch.from_numpy(x).float().to(dev), torch.from_numpy(fx["theta"]).float().to(dev),
            torch.from_numpy(f).float().to(dev).unsqueeze(0))
    assert out.shape == (B, Nmax, 1)
    (out * torch.from_numpy(G).float().to(dev)).sum().backward()
    grads = {k: p.grad.double().cpu().numpy() for k, p in m.named_parameters()}
    errs = check_parity(out.detach().double().cpu().numpy().reshape(B * Nmax, -1), grads, ref)
    assert not errs, errs


def test_configs2_widths_single_mesh():
    """configs[2] / configs[3] model (3-D, d=256, 8 experts, 4 blocks, 4-layer MLPs, one input
    function of 805 points) on one 2,048-point mesh."""
    fx, G = _random_case(5, CFG_3D, [2048], [[805]])
    m = build_model(fx["params"], fx["cfg"])
    out, grads = run_packed(m, fx, G)
    errs = check_parity(out, grads, fx)
    assert not errs, errs


@pytest.mark.timeout(300)
def test_configs1_exact_timed_shape():
    """configs[1] exactly as bench.py --workload cfg2 times it: one 10,000-point mesh, two input
    functions of 805 points, d=128, 4 experts, 4 blocks."""
    fx, G = _random_case(9, CFG_CFG2, [10000], [[805], [805]])
    m = build_model(fx["params"], fx["cfg"])
    out, grads = run_packed(m, fx, G)
    errs = check_parity(out, grads, fx)
    assert not errs, errs


@pytest.mark.timeout(300)
def test_configs4_variable_meshes_packed():
    """configs[4]-shaped packed batch: 16 meshes of U{1000..1400} points (seeded), main.py widths, one
    packed call; each mesh is an independent B=1 reference call (packed offsets, no padding)."""
    rng = np.random.default_rng(3)
    Ns = [int(v) for v in rng.integers(1000, 1401, 16)]
    fx, G = _random_case(13, CFG_MAIN, Ns, [[805] * 16])
    m = build_model(fx["params"], fx["cfg"])
    out, grads = run_packed(m, fx, G)
    errs = check_parity(out, grads, fx)
    assert not errs, errs
