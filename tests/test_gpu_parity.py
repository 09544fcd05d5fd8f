"""HIP path (libgnot_hip.so through the drop-in GNOT module) vs the reference's golden fixtures and
vs the CPU oracle.  Tolerances: golden_util.check_parity (1e-4 relative, fp32)."""
import numpy as np
import pytest
import torch

from golden_util import check_parity, fixture_names, load, model_args, rel
from oracle import gnot_oracle as O

pytestmark = pytest.mark.gpu


def build_model(fx_or_params, cfg):
    from gnot_amd import GNOT
    m = GNOT(*model_args(cfg)).cuda()
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)).float() for k, v in fx_or_params.items()})
    return m


def run_packed(m, fx, G):
    dev = torch.device("cuda")
    x = torch.from_numpy(fx["x"]).float().to(dev)
    theta = torch.from_numpy(fx["theta"]).float().to(dev)
    fns = [torch.from_numpy(f).float().to(dev) for f in fx["fns"]]
    m.zero_grad(set_to_none=True)
    out = m.forward_packed(x, fx["x_off"].tolist(), theta, fns, [o.tolist() for o in fx["fn_offs"]])
    (out * torch.from_numpy(G).float().to(dev)).sum().backward()
    torch.cuda.synchronize()
    grads = {k: p.grad.double().cpu().numpy() for k, p in m.named_parameters()}
    return out.detach().double().cpu().numpy(), grads


@pytest.fixture(params=["auto", "mfma"])
def attn_path(request, monkeypatch):
    """'auto': the size-based choice (VALU attention passes below 512 point chunks and VALU state
    reductions below 65,536 points, i.e. every fixture); 'mfma': GNOT_APPLY_MFMA_MIN=0 and
    GNOT_STATE_MFMA_MIN=0 force the fp32-MFMA apply / K-V backward (attn_mfma.hip) and state
    (state.hip) kernels wherever the head width has one."""
    if request.param == "mfma":
        monkeypatch.setenv("GNOT_APPLY_MFMA_MIN", "0")
        monkeypatch.setenv("GNOT_STATE_MFMA_MIN", "0")
    return request.param


@pytest.mark.parametrize("name", fixture_names())
def test_fixture_parity_packed(name, attn_path):
    fx = load(name)
    m = build_model(fx["params"], fx["cfg"])
    out, grads = run_packed(m, fx, fx["G"])
    errs = check_parity(out, grads, fx)
    assert not errs, errs


@pytest.mark.parametrize("name", [n for n in fixture_names() if load(n)["meta"]["mode"] == "padded"])
def test_fixture_parity_padded_call(name):
    """The reference calling convention: forward(x[B,N,in], theta, fns[I,B,M,F])."""
    fx = load(name)
    cfg = fx["cfg"]
    m = build_model(fx["params"], cfg)
    B = len(fx["x_off"]) - 1
    N = int(fx["x_off"][1])
    dev = torch.device("cuda")
    x = torch.from_numpy(fx["x"]).float().to(dev).view(B, N, -1)
    theta = torch.from_numpy(fx["theta"]).float().to(dev)
    I = cfg["n_input_functions"]
    fns = None
    if I > 0:
        M = int(fx["fn_offs"][0][1])
        fns = torch.stack([torch.from_numpy(f).float().view(B, M, -1) for f in fx["fns"]]).to(dev)
    out = m(x, theta, fns)
    assert out.shape == (B, N, cfg["out_dim"])
    (out * torch.from_numpy(fx["G"]).float().to(dev).view(B, N, -1)).sum().backward()
    grads = {k: p.grad.double().cpu().numpy() for k, p in m.named_parameters()}
    errs = check_parity(out.detach().double().cpu().numpy().reshape(B * N, -1), grads, fx)
    assert not errs, errs


def test_intermediates_match_oracle():
    """Stage-by-stage comparison (diagnostic when the end-to-end check fails)."""
    fx = load("cross1")
    cfg = fx["cfg"]
    m = build_model(fx["params"], cfg)
    out, _ = run_packed(m, fx, fx["G"])
    P = O.Params(fx["params"], np.float64)
    _, C = O.forward_sample(P, cfg, fx["x"], fx["theta"][0], fx["fns"])
    eng = m.engine()
    d = cfg["d"]
    N = fx["x"].shape[0]
    checks = {
        "scores": (C["scores"], cfg["n_expert"]),
        "query0": (C["x"][-1][2], d),
        "b0.cres": (C["blocks"][0]["cross"][2], d),
        "b0.query1": (C["blocks"][0]["self"][0], d),
        "b0.sres": (C["blocks"][0]["self"][2], d),
    }
    bad = []
    for name, (ref, cols) in checks.items():
        got = eng.debug_tensor(name, N, cols).double().cpu().numpy()
        e = rel(got, ref)
        if not e <= 1e-4:   # NaN fails
            bad.append(f"{name}: {e:.3e}")
    assert not bad, bad


def _random_case(seed, cfg, Ns, Ms):
    from gnot_amd import GNOT
    torch.manual_seed(seed)
    ref = GNOT(*model_args(cfg))
    params = {k: v.double().numpy() for k, v in ref.state_dict().items()}
    rng = np.random.default_rng(seed)
    x = rng.random((sum(Ns), cfg["input_dim"]))
    theta = rng.random((len(Ns), cfg["theta_dim"]))
    fns = [rng.random((sum(Ms[i]), cfg["input_func_dim"])) for i in range(cfg["n_input_functions"])]
    off = lambda L: np.concatenate([[0], np.cumsum(L)]).astype(np.int64)
    G = rng.standard_normal((sum(Ns), cfg["out_dim"]))
    fx = dict(params=params, cfg=cfg, x=x, x_off=off(Ns), theta=theta, fns=fns,
              fn_offs=[off(Ms[i]) for i in range(cfg["n_input_functions"])])
    out64, g64 = O.gnot_forward_backward(params, cfg, x, fx["x_off"], theta, fns, fx["fn_offs"], G=G)
    out32, g32 = O.gnot_forward_backward(params, cfg, x, fx["x_off"], theta, fns, fx["fn_offs"], G=G,
                                         dtype=np.float32)
    fx["out"] = out64
    fx["grads"] = g64
    fx["e32"] = {k: float(np.linalg.norm(g32[k].astype(np.float64) - g64[k])) for k in g64}
    return fx, G


@pytest.mark.parametrize("case", [
    # cfg2-like widths (BASELINE configs[1]: d=128, 4 experts, 8 heads, 2 input functions), small N
    dict(cfg=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=3, n_attn_layers=2, d=128,
                  n_mlp_num_layers=4, n_expert=4, n_head=8, n_input_functions=2),
         Ns=[517, 200], Ms=[[161, 90], [77, 130]]),
    # d=256 with 8 heads (dh=32) and 8 experts (cfg3 widths)
    dict(cfg=dict(input_dim=3, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=1, d=256,
                  n_mlp_num_layers=2, n_expert=8, n_head=8, n_input_functions=1),
         Ns=[300], Ms=[[97]]),
    # default main.py widths, no input functions (self-attention only)
    dict(cfg=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=2, n_attn_layers=1, d=256,
                  n_mlp_num_layers=4, n_expert=3, n_head=8, n_input_functions=0),
         Ns=[129, 64, 1], Ms=[]),
])
def test_random_config_vs_oracle(case, attn_path):
    fx, G = _random_case(3, case["cfg"], case["Ns"], case["Ms"])
    m = build_model(fx["params"], fx["cfg"])
    out, grads = run_packed(m, fx, G)
    errs = check_parity(out, grads, fx)
    assert not errs, errs


def test_repeated_steps_are_deterministic():
    fx = load("cross2_packed")
    m = build_model(fx["params"], fx["cfg"])
    o1, g1 = run_packed(m, fx, fx["G"])
    o2, g2 = run_packed(m, fx, fx["G"])
    assert np.array_equal(o1, o2)
    for k in g1:
        assert np.array_equal(g1[k], g2[k]), k


def _inputs(fx):
    dev = torch.device("cuda")
    return (torch.from_numpy(fx["x"]).float().to(dev), fx["x_off"].tolist(),
            torch.from_numpy(fx["theta"]).float().to(dev),
            [torch.from_numpy(f).float().to(dev) for f in fx["fns"]], [o.tolist() for o in fx["fn_offs"]])


def test_two_forwards_one_backward():
    """The reference builds one autograd graph per call (model.py:154-173): f(a) + f(b) -> backward
    sums both calls' gradients.  Two pending forwards use two engines (activation sets)."""
    fx = load("cross2_packed")
    m = build_model(fx["params"], fx["cfg"])
    _, g1 = run_packed(m, fx, fx["G"])
    x, xo, th, fns, fo = _inputs(fx)
    G = torch.from_numpy(fx["G"]).float().cuda()
    m.zero_grad(set_to_none=True)
    o1 = m.forward_packed(x, xo, th, fns, fo)
    o2 = m.forward_packed(x, xo, th, fns, fo)
    ((o1 * G).sum() + (o2 * G).sum()).backward()
    for k, p in m.named_parameters():
        assert np.array_equal(p.grad.double().cpu().numpy(), 2 * g1[k]), k


def test_eval_forward_between_forward_and_backward():
    """forward(train) -> forward(no_grad, another geometry) -> backward: the pending backward keeps its
    own activations (the evaluation runs on an engine with no pending backward)."""
    fx = load("cross2_packed")
    m = build_model(fx["params"], fx["cfg"])
    out0, g0 = run_packed(m, fx, fx["G"])
    x, xo, th, fns, fo = _inputs(fx)
    m.zero_grad(set_to_none=True)
    o = m.forward_packed(x, xo, th, fns, fo)
    with torch.no_grad():                       # a different geometry: the first half of the points
        n = max(1, xo[1] // 2)
        e = m.forward_packed(x[:n].contiguous(), [0, n], th[:1].contiguous(),
                             [f[: fo[i][1]].contiguous() for i, f in enumerate(fns)],
                             [[0, fo[i][1]] for i in range(len(fns))])
    assert torch.isfinite(e).all()
    (o * torch.from_numpy(fx["G"]).float().cuda()).sum().backward()
    assert np.array_equal(o.detach().double().cpu().numpy(), out0)
    for k, p in m.named_parameters():
        assert np.array_equal(p.grad.double().cpu().numpy(), g0[k]), k


def test_pending_backward_bound():
    """More pending training forwards than GNOT.max_pending_backwards: the oldest one's activations are
    reused and its backward raises; a forward whose graph was freed releases its engine."""
    fx = load("tiny_n_lt_h")
    m = build_model(fx["params"], fx["cfg"])
    m.set_max_pending_backwards(1)
    x, xo, th, fns, fo = _inputs(fx)
    o1 = m.forward_packed(x, xo, th, fns, fo)
    o2 = m.forward_packed(x, xo, th, fns, fo)
    with pytest.raises(RuntimeError, match="reused by a later forward"):
        o1.sum().backward()
    o2.sum().backward()
    m.set_max_pending_backwards(2)
    o3 = m.forward_packed(x, xo, th, fns, fo)
    del o3                                      # graph freed without a backward: its engine is free again
    o4 = m.forward_packed(x, xo, th, fns, fo)
    o5 = m.forward_packed(x, xo, th, fns, fo)
    (o4.sum() + o5.sum()).backward()
    assert len(m._extra) <= 1


def test_eval_no_grad_matches_training_forward():
    fx = load("d64_cross")
    m = build_model(fx["params"], fx["cfg"])
    out_t, _ = run_packed(m, fx, fx["G"])
    dev = torch.device("cuda")
    with torch.no_grad():
        out_e = m.forward_packed(torch.from_numpy(fx["x"]).float().to(dev), fx["x_off"].tolist(),
                                 torch.from_numpy(fx["theta"]).float().to(dev),
                                 [torch.from_numpy(f).float().to(dev) for f in fx["fns"]],
                                 [o.tolist() for o in fx["fn_offs"]])
    assert np.array_equal(out_e.double().cpu().numpy(), out_t)
