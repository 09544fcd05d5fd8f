"""The soft-MoE walk form (chain2.hip WALK, ChainArgs.walk): one workgroup runs every expert of its
points in order and sums in place (forward: query_out = query_in + sum_e s_e * MLP_e(a), model.py:128-131,
134-137; backward: d a = sum_e W_e0^T dz_e0), with no [P, E, d] stage and no moe_combine pass.

It sums in the same order and with the same roundings as the expert grid + moe_combine (s_e * y_e
rounded, then added left to right from the residual), so every output and parameter gradient must be
BITWISE equal to the expert-grid path -- with saved activations and with MoE recompute (whose walk
forward writes saves only).  GNOT_MOE_WALK forces the form (read at gnot_plan_set_batch).  The oracle
parity of the walk form at the headline's kernel selection is tests/test_gpu_headline.py."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(monkeypatch, walk, recompute, E, I, d=256, prec="fp32", fused="0"):
    from gnot_amd import GNOT
    monkeypatch.setenv("GNOT_MOE_WALK", walk)
    # fused="1": the opt-in fused combine (GNOT_MOE_FUSED, engine.cpp moe_fused), which needs serial weight
    # gradients; the default grid sums its stage with the moe_combine pass (bf16 mode: moe_combine_b16)
    monkeypatch.setenv("GNOT_MOE_FUSED", fused)
    monkeypatch.setenv("GNOT_WGRAD_OVERLAP", "0")
    dev = torch.device("cuda")
    torch.manual_seed(17)
    model = GNOT(3, 1, 3, 1, 2, d, 4, d, d, E, 8, I).to(dev)
    model.set_moe_recompute(recompute)
    model.set_precision(prec)
    g = torch.Generator(device="cpu").manual_seed(18)
    x_off = [0, 1500, 2093]                      # a partial last workgroup (2093 % 128 != 0)
    x = torch.rand(x_off[-1], 3, generator=g).to(dev)
    theta = torch.rand(2, 1, generator=g).to(dev)
    fns = [torch.rand(300, 3, generator=g).to(dev) for _ in range(I)]
    fn_offs = [[0, 120, 300] for _ in range(I)]
    tgt = torch.randn(x_off[-1], 1, generator=g).to(dev)
    out = model.forward_packed(x, x_off, theta, fns, fn_offs)
    ((out - tgt) ** 2).sum().backward()
    torch.cuda.synchronize()
    return out.detach().clone(), [p.grad.detach().clone() for p in model.parameters()]


@pytest.mark.parametrize("E,I,prec", [(8, 1, "fp32"), (3, 0, "fp32"), (2, 2, "fp32"), (8, 1, "bf16"), (3, 0, "bf16")])
def test_walk_form_bitwise_equals_expert_grid(monkeypatch, E, I, prec):
    """prec "bf16": the bf16 mode, whose MoE chains store bf16 saves / dZ / Linear inputs (ChainArgs.b16s)
    and whose MoE weight gradients run on pgemm_b16_kernel: the same equalities hold"""
    o0, g0 = _run(monkeypatch, "0", False, E, I, prec=prec)
    o1, g1 = _run(monkeypatch, "1", False, E, I, prec=prec)
    o2, g2 = _run(monkeypatch, "1", True, E, I, prec=prec)
    o3, g3 = _run(monkeypatch, "0", False, E, I, prec=prec, fused="1")   # the opt-in fused combine
    assert torch.isfinite(o0).all()
    diff = lambda a, b: f"max |diff| {float((a - b).abs().max()):.3e} of max {float(a.abs().max()):.3e}"
    assert torch.equal(o0, o1), "walk output: " + diff(o0, o1)
    assert torch.equal(o0, o2), "walk + recompute output: " + diff(o0, o2)
    assert torch.equal(o0, o3), "fused combine output: " + diff(o0, o3)
    for k, (a, b, c, f) in enumerate(zip(g0, g1, g2, g3)):
        assert torch.equal(a, b), f"parameter {k}: walk differs from the expert grid, " + diff(a, b)
        assert torch.equal(a, c), f"parameter {k}: walk + recompute differs from the expert grid, " + diff(a, c)
        assert torch.equal(a, f), f"parameter {k}: the fused combine differs from the combine pass, " + diff(a, f)

