"""MoE activation recompute (GNOT.set_moe_recompute): the backward re-runs each MoE call's expert
forward into one shared save buffer.  The kernels are deterministic, so outputs and every parameter
gradient must equal the plain (all activations saved) path BITWISE, for the d=256 bf16x6 chains
(configs[2] widths) and the d=64 fp32 chains, with input functions and without."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("d,E,I,prec", [(256, 8, 1, "fp32"), (64, 3, 0, "fp32"), (64, 2, 2, "fp32"), (256, 8, 1, "bf16")])
def test_recompute_matches_saved_activations_bitwise(d, E, I, prec):
    """prec "bf16": the bf16 mode's bf16 activation storage (the recompute rewrites the same bf16 saves)"""
    from gnot_amd import GNOT
    dev = torch.device("cuda")
    torch.manual_seed(7)
    model = GNOT(3, 1, 3, 1, 2, d, 4, d, d, E, 8 if d == 256 else 4, I).to(dev)
    model.set_precision(prec)
    g = torch.Generator(device="cpu").manual_seed(8)
    x_off = [0, 1500, 2048]
    x = torch.rand(x_off[-1], 3, generator=g).to(dev)
    theta = torch.rand(2, 1, generator=g).to(dev)
    fns = [torch.rand(300, 3, generator=g).to(dev) for _ in range(I)]
    fn_offs = [[0, 120, 300] for _ in range(I)]
    tgt = torch.randn(x_off[-1], 1, generator=g).to(dev)

    def run():
        model.zero_grad(set_to_none=True)
        out = model.forward_packed(x, x_off, theta, fns, fn_offs)
        ((out - tgt) ** 2).sum().backward()
        torch.cuda.synchronize()
        return out.detach().clone(), [p.grad.detach().clone() for p in model.parameters()]

    o0, g0 = run()
    model.set_moe_recompute(True)
    o1, g1 = run()
    model.set_moe_recompute(False)
    o2, g2 = run()
    assert torch.equal(o0, o1) and torch.equal(o0, o2)
    for a, b, c in zip(g0, g1, g2):
        assert torch.equal(a, b) and torch.equal(a, c)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_side_stream_weight_gradients_match_serial_bitwise(prec, monkeypatch):
    """GNOT_WGRAD_OVERLAP=1 (read when the plan is created): every weight-gradient group forked onto the
    side stream instead of the caller's stream -- the same kernels in the same order per group, so outputs
    and gradients are bitwise those of the serial default (configs[2] widths, input functions)."""
    from gnot_amd import GNOT
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(21)
    x_off = [0, 1700, 2300]
    x = torch.rand(x_off[-1], 3, generator=g).to(dev)
    theta = torch.rand(2, 1, generator=g).to(dev)
    fns = [torch.rand(300, 3, generator=g).to(dev)]
    tgt = torch.randn(x_off[-1], 1, generator=g).to(dev)
    res = []
    for overlap in ("0", "1"):
        monkeypatch.setenv("GNOT_WGRAD_OVERLAP", overlap)
        torch.manual_seed(7)
        model = GNOT(3, 1, 3, 1, 2, 256, 4, 256, 256, 8, 8, 1).to(dev)
        model.set_precision(prec)
        out = model.forward_packed(x, x_off, theta, fns, [[0, 120, 300]])
        ((out - tgt) ** 2).sum().backward()
        torch.cuda.synchronize()
        res.append((out.detach().clone(), [p.grad.detach().clone() for p in model.parameters()]))
    (o0, g0), (o1, g1) = res
    assert torch.equal(o0, o1)
    assert all(torch.equal(a, b) for a, b in zip(g0, g1))
