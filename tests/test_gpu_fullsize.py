"""configs[2] at its FULL size (one 262,144-point 3-D mesh, d=256, 8 experts, 4 blocks, 805 input-function
points) -- far past what the float64 oracle can run, so checked through size-independent properties:
finite outputs and gradients, bitwise-repeatable steps (deterministic reductions), an inference forward
(no saves) bitwise equal to the training forward, and a RelL2 loss that decreases over a few AdamW steps
on a fixed target (main.py:50-103).  Both arithmetics: fp32 (bf16x6) and the bf16 mode, each in its
default soft-MoE form (the expert grid and the moe_combine pass; bf16 mode: bf16 stage rows and moe_combine_b16)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

N, M = 262144, 805


@pytest.mark.timeout(300)
@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_configs2_full_size_properties(prec):
    from gnot_amd import GNOT
    from gnot_amd import train as gtrain
    dev = torch.device("cuda")
    torch.manual_seed(1234)
    model = GNOT(3, 1, 3, 1, 4, 256, 4, 256, 256, 8, 8, 1).to(dev)
    model.set_precision(prec)
    g = torch.Generator(device="cpu").manual_seed(100)
    x = torch.rand(N, 3, generator=g).to(dev)
    theta = torch.rand(1, 1, generator=g).to(dev)
    fns = [torch.rand(M, 3, generator=g).to(dev)]
    # a smooth target field of the coordinates (learnable, unlike noise)
    y = torch.sin(3.0 * x.sum(1, keepdim=True))
    x_off, fn_offs = [0, N], [[0, M]]
    loss_fn = gtrain.RelL2Loss()

    def step():
        model.zero_grad(set_to_none=True)
        out = model.forward_packed(x, x_off, theta, fns, fn_offs)
        loss = loss_fn(x_off, out, y)
        loss.backward()
        torch.cuda.synchronize()
        return out.detach().clone(), loss.item(), [p.grad.detach().clone() for p in model.parameters()]

    o1, l1, g1 = step()
    o2, l2, g2 = step()
    assert torch.isfinite(o1).all() and all(torch.isfinite(t).all() for t in g1)
    assert torch.equal(o1, o2) and l1 == l2
    assert all(torch.equal(a, b) for a, b in zip(g1, g2)), "repeated step differs bitwise"
    del o2, g2
    with torch.no_grad():                        # inference plan: no saves, the same arithmetic
        o3 = model.forward_packed(x, x_off, theta, fns, fn_offs)
    torch.cuda.synchronize()
    assert torch.equal(o1, o3), f"inference forward differs: {float((o1 - o3).abs().max()):.3e}"
    del o3

    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    losses = [l1]
    for _ in range(4):
        model.zero_grad(set_to_none=True)
        out = model.forward_packed(x, x_off, theta, fns, fn_offs)
        loss = loss_fn(x_off, out, y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    out = model.forward_packed(x, x_off, theta, fns, fn_offs)
    losses.append(loss_fn(x_off, out, y).item())
    assert all(torch.isfinite(torch.tensor(losses))), losses
    # monotone decrease from the first AdamW step on (the first two entries are the same weights)
    assert all(b < a for a, b in zip(losses[1:], losses[2:])), losses
    assert losses[-1] < 0.95 * losses[0], losses
