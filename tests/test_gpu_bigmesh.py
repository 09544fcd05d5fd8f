"""BASELINE configs[3] and configs[4] at their real sizes on ONE GPU.

Round 3's kernels addressed whole activation arrays through 32-bit buffer offsets, which capped a plan
at 1,398,101 points at d = 256; the chain and weight-gradient kernels now base every buffer resource at
their workgroup's (split's) first row.  These tests run past that bound:

* configs[4]: bench.py's exact batch -- 64 meshes of U{1k..50k} points (1,590,454 points) -- in ONE packed
  call with MoE recompute (the plain training workspace would need 336 GiB).  The smallest mesh is placed
  FIRST and the second smallest LAST (rows past 1.58 M, byte offsets past 4 GiB in the [P, 3d]
  projections); the upstream gradient is non-zero on those two meshes only.  Checks: three meshes'
  outputs equal B = 1 runs of that mesh alone (1e-6; the kernel selection differs with the batch size);
  the two edge meshes' outputs and EVERY parameter gradient match the float64 oracle of those two meshes
  at north_star's 1e-4 (packed samples are independent, reference main.py:60-89 without padding); a
  second backward is bitwise equal.
* configs[3]: the 1,048,576-point mesh forward (L = 4, bench.py's data and weights) against the
  fixture-pinned stock-torch port in fp32 under no_grad, executed by PyTorch-ROCm's own kernels (the CPU
  port needs minutes at this size; test_gpu_headline.py compares on the CPU at 262,144 points); then a
  training step of the whole mesh on one GPU (MoE recompute, as bench.py --workload cfg4 at N = 1):
  finite gradients, two steps bitwise equal.

Anchor: the all-point sums /root/reference/model.py:77-80, 98-101 over these point counts.
"""
import numpy as np
import pytest
import torch

from golden_util import check_parity, model_args, rel
from test_gpu_configs import CFG_3D, CFG_MAIN
from test_gpu_parity import build_model

pytestmark = pytest.mark.gpu


def _cfg5_batch():
    """bench.py's configs[4] batch at one rank (make_rank_batch, world 1), reordered: smallest mesh
    first, second smallest last, the rest in bench order."""
    import bench
    D = bench.make_rank_batch(bench.WORKLOADS["cfg5"], 0, 1, torch.device("cpu"))
    xo, fo = D["x_off"], D["fn_offs"][0]
    sizes = [xo[b + 1] - xo[b] for b in range(len(xo) - 1)]
    by_size = sorted(range(len(sizes)), key=lambda b: (sizes[b], b))
    first, last = by_size[0], by_size[1]
    order = [first] + [b for b in range(len(sizes)) if b not in (first, last)] + [last]
    pick = lambda t, off, bs: torch.cat([t[off[b]:off[b + 1]] for b in bs])
    offs = lambda off, bs: np.concatenate([[0], np.cumsum([off[b + 1] - off[b] for b in bs])]).astype(np.int64)
    batch = lambda bs: dict(x=pick(D["x"], xo, bs), x_off=offs(xo, bs), theta=D["theta"][bs],
                            fn=pick(D["fns"][0], fo, bs), fn_off=offs(fo, bs))
    return batch, order, sizes, (first, last)


@pytest.mark.timeout(600)
def test_configs4_full_64_mesh_batch_one_gpu():
    from oracle import gnot_oracle as O
    batch, order, sizes, (first, last) = _cfg5_batch()
    full = batch(order)
    P = int(full["x_off"][-1])
    assert len(order) == 64 and P == sum(sizes) and P > 1_398_101, P
    torch.manual_seed(1234)
    from gnot_amd import GNOT
    params = {k: v.double().numpy() for k, v in GNOT(*model_args(CFG_MAIN)).state_dict().items()}
    m = build_model(params, CFG_MAIN)
    m.set_moe_recompute(True)
    dev = torch.device("cuda")
    rng = np.random.default_rng(5)
    n0, n1 = sizes[first], sizes[last]
    G = np.zeros((P, 1))
    G[:n0] = rng.standard_normal((n0, 1))
    G[P - n1:] = rng.standard_normal((n1, 1))
    Gt = torch.from_numpy(G).float().to(dev)

    def step():
        m.zero_grad(set_to_none=True)
        out = m.forward_packed(full["x"].to(dev), full["x_off"].tolist(), full["theta"].to(dev), [full["fn"].to(dev)],
                               [full["fn_off"].tolist()])
        (out * Gt).sum().backward()
        torch.cuda.synchronize()
        return out.detach().double().cpu().numpy(), {k: p.grad.double().cpu().numpy() for k, p in m.named_parameters()}

    out, grads = step()
    assert np.isfinite(out).all() and all(np.isfinite(g).all() for g in grads.values())
    # meshes of the packed call == the same mesh alone (B = 1)
    xo = full["x_off"]
    for pos in (0, 31, 63):
        one = batch([order[pos]])
        with torch.no_grad():
            o1 = m.forward_packed(one["x"].to(dev), one["x_off"].tolist(), one["theta"].to(dev), [one["fn"].to(dev)],
                                  [one["fn_off"].tolist()]).double().cpu().numpy()
        e = rel(out[xo[pos]:xo[pos + 1]], o1)
        print(f"\nmesh {order[pos]} ({sizes[order[pos]]} points at rows {xo[pos]}..{xo[pos + 1]}): packed vs alone {e:.2e}")
        assert e < 1e-6, (pos, e)
    # the two edge meshes vs the float64 oracle: outputs and every parameter gradient
    two = batch([first, last])
    args = (params, CFG_MAIN, two["x"].double().numpy(), two["x_off"], two["theta"].double().numpy(),
            [two["fn"].double().numpy()], [two["fn_off"]])
    G2 = np.concatenate([G[:n0], G[P - n1:]])
    out64, g64 = O.gnot_forward_backward(*args, G=G2)
    _, g32 = O.gnot_forward_backward(*args, G=G2, dtype=np.float32)
    ref = dict(out=out64, grads=g64, e32={k: float(np.linalg.norm(g32[k].astype(np.float64) - g64[k])) for k in g64})
    got = np.concatenate([out[:n0], out[P - n1:]])
    errs = check_parity(got, grads, ref)
    print(f"edge meshes vs oracle: out rel {rel(got, out64):.3e}")
    assert not errs, errs
    # full-size determinism
    out2, grads2 = step()
    assert np.array_equal(out, out2)
    for k in grads:
        assert np.array_equal(grads[k], grads2[k]), k


def _cfg4_model_and_mesh(N):
    from gnot_amd import GNOT
    torch.manual_seed(1234)
    model = GNOT(3, 1, 3, 1, 4, 256, 4, 256, 256, 8, 8, 1)
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    g = torch.Generator(device="cpu").manual_seed(100)
    x = torch.rand(N, 3, generator=g)
    theta = torch.rand(1, 1, generator=g)
    fn = torch.rand(805, 3, generator=g)
    return model, sd, x, theta, fn


@pytest.mark.timeout(900)
def test_configs3_1m_point_mesh_one_gpu():
    from oracle import torch_port
    N, M = 1 << 20, 805
    model, sd, x, theta, fn = _cfg4_model_and_mesh(N)
    dev = torch.device("cuda")
    model = model.to(dev)
    args = lambda: (x.to(dev), [0, N], theta.to(dev), [fn.to(dev)], [[0, M]])
    with torch.no_grad():
        got = model.forward_packed(*args()).cpu()
    assert torch.isfinite(got).all()
    # training step of the whole mesh on one GPU (MoE recompute: 196 GiB of workspace instead of 476)
    model.set_moe_recompute(True)
    G = torch.randn(N, 1, generator=torch.Generator(device="cpu").manual_seed(7)).to(dev)

    def step():
        model.zero_grad(set_to_none=True)
        out = model.forward_packed(*args())
        (out * G).sum().backward()
        torch.cuda.synchronize()
        return out.detach().cpu(), torch.cat([p.grad.reshape(-1) for p in model.parameters()]).cpu()

    o1, g1 = step()
    o2, g2 = step()
    assert torch.equal(o1, got), "training forward != eval forward"
    assert torch.isfinite(g1).all()
    assert torch.equal(o1, o2) and torch.equal(g1, g2)
    del model
    torch.cuda.empty_cache()
    # the fixture-pinned stock-torch port (oracle/torch_port.py), executed by PyTorch-ROCm's own fp32
    # kernels (rocBLAS / hipBLASLt GEMMs, ATen softmax / GELU / reductions) on the GPU: an independent
    # implementation of the same arithmetic; on the host's CPU cores the 1M-point forward alone takes
    # minutes (the 262,144-point CPU comparison is test_gpu_headline.py's)
    with torch.no_grad():
        sdg = {k: v.to(dev) for k, v in sd.items()}
        ref = torch_port.gnot_forward(sdg, dict(CFG_3D, n_attn_hidden_dim=256), x[None].to(dev), theta.to(dev),
                                      [fn[None].to(dev)])[0].cpu()
    e = rel(got.double().numpy(), ref.double().numpy())
    print(f"\n1,048,576-point forward vs the stock-torch port (PyTorch-ROCm fp32 kernels): rel {e:.3e}")
    assert e < 1e-4, e
