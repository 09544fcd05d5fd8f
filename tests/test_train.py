"""The training step around the path: OneCycle schedule arithmetic
vs torch's OneCycleLR (CPU), and on the GPU the native RelL2 loss / gradient vs the reference
formula (loss.py:14-23) and FlatAdamW vs torch.optim.AdamW."""
import numpy as np
import pytest
import torch

from gnot_amd import train


@pytest.mark.parametrize("epochs,spe", [(100, 275), (3, 7)])
def test_onecycle_matches_torch(epochs, spe):
    p = torch.nn.Parameter(torch.zeros(3))
    opt = torch.optim.AdamW([p], lr=1e-3)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=1e-3, steps_per_epoch=spe, epochs=epochs)
    mine = train.OneCycle(1e-3, epochs, spe)
    for _ in range(min(epochs * spe - 1, 400)):
        lr, b1 = mine.values()
        g = opt.param_groups[0]
        assert abs(lr - g["lr"]) <= 1e-12 * max(1.0, g["lr"]) and abs(b1 - g["betas"][0]) <= 1e-12
        sched.step()
        mine.step()


def test_reference_schedule_quirk_keeps_lr_near_initial():
    """main.py:52/106: OneCycleLR sized per batch but stepped per epoch."""
    s = train.OneCycle(1e-3, epochs=100, steps_per_epoch=275)
    lrs = []
    for _ in range(100):
        lrs.append(s.values()[0])
        s.step()
    assert abs(lrs[0] - 1e-3 / 25) < 1e-15 and max(lrs) < 1e-3 / 25 * 1.01


def rel_l2_reference(pred, tgt, off):
    """loss.py:14-23 with dgl SumPooling = per-sample sums (float64)."""
    vals = []
    for b in range(len(off) - 1):
        p, t = pred[off[b]:off[b + 1]], tgt[off[b]:off[b + 1]]
        vals.append(np.sqrt(((p - t) ** 2).sum(0) / (t ** 2).sum(0)))
    return float(np.mean(vals))


@pytest.mark.gpu
@pytest.mark.parametrize("sizes,C", [([10000], 1), ([37, 1, 5000, 2049], 3), ([4097, 4096], 2)])
def test_native_rel_l2_loss_and_grad(sizes, C):
    rng = np.random.default_rng(0)
    off = np.concatenate([[0], np.cumsum(sizes)]).tolist()
    pred = rng.standard_normal((off[-1], C))
    tgt = rng.standard_normal((off[-1], C))
    dev = torch.device("cuda")
    pt = torch.tensor(pred, dtype=torch.float32, device=dev, requires_grad=True)
    loss = train.RelL2Loss()(off, pt, torch.tensor(tgt, dtype=torch.float32, device=dev))
    loss.backward()
    ref = rel_l2_reference(pred, tgt, off)
    assert abs(float(loss) - ref) <= 1e-5 * ref
    # gradient: autograd of the same formula in float64
    p64 = torch.tensor(pred, dtype=torch.float64, requires_grad=True)
    t64 = torch.tensor(tgt, dtype=torch.float64)
    seg = torch.repeat_interleave(torch.arange(len(sizes)), torch.tensor(sizes))
    num = torch.zeros(len(sizes), C, dtype=torch.float64).index_add(0, seg, (p64 - t64) ** 2)
    den = torch.zeros(len(sizes), C, dtype=torch.float64).index_add(0, seg, t64 ** 2)
    (num / den).sqrt().mean().backward()
    g = pt.grad.double().cpu().numpy()
    r = p64.grad.numpy()
    assert np.linalg.norm(g - r) <= 1e-5 * np.linalg.norm(r)


@pytest.mark.gpu
def test_flat_adamw_matches_torch_adamw_with_onecycle():
    from gnot_amd import GNOT
    dev = torch.device("cuda")
    torch.manual_seed(0)
    a = GNOT(2, 1, 3, 1, 1, 32, 2, 32, 32, 2, 4, 1).to(dev)
    b = GNOT(2, 1, 3, 1, 1, 32, 2, 32, 32, 2, 4, 1).to(dev)
    b.load_state_dict(a.state_dict())
    flat = train.flatten_parameters(b)
    opt_a = torch.optim.AdamW(a.parameters(), lr=1e-3, foreach=False)
    sch_a = torch.optim.lr_scheduler.OneCycleLR(opt_a, max_lr=1e-3, steps_per_epoch=4, epochs=3)
    opt_b = train.FlatAdamW(flat, lr=1e-3, schedule=train.OneCycle(1e-3, 3, 4))
    g = torch.Generator(device="cpu").manual_seed(1)
    for _ in range(10):
        grads = [torch.randn(p.shape, generator=g).to(dev) * 1e-2 for p in a.parameters()]
        for p, gr in zip(a.parameters(), grads):
            p.grad = gr.clone()
        opt_a.step()
        sch_a.step()
        # the flat gradient in the arena layout: (W, b) of every Linear in canonical order
        gmap = {n: gr for (n, _), gr in zip(a.named_parameters(), grads)}
        lin_names = []
        for l in b.linears():
            for p in (l.weight, l.bias):
                lin_names.append(next(n for n, q in b.named_parameters() if q is p))
        gflat = torch.cat([gmap[n].reshape(-1) for n in lin_names])
        opt_b.step(gflat)
        opt_b.schedule.step()
    torch.cuda.synchronize()
    for (n, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        err = (pa - pb).abs().max().item()
        assert err <= 1e-6 * max(1.0, pa.abs().max().item()), (n, err)
