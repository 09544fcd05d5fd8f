"""The reference training loop (main.py:50-153) through gnot_amd.train.fit / evaluate, against a
stock-torch replica of the reference step (torch_port forward + autograd, torch.optim.AdamW +
OneCycleLR stepped per epoch, RelL2 of loss.py:14-23) on the same batches:
  * per-epoch train losses and per-epoch test metrics (main.py:108-147) equal the replica's,
  * the best checkpoint round-trips through torch.save / torch.load(weights_only=True) with the keys of
    the reference state_dict AND the values the model held when it was saved,
for packed batches (collate_packed) and for main.py's zero-padded batches (collate_padded, pad rows in
the attention sums)."""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CFG = (2, 1, 3, 1, 1, 32, 2, 32, 32, 2, 4, 1)
TCFG = dict(n_mlp_num_layers=2, n_expert=2, n_head=4, n_attn_layers=1, n_input_functions=1)


def _loaders(padded):
    from gnot_amd import data
    rng = np.random.default_rng(3)
    samples = [data.synthetic_sample(rng, int(rng.integers(40, 120)), fn_points=(int(rng.integers(10, 30)),))
               for _ in range(6)]
    test = [data.synthetic_sample(rng, int(rng.integers(40, 120)), fn_points=(int(rng.integers(10, 30)),))
            for _ in range(4)]
    coll = data.collate_padded if padded else data.collate_packed
    mk = lambda s: torch.utils.data.DataLoader(data.NS2dData(s), batch_size=2, shuffle=False, collate_fn=coll)
    return mk(samples), mk(test)


def _replica_out(torch_port, p, b, dev):
    """reference forward of one batch -> (packed prediction, packed offsets)."""
    if "counts" in b:      # padded: ONE B-sample call, pad rows inside the attention sums (main.py:84)
        out = torch_port.gnot_forward(p, TCFG, b["x"].to(dev), b["theta"].to(dev), [f.to(dev) for f in b["fns"]])
        counts = b["counts"]
        off = np.concatenate([[0], np.cumsum(counts)]).tolist()
        return torch.cat([out[i, :n] for i, n in enumerate(counts)]), off
    outs = []
    for i in range(len(b["x_off"]) - 1):          # packed: one unpadded B=1 call per sample
        s, e = b["x_off"][i], b["x_off"][i + 1]
        fo = b["fn_offs"][0]
        outs.append(torch_port.gnot_forward(p, TCFG, b["x"][s:e][None].to(dev), b["theta"][i:i + 1].to(dev),
                                            [b["fns"][0][fo[i]:fo[i + 1]][None].to(dev)])[0])
    return torch.cat(outs), b["x_off"]


def _rel_l2(out, y, off):
    tot = [(((out[s:e] - y[s:e]) ** 2).sum(0) / (y[s:e] ** 2).sum(0)).sqrt() for s, e in zip(off[:-1], off[1:])]
    return torch.stack(tot).mean()


def _replica(init, train_loader, test_loader, epochs, dev):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import torch_port
    p = {k: v.clone().requires_grad_(True) for k, v in init.items()}
    opt = torch.optim.AdamW(list(p.values()), lr=1e-3, foreach=False)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=1e-3, steps_per_epoch=len(train_loader), epochs=epochs)
    train, test, snaps = [], [], []
    for _ in range(epochs):
        losses = []
        for b in train_loader:
            opt.zero_grad()
            out, off = _replica_out(torch_port, p, b, dev)
            loss = _rel_l2(out, b["y"].to(dev), off)
            loss.backward()
            opt.step()
            losses.append(float(loss))
        sched.step()
        train.append(np.mean(losses))
        with torch.no_grad():
            vals = []
            for b in test_loader:
                out, off = _replica_out(torch_port, p, b, dev)
                vals.append(float(_rel_l2(out, b["y"].to(dev), off)))
        test.append(np.mean(vals))
        snaps.append({k: v.detach().clone() for k, v in p.items()})
    return train, test, snaps


@pytest.mark.parametrize("padded", [False, True], ids=["packed", "padded"])
def test_fit_evaluate_checkpoint_match_torch_reference(tmp_path, padded):
    from gnot_amd import GNOT, train
    dev = torch.device("cuda")
    train_loader, test_loader = _loaders(padded)
    torch.manual_seed(0)
    model = GNOT(*CFG).to(dev)
    init = {k: v.detach().clone() for k, v in model.state_dict().items()}
    epochs = 3
    ref_train, ref_test, ref_snaps = _replica(init, train_loader, test_loader, epochs, dev)

    got_train, got_test, held = [], [], []

    def log(msg):
        if "Loss" in msg:
            got_train.append(float(msg.split(": ")[1]))
        if "Test Metric" in msg:       # logged just before a possible checkpoint save
            got_test.append(float(msg.split(": ")[1]))
            held.append({k: v.detach().clone() for k, v in model.state_dict().items()})

    ckpt = os.path.join(tmp_path, "best_model.pth")
    hist_train, hist_test = train.fit(model, train_loader, test_loader, epochs=epochs, checkpoint=ckpt, log=log)
    assert hist_train == got_train and hist_test == got_test
    assert np.allclose(got_train, ref_train, rtol=1e-4, atol=0), (got_train, ref_train)
    assert np.allclose(got_test, ref_test, rtol=1e-4, atol=0), (got_test, ref_test)
    # evaluate() on its own equals the replica's metric of the final weights
    assert np.isclose(train.evaluate(model, test_loader), ref_test[-1], rtol=1e-4, atol=0)

    # the best checkpoint: reference keys, and exactly the values held at the best epoch
    best = int(np.argmin(got_test))
    fresh = GNOT(*CFG)
    train.load_checkpoint(fresh, ckpt)
    sd = fresh.state_dict()
    assert list(sd.keys()) == list(init.keys())
    for k in sd:
        assert torch.equal(sd[k], held[best][k].cpu()), k
        # and the replica's weights at that epoch, norm-wise (AdamW normalises each update, so an element
        # whose gradient is at fp32 noise level may step differently; the tensor as a whole may not)
        r = ref_snaps[best][k].cpu()
        assert float((sd[k] - r).norm() / r.norm().clamp_min(1e-12)) < 1e-3, k
