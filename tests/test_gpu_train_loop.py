"""The reference training loop (main.py:50-153) through gnot_amd.train.fit on packed NS2d batches:
per-step losses equal a stock-torch replica of the reference step (torch_port forward + autograd,
torch.optim.AdamW + OneCycleLR stepped per epoch, RelL2 of loss.py:14-23) on the same batches, and
the best checkpoint round-trips through torch.save / torch.load(weights_only=True)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup():
    from gnot_amd import GNOT, data
    rng = np.random.default_rng(3)
    samples = [data.synthetic_sample(rng, int(rng.integers(40, 120)), fn_points=(int(rng.integers(10, 30)),))
               for _ in range(6)]
    ds = data.NS2dData(samples)
    loader = torch.utils.data.DataLoader(ds, batch_size=2, shuffle=False, collate_fn=data.collate_packed)
    torch.manual_seed(0)
    cfg = (2, 1, 3, 1, 1, 32, 2, 32, 32, 2, 4, 1)
    return GNOT, cfg, ds, loader


def test_fit_matches_torch_reference_steps(tmp_path):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import torch_port
    from gnot_amd import train
    GNOT, cfg, ds, loader = _setup()
    dev = torch.device("cuda")
    model = GNOT(*cfg).to(dev)
    init = {k: v.detach().clone() for k, v in model.state_dict().items()}
    # reference replica: same init, same batches, torch AdamW + OneCycleLR stepped per epoch
    p = {k: v.clone().requires_grad_(True) for k, v in init.items()}
    opt = torch.optim.AdamW(list(p.values()), lr=1e-3, foreach=False)
    sched = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=1e-3, steps_per_epoch=len(loader), epochs=2)
    tcfg = dict(n_mlp_num_layers=2, n_expert=2, n_head=4, n_attn_layers=1, n_input_functions=1)
    ref_losses = []
    for epoch in range(2):
        for b in loader:
            opt.zero_grad()
            tot = []
            outs = []
            for i in range(len(b["x_off"]) - 1):          # one unpadded B=1 reference call per sample
                s, e = b["x_off"][i], b["x_off"][i + 1]
                fo = b["fn_offs"][0]
                o = torch_port.gnot_forward(p, tcfg, b["x"][s:e][None].to(dev), b["theta"][i:i + 1].to(dev),
                                            [b["fns"][0][fo[i]:fo[i + 1]][None].to(dev)])[0]
                outs.append(o)
            out = torch.cat(outs)
            y = b["y"].to(dev)
            for i in range(len(b["x_off"]) - 1):
                s, e = b["x_off"][i], b["x_off"][i + 1]
                tot.append((((out[s:e] - y[s:e]) ** 2).sum(0) / (y[s:e] ** 2).sum(0)).sqrt())
            loss = torch.stack(tot).mean()
            loss.backward()
            opt.step()
            ref_losses.append(float(loss))
        sched.step()
    got = []
    ckpt = os.path.join(tmp_path, "best_model.pth")
    train.fit(model, loader, loader, epochs=2, checkpoint=ckpt,
              log=lambda msg: got.append(float(msg.split(": ")[1])) if "Loss" in msg else None)
    ref_epoch = [np.mean(ref_losses[:3]), np.mean(ref_losses[3:])]
    assert np.allclose(got, ref_epoch, rtol=1e-4, atol=0), (got, ref_epoch)
    # the best checkpoint is a reference-compatible state_dict
    fresh = GNOT(*cfg)
    train.load_checkpoint(fresh, ckpt)
    assert list(fresh.state_dict().keys()) == list(init.keys())
