#!/usr/bin/env python3
"""Train GNOT on NS2d-format data with the MI355X core: the reference's main.py (argparse flags of
main.py:15-23, batch 4, AdamW lr 1e-3, OneCycleLR stepped per epoch, RelL2 metric, best checkpoint)
with plain tensors instead of dgl graphs.  Batches are zero-padded exactly like main.py:60-89 by
default (the pad rows enter the attention sums, as in the reference); --packed uses packed offsets.

    python scripts/train_ns2d.py --train train.pkl --test test.pkl [--epochs 100 ...]
    python scripts/train_ns2d.py --synthetic 64 --epochs 2          # generated meshes, same format
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnot-replication_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gnot_amd import GNOT, data, train  # noqa: E402


def main():
    ap = argparse.ArgumentParser(description="GNOT (MI355X)")
    ap.add_argument("--gpu_id", type=int, default=0)
    ap.add_argument("--n_attn_layers", type=int, default=4)
    ap.add_argument("--n_attn_hidden_dim", type=int, default=256)
    ap.add_argument("--n_mlp_num_layers", type=int, default=4)
    ap.add_argument("--n_mlp_hidden_dim", type=int, default=256)
    ap.add_argument("--n_input_hidden_dim", type=int, default=256)
    ap.add_argument("--n_expert", type=int, default=3)
    ap.add_argument("--n_head", type=int, default=8)
    ap.add_argument("--epochs", type=int, default=100)
    ap.add_argument("--train")
    ap.add_argument("--test")
    ap.add_argument("--synthetic", type=int, default=0, help="generate this many training meshes instead")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--per-batch-schedule", action="store_true", help="step OneCycleLR per batch (main.py steps it per epoch)")
    ap.add_argument("--checkpoint", default="best_model.pth")
    ap.add_argument("--packed", action="store_true",
                    help="packed batches (per-sample exact); default: main.py's zero-padded batches")
    args = ap.parse_args()
    if args.synthetic:
        rng = np.random.default_rng(0)
        tr = data.NS2dData([data.synthetic_sample(rng, int(rng.integers(1000, 4000))) for _ in range(args.synthetic)])
        te = data.NS2dData([data.synthetic_sample(rng, int(rng.integers(1000, 4000))) for _ in range(max(4, args.synthetic // 8))])
    else:
        tr, te = data.NS2dData(args.train), data.NS2dData(args.test)
    x0, y0, th0, f0 = tr[0]
    dev = torch.device("cuda", args.gpu_id)
    model = GNOT(x0.shape[1], len(np.atleast_1d(th0)), f0[0].shape[1], y0.shape[1], args.n_attn_layers,
                 args.n_attn_hidden_dim, args.n_mlp_num_layers, args.n_mlp_hidden_dim, args.n_input_hidden_dim,
                 args.n_expert, args.n_head, len(f0)).to(dev)
    dl = lambda ds, sh: torch.utils.data.DataLoader(ds, batch_size=args.batch, shuffle=sh,
                                                    collate_fn=data.collate_packed if args.packed
                                                    else data.collate_padded)
    _, test = train.fit(model, dl(tr, True), dl(te, False), epochs=args.epochs,
                        per_epoch_schedule=not args.per_batch_schedule, checkpoint=args.checkpoint)
    print(f"\nBest Test Metric: {min(test)}")


if __name__ == "__main__":
    main()
