"""Generate the golden GNOT fixtures from the reference implementation.

Test infrastructure only.  Run HERE (the survey container), never on the GPU box:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [case ...]

It imports `/root/reference/model.py` unchanged (it only depends on torch), builds
`GNOT(...)` (model.py:142-173) in float64, runs forward + backward with a fixed upstream
gradient G (loss = sum(out * G)), and stores inputs, the state_dict, the output and every
parameter gradient as plain arrays in `tests/golden/<case>.npz` (no pickles).

Two calling conventions are captured:
  * "padded": ONE batched reference call on zero-padded tensors, exactly as main.py:60-84 builds
    them (pad to the batch max N, pad every input function to one common max M, utils.py:3-4).
  * "packed": one B=1 unpadded reference call per sample (what packed offsets must reproduce,
    SURVEY.md §0.3); the outputs are concatenated and the gradients summed over samples.

Every array is stored packed ([sum rows, feat] + offsets[B+1]) so the oracle and the GPU path
read one format; for "padded" cases every sample has the padded length.
"""
import json
import os
import sys

import numpy as np
import torch

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

CASES = [
    # name, mode, model cfg, lengths
    dict(name="self_only_pad", mode="padded",
         cfg=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=2, n_attn_layers=2,
                  d=32, n_mlp_num_layers=2, n_expert=2, n_head=4, n_input_functions=0),
         N=[37, 30], M=[]),
    dict(name="cross1", mode="padded",
         cfg=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=2,
                  d=32, n_mlp_num_layers=4, n_expert=3, n_head=2, n_input_functions=1),
         N=[53], M=[[29]]),
    dict(name="cross2_packed", mode="packed",
         cfg=dict(input_dim=3, theta_dim=2, input_func_dim=3, out_dim=3, n_attn_layers=1,
                  d=32, n_mlp_num_layers=3, n_expert=2, n_head=1, n_input_functions=2),
         N=[41, 17, 26], M=[[19, 7, 11], [13, 22, 5]]),
    dict(name="main_pad_h8", mode="padded",
         cfg=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=2,
                  d=32, n_mlp_num_layers=2, n_expert=3, n_head=8, n_input_functions=1),
         N=[40, 25, 33], M=[[20, 12, 17]]),
    dict(name="d64_cross", mode="padded",
         cfg=dict(input_dim=2, theta_dim=1, input_func_dim=4, out_dim=2, n_attn_layers=1,
                  d=64, n_mlp_num_layers=2, n_expert=2, n_head=4, n_input_functions=1),
         N=[70], M=[[33]]),
    dict(name="tiny_n_lt_h", mode="packed",
         cfg=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=1,
                  d=32, n_mlp_num_layers=1, n_expert=1, n_head=8, n_input_functions=1),
         N=[3, 5], M=[[5, 2]]),
    dict(name="cross1_sharp", mode="packed", sharp=6.0,
         cfg=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=2, n_attn_layers=2,
                  d=32, n_mlp_num_layers=2, n_expert=3, n_head=2, n_input_functions=1),
         N=[45, 31], M=[[23, 9]]),
    dict(name="self_sharp_h8", mode="padded", sharp=6.0,
         cfg=dict(input_dim=3, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=1,
                  d=64, n_mlp_num_layers=2, n_expert=2, n_head=8, n_input_functions=0),
         N=[38, 38], M=[]),
    dict(name="d48_h3_self", mode="packed",
         cfg=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=2, n_attn_layers=1,
                  d=48, n_mlp_num_layers=2, n_expert=2, n_head=3, n_input_functions=0),
         N=[29, 18], M=[]),
    # round 6: the BASELINE workloads' head shapes.  Multi-head dh = 32 (the headline's attention kernels
    # are templated on dh; configs[2] runs dh = 32 with H = 8)
    dict(name="d64_h2_mh", mode="packed", sharp=4.0, fp32_params=True,
         cfg=dict(input_dim=3, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=2,
                  d=64, n_mlp_num_layers=2, n_expert=3, n_head=2, n_input_functions=1),
         N=[150, 97], M=[[60, 41]]),
    # configs[2]'s expert count and MLP depth (E = 8, nl = 4) at a small width
    dict(name="d32_e8_nl4", mode="padded", fp32_params=True,
         cfg=dict(input_dim=3, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=2,
                  d=32, n_mlp_num_layers=4, n_expert=8, n_head=4, n_input_functions=1),
         N=[80, 64], M=[[30, 25]]),
    # configs[1]'s shape: d = 128, 8 heads (dh = 16), 4 experts, 2 input functions (one block)
    dict(name="d128_h8_e4_i2", mode="packed", sharp=3.0, fp32_params=True,
         cfg=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=1,
                  d=128, n_mlp_num_layers=1, n_expert=4, n_head=8, n_input_functions=2),
         N=[120, 75], M=[[50, 30], [44, 20]]),
    # round 6: one head of 128 (attn.hip's wide forms: 16 lanes per head, quads round-robin)
    dict(name="d128_h1_wide", mode="packed", sharp=3.0, fp32_params=True,
         cfg=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=1,
                  d=128, n_mlp_num_layers=1, n_expert=2, n_head=1, n_input_functions=1),
         N=[60, 41], M=[[30, 17]]),
    # padded heads (4 heads of 25, run as heads of 28 at an internal width of 112), padded calling convention
    dict(name="d100_h4_padheads", mode="padded", sharp=3.0, fp32_params=True,
         cfg=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=2, n_attn_layers=1,
                  d=100, n_mlp_num_layers=1, n_expert=2, n_head=4, n_input_functions=1),
         N=[40, 27], M=[[19, 12]]),
]


def build_model(model_mod, c):
    d = c["d"]
    return model_mod.GNOT(c["input_dim"], c["theta_dim"], c["input_func_dim"], c["out_dim"],
                          c["n_attn_layers"], d, c["n_mlp_num_layers"], d, d,
                          c["n_expert"], c["n_head"], c["n_input_functions"]).double()


def sharpen(model, factor):
    """Scale every attention query/key projection so the feature softmaxes are far from uniform.
    At nn.Linear's default init q and k are nearly uniform and the key-path gradients are ~1e-13
    (pure cancellation); these cases keep the attention gradients well conditioned."""
    with torch.no_grad():
        for name, p in model.named_parameters():
            if ".query." in name or ".key." in name:
                p.mul_(factor)


def forward_backward(model, case, xs, theta, fns, Gs):
    """Run the reference on the case's inputs (backward included); returns per-sample outputs."""
    I = len(fns)
    B = len(xs)
    model.zero_grad()
    if case["mode"] == "padded":
        nmax = max(t.shape[0] for t in xs)
        mmax = max([t.shape[0] for row in fns for t in row], default=0)
        pad = lambda t, L: torch.nn.functional.pad(t, (0, 0, 0, L - t.shape[0]))  # utils.py:3-4
        X = torch.stack([pad(t, nmax) for t in xs])
        F = torch.stack([torch.stack([pad(t, mmax) for t in row]) for row in fns]) if I > 0 else None
        out = model(X, theta, F)
        (out * torch.stack([pad(t, nmax) for t in Gs])).sum().backward()
        return [out[b].detach() for b in range(B)]
    outs = []
    for b in range(B):
        F = [fns[i][b].unsqueeze(0) for i in range(I)] if I > 0 else None
        o = model(xs[b].unsqueeze(0), theta[b:b + 1], F)[0]
        (o * Gs[b]).sum().backward()
        outs.append(o.detach())
    return outs


def run_case(model_mod, case, seed):
    c = case["cfg"]
    torch.manual_seed(seed)
    model = build_model(model_mod, c)
    if case.get("sharp"):
        sharpen(model, case["sharp"])
    if case.get("fp32_params"):
        # fp32-representable weights, stored as float32 (exact): halves the fixture, and the fp32 GPU path
        # runs on exactly the weights the float64 reference used
        with torch.no_grad():
            for p in model.parameters():
                p.copy_(p.float().double())
    g = torch.Generator().manual_seed(1000 + seed)
    I = c["n_input_functions"]
    Ns = case["N"]
    B = len(Ns)
    Ms = case["M"]  # Ms[i][b]
    xs = [torch.rand(n, c["input_dim"], generator=g, dtype=torch.float64) for n in Ns]
    theta = torch.rand(B, c["theta_dim"], generator=g, dtype=torch.float64)
    fns = [[torch.rand(Ms[i][b], c["input_func_dim"], generator=g, dtype=torch.float64)
            for b in range(B)] for i in range(I)]
    Gs = [torch.randn(n, c["out_dim"], generator=g, dtype=torch.float64) for n in Ns]

    outs = forward_backward(model, case, xs, theta, fns, Gs)
    grads64 = {k: p.grad.clone() for k, p in model.named_parameters()}
    # the reference's own fp32 error (same weights/inputs, float32): the conditioning yardstick
    m32 = build_model(model_mod, c).float()
    m32.load_state_dict({k: v.float() for k, v in model.state_dict().items()})
    outs32 = forward_backward(m32, case, [t.float() for t in xs], theta.float(),
                              [[t.float() for t in row] for row in fns], [t.float() for t in Gs])
    if case["mode"] == "padded":
        nmax = max(Ns)
        mmax = max([m for row in Ms for m in row], default=0)
        pad = lambda t, L: torch.nn.functional.pad(t, (0, 0, 0, L - t.shape[0]))  # utils.py:3-4
        xs = [pad(t, nmax) for t in xs]
        Gs = [pad(t, nmax) for t in Gs]
        fns = [[pad(t, mmax) for t in row] for row in fns]
        Ns_store = [nmax] * B
        Ms_store = [[mmax] * B for _ in range(I)]
    else:
        Ns_store = Ns
        Ms_store = Ms

    arrs = {}
    cat = lambda ts: torch.cat(ts).numpy() if ts else np.zeros((0,))
    off = lambda lens: np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    arrs["x"] = cat(xs)
    arrs["x_off"] = off(Ns_store)
    arrs["theta"] = theta.numpy()
    for i in range(I):
        arrs[f"fn{i}"] = cat(fns[i])
        arrs[f"fn{i}_off"] = off(Ms_store[i])
    arrs["G"] = cat(Gs)
    arrs["out"] = cat(outs)
    for k, v in model.state_dict().items():
        arrs["p." + k] = v.float().numpy() if case.get("fp32_params") else v.numpy()
    for k, p in model.named_parameters():
        arrs["g." + k] = grads64[k].numpy()
        g32 = dict(m32.named_parameters())[k].grad.double()
        arrs["e32." + k] = np.array(float((g32 - grads64[k]).norm()))
    arrs["e32.out"] = np.array(float((torch.cat(outs32).double() - torch.cat(outs)).abs().max()))
    meta = dict(case)
    meta["seed"] = seed
    meta["real_N"] = Ns
    arrs["meta"] = np.array(json.dumps(meta))
    return arrs


def main():
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    import model as model_mod  # /root/reference/model.py
    only = set(sys.argv[1:])               # optional: case names to (re)generate
    for case in CASES:
        if only and case["name"] not in only:
            continue
        arrs = run_case(model_mod, case, seed=7)
        path = os.path.join(HERE, case["name"] + ".npz")
        np.savez_compressed(path, **arrs)
        print(f"{case['name']}: {os.path.getsize(path)/1024:.1f} KiB, out {arrs['out'].shape}")


if __name__ == "__main__":
    main()
