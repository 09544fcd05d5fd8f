"""Stock-torch CPU restatement of the reference GNOT — TEST/BASELINE INFRASTRUCTURE ONLY.

Used for exactly one thing: `bench.py`'s `cpu_baseline` leg (the reference's CPU path timed on the
GPU box's host cores, BASELINE.md "CPU-baseline plan": stock-torch math identical to the reference,
validated against the golden fixtures — tests/test_oracle.py::test_torch_port_matches_fixtures).
The reference module itself cannot travel to the GPU box, so this is the same arithmetic written
functionally over a state_dict (same op sequence: Linear + exact GELU MLPs, feature softmax,
k_sum / K^T V / alpha, head-major scramble, soft-MoE mix), run by torch's CPU kernels and autograd.

Anchors: MLP model.py:5-18; LinearAttention model.py:53-107; block model.py:126-139;
GNOT.forward model.py:154-173.
"""
import torch
import torch.nn.functional as F


def _mlp(p, prefix, h, n_lin):
    for j in range(n_lin):
        h = F.linear(h, p[f"{prefix}.layers.{2 * j}.weight"], p[f"{prefix}.layers.{2 * j}.bias"])
        if j < n_lin - 1:
            h = F.gelu(h)
    return h


def _heads(t, H):
    B, L, d = t.shape
    return t.view(B, L, H, d // H).transpose(1, 2)          # [B, H, L, dh]


def _attention(p, prefix, query, srcs, H, key_names, value_names):
    B, N, d = query.shape
    q = torch.softmax(_heads(F.linear(query, p[prefix + ".query.weight"], p[prefix + ".query.bias"]), H), -1)
    acc = 0
    for i, src in enumerate(srcs):
        k = torch.softmax(_heads(F.linear(src, p[key_names[i] + ".weight"], p[key_names[i] + ".bias"]), H), -1)
        v = _heads(F.linear(src, p[value_names[i] + ".weight"], p[value_names[i] + ".bias"]), H)
        z = k.sum(2, keepdim=True)
        state = k.transpose(-2, -1) @ v
        acc = acc + (q @ state) / (q * z).sum(-1, keepdim=True)
    res = (q + acc / len(srcs)).reshape(B, N, d)              # head-major flat order (the scramble)
    return F.linear(res, p[prefix + ".fc_out.weight"], p[prefix + ".fc_out.bias"])


def gnot_forward(p, cfg, x, theta, fns):
    """x [B,N,in], theta [B,th], fns list of [B,M,F] (tensors); p: state_dict of tensors."""
    n_lin = max(cfg["n_mlp_num_layers"], 1) + 1
    E, H, L, I = cfg["n_expert"], cfg["n_head"], cfg["n_attn_layers"], cfg["n_input_functions"]
    s = torch.softmax(_mlp(p, "gating", x, n_lin), -1)
    xin = torch.cat([x, theta[:, None, :].expand(-1, x.shape[1], -1)], -1)
    query = _mlp(p, "x", xin, n_lin)
    enc = [_mlp(p, f"input_func_mlps.{i}", fns[i], n_lin) for i in range(I)]
    for l in range(L):
        pre = f"blocks.{l}"
        if I > 0:
            kn = [f"{pre}.cross_attention.key.{i}" for i in range(I)]
            vn = [f"{pre}.cross_attention.value.{i}" for i in range(I)]
            a = _attention(p, pre + ".cross_attention", query, enc, H, kn, vn)
        else:
            a = _attention(p, pre + ".cross_attention", query, [query], H, [pre + ".cross_attention.key"],
                           [pre + ".cross_attention.value"])
        query = query + sum(s[..., e:e + 1] * _mlp(p, f"{pre}.ffn1.{e}", a, n_lin) for e in range(E))
        b = _attention(p, pre + ".self_attention", query, [query], H, [pre + ".self_attention.key"],
                       [pre + ".self_attention.value"])
        query = query + sum(s[..., e:e + 1] * _mlp(p, f"{pre}.ffn2.{e}", b, n_lin) for e in range(E))
    return _mlp(p, "out", query, n_lin)
