"""Multi-GPU host logic on CPU: shard ranges, the scramble all-to-all tables (C ABI, no GPU), LPT
sample balancing, and world_size-2 gloo runs of the point-sharded attention algebra and the sharded
RelL2 loss through the product's own collective glue (gnot_amd.parallel.PointShardComm)."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gnot_amd import parallel as par


# ------------------------------------------------------------------ tables (single process)
@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
def test_shard_ranges_tile_the_sample(world):
    for n in (0, 1, 7, 10, 1000, 1_048_576):
        rs = [par.shard_range(n, r, world) for r in range(world)]
        assert rs[0][0] == 0 and rs[-1][1] == n
        assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
        assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1


def _simulate_exchange(n_global, H, dh, world):
    """Run every rank's send/recv segments in-process; returns per-rank token buffers and the ids."""
    plans = [par.exchange_plan(n_global, H, dh, r, world) for r in range(world)]
    d = H * dh
    ident = lambda b, h, n: (b * 1000 + h) * 100000 + n       # unique per (sample, head, point)
    hms, sends = [], []
    for r in range(world):
        off, ranges = par.shard_offsets(n_global, r, world)
        hm = np.zeros(off[-1] * d)
        for b, (lo, hi) in enumerate(ranges):
            cnt = hi - lo
            for h in range(H):
                for i in range(cnt):
                    base = off[b] * d + (h * cnt + i) * dh
                    hm[base: base + dh] = ident(b, h, lo + i) * 10 + np.arange(dh)
        sc, rc, segs = plans[r]
        send = np.zeros(sum(sc))
        for dirn, loc, buf, ln in segs:
            if dirn == 0:
                send[buf: buf + ln] = hm[loc: loc + ln]
        hms.append(hm)
        sends.append(send)
    toks = []
    for t in range(world):
        pieces = []
        for s in range(world):
            sc = plans[s][0]
            start = sum(sc[:t])
            pieces.append(sends[s][start: start + sc[t]])
        recv = np.concatenate(pieces) if pieces else np.zeros(0)
        assert recv.size == sum(plans[t][1])
        off, _ = par.shard_offsets(n_global, t, world)
        tok = np.full(off[-1] * d, -1.0)
        for dirn, loc, buf, ln in plans[t][2]:
            if dirn == 1:
                tok[loc: loc + ln] = recv[buf: buf + ln]
        toks.append(tok)
    return plans, hms, toks, ident


@pytest.mark.parametrize("world,H,dh,ns", [(1, 8, 4, [13]), (2, 8, 4, [37, 30]), (3, 3, 8, [29, 5, 18]),
                                            (4, 1, 4, [9]), (5, 8, 4, [3, 41]), (8, 8, 4, [100])])
def test_exchange_realises_the_reference_scramble(world, H, dh, ns):
    """Token n' of sample b = flat rows n'H .. n'H+H-1 of the head-major [H, N, dh] array
    (model.py:81 / 103-104); after the all-to-all every rank holds exactly its tokens."""
    plans, hms, toks, ident = _simulate_exchange(ns, H, dh, world)
    for t in range(world):
        off, ranges = par.shard_offsets(ns, t, world)
        for b, (lo, hi) in enumerate(ranges):
            N = ns[b]
            for i, tokn in enumerate(range(lo, hi)):
                for jj in range(H):
                    r = tokn * H + jj
                    h, n = divmod(r, N)
                    base = (off[b] + i) * H * dh + jj * dh
                    assert np.array_equal(toks[t][base: base + dh], ident(b, h, n) * 10 + np.arange(dh))
    # send/recv volumes are consistent between every pair of ranks
    for s in range(world):
        for t in range(world):
            assert plans[s][0][t] == plans[t][1][s]


def test_lpt_partition_balances_and_covers():
    rng = np.random.default_rng(0)
    sizes = list(rng.integers(1000, 50000, size=64))          # BASELINE configs[4]: 64 meshes, 1k-50k
    parts = par.lpt_partition(sizes, 8)
    assert sorted(i for p in parts for i in p) == list(range(64))
    loads = [sum(sizes[i] for i in p) for p in parts]
    assert max(loads) - min(loads) <= max(sizes)
    assert max(loads) / (sum(sizes) / 8) < 1.05
    assert parts == par.lpt_partition(sizes, 8)               # deterministic


# ------------------------------------------------------------------ gloo world_size 2
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(world, fn, *args):
    port = _free_port()
    mp.start_processes(_entry, args=(world, port, fn, args), nprocs=world, join=True, start_method="spawn")


def _entry(rank, world, port, fn, args):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fn(rank, world, *args)
    finally:
        dist.destroy_process_group()


def _sharded_attention(rank, world, I, seed):
    """One self-attention call (model.py:88-106) of a mesh point-sharded over `world` gloo ranks,
    computed with the oracle's algebra, the engine's exchange tables and PointShardComm's
    callbacks on a CPU 'workspace'; compared with the unsharded oracle call."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import gnot_oracle as O
    rng = np.random.default_rng(seed)
    H, dh, N = 4, 8, 23
    d = H * dh
    params = {}
    for name in ("a.query", "a.key", "a.value", "a.fc_out"):
        params[name + ".weight"] = rng.standard_normal((d, d)) * 0.5
        params[name + ".bias"] = rng.standard_normal(d) * 0.1
    P = O.Params(params, np.float64)
    query = rng.standard_normal((N, d))
    ref, _ = O.attn_fwd(P, "a", query, None, H, ["a.key"], ["a.value"])

    lo, hi = par.shard_range(N, rank, world)
    ql = query[lo:hi]
    q = O.softmax(O.to_heads(P.linear("a.query", ql), H), -1)
    k = O.softmax(O.to_heads(P.linear("a.key", ql), H), -1)
    v = O.to_heads(P.linear("a.value", ql), H)
    # "workspace": [state | hm | send | recv | tok] float32 regions of one CPU tensor
    n_state = H * (dh * dh + dh)
    nloc = (hi - lo) * d
    ws = torch.zeros(4 * (n_state + 4 * nloc + 64), dtype=torch.uint8)
    f = ws.view(torch.float32)
    comm = par.PointShardComm()
    comm.ws = ws
    st = np.concatenate([np.concatenate([(k[h].T @ v[h]).ravel(), k[h].sum(0)]) for h in range(H)])
    f[:n_state] = torch.from_numpy(st)
    assert comm._allreduce(None, ws.data_ptr(), n_state, None) == 0      # S, z over all ranks
    st = f[:n_state].double().numpy().reshape(H, dh * dh + dh)
    S = st[:, : dh * dh].reshape(H, dh, dh)
    z = st[:, dh * dh:][:, None, :]
    o = (q @ S) / (q * z).sum(-1, keepdims=True)
    hm_off, send_off, recv_off = n_state, n_state + nloc, n_state + 2 * nloc
    tok_off = n_state + 3 * nloc
    f[hm_off: hm_off + nloc] = torch.from_numpy((q + o).ravel())       # head-major local [H, n, dh]
    sc, rc, segs = par.exchange_plan([N], H, dh, rank, world)
    for dirn, loc, buf, ln in segs:
        if dirn == 0:
            f[send_off + buf: send_off + buf + ln] = f[hm_off + loc: hm_off + loc + ln]
    SC = (ctypes.c_int64 * world)(*sc)
    RC = (ctypes.c_int64 * world)(*rc)
    assert comm._alltoallv(None, ws.data_ptr() + 4 * send_off, SC, ws.data_ptr() + 4 * recv_off, RC, None) == 0
    for dirn, loc, buf, ln in segs:
        if dirn == 1:
            f[tok_off + loc: tok_off + loc + ln] = f[recv_off + buf: recv_off + buf + ln]
    res = f[tok_off: tok_off + nloc].double().numpy().reshape(hi - lo, d)
    out = P.linear("a.fc_out", res)
    err = np.abs(out - ref[lo:hi]).max()
    assert err < 1e-5, err


@pytest.mark.parametrize("world", [2, 3])
def test_point_sharded_attention_gloo(world):
    _run(world, _sharded_attention, 0, 5)


def _sharded_loss(rank, world):
    torch.manual_seed(0)
    B, N, C = 2, 11, 2
    out = torch.randn(B * N, C, dtype=torch.float64, requires_grad=True)
    tgt = torch.randn(B * N, C, dtype=torch.float64)
    seg = torch.arange(B).repeat_interleave(N)
    # unsharded reference (loss.py:14-23)
    num = torch.zeros(B, C, dtype=torch.float64).index_add(0, seg, (out - tgt) ** 2)
    den = torch.zeros(B, C, dtype=torch.float64).index_add(0, seg, tgt ** 2)
    ref = (num / den).sqrt().mean()
    ref.backward()
    g_ref = out.grad.clone()
    # this rank's slice of every sample
    idx = torch.cat([torch.arange(b * N + par.shard_range(N, rank, world)[0], b * N + par.shard_range(N, rank, world)[1])
                     for b in range(B)])
    ol = out.detach()[idx].clone().requires_grad_(True)
    loss = par.rel_l2_loss_sharded(ol, tgt[idx], seg[idx], B)
    loss.backward()
    assert abs(float(loss) - float(ref)) < 1e-12
    assert torch.allclose(ol.grad, g_ref[idx], rtol=0, atol=1e-12)


def test_sharded_rel_l2_loss_gloo():
    _run(2, _sharded_loss)
