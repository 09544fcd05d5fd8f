"""Point-sharded GNOT forward + backward through the HIP engine (gnot_plan_set_shard + the
PointShardComm callbacks): `world` processes share cuda:0 over gloo (host-staged collectives, the
box has one GPU), each owns a contiguous slice of every sample's points.  The
gathered outputs and the rank-summed parameter gradients must match the unsharded CPU oracle."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _case(cfg, Ns, Ms, seed):
    from golden_util import model_args
    from gnot_amd import GNOT
    from oracle import gnot_oracle as O
    torch.manual_seed(seed)
    ref = GNOT(*model_args(cfg))
    params = {k: v.double().numpy() for k, v in ref.state_dict().items()}
    rng = np.random.default_rng(seed)
    x = rng.random((sum(Ns), cfg["input_dim"]))
    theta = rng.random((len(Ns), cfg["theta_dim"]))
    fns = [rng.random((sum(Ms[i]), cfg["input_func_dim"])) for i in range(cfg["n_input_functions"])]
    off = lambda L: np.concatenate([[0], np.cumsum(L)]).astype(np.int64)
    G = rng.standard_normal((sum(Ns), cfg["out_dim"]))
    fx = dict(params=params, cfg=cfg, x=x, x_off=off(Ns), theta=theta, fns=fns,
              fn_offs=[off(Ms[i]) for i in range(cfg["n_input_functions"])], G=G)
    out64, g64 = O.gnot_forward_backward(params, cfg, x, fx["x_off"], theta, fns, fx["fn_offs"], G=G)
    out32, g32 = O.gnot_forward_backward(params, cfg, x, fx["x_off"], theta, fns, fx["fn_offs"], G=G,
                                         dtype=np.float32)
    fx["out"], fx["grads"] = out64, g64
    fx["e32"] = {k: float(np.linalg.norm(g32[k].astype(np.float64) - g64[k])) for k in g64}
    return fx


def _rank(rank, world, port, cfg, Ns, Ms, q, backend="gloo", fx=None, env=None):
    """One rank: its slice of every sample through the sharded engine; rank 0 gathers and checks.  `fx`
    (with fx["G"]): a precomputed case (else _case(cfg, Ns, Ms)); `env`: environment for the rank."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "gnot-replication_amd"), os.path.join(ROOT, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.update(env or {})
    if backend == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from golden_util import check_parity, model_args
        from gnot_amd import GNOT
        from gnot_amd import parallel as par
        if fx is None:
            fx = _case(cfg, Ns, Ms, seed=11)
        dev = torch.device("cuda", 0)
        m = GNOT(*model_args(cfg)).to(dev)
        m.load_state_dict({k: torch.from_numpy(v).float() for k, v in fx["params"].items()})
        m.set_point_shard(par.PointShardComm(stage_via_host=backend != "nccl"))
        loc_off, ranges = par.shard_offsets(Ns, rank, world)
        rows = np.concatenate([np.arange(fx["x_off"][b] + lo, fx["x_off"][b] + hi) for b, (lo, hi) in enumerate(ranges)])
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).float().to(dev)
        out = m.forward_packed(t(fx["x"][rows]), loc_off, t(fx["theta"]), [t(f) for f in fx["fns"]],
                               [o.tolist() for o in fx["fn_offs"]], n_global=Ns)
        (out * t(fx["G"][rows])).sum().backward()
        flat = m.engine().grad_flat
        if backend == "nccl":
            dist.all_reduce(flat)              # parameter gradients: sum over ranks (RCCL)
        else:
            h = flat.cpu()
            dist.all_reduce(h)                 # parameter gradients: sum over ranks
            flat.copy_(h.to(dev))
        torch.cuda.synchronize()
        outs = [None] * world
        dist.all_gather_object(outs, (rows, out.detach().double().cpu().numpy()))
        if rank == 0:
            full = np.zeros_like(fx["out"])
            for r_rows, o in outs:
                full[r_rows] = o
            grads = {k: p.grad.double().cpu().numpy() for k, p in m.named_parameters()}
            q.put(check_parity(full, grads, fx))
    except Exception as e:  # report instead of hanging the other rank's collectives
        if rank == 0:
            q.put([f"rank0 exception: {e!r}"])
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,case", [
    (2, dict(cfg=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=2, n_attn_layers=2, d=64,
                      n_mlp_num_layers=2, n_expert=3, n_head=8, n_input_functions=1),
             Ns=[150, 97], Ms=[[40, 31]])),
    (2, dict(cfg=dict(input_dim=3, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=1, d=64,
                      n_mlp_num_layers=2, n_expert=2, n_head=4, n_input_functions=0),
             Ns=[131], Ms=[])),
    (3, dict(cfg=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=1, d=32,
                      n_mlp_num_layers=2, n_expert=2, n_head=8, n_input_functions=2),
             Ns=[64, 5], Ms=[[20, 9], [7, 12]])),
])
def test_point_sharded_gnot_matches_oracle(world, case):
    _run_sharded_case(world, case)


@pytest.mark.parametrize("world,case", [
    # padded hidden widths (the kernels run D > d with exact-zero pad columns; the scramble rows, the states
    # and the exchange tables use the real width d = H * dh): d = 100 (5 heads of 20, kernels at 112) and
    # d = 208 (13 heads of 16, the d = 256 kernels)
    (2, dict(cfg=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=2, n_attn_layers=2, d=100,
                      n_mlp_num_layers=2, n_expert=3, n_head=5, n_input_functions=1),
             Ns=[150, 97], Ms=[[40, 31]])),
    (3, dict(cfg=dict(input_dim=3, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=1, d=208,
                      n_mlp_num_layers=2, n_expert=2, n_head=13, n_input_functions=0),
             Ns=[131, 40], Ms=[])),
    # padded HEADS: 4 heads of 25 (run as heads of 28; the scramble exchange at the real head width)
    (2, dict(cfg=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=2, n_attn_layers=1, d=100,
                      n_mlp_num_layers=2, n_expert=2, n_head=4, n_input_functions=1),
             Ns=[121, 66], Ms=[[33, 20]])),
    # heads of 25 padded to 28 past an internal 192: kernels at 320 (one Linear at a time)
    (2, dict(cfg=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=1, d=250,
                      n_mlp_num_layers=2, n_expert=2, n_head=10, n_input_functions=1),
             Ns=[90, 61], Ms=[[30, 22]])),
    # d = 576 (kernels at 640: K-split projections; the exchange at the real width)
    (2, dict(cfg=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=1, d=576,
                      n_mlp_num_layers=2, n_expert=2, n_head=9, n_input_functions=1),
             Ns=[70, 45], Ms=[[25, 18]])),
    # one head of 128 (attn.hip's wide forms; the state all-reduce and scramble exchange at dh = 128)
    (2, dict(cfg=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=1, d=128,
                      n_mlp_num_layers=2, n_expert=2, n_head=1, n_input_functions=1),
             Ns=[140, 57], Ms=[[30, 22]])),
])
def test_point_sharded_padded_widths(world, case):
    _run_sharded_case(world, case)


def _run_sharded_case(world, case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, case["cfg"], case["Ns"], case["Ms"], q))
             for r in range(world)]
    for p in procs:
        p.start()
    errs = q.get(timeout=100)
    for p in procs:
        p.join(timeout=30)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert not errs, errs


def test_point_sharded_gnot_rccl_path():
    """The RCCL branch of PointShardComm (collectives issued on the engine's stream through a torch
    ExternalStream, no host staging) at world size 1 -- the only RCCL world a one-GPU box can form: the
    state all-reduces and scramble all-to-alls run through RCCL on device buffers, the result must still
    match the oracle.  (N > 1 ranks over RCCL runs in the driver's multi-GPU bench.)"""
    case = dict(cfg=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=2, n_attn_layers=2, d=64,
                         n_mlp_num_layers=2, n_expert=3, n_head=8, n_input_functions=1),
                Ns=[150, 97], Ms=[[40, 31]])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rank, args=(0, 1, _free_port(), case["cfg"], case["Ns"], case["Ms"], q, "nccl"))
    p.start()
    errs = q.get(timeout=100)
    p.join(timeout=30)
    assert p.exitcode == 0, p.exitcode
    assert not errs, errs


@pytest.mark.timeout(600)
@pytest.mark.parametrize("overlap", ["auto", "0"])
def test_point_sharded_configs3_widths_70k_points(mid_case, overlap):
    """configs[3]'s model widths (d=256, 8 heads, 8 experts, 4-layer MLPs, one 805-point input function;
    L = 1 block) on one 70,000-point mesh split over 2 ranks (35,000 points each, gloo host staging on one
    GPU) vs the float64 oracle at 1e-4: the sharded run takes the kernels a 1M / 8 rank does -- the MFMA
    attention apply / K-V backward (>= 8,192 points), the MFMA state partials (GNOT_STATE_MFMA_MIN=16384
    in the ranks: per-rank groups of 35,000 points), the wide weight gradients -- and real exchange
    tables (the scramble of 8 heads over 70,000 points is 16 runs per rank pair).  Anchor: the all-point
    state sums model.py:98-100 (all-reduced) and the head-major reshape model.py:103-104 (all-to-all).
    overlap "auto": 35,000 points per rank fork their weight gradients onto the side stream; "0"
    (GNOT_WGRAD_OVERLAP=0) runs them serially on the caller's stream, the form every N > 1 bench rank of
    configs[2]/[3] takes.  With the opt-in fused soft-MoE combine (an inter-workgroup hand-off) this setting
    -- the other rank's process and side2's input-function branch sharing the GPU -- returned wrong block-0
    cross-attention gradients in round 4 (r04sf) and again in round 5 (r05c, all gradients 5.5e2 off); the
    default combine pass has no hand-off."""
    fx, G = mid_case
    fx = dict(fx, G=G)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    env = {"GNOT_STATE_MFMA_MIN": "16384"}
    if overlap != "auto":
        env["GNOT_WGRAD_OVERLAP"] = overlap
    procs = [ctx.Process(target=_rank, args=(r, world, port, fx["cfg"], [int(fx["x_off"][-1])], [[805]], q),
                         kwargs=dict(fx=fx, env=env))
             for r in range(world)]
    for p in procs:
        p.start()
    errs = q.get(timeout=400)
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert not errs, errs


def _rank_input_grads(rank, world, port, cfg, Ns, Ms, q):
    """Input gradients of a point-sharded batch: each rank differentiates its slice of x; theta and the
    (replicated) input functions get one partial per rank, summed over the ranks inside gnot_input_grads."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "gnot-replication_amd"), os.path.join(ROOT, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from golden_util import model_args
        from gnot_amd import GNOT
        from gnot_amd import parallel as par
        from test_gpu_input_grads import _port_grads, _rel
        torch.manual_seed(5)
        m = GNOT(*model_args(cfg))
        sd64 = {k: v.detach().double() for k, v in m.state_dict().items()}
        dev = torch.device("cuda", 0)
        m = m.to(dev)
        m.set_point_shard(par.PointShardComm(stage_via_host=True))
        rng = np.random.default_rng(3)
        I = cfg["n_input_functions"]
        xs = [rng.random((n, cfg["input_dim"])) for n in Ns]
        thetas = [rng.random(cfg["theta_dim"]) for _ in Ns]
        fns_ps = [[rng.random((Ms[i][b], cfg["input_func_dim"])) for i in range(I)] for b in range(len(Ns))]
        Gs = [rng.standard_normal((n, cfg["out_dim"])) for n in Ns]
        loc_off, ranges = par.shard_offsets(Ns, rank, world)
        t = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float32, device=dev)
        x = t(np.concatenate([xs[b][lo:hi] for b, (lo, hi) in enumerate(ranges)])).requires_grad_(True)
        th = t(np.stack(thetas)).requires_grad_(True)
        fns = [t(np.concatenate([fns_ps[b][i] for b in range(len(Ns))])).requires_grad_(True) for i in range(I)]
        fn_offs = [np.concatenate([[0], np.cumsum([Ms[i][b] for b in range(len(Ns))])]).tolist() for i in range(I)]
        G = t(np.concatenate([Gs[b][lo:hi] for b, (lo, hi) in enumerate(ranges)]))
        out = m.forward_packed(x, loc_off, th, fns, fn_offs, n_global=Ns)
        (out * G).sum().backward()
        torch.cuda.synchronize()
        got = (x.grad.double().cpu().numpy(), th.grad.double().cpu().numpy(), [f.grad.double().cpu().numpy() for f in fns])
        parts = [None] * world
        dist.all_gather_object(parts, (ranges, got))
        if rank == 0:
            rx, rt, rf = _port_grads(cfg, sd64, xs, thetas, fns_ps, Gs)
            dx = [np.zeros_like(r) for r in rx]
            for rgs, (gx, _, _) in parts:
                k = 0
                for b, (lo, hi) in enumerate(rgs):
                    dx[b][lo:hi] = gx[k:k + hi - lo]
                    k += hi - lo
            errs = []
            e = _rel(np.concatenate(dx), np.concatenate(rx))
            if not e <= 1e-4:   # NaN fails
                errs.append(f"dx {e:.3e}")
            for r, (_, (_, gt, gf)) in enumerate(parts):   # every rank holds the rank sums
                e = _rel(gt, np.stack(rt))
                if not e <= 1e-4:   # NaN fails
                    errs.append(f"rank {r} dtheta {e:.3e}")
                for i in range(I):
                    e = _rel(gf[i], np.concatenate([rf[b][i] for b in range(len(Ns))]))
                    if not e <= 1e-4:   # NaN fails
                        errs.append(f"rank {r} dfn{i} {e:.3e}")
            q.put(errs)
    except Exception as e:
        if rank == 0:
            q.put([f"rank0 exception: {e!r}"])
        raise
    finally:
        dist.destroy_process_group()


def test_point_sharded_input_grads():
    """dx (this rank's rows), dtheta and the input-function gradients (rank sums) of a batch point-sharded
    over 2 ranks vs float64 autograd of the stock-torch port (one reference call per sample) at 1e-4."""
    cfg = dict(input_dim=2, theta_dim=2, input_func_dim=3, out_dim=1, n_attn_layers=2, d=64,
               n_mlp_num_layers=3, n_expert=3, n_head=4, n_input_functions=1)
    Ns, Ms = [300, 173], [[120, 77]]
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_input_grads, args=(r, world, port, cfg, Ns, Ms, q)) for r in range(world)]
    for p in procs:
        p.start()
    errs = q.get(timeout=200)
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert not errs, errs


@pytest.mark.parametrize("which", ["default", "external0", "side"])
def test_comm_stream_orders_after_kernels(which):
    """PointShardComm runs its collectives under the stream the engine hands it (parallel.PointShardComm._on).
    Whatever that handle is -- 0 for a caller on torch's default (null) stream, or a side stream -- a copy
    issued under it must see the result of the long kernel queued just before on that stream.  "external0"
    is the round-4 form (ExternalStream(0)), kept here as the record of what the test checks; the product
    path maps handle 0 to torch.cuda.default_stream."""
    dev = torch.device("cuda", 0)
    torch.cuda.synchronize()
    s = torch.cuda.Stream(dev) if which == "side" else torch.cuda.default_stream(dev)
    a = torch.randn(4096, 4096, device=dev)
    ok = True
    for _ in range(3):
        with torch.cuda.stream(s):
            t = torch.zeros(1, device=dev)
            b = a
            for _ in range(8):
                b = b @ a / 64.0          # ~10 ms of queued work before the last write
            t.fill_(1.0)
        if which == "external0":
            ctx = torch.cuda.stream(torch.cuda.ExternalStream(0, device=dev))
        elif which == "default":
            from gnot_amd import parallel as par
            c = par.PointShardComm.__new__(par.PointShardComm)
            c.ws = t
            ctx = c._on(0)
        else:
            from gnot_amd import parallel as par
            c = par.PointShardComm.__new__(par.PointShardComm)
            c.ws = t
            ctx = c._on(s.cuda_stream)
        with ctx:
            h = t.cpu()
        ok = ok and float(h[0]) == 1.0
        torch.cuda.synchronize()
    if which == "external0" and not ok:
        pytest.xfail("ExternalStream(0) does not order after the null stream's kernels on this stack")
    assert ok
