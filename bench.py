#!/usr/bin/env python3
"""GNOT fwd+bwd training-step benchmark on MI355X (the driver's bench contract).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Default workload = BASELINE.json configs[2], the largest configuration that fits one GPU: a synthetic
3-D mesh of 262,144 query points, GNOT with d=256, 8 experts, 8 heads, 4 blocks, 4-layer MLPs and one
input function of 805 points, fp32 arithmetic (the reference computes in fp32; the MoE GEMMs run on
bf16 MFMA with an exact three-piece split, fp32-level results).  A step = pack weights -> GNOT forward
(gnot_amd, HIP) -> RelL2 loss (loss.py:14-23) -> backward to every parameter gradient (N>1: summed
over the ranks by RCCL group by group inside the backward, overlapped with it) -> AdamW step, captured
in hipGraphs (RCCL kernels included).
At N>1 ranks the default workload is configs[3], north_star's scaling target: ONE 1,048,576-point mesh
point-sharded over the ranks (strong scaling: 1M / N points per GPU; every attention call all-reduces
its states and runs the scramble all-to-all over RCCL).  --workload cfg3 at N>1
point-shards one mesh of N x 262,144 points instead (weak scaling).  Other workloads (--workload):
cfg1 = configs[0] (main.py widths, batch 4 x 4096), cfg2 = configs[1] (d=128, 4 experts, 2 input
functions, 10k points), cfg4 = configs[3] (at N=1: the whole 1M mesh on one GPU, MoE recompute),
cfg5 = configs[4] (64 variable meshes, LPT sample-DP).  --points / --meshes resize.

value = all query points processed by all ranks / max-over-ranks wall time of the K timed steps.
roofline: the kernel class with the most device time in an untimed profiled step (normally the
weight-gradient GEMMs or the MoE chain backward), timed live with hipEvents on the stream it runs on
during the timed steps; achieved = its algorithmic FLOPs per launch / average launch duration; frac =
achieved / the peak of the pipe the kernel issues on (bf16x6: 2.5 PFLOP/s / 6; bf16 mode: 2.5 PFLOP/s;
HBM-bound classes: 8 TB/s, MI355X_MICROARCH.md).
cpu_baseline: the stock-torch CPU port of the reference (oracle/torch_port.py) on this host's cores, on
a bounded sample of the same model (one mesh of at most 16,384 points), rank 0 at N=1 only.
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gnot-replication_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_16x16x4_f32 / 32x32x2, dense
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: "Peak BF16/FP16 MFMA ~2.5 PF dense" (no sparsity)
HBM_PEAK_GBS = 8000.0


def pmc_traffic(workload, kind, launches_per_step):
    """Mean HBM bytes per launch of the roofline class, from rocprofv3 PMC passes of the same bench command
    (profiles/pmc_traffic.json, written by scripts/pmc_traffic.py: FETCH_SIZE x 2 for the gfx950 half-count
    of wide streaming reads + WRITE_SIZE, MI355X_MICROARCH.md HBM section, summed over ALL of the class's
    dispatches of a step and divided by their count -- the same per-launch mean as `achieved`).  None
    when no entry exists, or the entry was measured on other kernels: its source hash (gnot_amd._lib.
    source_hash over the library's sources) differs from this tree's, or its launches per step differ."""
    from gnot_amd import _lib
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        e = json.load(open(path))[f"{workload}/{kind}"]
    except (OSError, KeyError, ValueError):
        return None
    sh = _lib.source_hash()
    if sh is None or e.get("source_hash") != sh or e.get("launches_per_step") != launches_per_step:
        return None
    return e["bytes_per_launch"]


WORKLOADS = {
    # BASELINE.json configs[1]
    "cfg2": dict(model=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=4,
                            n_attn_hidden_dim=128, n_mlp_num_layers=4, n_mlp_hidden_dim=128,
                            n_input_hidden_dim=128, n_expert=4, n_head=8, n_input_functions=2),
                 N=10000, M=805, B=1,
                 desc="configs[1]: GNOT 4-layer, 4-expert, d=128, 8 heads, 2 input functions, "
                      "2-D irregular mesh of {N} points/sample (805 points per input function), {dtype} fwd+bwd"),
    # BASELINE.json configs[2]: synthetic 3-D mesh, 256k points, d=256, 8 experts (the reference config
    # names bf16 training: --dtype bf16; the default computes the reference's fp32, bf16x6-exact)
    "cfg3": dict(model=dict(input_dim=3, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=4,
                            n_attn_hidden_dim=256, n_mlp_num_layers=4, n_mlp_hidden_dim=256,
                            n_input_hidden_dim=256, n_expert=8, n_head=8, n_input_functions=1),
                 N=262144, M=805, B=1, shard_weak=True,
                 desc="configs[2]: synthetic 3-D mesh of {N} points, d=256, 8 experts, 8 heads, "
                      "1 input function (805 points), {dtype} fwd+bwd"),
    # BASELINE.json configs[3]: ONE 1M-point mesh point-sharded over the ranks (strong scaling)
    "cfg4": dict(model=dict(input_dim=3, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=4,
                            n_attn_hidden_dim=256, n_mlp_num_layers=4, n_mlp_hidden_dim=256,
                            n_input_hidden_dim=256, n_expert=8, n_head=8, n_input_functions=1),
                 N=1048576, M=805, B=1, shard=True,
                 desc="configs[3]: synthetic 3-D mesh of {N} points point-sharded over the GPUs "
                      "(state all-reduce + scramble all-to-all over RCCL), d=256, 8 experts, {dtype} fwd+bwd"),
    # BASELINE.json configs[4]: 64 variable meshes (1k-50k points, packed), sample-DP with LPT balancing
    "cfg5": dict(model=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=4,
                            n_attn_hidden_dim=256, n_mlp_num_layers=4, n_mlp_hidden_dim=256,
                            n_input_hidden_dim=256, n_expert=3, n_head=8, n_input_functions=1),
                 N=0, M=805, B=64, variable=(1000, 50000),
                 desc="configs[4]: {B} meshes of U{{1k..50k}} points (seeded), packed offsets, sample-DP over the "
                      "GPUs with longest-processing-time balancing, main.py widths, {dtype} fwd+bwd"),
    # BASELINE.json configs[0] (main.py defaults, ~1-4k points/sample, batch 4)
    "cfg1": dict(model=dict(input_dim=2, theta_dim=1, input_func_dim=3, out_dim=1, n_attn_layers=4,
                            n_attn_hidden_dim=256, n_mlp_num_layers=4, n_mlp_hidden_dim=256,
                            n_input_hidden_dim=256, n_expert=3, n_head=8, n_input_functions=1),
                 N=4096, M=805, B=4,
                 desc="configs[0]: main.py defaults d=256, 3 experts, 8 heads, 1 input function, "
                      "batch {B} x {N} points, {dtype} fwd+bwd"),
}


def rel_l2_loss(out, tgt, seg, B):
    """RelL2Loss (loss.py:14-23): mean over samples x channels of sqrt(sum (p-t)^2 / sum t^2)."""
    C = out.shape[1]
    num = torch.zeros(B, C, device=out.device).index_add_(0, seg, (out - tgt) ** 2)
    den = torch.zeros(B, C, device=out.device).index_add_(0, seg, tgt ** 2)
    return (num / den).sqrt().mean()


def make_rank_batch(w, rank, world, device, force_shard=False):
    """This rank's share of the step's data, the loss normaliser and the step's total point count.
    sample-DP: `B` meshes of `N` points per rank (seeded by rank); configs[4]: the rank's LPT share of
    64 variable meshes; point-shard (configs[3]): the rank's slice of ONE mesh (every rank generates
    the same global mesh and keeps its gnot_amd.parallel.shard_range)."""
    from gnot_amd import parallel as par
    m = w["model"]
    if w.get("variable"):
        g = torch.Generator(device="cpu").manual_seed(0)
        lo, hi = w["variable"]
        sizes = torch.randint(lo, hi + 1, (w["B"],), generator=g).tolist()
        mine = par.lpt_partition(sizes, world)[rank]
        xs, ys, fl, th = [], [], [], []
        for b in mine:                                    # every mesh's data is seeded by its index
            gb = torch.Generator(device="cpu").manual_seed(1000 + b)
            xs.append(torch.rand(sizes[b], m["input_dim"], generator=gb))
            th.append(torch.rand(1, m["theta_dim"], generator=gb))
            fl.append([torch.rand(w["M"], m["input_func_dim"], generator=gb) for _ in range(m["n_input_functions"])])
            ys.append(torch.randn(sizes[b], m["out_dim"], generator=gb))
        Bl = len(mine)
        x_off = [0]
        for xb in xs:
            x_off.append(x_off[-1] + xb.shape[0])
        fns = [torch.cat([fl[k][i] for k in range(Bl)]) for i in range(m["n_input_functions"])]
        fn_offs = [[k * w["M"] for k in range(Bl + 1)] for _ in range(m["n_input_functions"])]
        seg = torch.repeat_interleave(torch.arange(Bl), torch.tensor([xb.shape[0] for xb in xs]))
        to = lambda t: t.to(device)
        return dict(x=to(torch.cat(xs)), x_off=x_off, theta=to(torch.cat(th)), fns=[to(f) for f in fns],
                    fn_offs=fn_offs, y=to(torch.cat(ys)), seg=to(seg), B=Bl, norm=w["B"], n_global=None,
                    step_points=sum(sizes), mesh_points=f"{min(sizes)}..{max(sizes)}", meshes=w["B"])
    if w.get("shard") or (w.get("shard_weak") and (world > 1 or force_shard)):
        w = dict(w, N=w["N"] * (world if w.get("shard_weak") else 1))     # weak: N points per rank
        x, x_off, theta, fns, fn_offs, y, seg = make_batch(w, 100, torch.device("cpu"))
        lo, hi = par.shard_range(w["N"], rank, world)
        to = lambda t: t.to(device)
        return dict(x=to(x[lo:hi]), x_off=[0, hi - lo], theta=to(theta), fns=[to(f) for f in fns], fn_offs=fn_offs,
                    y=to(y[lo:hi]), seg=to(seg[lo:hi]), B=1, norm=1,
                    n_global=[w["N"]] if (world > 1 or force_shard) else None,
                    step_points=w["N"],
                    mesh_points=f"{w['N']:,} ({hi - lo:,} on this GPU)", meshes=1)
    x, x_off, theta, fns, fn_offs, y, seg = make_batch(w, 100 + rank, device)
    return dict(x=x, x_off=x_off, theta=theta, fns=fns, fn_offs=fn_offs, y=y, seg=seg, B=w["B"],
                norm=w["B"] * world, n_global=None, step_points=w["B"] * w["N"] * world, mesh_points=f"{w['N']:,}",
                meshes=w["B"])


def permuted_batch(D, k):
    """The rank's variable-mesh batch with its meshes in the k-th seeded random order (new packed
    offsets, same data): main.py:41's shuffle=True re-batching, which changes the geometry every step."""
    B = D["B"]
    order = torch.randperm(B, generator=torch.Generator(device="cpu").manual_seed(500 + k)).tolist()
    xo, fo = D["x_off"], D["fn_offs"]
    pick = lambda t, off: torch.cat([t[off[b]:off[b + 1]] for b in order])
    x_off = [0]
    for b in order:
        x_off.append(x_off[-1] + xo[b + 1] - xo[b])
    fn_offs = []
    for o in fo:
        n = [0]
        for b in order:
            n.append(n[-1] + o[b + 1] - o[b])
        fn_offs.append(n)
    return dict(x=pick(D["x"], xo), x_off=x_off, theta=D["theta"][order], y=pick(D["y"], xo),
                fns=[pick(f, o) for f, o in zip(D["fns"], fo)], fn_offs=fn_offs)


def make_batch(w, seed, device):
    g = torch.Generator(device="cpu").manual_seed(seed)
    m = w["model"]
    B, N, M = w["B"], w["N"], w["M"]
    x = torch.rand(B * N, m["input_dim"], generator=g)
    theta = torch.rand(B, m["theta_dim"], generator=g)
    fns = [torch.rand(B * M, m["input_func_dim"], generator=g) for _ in range(m["n_input_functions"])]
    y = torch.randn(B * N, m["out_dim"], generator=g)
    x_off = [b * N for b in range(B + 1)]
    fn_offs = [[b * M for b in range(B + 1)] for _ in range(m["n_input_functions"])]
    seg = torch.repeat_interleave(torch.arange(B), N)
    to = lambda t: t.to(device)
    return to(x), x_off, to(theta), [to(f) for f in fns], fn_offs, to(y), to(seg)


CPU_SAMPLE_POINTS = 16384      # bound on the CPU sample (points per step; ~10-30 s of host work)


def host_cores():
    """(threads to use, description): the physical cores among the CPUs this process may run on
    (sched_getaffinity + sysfs topology: one thread per core, no SMT siblings), capped by the cgroup CPU
    quota (a GPU box grants a share of a larger machine), as BASELINE.md's CPU plan asks."""
    cpus = sorted(os.sched_getaffinity(0))
    cores = set()
    for c in cpus:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            cores.add((open(base + "physical_package_id").read().strip(), open(base + "core_id").read().strip()))
        except OSError:
            cores.add(("?", str(c)))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    n = len(cores) if quota is None else min(len(cores), quota)
    desc = (f"{n} threads = physical cores available to the process ({len(cpus)} CPUs in the affinity mask, "
            f"{len(cores)} physical cores" + (f", cgroup CPU quota {quota}" if quota is not None else "") + ")")
    return n, desc


def cpu_baseline(w, steps=5, warmup=2):
    """Reference CPU path (stock torch, oracle/torch_port.py) on this host's cores, on a BOUNDED sample
    of the workload: the same model, one step over at most CPU_SAMPLE_POINTS query points (pts/s of
    this linear-attention model is flat in the mesh size).  BASELINE.md's plan:
    torch.set_num_threads(physical cores), 2 warm-up steps, median of 5."""
    from oracle import torch_port
    from gnot_amd import GNOT
    m = w["model"]
    nthreads, cores_desc = host_cores()
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(nthreads)
    torch.manual_seed(0)
    mod = GNOT(*[m[k] for k in ("input_dim", "theta_dim", "input_func_dim", "out_dim", "n_attn_layers",
                                "n_attn_hidden_dim", "n_mlp_num_layers", "n_mlp_hidden_dim",
                                "n_input_hidden_dim", "n_expert", "n_head", "n_input_functions")])
    p = {k: v.detach().clone().requires_grad_(True) for k, v in mod.state_dict().items()}
    cfg = dict(m, d=m["n_attn_hidden_dim"])
    B = max(1, min(w["B"], 4))
    N = w["N"] if w["N"] > 0 else 4096
    N = min(N, CPU_SAMPLE_POINTS // B)
    ws = dict(w, B=B, N=N)
    x, x_off, theta, fns, fn_offs, y, seg = make_batch(ws, 0, torch.device("cpu"))
    M = w["M"]
    xb = x.view(B, N, -1)
    fb = [f.view(B, M, -1) for f in fns]
    times = []
    for it in range(warmup + steps):
        t0 = time.perf_counter()
        out = torch_port.gnot_forward(p, cfg, xb, theta, fb).reshape(B * N, -1)
        loss = rel_l2_loss(out, y, seg, B)
        for v in p.values():
            v.grad = None
        loss.backward()
        if it >= warmup:
            times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    torch.set_num_threads(prev_threads)
    return dict(value=round(B * N / med, 1), unit="points/s", cores=nthreads, kind="port",
                sample=f"bounded sample of the workload: same model, {B} mesh(es) x {N} points ({M} input-function "
                       f"points), stock-torch fp32 CPU port of the reference (oracle/torch_port.py, fixture-"
                       f"validated), fwd+RelL2+bwd, median of {steps} steps after {warmup} warm-up; {cores_desc}; "
                       f"points/s is flat in the mesh size (linear attention)")


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, script=None, argv=None):
    """`python bench.py --gpus N` without a launcher: start N rank processes of this same command (one
    per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in their environment) as CHILDREN -- no exec, and no GPU
    call in this parent -- wait for all, and return the first non-zero exit code (the other ranks are
    then ended by PID).  Only rank 0 prints the JSON line."""
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=port,
                   GNOT_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)]
                                      + list(sys.argv[1:] if argv is None else argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                print(f"[bench] rank {procs.index(p)} exited with {code}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    for p in procs:
        p.wait()
    return rc


def resolve_world(args):
    """(world, rank, local rank) of this process, or an exit: `--gpus N` with no WORLD_SIZE in the
    environment spawns N ranks (spawn_ranks); with one (torchrun, or spawn_ranks' children) it must equal
    --gpus.  N above the visible device count needs GNOT_BENCH_ONE_GPU=1 (every rank on cuda:0).
    torch.cuda.device_count() does not initialise the GPU on this image."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        n = args.gpus or 1
        if n > 1:
            if n > torch.cuda.device_count() and not os.environ.get("GNOT_BENCH_ONE_GPU"):
                raise SystemExit(f"bench.py: --gpus {n} but {torch.cuda.device_count()} GPU(s) visible "
                                 "(GNOT_BENCH_ONE_GPU=1 runs every rank on cuda:0)")
            raise SystemExit(spawn_ranks(n))
        return 1, 0, 0
    world = int(env_world)
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (launcher and flag disagree)")
    if world > torch.cuda.device_count() and not os.environ.get("GNOT_BENCH_ONE_GPU"):
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but {torch.cuda.device_count()} GPU(s) visible "
                         "(GNOT_BENCH_ONE_GPU=1 runs every rank on cuda:0)")
    return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU).  Without a launcher, N > 1 spawns the N rank processes itself; "
                         "under torchrun it must equal WORLD_SIZE.  Default: WORLD_SIZE, else 1")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default=None, choices=sorted(WORKLOADS),
                    help="default: cfg3 (configs[2], one 262,144-point mesh) at one GPU; cfg4 (configs[3], ONE "
                         "1,048,576-point mesh point-sharded over the GPUs: north_star's strong-scaling curve) at N > 1")
    ap.add_argument("--points", type=int, default=0, help="override points per sample")
    ap.add_argument("--meshes", type=int, default=0, help="cfg5: override the number of meshes")
    ap.add_argument("--roofline-kernel", default="auto", choices=["auto", "moe_fwd", "moe_bwd", "wgrad", "wgrad_b16"],
                    help="kernel class timed live for the roofline (auto: the one with the most device time)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of hipGraph replay")
    ap.add_argument("--torch-adamw", action="store_true", help="torch's fused AdamW instead of the native one")
    ap.add_argument("--breakdown", action="store_true", help="print per-kernel-class device time to stderr")
    ap.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32",
                    help="fp32: the reference's arithmetic (bf16x6-exact MFMA); bf16: configs[2]'s bf16 training "
                         "(one RNE bf16 operand per MFMA in the chains / projections / weight gradients up to d=256, "
                         "fp32 accumulation; at d=256 the soft-MoE chains keep their saves, dZ and Linear inputs in "
                         "bf16; north_star's 1e-2 bar, tests/test_gpu_bf16.py)")
    ap.add_argument("--fp32-only", action="store_true",
                    help="skip the companion bf16-mode measurement of the default fp32 run (configs[2], N=1)")
    ap.add_argument("--recompute", choices=["auto", "on", "off"], default="auto",
                    help="MoE activation recompute (GNOT.set_moe_recompute); auto: on when the plain workspace "
                         "would not fit the GPU (configs[3]'s 1M-point mesh on one GPU)")
    ap.add_argument("--vary-geometry", action="store_true",
                    help="variable-mesh workloads: a new mesh order (hence new packed offsets) every step, as "
                         "main.py:41's shuffled DataLoader does; eager launches")
    args = ap.parse_args()

    world, rank, local = resolve_world(args)
    # rehearsal knobs for the multi-process path on a one-GPU box (the real run is RCCL, one GPU per
    # rank): GNOT_BENCH_BACKEND=gloo (host-staged collectives) and GNOT_BENCH_ONE_GPU=1 (every rank on
    # cuda:0)
    backend = os.environ.get("GNOT_BENCH_BACKEND", "nccl")
    if os.environ.get("GNOT_BENCH_ONE_GPU"):
        local = 0
    # GNOT_BENCH_FORCE_SHARD=1: run the point-shard path (engine callbacks, RCCL collectives, the per-group
    # gradient all-reduce, all captured in the step's hipGraph) even at one rank -- the N=1 reference of
    # the sharded step the multi-GPU runs take
    force_shard = os.environ.get("GNOT_BENCH_FORCE_SHARD") == "1"
    if world > 1 or force_shard:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    if args.workload is None:
        args.workload = "cfg3" if world == 1 else "cfg4"
    w = dict(WORKLOADS[args.workload])
    if args.points:
        w["N"] = args.points
    if args.meshes:
        w["B"] = args.meshes
    from gnot_amd import GNOT
    m = w["model"]
    torch.manual_seed(1234)                       # same initial weights on every rank
    model = GNOT(*[m[k] for k in ("input_dim", "theta_dim", "input_func_dim", "out_dim", "n_attn_layers",
                                  "n_attn_hidden_dim", "n_mlp_num_layers", "n_mlp_hidden_dim",
                                  "n_input_hidden_dim", "n_expert", "n_head", "n_input_functions")]).to(device)
    shard = bool(w.get("shard") or w.get("shard_weak")) and (world > 1 or force_shard)
    # the point-shard exchanges and the per-group gradient all-reduces run inside the engine's launch sequence
    # (RCCL through callbacks on the engine's stream): RCCL kernels are graph-capturable, so the multi-rank
    # step is captured too; the host-staged gloo rehearsal stays eager
    use_graph = not args.no_graph and not ((world > 1 or shard) and backend != "nccl")
    from gnot_amd import train as gtrain
    # main.py:50-51 AdamW(lr=1e-3): one native update over the flat parameter arena (gnot_adamw_step),
    # or torch's fused multi-tensor AdamW (--torch-adamw; capturable keeps its step count on device)
    if args.torch_adamw:
        opt = torch.optim.AdamW(model.parameters(), lr=1e-3, fused=True, capturable=use_graph)
    else:
        opt = gtrain.FlatAdamW(gtrain.flatten_parameters(model), lr=1e-3)
    loss_fn = gtrain.RelL2Loss()
    D = make_rank_batch(w, rank, world, device, force_shard)
    x, x_off, theta, fns, fn_offs, y, seg, B = (D[k] for k in ("x", "x_off", "theta", "fns", "fn_offs", "y", "seg", "B"))
    eng = model.engine()
    eng.param_grads = bool(args.torch_adamw)      # the native AdamW reads the gradient arena directly
    recompute = args.recompute == "on"
    if args.recompute == "auto":
        # the plan's training workspace for this rank's geometry vs ~90 % of the free device memory
        import ctypes
        from gnot_amd import _lib
        lib = _lib.load()
        nx = D["x_off"]
        B_ = len(nx) - 1
        flat = [v for o in D["fn_offs"] for v in o]
        _lib.check(lib.gnot_plan_set_batch(eng.plan, B_, (ctypes.c_int64 * (B_ + 1))(*nx),
                                           (ctypes.c_int64 * max(1, len(flat)))(*flat) if flat else None, 1))
        need = lib.gnot_plan_workspace_bytes(eng.plan)
        free, _ = torch.cuda.mem_get_info(device)
        # headroom for RCCL's buffers, the point-shard exchange tensors and allocator slack: 12 GiB (at N = 2 a
        # configs[3] rank holds 524,288 points: 238 GiB of workspace, which fits a 288 GB MI355X without the
        # recompute that would cost ~25 % of its step)
        recompute = need > free - 12 * 2 ** 30
        eng.geom = None
    model.set_moe_recompute(recompute)
    model.set_precision(args.dtype)
    batches = None
    if args.vary_geometry:
        if not w.get("variable"):
            raise SystemExit("--vary-geometry needs a variable-mesh workload (cfg5)")
        batches = [permuted_batch(D, k) for k in range(max(args.warmup, 2) + 3 + args.steps)]
        use_graph = False                         # every step binds a new geometry
    it = {"k": 0}
    comm = None
    if world > 1 or shard:
        from gnot_amd import parallel as par
        comm = par.PointShardComm(stage_via_host=backend != "nccl")
    if shard:
        model.set_point_shard(comm)
    if (world > 1 or force_shard) and os.environ.get("GNOT_BENCH_FLAT_ALLREDUCE") != "1":
        # the parameter gradients are summed over the ranks INSIDE the backward, one collective per weight-
        # gradient group as soon as it is written (overlapped with the rest of the backward; SURVEY.md
        # section 5); GNOT_BENCH_FLAT_ALLREDUCE=1: one all-reduce of the flat buffer after the backward
        model.set_grad_allreduce(comm)

    # one training step = [forward + RelL2 + backward (N>1: gradients summed over the ranks group by group
    # inside it)] -> [AdamW].  With hipGraphs the two bracketed parts are captured once and replayed
    # (RCCL kernels included); GNOT_BENCH_FLAT_ALLREDUCE=1 keeps one eager all-reduce of the flat gradient
    # buffer between them instead.
    def fwd_bwd():
        nonlocal x, x_off, theta, fns, fn_offs, y
        if batches is not None:
            bt = batches[it["k"] % len(batches)]
            it["k"] += 1
            x, x_off, theta, fns, fn_offs, y = (bt[k] for k in ("x", "x_off", "theta", "fns", "fn_offs", "y"))
        out = model.forward_packed(x, x_off, theta, fns, fn_offs, n_global=D["n_global"])
        if shard:
            from gnot_amd import parallel as par
            loss = par.rel_l2_loss_sharded(out, y, seg, B, stage_via_host=backend != "nccl")
        else:
            # native RelL2 (loss.py:14-23); mean over ALL samples of the step: local sum / global count
            loss = loss_fn(x_off, out, y) * (B / D["norm"])
        if args.torch_adamw:
            opt.zero_grad(set_to_none=True)
        loss.backward()
        return loss

    def opt_step():
        if args.torch_adamw:
            opt.step()
        else:
            opt.launch(eng.grad_flat)

    def allreduce():
        if world > 1 and eng.grad_comm is None:
            dist.all_reduce(eng.grad_flat, op=dist.ReduceOp.SUM)

    def eager_step():
        fwd_bwd()
        allreduce()
        if not args.torch_adamw:
            opt.prepare()
        opt_step()

    def roofline(M, dtype):
        """the device-time-dominant kernel class of a measure() run.  `frac` = achieved / the peak of the pipe
        the kernel ISSUES on (never above 1): the fp32 path's bf16x6 kernels run six bf16 MFMAs per fp32
        block product, so their ceiling is 2.5 PFLOP/s / 6 = 416.7 TFLOP/s of fp32-equivalent work; the bf16
        mode's one-piece kernels 2.5 PFLOP/s; the HBM-bound bf16-row weight gradients 8 TB/s.
        `vs_fp32_mfma_peak` = achieved / the v_mfma_f32 rate (157.3), the fp32 arithmetic's own MFMA peak."""
        avg_ms = M["kms"] / max(M["klaunch"], 1)
        flops_launch = M["kflops"] / max(M["klaunch"], 1)
        ach = flops_launch / (avg_ms * 1e-3) / 1e12 if M["klaunch"] and M["kms"] > 0 else 0.0
        form = "bf16x6" if dtype == "fp32" else "bf16"
        d256 = m["n_attn_hidden_dim"] == 256
        names = ({"moe_fwd": f"chain2_fwd_kernel (fused MoE expert chains, forward, {form} MFMA)",
                  "moe_bwd": f"chain2_bwd_kernel (fused MoE expert chains, backward, {form} MFMA)",
                  "wgrad": f"pgemm_x6w_kernel+pgemm_reduce_kernel (weight gradients, 256x256 {form} MFMA)",
                  "wgrad_b16": "pgemm_b16_kernel+pgemm_reduce_kernel (soft-MoE weight gradients on bf16 rows, "
                               "LDS-DMA + ds_read_b64_tr_b16, bf16 MFMA)"}
                 if d256 else
                 {"moe_fwd": f"chain_fwd_kernel (fused MoE expert chains, forward, {form} MFMA)",
                  "moe_bwd": f"chain_bwd_kernel (fused MoE expert chains, backward, {form} MFMA)",
                  # d <= 128: the wide kernel's design at a 128 x 128 output (engine.cpp wgrad128_on)
                  "wgrad": (f"pgemm_x6w_kernel<TW=128>+pgemm_reduce_kernel (weight gradients, 128x128 {form} MFMA)"
                            if m["n_attn_hidden_dim"] <= 128 else
                            f"pgemm_x6_kernel+pgemm_reduce_kernel (weight gradients, {form} MFMA)")})
        rk = M["rkind"]
        if dtype == "bf16" and m["n_attn_hidden_dim"] <= 256:
            pipe, pipe_peak = "bf16 MFMA (one product per block)", BF16_MFMA_PEAK_TFLOPS
        else:
            pipe, pipe_peak = "bf16 MFMA, six per fp32 block product (bf16x6)", BF16_MFMA_PEAK_TFLOPS / 6
        traffic = None
        if not args.points:
            # entries: "<workload>/<class>" (fp32), "<workload>/bf16/<class>" (bf16 mode)
            traffic = pmc_traffic(args.workload if dtype == "fp32" else f"{args.workload}/bf16", rk,
                                  M["klaunch_step"])
        if rk == "wgrad_b16":
            # HBM-bound: every job is a 256 x 256 Linear reading (out + in) * 2 B of bf16 rows per point for
            # 2 * out * in flops, so algorithmic bytes = flops / 128
            gbs = flops_launch / 128.0 / (avg_ms * 1e-3) / 1e9 if M["klaunch"] and M["kms"] > 0 else 0.0
            return {
                "kernel": names[rk], "class": rk,
                "class_ms_per_step": {k: round(v[0], 3) for k, v in M["kinds"].items()},
                "bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
                "tflops": round(ach, 3), "frac_mfma": round(ach / BF16_MFMA_PEAK_TFLOPS, 4),
                "avg_launch_us": round(avg_ms * 1e3, 2), "bytes_per_launch": flops_launch / 128.0,
                "flops_per_launch": flops_launch, "launches": M["klaunch"],
            }
        return {
            "kernel": names[rk],
            "class": rk,
            "class_ms_per_step": {k: round(v[0], 3) for k, v in M["kinds"].items()},
            "bound": "mfma",
            "achieved": round(ach, 3),
            "peak": round(pipe_peak, 2),
            "unit": "TFLOP/s",
            "frac": round(ach / pipe_peak, 4),
            "pipe": pipe,
            "vs_fp32_mfma_peak": round(ach / FP32_MFMA_PEAK_TFLOPS, 4),
            "traffic": traffic,
            # the measured HBM bytes per launch (PMC) over the live launch time: how far the class is from
            # the memory side of its roofline (the one-piece bf16 chains are nearer to it than to the MFMA's)
            "traffic_gbs": round(traffic / (avg_ms * 1e-3) / 1e9, 1) if traffic and avg_ms > 0 else None,
            "traffic_frac_hbm": round(traffic / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if traffic and avg_ms > 0 else None,
            "avg_launch_us": round(avg_ms * 1e3, 2),
            "flops_per_launch": flops_launch,
            "launches": M["klaunch"],
        }

    M_graph = {"on": False, "fail": None}

    def rebuild_engine():
        """a fresh engine (plan, streams, workspace) with this run's settings (GNOT.engine() copies the
        module's comm / grad-comm / recompute / precision settings into it)"""
        nonlocal eng
        model._engine = None
        eng = model.engine()
        eng.param_grads = bool(args.torch_adamw)

    def measure():
        """warm-up, class profile, capture, K timed steps -> timing of the current precision"""
        # warm-up (also the capture warm-up: allocations, plan binding, optimizer state)
        side = torch.cuda.Stream(device)
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):
            for _ in range(max(args.warmup, 2)):
                eager_step()
        torch.cuda.current_stream(device).wait_stream(side)
        torch.cuda.synchronize()
        print("[bench] warm-up done", file=sys.stderr, flush=True)
        # which kernel class dominates device time: one profiled eager step per class (untimed)
        kinds = {}
        classes = ("moe_fwd", "moe_bwd", "wgrad") + (("wgrad_b16",) if eng.bf16 and m["n_attn_hidden_dim"] == 256 else ())
        for kind in classes:
            eng.profile_enable(kind)
            eager_step()
            kinds[kind] = eng.profile_read()
            if args.breakdown:
                ms, n, fl = kinds[kind]
                print(f"[breakdown] {kind}: {ms:.3f} ms/step over {n} launches, "
                      f"{fl / ms / 1e9 if ms else 0:.1f} TFLOP/s", file=sys.stderr)
        eng.profile_enable("")
        torch.cuda.synchronize()
        rkind = args.roofline_kernel
        if rkind == "auto":
            # the class with the most device time; the weight gradients run on the caller's stream after
            # their chain backward (engine.cpp serial_wgrad), so every class time is its own serial cost.
            # bf16 mode: the soft-MoE weight gradients are their own class (wgrad_b16)
            pick = list(kinds)
            rkind = max(pick, key=lambda k: kinds[k][0])

        step = eager_step
        if use_graph:
            # the roofline kernel's hipEvent pairs are recorded inside the captured graph, so the timed
            # replays carry them (the pool of events exists from one eager profiled step)
            eng.profile_enable(rkind)
            eager_step()
            eng.profile_read()
            torch.cuda.synchronize()
            eng.profile_enable(rkind)
            g_fb, g_opt = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            print("[bench] capturing", file=sys.stderr, flush=True)
            if comm is not None and int(os.environ.get("GNOT_BENCH_FAIL_CAPTURE", "0")) > 0:
                # test knob: the n-th collective callback issued under capture fails (1: the forward's first)
                comm.fail_next_captured = int(os.environ["GNOT_BENCH_FAIL_CAPTURE"])
            try:
                with torch.cuda.graph(g_fb):
                    fwd_bwd()
                with torch.cuda.graph(g_opt, pool=g_fb.pool()):
                    opt_step()
                torch.cuda.synchronize()
                captured = True
            except Exception as ex:           # e.g. a collective the communicator cannot capture: stay eager
                print(f"[bench] capture failed ({ex!r}); eager steps", file=sys.stderr, flush=True)
                captured = False
                M_graph["fail"] = f"{type(ex).__name__}: {str(ex).splitlines()[0][:160] if str(ex) else ''}"
                try:
                    torch.cuda.synchronize()
                except Exception as ex2:
                    print(f"[bench] synchronize after the failed capture: {ex2!r}", file=sys.stderr, flush=True)
            if world > 1:
                # every rank replays, or every rank runs eager: a rank whose capture failed must not pair its
                # eager collectives with its peers' graph replays
                ok = torch.tensor([1.0 if captured else 0.0], device=device)
                dist.all_reduce(ok, op=dist.ReduceOp.MIN)
                if captured and ok.item() < 1.0:
                    captured = False
                    M_graph["fail"] = "a peer rank's capture failed"
            if not captured:
                # the failed capture may have left the plan's side streams (and its events) in an invalidated
                # capture state: discard the engine -- new plan, streams and workspace -- before eager steps
                rebuild_engine()
                g_fb = g_opt = None
                torch.cuda.synchronize()
                eng.profile_enable(rkind)
                eager_step()                  # the new plan's event pool for the profiled class
                eng.profile_read()
                torch.cuda.synchronize()
                eng.profile_enable(rkind)
            print("[bench] captured" if captured else "[bench] eager", file=sys.stderr, flush=True)

            def graph_step():
                g_fb.replay()
                allreduce()
                if not args.torch_adamw:
                    opt.prepare()         # this step's AdamW hyper-parameters -> device (outside the graph)
                g_opt.replay()
            if captured:
                step = graph_step
                M_graph["on"] = True
            for _ in range(2):
                step()
            torch.cuda.synchronize()
        else:
            eng.profile_enable(rkind)

        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        # eager: summed over every timed step; graph: the events hold the LAST replay's launches, and
        # launches/flops are those of one step -> both give the average launch duration
        kms, klaunch, kflops = eng.profile_read()
        eng.profile_enable("")
        if world > 1:
            t = torch.tensor([elapsed], device=device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return dict(elapsed=elapsed, kinds=kinds, rkind=rkind, kms=kms, klaunch=klaunch, kflops=kflops,
                    klaunch_step=kinds[rkind][1])

    M0 = measure()
    elapsed, kinds, rkind, kms, klaunch, kflops = (M0[k] for k in ("elapsed", "kinds", "rkind", "kms", "klaunch", "kflops"))
    pts = D["step_points"] * args.steps
    result = {
        "metric": "mesh points/sec (GNOT fwd+bwd, whole node)",
        "value": round(pts / elapsed, 1),
        "unit": "points/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if (w.get("shard") and world > 1) else "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic: coords/theta/input-function rows U[0,1], targets N(0,1), seeded per rank; "
                "random-init weights (torch.manual_seed)",
        "config": {"workload": w["desc"].format(N=D["mesh_points"], B=D["meshes"], dtype=args.dtype),
                   "points_per_step": D["step_points"], "samples_per_gpu": B,
                   "input_function_points": w["M"], "hidden": m["n_attn_hidden_dim"], "experts": m["n_expert"],
                   "heads": m["n_head"], "blocks": m["n_attn_layers"], "mlp_layers": m["n_mlp_num_layers"],
                   "input_functions": m["n_input_functions"],
                   "geometry": "new mesh order every step (--vary-geometry)" if batches is not None else "fixed",
                   "moe_recompute": recompute,
                   "parallelism": (f"point-shard{world}" if shard else f"sample-dp{world}") if (world > 1 or shard) else "single",
                   "step": "pack+fwd+RelL2+bwd+AdamW (native loss, " + ("torch fused AdamW" if args.torch_adamw else "native flat AdamW") + ")" + (" (hipGraph replay)" if M_graph["on"] else " (eager)")
                           + (f"; graph capture failed ({M_graph['fail']}): fresh engine, eager steps" if M_graph["fail"] else "")},
        "roofline": roofline(M0, args.dtype),
    }
    if (args.dtype == "fp32" and not args.fp32_only and world == 1 and m["n_attn_hidden_dim"] == 256
            and batches is None and not args.torch_adamw):
        # BASELINE configs[2] names bf16 training: the same workload in the bf16 arithmetic mode, timed the
        # same way on the same model and optimizer (the headline `value` above stays the fp32 path)
        model.set_precision("bf16")
        M1 = measure()
        result["bf16_mode"] = {
            "value": round(D["step_points"] * args.steps / M1["elapsed"], 1),
            "ms_per_step": round(M1["elapsed"] / args.steps * 1e3, 4),
            "dtype": "bf16",
            "arithmetic": "one RNE bf16 operand per MFMA in the d=256 chains / projections / weight gradients, "
                          "fp32 accumulation; bf16 storage of the soft-MoE chains' saves, dZ and Linear inputs "
                          "(GNOT.set_precision('bf16'); tests/test_gpu_bf16.py: "
                          "1e-2 of the fp64 oracle)",
            "roofline": roofline(M1, "bf16"),
        }
        model.set_precision("fp32")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(w)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
