"""Gradient all-reduce overlapped with the backward (GNOT.set_grad_allreduce -> gnot_plan_set_grad_comm).

Two processes share cuda:0 over gloo (host-staged collectives; the box has one GPU).  Sample data
parallel, as bench.py runs configs[0]/[1]/[4] at N > 1: every rank runs its OWN meshes, and the
parameter gradients are summed over the ranks.  Summed group by group inside the backward (one
collective per weight-gradient group, issued as soon as the group is written), the gradients must be
BITWISE those of the plain path -- the backward alone, then one all-reduce of the flat gradient buffer
(two ranks: every element is the same a + b).  d = 64 (chain.hip, the 128-tile weight gradients) and
d = 256 with 8 experts (chain2.hip, the wide weight-gradient kernels), fp32 and bf16 mode.

The plans have ~1.5k points, below the size from which the engine runs its weight gradients serially
(kWgradSerialPoints), so by default they fork the weight gradients onto the side stream and sum the soft-MoE
experts with the moe_combine pass.  GNOT_WGRAD_OVERLAP=0 forces the serial form: each group's collective
is then issued on the comm stream right behind the caller's stream, and at d = 256 the expert grid sums
its experts with the FUSED combine (inter-workgroup hand-off, chain2.hip moe_combine_last) while the
collectives of earlier groups and the other rank's kernels run beside it -- the setting of every N > 1
bench run of configs[2]/[3].  Both forms must give the flat all-reduce's bits -- also when the ranks take DIFFERENT forms ("mixed":
serial_wgrad() is decided per rank from its local point count, so uneven sample-DP shares can split the
ranks): every rank must still issue its gradient collectives in the same order (engine.cpp flushes the
deferred groups before the input-function branch issues its own).
The reference is single-device (main.py:27); SURVEY.md section 5 asks for the overlap.
"""
import os
import socket
import sys

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


def _rank(rank, world, port, d, E, prec, overlap, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "gnot-replication_amd"), os.path.join(ROOT, "tests")]
    if overlap == "mixed":          # rank 0 forks its weight gradients, rank 1 runs them serially
        overlap = "1" if rank == 0 else "0"
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GNOT_WGRAD_OVERLAP=overlap)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gnot_amd import GNOT
        from gnot_amd import parallel as par
        dev = torch.device("cuda", 0)
        torch.manual_seed(3)                                 # the same weights on every rank
        m = GNOT(2, 1, 3, 1, 2, d, 3, d, d, E, 8 if d == 256 else 4, 1).to(dev)
        m.set_precision(prec)
        g = torch.Generator(device="cpu").manual_seed(100 + rank)   # this rank's own meshes
        x_off = [0, 900 + 37 * rank, 1500 + 11 * rank]
        x = torch.rand(x_off[-1], 2, generator=g).to(dev)
        theta = torch.rand(2, 1, generator=g).to(dev)
        fns = [torch.rand(200, 3, generator=g).to(dev)]
        G = torch.randn(x_off[-1], 1, generator=g).to(dev)

        def step():
            m.zero_grad(set_to_none=True)
            out = m.forward_packed(x, x_off, theta, fns, [[0, 90, 200]])
            (out * G).sum().backward()
            torch.cuda.synchronize()

        step()                                               # plain: backward, then ONE flat all-reduce
        h = m.engine().grad_flat.cpu()
        dist.all_reduce(h)
        ref = h.clone()
        m.set_grad_allreduce(par.PointShardComm(stage_via_host=True))
        step()                                               # summed group by group inside the backward
        flat = m.engine().grad_flat.cpu()                    # the .grad tensors are views of it
        q.put((rank, bool(torch.equal(flat, ref)), float((flat - ref).abs().max()), bool(torch.isfinite(flat).all())))
    except Exception as e:
        q.put((rank, False, repr(e), False))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("overlap", ["1", "0", "mixed"])
@pytest.mark.parametrize("d,E,prec", [(64, 3, "fp32"), (256, 8, "fp32"), (256, 8, "bf16")])
def test_overlapped_grad_allreduce_equals_flat_allreduce(d, E, prec, overlap):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, d, E, prec, overlap, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=200) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    for rank, equal, diff, finite in res:
        assert equal and finite, (rank, diff)
