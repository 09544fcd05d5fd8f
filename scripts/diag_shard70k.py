#!/usr/bin/env python3
"""Diagnostic: the 2-rank point-sharded 70k case of tests/test_gpu_shard.py under several environments,
one oracle computation for all.  Prints, per variant, the output error and the per-tensor gradient errors
(relative, worst first).   python scripts/diag_shard70k.py "GNOT_WGRAD_OVERLAP=0" "GNOT_WGRAD_OVERLAP=1" ..."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnot-replication_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _rank(rank, world, port, fx, env, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "gnot-replication_amd"), os.path.join(ROOT, "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **env)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from golden_util import model_args
        from gnot_amd import GNOT
        from gnot_amd import parallel as par
        dev = torch.device("cuda", 0)
        cfg = fx["cfg"]
        m = GNOT(*model_args(cfg)).to(dev)
        m.load_state_dict({k: torch.from_numpy(v).float() for k, v in fx["params"].items()})
        m.set_point_shard(par.PointShardComm(stage_via_host=True))
        Ns = [int(fx["x_off"][-1])]
        loc_off, ranges = par.shard_offsets(Ns, rank, world)
        rows = np.concatenate([np.arange(fx["x_off"][b] + lo, fx["x_off"][b] + hi) for b, (lo, hi) in enumerate(ranges)])
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).float().to(dev)
        print(f"[rank {rank}] torch current stream {torch.cuda.current_stream(dev)} ptr {torch.cuda.current_stream(dev).cuda_stream}",
              flush=True)
        res = []
        names = ["x", "xin", "scores", "query0", "fnenc0", "b0.cq", "b0.ckv0", "b0.cstate0", "b0.cres", "b0.a",
                 "b0.query1", "b0.sq", "b0.sstate", "b0.sres", "b0.bb", "b0.query2", "xa", "xb"]
        for it in range(int(env.get("DIAG_STEPS", "1"))):
            out = m.forward_packed(t(fx["x"][rows]), loc_off, t(fx["theta"]), [t(f) for f in fx["fns"]],
                                   [o.tolist() for o in fx["fn_offs"]], n_global=Ns)
            torch.cuda.synchronize()
            eng = m.engine()
            bad = []
            for nm in names:
                try:
                    ptr, ld = eng.debug_ptr(nm)
                except Exception:
                    continue
                off = ptr - eng.ws.data_ptr()
                cnt = {"x": 1, "xin": 1, "scores": 1, "fnenc0": 1, "b0.ckv0": 1, "b0.cstate0": 0, "b0.sstate": 0}.get(nm)
                rowsn = len(rows) if nm not in ("fnenc0", "b0.ckv0", "b0.cstate0", "b0.sstate") else (805 if nm in ("fnenc0", "b0.ckv0") else 1)
                n = rowsn * ld if nm not in ("b0.cstate0", "b0.sstate") else 8 * (32 * 32 + 32)
                v = eng.ws[off: off + 4 * n].view(torch.float32)
                nf = int((~torch.isfinite(v)).sum())
                if nf:
                    bad.append(f"{nm}:{nf}/{n}")
            print(f"[rank {rank} step {it}] forward out finite {bool(torch.isfinite(out).all())}; non-finite buffers: {bad}",
                  flush=True)
            m.zero_grad(set_to_none=True)
            (out * t(fx["G"][rows])).sum().backward()
            torch.cuda.synchronize()
            print(f"[rank {rank} step {it}] grads finite {bool(torch.isfinite(m.engine().grad_flat).all())}", flush=True)
            h = m.engine().grad_flat.cpu()
            dist.all_reduce(h)
            m.engine().grad_flat.copy_(h.to(dev))
            torch.cuda.synchronize()
            outs = [None] * world
            dist.all_gather_object(outs, (rows, out.detach().double().cpu().numpy()))
            if rank == 0:
                full = np.zeros_like(fx["out"])
                for r_rows, o in outs:
                    full[r_rows] = o
                rel = lambda a, b: float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))
                grads = {k: p.grad.double().cpu().numpy() for k, p in m.named_parameters()}
                errs = sorted(((rel(grads[k], fx["grads"][k]), k) for k in grads), reverse=True)
                res.append((rel(full, fx["out"]), errs))
        if rank == 0:
            q.put(res)
    except Exception as e:
        if rank == 0:
            q.put(repr(e))
        raise
    finally:
        dist.destroy_process_group()


def main():
    from test_gpu_configs import CFG_3D
    from test_gpu_parity import _random_case
    import socket
    t0 = time.time()
    print("oracle ...", flush=True)
    fx, G = _random_case(31, dict(CFG_3D, n_attn_layers=1), [70000], [[805]])
    fx = dict(fx, G=G)
    print(f"oracle done {time.time() - t0:.0f} s", flush=True)
    ctx = mp.get_context("spawn")
    for spec in sys.argv[1:]:
        env = dict(kv.split("=", 1) for kv in spec.split(",") if kv)
        env.setdefault("GNOT_STATE_MFMA_MIN", "16384")
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        q = ctx.Queue()
        procs = [ctx.Process(target=_rank, args=(r, 2, port, fx, env, q)) for r in range(2)]
        for p in procs:
            p.start()
        res = q.get(timeout=300)
        for p in procs:
            p.join(timeout=60)
        print(f"=== {spec}  exitcodes {[p.exitcode for p in procs]}", flush=True)
        if isinstance(res, str):
            print(res)
            continue
        for it, (eo, errs) in enumerate(res):
            bad = [(e, k) for e, k in errs if e > 1e-4]
            print(f"  step {it}: output rel {eo:.2e}; {len(bad)} tensors > 1e-4; worst: "
                  + ", ".join(f"{k} {e:.2e}" for e, k in errs[:12]), flush=True)


if __name__ == "__main__":
    main()
