"""The one-shot all-reduce + RMSNorm collective (csrc/allreduce.hip) as a TP decode step runs it:
captured in a hipGraph, 2 x L calls per replay (A1 / A2 of every layer), ranks as processes sharing
the one GPU of the test box (RCCL refuses duplicate-device ranks; the IPC kernels do not care).  It
bounds the collective share of a Llama-3-70B TP = 8 decode step that the virtual-rank timing leaves
out (profiles/r6/virtual_rank/).  On one GPU the peers' buffers are local HBM
rather than xGMI links, and the ranks' kernels share the CUs, so the numbers are a floor for the
kernel + handshake cost, not an xGMI measurement.

    python scripts/bench_custom_ar.py [--world 2] [--rows 1,8,64,256] [--layers 80]

Per row count: the graph with bf16 inputs (the splitk_reduce kernel ahead of each call, as before
round 6) and with split-K partial slabs reduced inside the collective (round 6).
"""
import argparse
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, rows_list, layers, split, q):
    try:
        sys.path.insert(0, ROOT)
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from ai_agent_kubectl_amd import ops
        from ai_agent_kubectl_amd.parallel.custom_allreduce import OneShotAllReduce
        ar = OneShotAllReduce(device="cuda:0")
        H = 8192
        w = torch.ones(H, dtype=torch.bfloat16, device="cuda")
        out = {}
        for rows in rows_list:
            res = torch.zeros(rows, H, dtype=torch.bfloat16, device="cuda")
            P = (torch.randn(split, rows, H, device="cuda") * 0.01).to(torch.bfloat16)
            sk = ops.SplitK(P, split)
            t = torch.empty(rows, H, dtype=torch.bfloat16, device="cuda")
            graphs = {}
            for mode in ("reduce_then_ar", "fused_splitk"):
                for _ in range(2):   # warm the kernels before capture
                    if mode == "fused_splitk":
                        ar.all_reduce_rmsnorm(sk, w, 1e-5, res)
                    else:
                        t.copy_(sk.resolve())
                        ar.all_reduce_rmsnorm(t, w, 1e-5, res)
                torch.cuda.synchronize()
                dist.barrier()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(2 * layers):
                        if mode == "fused_splitk":
                            ar.all_reduce_rmsnorm(sk, w, 1e-5, res)
                        else:
                            ops.rmsnorm(sk, w, 1e-5)   # stands in for the splitk_reduce launch + HBM pass
                            ar.all_reduce_rmsnorm(t, w, 1e-5, res)
                graphs[mode] = g
            for mode, g in graphs.items():
                torch.cuda.synchronize()
                dist.barrier()
                g.replay()   # warm replay
                torch.cuda.synchronize()
                dist.barrier()
                reps = 10
                t0 = time.perf_counter()
                for _ in range(reps):
                    g.replay()
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / reps
                dist.barrier()
                out[(rows, mode)] = dt * 1e3
        ar.check()
        q.put((rank, out, None))
    except Exception:
        import traceback
        q.put((rank, None, traceback.format_exc()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--rows", default="1,8,64,256")
    ap.add_argument("--layers", type=int, default=80)
    ap.add_argument("--split", type=int, default=4)
    args = ap.parse_args()
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    rows = [int(r) for r in args.rows.split(",")]
    procs = [ctx.Process(target=_rank, args=(r, args.world, port, rows, args.layers, args.split, q))
             for r in range(args.world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(args.world):
            r, val, tb = q.get(timeout=600)
            if tb:
                print(f"rank {r} failed:\n{tb}", flush=True)
                sys.exit(1)
            res[r] = val
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.terminate()
    print(f"world {args.world}, {2 * args.layers} all-reduce + RMSNorm calls per graph replay, hidden 8192, "
          f"split-K {args.split} bf16 partials; max over ranks:")
    for n in rows:
        a = max(res[r][(n, "reduce_then_ar")] for r in res)
        b = max(res[r][(n, "fused_splitk")] for r in res)
        print(f"  rows {n:4d} ({n * 16} KiB per call): reduce + AR {a:7.3f} ms ({a / (2 * args.layers) * 1e3:6.2f} us/call)"
              f" | fused split-K AR {b:7.3f} ms ({b / (2 * args.layers) * 1e3:6.2f} us/call)", flush=True)


if __name__ == "__main__":
    main()
