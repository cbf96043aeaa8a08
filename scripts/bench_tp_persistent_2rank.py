"""Decode-step time of a real TP = 2 group whose two ranks share the one GPU of the test box: the
bucket-1 decode hipGraph replayed on both ranks at once, (a) the persistent all-layers kernel with its
in-kernel all-reduce (KA_PERSISTENT_TP=1) against (b) the kernel chain with the one-shot IPC all-reduce
+ RMSNorm kernels.  Both persistent grids are capped at 120 workgroups (KA_PD_GRID) so both ranks are
resident; the peers' buffers are local HBM here, not xGMI links, so this bounds the protocol's cost
(flags, fences, the extra exchange) rather than measuring an 8-GPU node.

    python scripts/bench_tp_persistent_2rank.py [--model llama3-70b-8l] [--reps 50]
"""
import argparse
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rank(rank, world, port, model, reps, persistent, q):
    try:
        sys.path.insert(0, ROOT)
        os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=str(port), KA_CUSTOM_AR="1", KA_TP_OVERLAP="0", KA_PD_GRID="120",
                          KA_PERSISTENT_TP="1" if persistent else "0", KA_PERSISTENT_DECODE="1" if persistent else "0")
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine
        from ai_agent_kubectl_amd.engine.sequence import SamplingParams
        from ai_agent_kubectl_amd.llm.engine_backend import EngineLLM
        from ai_agent_kubectl_amd.parallel.comm import make_comm
        comm = make_comm(None)
        eng = build_engine(EngineOptions(model=model, device="cuda:0", tp_rank=rank, tp_size=world, max_batch=2,
                                         graph_buckets=(1,), kv_cache_tokens=4096, max_model_len=256,
                                         gpu_mem_fraction=0.3), comm=comm)
        r = eng.runner
        r.capture_graphs(autotune=False)
        m = r.model
        assert bool(r.graph_persistent.get(1)) == persistent, r.graph_persistent
        if rank == 0:
            be = EngineLLM(eng, max_new_tokens=4, ignore_eos=True)
            eng.generate_blocking([be.prompt_ids("list all pods in kube-system")],
                                  SamplingParams(max_new_tokens=4, ignore_eos=True), forced_prefix=be._forced)
            r.stop_workers()
        else:
            r.worker_loop()
        # both ranks now hold the same last (B = 1 decode) staging image: replay it together
        g = r.graphs[1]
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        comm.custom_ar.check()
        err = m.persistent_err() if persistent else 0
        q.put((rank, (ms, err, len(m.layers)), None))
    except Exception:
        import traceback
        q.put((rank, None, traceback.format_exc()))


def run(model, reps, persistent):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, model, reps, persistent, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rk, val, tb = q.get(timeout=900)
        if tb:
            raise RuntimeError(f"rank {rk}:\n{tb}")
        res[rk] = val
    for p in procs:
        p.join(timeout=60)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b-8l")
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    for persistent in (True, False, True, False):
        t0 = time.time()
        res = run(args.model, args.reps, persistent)
        L = res[0][2]
        name = "persistent + in-kernel all-reduce" if persistent else "kernel chain + one-shot all-reduce kernels"
        print(f"TP=2 (2 ranks, one GPU), {args.model}, B=1 decode graph: {name}: "
              + ", ".join(f"rank {k} {v[0]:.3f} ms ({v[0] * 1000 / L:.1f} us/layer, err {v[1]})" for k, v in sorted(res.items()))
              + f"  [{time.time() - t0:.0f} s]", flush=True)


if __name__ == "__main__":
    main()
