"""One-shot all-reduce (csrc/allreduce.hip) with 2 ranks sharing the single GPU of the test box.

Both processes map each other's uncached buffers through hipIpc handles and run the kernel
concurrently on the same device, so the IPC mapping, the flag handshake, the epoch / half
alternation and hipGraph replay are exercised; the xGMI (multi-GPU) transport itself needs the
8-GPU node (validated by the driver's TP runs, not here).
"""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        from ai_agent_kubectl_amd.parallel.custom_allreduce import OneShotAllReduce
        ar = OneShotAllReduce(None, "cuda:0", cap_elems=1 << 20)
        errs = []
        for it, n in enumerate([8, 4096, 8192 * 8, 4096 * 256, 1 << 20, 16]):
            g = torch.Generator().manual_seed(1000 + it)
            parts = [torch.randn(n, generator=g).to(torch.bfloat16) for _ in range(world)]
            want = sum(p.float() for p in parts)
            t = parts[rank].cuda()
            ar.all_reduce(t)
            torch.cuda.synchronize()
            errs.append((t.float().cpu() - want).abs().max().item())
        # fused all-reduce + residual add + RMSNorm == all-reduce then the RMSNorm kernel, bit for bit
        from ai_agent_kubectl_amd import ops
        for rows, hidden in ((1, 4096), (3, 8192), (70, 4096)):
            g = torch.Generator().manual_seed(77 + rows)
            parts = [torch.randn(rows, hidden, generator=g).to(torch.bfloat16) for _ in range(world)]
            res0 = torch.randn(rows, hidden, generator=g).to(torch.bfloat16).cuda()
            wgt = (torch.rand(hidden, generator=g) + 0.5).to(torch.bfloat16).cuda()
            t1, r1 = parts[rank].cuda(), res0.clone()
            ar.all_reduce(t1)
            want_out = ops.rmsnorm(t1, wgt, 1e-5, residual=r1)
            t2, r2 = parts[rank].cuda(), res0.clone()
            got_out = ar.all_reduce_rmsnorm(t2, wgt, 1e-5, r2)
            torch.cuda.synchronize()
            errs.append(0.0 if torch.equal(got_out, want_out) and torch.equal(r2, r1) else 1.0)
            # split-K partial slabs reduced inside the collective (round 6: a TP rank's O / down hand
            # their partials to it) == splitk_reduce's bf16 sum then the collective, bit for bit
            for pdt, split in ((torch.float32, 4), (torch.bfloat16, 8), (torch.bfloat16, 2)):
                slabs = (torch.randn(split, rows, hidden, generator=g) * 0.3).to(pdt).cuda()
                r3, r4 = res0.clone(), res0.clone()
                acc = slabs[0].float()
                for z in range(1, split):   # the kernel's order: fp32, slab 0 first
                    acc = acc + slabs[z].float()
                want3 = ar.all_reduce_rmsnorm(acc.to(torch.bfloat16), wgt, 1e-5, r3)
                got4 = ar.all_reduce_rmsnorm(ops.SplitK(slabs, split), wgt, 1e-5, r4)
                torch.cuda.synchronize()
                errs.append(0.0 if torch.equal(got4, want3) and torch.equal(r4, r3) else 1.0)
            t3 = torch.arange(rows * 4, dtype=torch.int32, device="cuda").view(rows, 4) + 1000 * rank
            gath = ar.all_gather(t3)
            errs.append(0.0 if all(torch.equal(gath[p], t3 - 1000 * rank + 1000 * p) for p in range(world)) else 1.0)
        # hipGraph capture + replay (epoch read from device memory each replay)
        x = torch.zeros(4096, dtype=torch.bfloat16, device="cuda")
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                ar.all_reduce(x)
        dist.barrier()
        for rep in range(5):
            x.fill_(float(rank + 1 + rep))
            torch.cuda.synchronize()
            dist.barrier()
            g.replay()
            torch.cuda.synchronize()
            want = sum(float(r + 1 + rep) for r in range(world))
            errs.append((x.float() - want).abs().max().item())
        ar.check()
        dist.barrier()
        ar.close()
        q.put((rank, errs, None))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, None, traceback.format_exc()))


def test_oneshot_allreduce_two_ranks_one_gpu():
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, errs, tb in res:
        assert tb is None, tb
        assert max(errs) < 0.1, (rank, errs)
