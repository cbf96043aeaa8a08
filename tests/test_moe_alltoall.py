"""Expert-parallel all-to-all dispatch / combine (models/moe.py `moe_alltoall` and
the shape-static, graph-capturable `moe_alltoall_static`)
over real torch.distributed process groups (gloo, world_size 2 and 4): the token-sharded
all-to-all path must equal the single-process MoE over all experts, including shards that are
short or empty (T not divisible by, or smaller than, the world size)."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _weights(cfg, seed=0):
    g = torch.Generator().manual_seed(seed)
    H, I, E = cfg.hidden, cfg.intermediate, cfg.num_experts
    return {"router": torch.randn(E, H, generator=g) * 0.2,
            "w13": torch.randn(E, 2 * I, H, generator=g) * H ** -0.5,
            "w2": torch.randn(E, H, I, generator=g) * I ** -0.5}


def _worker(rank, world, port, T_list, queue):
    sys.path.insert(0, ROOT)
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    import torch.distributed as dist
    from ai_agent_kubectl_amd.models.config import get_config
    from ai_agent_kubectl_amd.models.moe import moe_alltoall, moe_alltoall_static, moe_forward
    from ai_agent_kubectl_amd.parallel.comm import make_comm
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = make_comm(None)
    cfg = get_config("tiny-mixtral")
    full = _weights(cfg)
    el = cfg.num_experts // world
    L = {"router": full["router"], "w13": full["w13"][rank * el:(rank + 1) * el].contiguous(),
         "w2": full["w2"][rank * el:(rank + 1) * el].contiguous()}
    outs = []
    for T in T_list:
        x = torch.randn(T, cfg.hidden, generator=torch.Generator().manual_seed(T))
        y = moe_alltoall(x, L, cfg, comm)
        y2, combined = moe_forward(x, L, cfg, rank, world, False, comm)   # the model's entry point
        assert combined
        # all-reduce combine of the per-rank partials (the decode path) for comparison
        part, combined = moe_forward(x, L, cfg, rank, world, True, comm)
        assert not combined
        comm.all_reduce(part)
        y3 = moe_alltoall_static(x, L, cfg, comm)   # shape-static splits (graph-capturable form)
        os.environ["MOE_DISPATCH"] = "a2a-static"
        y4, combined = moe_forward(x, L, cfg, rank, world, True, comm)   # decode goes through it too
        assert combined
        del os.environ["MOE_DISPATCH"]
        outs.append(tuple(t.numpy() for t in (y, y2, part, y3, y4)))
    queue.put((rank, outs))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_moe_alltoall_matches_single_process(world):
    sys.path.insert(0, ROOT)
    from ai_agent_kubectl_amd.models.config import get_config
    from ai_agent_kubectl_amd.models.moe import moe_grouped
    cfg = get_config("tiny-mixtral")
    T_list = [1, 3, 8, 37]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, T_list, q)) for r in range(world)]
    for p in procs:
        p.start()
    import queue as _queue
    import time
    res, t0 = {}, time.time()
    while len(res) < world:
        try:
            r, outs = q.get(timeout=2)
            res[r] = outs
        except _queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead and time.time() - t0 < 180, f"worker failed: {dead}"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    W = _weights(cfg)
    for i, T in enumerate(T_list):
        x = torch.randn(T, cfg.hidden, generator=torch.Generator().manual_seed(T))
        ref = moe_grouped(x, W, cfg, 0, 1)
        for r in range(world):
            y, y2, part, y3, y4 = (torch.from_numpy(a) for a in res[r][i])
            torch.testing.assert_close(y3, ref, rtol=1e-4, atol=1e-4)
            torch.testing.assert_close(y4, ref, rtol=1e-4, atol=1e-4)
            torch.testing.assert_close(y, ref, rtol=1e-4, atol=1e-4)
            torch.testing.assert_close(y2, ref, rtol=1e-4, atol=1e-4)
            torch.testing.assert_close(part, ref, rtol=1e-4, atol=1e-4)
