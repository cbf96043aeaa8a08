"""Real multi-process tensor parallelism over torch.distributed (gloo on CPU, world_size 2).

Exercises exactly the code that runs over RCCL on MI355X: TorchComm all-reduce / all-gather /
broadcast, the runner's driver (rank 0: scheduler + metadata broadcast) / worker (`worker_loop`)
protocol, vocab-parallel argmax and expert-parallel Mixtral.  Tokens must equal the TP=1 run.
"""
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


def _worker(rank, world, port, model, queue):
    sys.path.insert(0, ROOT)
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    torch.set_num_threads(2)
    from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine
    from ai_agent_kubectl_amd.engine.sequence import SamplingParams
    from ai_agent_kubectl_amd.llm.engine_backend import EngineLLM
    from ai_agent_kubectl_amd.parallel.launch import init_tp
    comm, r = init_tp(world, backend="gloo")
    eng = build_engine(EngineOptions(model=model, device="cpu", tp_rank=r, tp_size=world, max_batch=4,
                                     graph_buckets=(1, 2, 4), kv_cache_tokens=4096, max_model_len=256), comm=comm)
    if r != 0:
        eng.runner.worker_loop()
        queue.put((r, None))
        return
    be = EngineLLM(eng, max_new_tokens=6, ignore_eos=True)
    params = SamplingParams(max_new_tokens=6, ignore_eos=True)
    seqs = eng.generate_blocking([be.prompt_ids(q) for q in ("list pods", "get nodes in prod", "scale web to 2")],
                                 params, forced_prefix=be._forced)
    eng.runner.stop_workers()
    queue.put((0, [s.output_ids for s in seqs]))


def _run_tp(model, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, model, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, toks = q.get(timeout=120)
        out[r] = toks
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out[0]


@pytest.mark.slow
@pytest.mark.parametrize("model", ["tiny-llama", "tiny-mixtral"])
def test_tp2_gloo_matches_tp1(model):
    tp1 = _run_tp(model, 1)
    tp2 = _run_tp(model, 2)
    assert tp1 == tp2


def _lookahead_worker(rank, world, port, queue):
    """Rank 0 steps the engine by hand with arrivals while steps are in flight (KA_TP_OVERLAP=force:
    gloo stands in for RCCL): prefill / mixed steps are queued async, steps are scheduled ahead of
    the in-flight readback and their placeholder inputs fixed up on rank 0's device before the
    staging broadcast.  Lookahead on must sample what lookahead off samples."""
    sys.path.insert(0, ROOT)
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), KA_TP_OVERLAP="force")
    torch.set_num_threads(2)
    try:
        from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine
        from ai_agent_kubectl_amd.engine.sequence import SamplingParams
        from ai_agent_kubectl_amd.llm.engine_backend import EngineLLM
        from ai_agent_kubectl_amd.parallel.launch import init_tp
        comm, r = init_tp(world, backend="gloo")
        eng = build_engine(EngineOptions(model="tiny-llama", device="cpu", tp_rank=r, tp_size=world, max_batch=4,
                                         graph_buckets=(1, 2, 4), kv_cache_tokens=4096, max_model_len=256),
                           comm=comm)
        if r != 0:
            eng.runner.worker_loop()
            queue.put((r, None, None))
            return
        assert eng.runner.can_lookahead() and eng.runner.can_overlap_prefill(2)
        be = EngineLLM(eng, max_new_tokens=6, ignore_eos=True)
        prompts = [be.prompt_ids(q) for q in ("list pods", "get svc -A", "top nodes", "describe pod web-1",
                                              "logs api", "get services in namespace kube-system -o wide")]
        sch = eng.scheduler
        sch.gather_max_s, sch.prefill_max_wait_s = 0.0, 0.0
        sch.max_batched_tokens, sch.min_chunk = 24, 4   # chunked prompts: mixed steps
        n_async = [0]
        launch = eng.runner.launch_prefill_async

        def counted(batch):
            n_async[0] += 1
            return launch(batch)
        eng.runner.launch_prefill_async = counted

        def run(lookahead, k):
            eng.lookahead = lookahead
            eng.bm.reset_prefix_cache()
            p = SamplingParams(max_new_tokens=7, ignore_eos=True)
            seqs = [eng.submit(x, p, None, forced_prefix=be._forced) for x in prompts[:2]]
            for i in range(500):
                if i == k:
                    seqs += [eng.submit(x, p, None, forced_prefix=be._forced) for x in prompts[2:]]
                eng.step()
                if i >= k and all(s.finished for s in seqs) and eng._inflight is None:
                    break
            assert all(s.finished for s in seqs) and eng.healthy
            return [list(s.output_ids) for s in seqs]

        res = []
        for k in (1, 3, 5):
            on, off = run(True, k), run(False, k)
            res.append(on == off)
        eng.runner.stop_workers()
        queue.put((0, (res, eng.lookahead_steps, n_async[0]), None))
    except Exception:
        import traceback
        queue.put((rank, None, traceback.format_exc()))


@pytest.mark.slow
def test_tp2_lookahead_and_prefill_overlap_match_sync():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_lookahead_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(2):
            r, val, tb = q.get(timeout=300)
            assert tb is None, tb
            out[r] = val
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.terminate()
    res, lookahead_steps, async_prefills = out[0]
    assert all(res), res
    assert lookahead_steps > 0 and async_prefills > 0
