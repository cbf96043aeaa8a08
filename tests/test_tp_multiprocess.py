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
