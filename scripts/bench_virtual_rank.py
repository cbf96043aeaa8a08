"""One rank of a tensor-parallel engine on ONE GPU: the per-rank shard of Llama-3-70B at TP = 8 (or of
Mixtral-8x7B at EP = TP = 8), its all-reduces / all-gathers left out (parallel/comm.py VirtualRankComm),
timed the way the serving path runs it: the decode hipGraph of each batch bucket replayed, and one
eager prefill step of ~4k tokens.  What a real TP = 8 step adds on top is the collectives' time
(2 all-reduces per layer of B x H x 2 bytes, the argmax all-gather).

    python scripts/bench_virtual_rank.py --model llama3-70b --tp 8 --buckets 1,8,64,256

KA_GEMM_PLAN=write (with PLAN_COPY_TO=dir) tunes and persists the shard shapes' plans
(ops/tuned/gemm_plan_mi355x.json), so engine start at TP = 8 loads every plan without timing.
"""
import argparse
import os
import shutil
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd import ops  # noqa: E402
from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine  # noqa: E402
from ai_agent_kubectl_amd.engine.sequence import SamplingParams, Sequence  # noqa: E402
from ai_agent_kubectl_amd.llm.engine_backend import EngineLLM  # noqa: E402
from ai_agent_kubectl_amd.ops.autotune import DEFAULT_PLAN_FILE  # noqa: E402
from ai_agent_kubectl_amd.parallel.comm import VirtualRankComm  # noqa: E402


def _heartbeat():
    t0 = time.time()
    while True:
        time.sleep(30)
        print(f"... {time.time() - t0:.0f} s", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--tp", type=int, default=8)
    ap.add_argument("--buckets", default="1,8,64,256")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--prefill-seqs", type=int, default=32, help="sequences of the timed prefill step")
    ap.add_argument("--device", default="cuda", help="cpu: a logic check of the script (no graphs, no timing)")
    args = ap.parse_args()
    threading.Thread(target=_heartbeat, daemon=True).start()
    buckets = tuple(int(b) for b in args.buckets.split(","))
    comm = VirtualRankComm(args.tp)
    t0 = time.time()
    eng = build_engine(EngineOptions(model=args.model, device=args.device, tp_rank=0, tp_size=args.tp, ep_size=args.tp,
                                     max_batch=max(buckets + (args.prefill_seqs,)), graph_buckets=buckets,
                                     kv_cache_tokens=65536, max_model_len=512), comm=comm)
    r, m = eng.runner, eng.runner.model
    print(f"{args.model} rank 0 of TP={args.tp}: {len(m.layers)} layers, hq={m.hq} hkv={m.hkv}, built in "
          f"{time.time() - t0:.1f} s; weights {sum(w.numel() * w.element_size() for w in m.W.values()) / 2**30:.1f} GiB",
          flush=True)
    t0 = time.time()
    r.capture_graphs(autotune=True)
    plan = getattr(r, "gemm_plan", {})
    print(f"plans + graphs in {time.time() - t0:.1f} s; gemm plan: "
          f"{plan.get('from', 'tuned at start') if isinstance(plan, dict) else plan}", flush=True)
    if os.environ.get("PLAN_COPY_TO"):
        os.makedirs(os.environ["PLAN_COPY_TO"], exist_ok=True)
        shutil.copy(DEFAULT_PLAN_FILE, os.environ["PLAN_COPY_TO"])
    be = EngineLLM(eng, max_new_tokens=64, ignore_eos=True)
    sch = eng.scheduler
    sch.gather_max_s = 0.0
    sch.prefill_max_wait_s = 0.0
    params = SamplingParams(max_new_tokens=64, ignore_eos=True)
    n = max(max(buckets), args.prefill_seqs)
    sync = torch.cuda.synchronize if args.device.startswith("cuda") else (lambda: None)
    with torch.inference_mode():
        # one warm prefill (the instruction blocks become prefix-cache hits), then a timed cold one
        for i in range(n):
            sch.add(Sequence(prompt_ids=be.prompt_ids(f"list pods in namespace team-{i} sorted by age"), params=params))
        steps, tok, dt = 0, 0, 0.0
        while sch.waiting:
            b = sch.schedule()
            sync()
            t1 = time.perf_counter()
            out = r.execute(b)
            sync()
            if steps > 0 or len(b.seqs) > 1:
                dt += time.perf_counter() - t1
                tok += b.num_tokens
            steps += 1
            eng._apply(b, out)
            sch.on_step_done(b)
        print(f"prefill: {tok} tokens in {dt * 1e3:.1f} ms over {steps} steps ({tok / max(dt, 1e-9):.0f} tok/s, "
              f"eager, collectives left out)", flush=True)
        batch = sch.schedule()
        assert batch.is_decode
        calls0, bytes0 = comm.allreduce_calls, comm.allreduce_bytes
        out = []
        for B in buckets:
            sub = type(batch)(batch.seqs[:B], [1] * B, is_decode=True)
            r._pack_decode(sub, B)
            nc = r._off["bt"] + B * r.max_blocks
            r.d_stage[:nc].copy_(r.h_stage[:nc])
            if B == buckets[0]:   # collectives a real group would run per decode step (one eager step)
                r._decode_forward(B)
                sync()
                calls, nbytes = comm.allreduce_calls - calls0, comm.allreduce_bytes - bytes0
            g = r.graphs.get(B)
            if g is None:   # CPU logic check
                r._decode_forward(B)
                out.append(f"B={B}: eager ok")
                continue
            for _ in range(5):
                g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            out.append(f"B={B}: {e0.elapsed_time(e1) / args.reps:.3f} ms")
        print(f"decode graph replay, one rank of TP={args.tp} (collectives left out): " + ", ".join(out), flush=True)
        print(f"per decode step a real group adds {calls} all-reduces ({nbytes / max(calls, 1) / 1024:.1f} KiB each "
              f"at B={buckets[0]}) and one argmax all-gather", flush=True)


if __name__ == "__main__":
    main()
