"""Per-phase GPU profile of the bench workload: one prefill step admitting C requests at once
(prefix-cached instruction blocks, sub-block reuse) and C-row decode steps (hipGraph replay).

Drives the engine step by step on this thread and wraps each phase in torch.profiler, printing
wall ms per phase and the top kernels by GPU time, so prefill and decode costs can be attributed
separately (a whole-run rocprofv3 trace mixes in model build, autotune and warm-up).

  python scripts/phase_profile.py [--concurrency 256] [--model llama3-8b]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine  # noqa: E402
from ai_agent_kubectl_amd.engine.sequence import SamplingParams, Sequence  # noqa: E402
from ai_agent_kubectl_amd.llm.engine_backend import EngineLLM  # noqa: E402
import bench  # noqa: E402


def table(prof, n=25):
    rows = []
    for e in prof.key_averages():
        t = getattr(e, "device_time_total", None) or getattr(e, "cuda_time_total", 0)
        if t > 0 and e.key and not e.key.startswith("ProfilerStep"):
            rows.append((t, e.count, e.key))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows if not r[2].startswith("aten::") and not r[2].startswith("cuda"))
    out = [f"  device total (kernels) {tot / 1e3:.2f} ms"]
    for t, c, k in rows[:n]:
        out.append(f"  {t / 1e3:9.3f} ms  n={c:5d}  avg={t / max(1, c):8.1f} us  {k[:100]}")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--concurrency", type=int, default=256)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--decode-steps", type=int, default=8)
    ap.add_argument("--budget", type=int, default=0, help="tokens per step (0: the model's default, as bench.py)")
    ap.add_argument("--prefill-steps", type=int, default=3, help="mixed steps profiled one by one")
    a = ap.parse_args()
    C = a.concurrency
    buckets = tuple(b for b in (1, 8, 16, 32, 64, 128, 192, 256, 384, 512) if b <= C) + ((C,) if C not in (1, 8, 16, 32, 64, 128, 192, 256, 384, 512) else ())
    eng = build_engine(EngineOptions(model=a.model, device="cuda:0", max_batch=C, graph_buckets=buckets,
                                     kv_cache_tokens=max(65536, C * 528), max_model_len=512, ignore_eos=True,
                                     max_batched_tokens=a.budget))
    eng.runner.capture_graphs()
    be = EngineLLM(eng, max_new_tokens=16, ignore_eos=True)
    params = SamplingParams(max_new_tokens=16, ignore_eos=True)
    eng.scheduler.gather_max_s = 0.0
    for w in range(2):   # warm: publish the instruction blocks, exercise the plans
        eng.generate_blocking([be.prompt_ids(bench.make_query(0, w, i)) for i in range(C)], params,
                              forced_prefix=be._forced)
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]

    def one_step():
        batch = eng.scheduler.schedule()
        toks = eng.runner.execute(batch)
        eng._apply(batch, toks)
        eng.scheduler.on_step_done(batch)
        return batch

    def admit(wave):
        for i in range(C):
            eng.scheduler.add(Sequence(prompt_ids=be.prompt_ids(bench.make_query(0, wave, i)), params=params,
                                       forced_prefix=list(be._forced)))

    # wave 9 unprofiled: the wall time of each admission (mixed) step, the profiler's hooks off
    admit(9)
    torch.cuda.synchronize()
    walls = []
    while True:
        t0 = time.perf_counter()
        b = one_step()
        torch.cuda.synchronize()
        if b.is_decode:
            break
        walls.append((b.num_tokens, len(b.seqs), (time.perf_counter() - t0) * 1e3))
    print("MIXED steps, unprofiled (tokens, seqs, wall ms):", [(n, q, round(w, 2)) for n, q, w in walls])
    while eng.scheduler.has_work():
        one_step()
    # wave 10 profiled step by step: device time per kernel of each admission step
    admit(10)
    torch.cuda.synchronize()
    for _ in range(a.prefill_steps):
        with torch.profiler.profile(activities=acts) as prof_p:
            t0 = time.perf_counter()
            b = one_step()
            torch.cuda.synchronize()
            tp = time.perf_counter() - t0
        print(f"PREFILL step: {len(b.seqs)} seqs, {b.num_tokens} tokens, decode={b.is_decode}, "
              f"{len(b.copies)} block copies, wall {tp * 1e3:.2f} ms under the profiler")
        print(table(prof_p))
        if b.is_decode:
            break
    while not b.is_decode:
        b = one_step()
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=acts) as prof_d:
        t0 = time.perf_counter()
        for _ in range(a.decode_steps):
            b = one_step()
        torch.cuda.synchronize()
        td = (time.perf_counter() - t0) / a.decode_steps
    print(f"DECODE steps: B={len(b.seqs)} decode={b.is_decode} wall {td * 1e3:.3f} ms/step")
    print(table(prof_d, 30))
    # eager (non-graph) decode for per-kernel attribution inside the graph
    graphs = eng.runner.graphs
    eng.runner.graphs = {}
    with torch.profiler.profile(activities=acts) as prof_e:
        t0 = time.perf_counter()
        for _ in range(2):
            one_step()
        torch.cuda.synchronize()
        te = (time.perf_counter() - t0) / 2
    eng.runner.graphs = graphs
    print(f"DECODE eager (attribution): {te * 1e3:.3f} ms/step")
    print(table(prof_e, 30))


if __name__ == "__main__":
    main()
