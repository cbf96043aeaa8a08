"""Full-size model validation on ONE MI355X (288 GB HBM3E): Llama-3-70B (141 GB bf16) and
Mixtral-8x7B (93 GB) fit at TP=1, so the real-geometry forward, hipGraph decode and SAFE_DECODE
output can be checked on the single-GPU box; TP=8 itself needs the 8-GPU node.

Prints one JSON line per model: build time, memory, prefill ms, decode ms/step at batch 1 / 32 /
128 (bucketed hipGraph replays) and a sample reply that must pass the reference's validator.
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine  # noqa: E402
from ai_agent_kubectl_amd.engine.sequence import SamplingParams  # noqa: E402
from ai_agent_kubectl_amd.llm.engine_backend import EngineLLM  # noqa: E402
from ai_agent_kubectl_amd.safety import is_safe_kubectl_command  # noqa: E402


def run(model, batches=(1, 32, 128)):
    t0 = time.perf_counter()
    eng = build_engine(EngineOptions(model=model, device="cuda:0", max_batch=max(batches), graph_buckets=batches,
                                     kv_cache_tokens=65536, max_model_len=512))
    cap = eng.runner.capture_graphs()
    build = time.perf_counter() - t0
    be = EngineLLM(eng, max_new_tokens=16, ignore_eos=True)
    out = {"model": model, "build_s": round(build, 1), "graph_capture_s": round(cap, 1),
           "mem_alloc_gb": round(torch.cuda.memory_allocated() / 2**30, 1)}
    params = SamplingParams(max_new_tokens=16, ignore_eos=True)
    for B in batches:
        qs = [be.prompt_ids(f"team-{B}-{i}: list all pods in namespace prod") for i in range(B)]
        st0 = dict(eng.runner.stats)
        t = time.perf_counter()
        seqs = eng.generate_blocking(qs, params, forced_prefix=be._forced)
        el = time.perf_counter() - t
        st = {k: eng.runner.stats[k] - st0[k] for k in st0}
        out[f"b{B}_decode_ms_per_step"] = round(st["decode_ms"] / max(1, st["decode_steps"]), 3)
        out[f"b{B}_prefill_ms"] = round(st["prefill_ms"] / max(1, st["prefill_steps"]), 2)
        out[f"b{B}_total_s"] = round(el, 3)
        txt = be.tok.decode(seqs[0].output_ids)
        assert is_safe_kubectl_command(txt), txt
        out["sample"] = txt
    print(json.dumps(out), flush=True)
    del eng, be
    torch.cuda.empty_cache()


if __name__ == "__main__":
    for m in (sys.argv[1:] or ["llama3-70b", "mixtral-8x7b"]):
        run(m)
