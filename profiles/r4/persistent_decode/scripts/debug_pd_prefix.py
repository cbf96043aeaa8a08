"""Debug: cold vs warm (prefix-cached) generation through the persistent batch-1 decode kernel,
eager and with graphs, repeated, against the kernel chain."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine  # noqa: E402
from ai_agent_kubectl_amd.engine.sequence import SamplingParams  # noqa: E402
from ai_agent_kubectl_amd.llm.engine_backend import EngineLLM  # noqa: E402

Q = "list all pods in the kube-system namespace"


def run(graphs, persistent, buckets=(1, 2, 4, 8)):
    print("buckets", buckets, "lookahead", os.environ.get("KA_LOOKAHEAD"), flush=True)
    opts = EngineOptions(model="llama3-8b-2l", device="cuda", max_batch=max(buckets), graph_buckets=buckets,
                         kv_cache_tokens=16384, max_model_len=512, use_graphs=graphs)
    eng = build_engine(opts)
    eng.runner.model.persistent = persistent
    m = eng.runner.model
    orig = m._forward_persistent

    def wrapped(*a, **k):
        if m._pd is None:
            print("  _pd created; capturing:", torch.cuda.is_current_stream_capturing(), flush=True)
        return orig(*a, **k)
    m._forward_persistent = wrapped
    if graphs:
        eng.runner.capture_graphs()
    be = EngineLLM(eng, max_new_tokens=8, ignore_eos=True)
    params = SamplingParams(max_new_tokens=8, ignore_eos=True)
    outs = []
    for i in range(4):
        s = eng.generate_blocking([be.prompt_ids(Q)], params, forced_prefix=be._forced)[0]
        outs.append((s.num_cached_prompt, s.output_ids))
        if persistent and m._pd is not None:
            print("  err after generate", i, m.persistent_err(), "ws", hex(m._pd[1].data_ptr()), flush=True)
    m = eng.runner.model
    print(f"graphs={graphs} persistent={persistent} err={m.persistent_err() if persistent else 0}", flush=True)
    for c, o in outs:
        print(f"   cached {c:3d}: {o}", flush=True)
    del eng
    torch.cuda.empty_cache()


if __name__ == "__main__":
    run(True, True, (1,))
    run(True, True, (1, 2))
    run(True, True, (2, 1))
