"""Bitwise repeatability of the hand-written kernels that wait for LDS-DMA with counted vmcnt: the
persistent decode kernel (per-wave weight rings), the gemm_mfma ring kernels and gemm_big.  Each
kernel's result has one fixed summation order, so every repeat of a launch must be bit-identical;
a piece read before it landed (the hazard of profiles/r5/gemm_big_clamp/) shows as a mismatch.
Every repeat follows an unrelated GEMM, the pattern that exposed the gemm_big hazard.  GPU only.

    python scripts/determinism_stress.py [--reps N]
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ai_agent_kubectl_amd import ops  # noqa: E402

BF, DEV = torch.bfloat16, "cuda"
ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=100)
ap.add_argument("--skip-model", action="store_true")
args = ap.parse_args()
torch.manual_seed(0)
other = torch.randn(4096, 4096, device=DEV, dtype=BF)
wo = (torch.randn(4096, 4096, device=DEV) / 64).to(BF)
total = 0


def repeat(name, fn):
    global total
    first = fn().clone()
    bad = 0
    for _ in range(args.reps - 1):
        torch.nn.functional.linear(other, wo)
        bad += int(not torch.equal(fn(), first))
    total += bad
    print(f"{name}: {bad} of {args.reps - 1} repeats differ", flush=True)


# gemm_big (drained waits) and gemm_mfma ring kernels (counted waits) at the engine's shapes
for (M, N, K) in [(4096, 1152, 4096), (2944, 6144, 4096), (4096, 4096, 4096)]:
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(BF)
    repeat(f"gemm_big {M}x{N}x{K}", lambda: ops.linear_big(x, w))
for (M, N, K) in [(256, 6144, 4096), (256, 4096, 14336), (64, 28672, 4096), (8, 4096, 4096)]:
    x = torch.randn(M, K, device=DEV, dtype=BF)
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(BF)
    for cfg in (2, 5, 19):
        try:
            ops.linear_gm(x, w, cfg, 1)
        except (ValueError, RuntimeError):
            continue
        repeat(f"gemm_mfma cfg {cfg} {M}x{N}x{K}", lambda: ops.linear_gm(x, w, cfg, 1))

if not args.skip_model:
    # the persistent all-layers decode kernel, full-depth Llama-3-8B, B = 1 and 2
    from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine
    from ai_agent_kubectl_amd.engine.sequence import Sequence
    from ai_agent_kubectl_amd.engine.sequence import SamplingParams
    from ai_agent_kubectl_amd.llm.engine_backend import EngineLLM
    from ai_agent_kubectl_amd.models.llama import AttnMeta
    eng = build_engine(EngineOptions(model="llama3-8b", device=DEV, max_batch=2, graph_buckets=(1, 2),
                                     kv_cache_tokens=8192, max_model_len=512, use_graphs=False))
    be = EngineLLM(eng, max_new_tokens=16, ignore_eos=True)
    sch, r = eng.scheduler, eng.runner
    sch.gather_max_s = 0.0
    sch.prefill_max_wait_s = 0.0
    m = r.model
    with torch.inference_mode():
        for q in ("list all pods in kube-system", "show services in namespace prod"):
            sch.add(Sequence(prompt_ids=be.prompt_ids(q), params=SamplingParams(max_new_tokens=16, ignore_eos=True)))
        while sch.waiting:
            b = sch.schedule()
            eng._apply(b, r.execute(b))
            sch.on_step_done(b)
        batch = sch.schedule()
        for B in (1, 2):
            r._pack_decode(batch, B)
            n = r._off["bt"] + B * r.max_blocks
            r.d_stage[:n].copy_(r.h_stage[:n])
            meta = AttnMeta(positions=r._view("pos", B), slot_mapping=r._view("slots", B),
                            block_tables=r._view("bt", B), ctx_lens=r._view("ctx", B),
                            logits_indices=r.d_logits_idx[:B], is_decode=True)
            ids = r._view("ids", B)
            m.persistent = True
            assert m.persistent_ok(B)
            kc, vc = r.k_cache.clone(), r.v_cache.clone()

            def step():
                kc.copy_(r.k_cache)
                vc.copy_(r.v_cache)
                h = m.forward(ids, meta, kc, vc)
                return h

            repeat(f"persistent decode B={B} (32 layers)", step)
            assert m.persistent_err() == 0
print(f"TOTAL differing repeats: {total}", flush=True)
