"""Debug: the captured B = 1 decode graph with the persistent kernel, replayed step after step,
against eager persistent forwards of the same steps (error word and token per step)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine  # noqa: E402
from ai_agent_kubectl_amd.engine.sequence import SamplingParams, Sequence  # noqa: E402
from ai_agent_kubectl_amd.llm.engine_backend import EngineLLM  # noqa: E402
from ai_agent_kubectl_amd.models.llama import AttnMeta  # noqa: E402


def main():
    eng = build_engine(EngineOptions(model="llama3-8b-2l", device="cuda", max_batch=1, graph_buckets=(1,),
                                     kv_cache_tokens=8192, max_model_len=512, use_graphs=True))
    r, m, sch = eng.runner, eng.runner.model, eng.scheduler
    m.persistent = True
    r.capture_graphs(autotune=False)
    be = EngineLLM(eng, max_new_tokens=16, ignore_eos=True)
    sch.gather_max_s = 0.0
    with torch.inference_mode():
        sch.add(Sequence(prompt_ids=be.prompt_ids("list all pods in kube-system"),
                         params=SamplingParams(max_new_tokens=16, ignore_eos=True)))
        b = sch.schedule()
        eng._apply(b, r.execute(b))
        sch.on_step_done(b)
        for step in range(8):
            batch = sch.schedule()
            r._pack_decode(batch, 1)
            n = r._off["bt"] + r.max_blocks
            r.d_stage[:n].copy_(r.h_stage[:n])
            meta = AttnMeta(positions=r._view("pos", 1), slot_mapping=r._view("slots", 1),
                            block_tables=r._view("bt", 1), ctx_lens=r._view("ctx", 1),
                            logits_indices=r.d_logits_idx[:1], is_decode=True)
            kc, vc = r.k_cache.clone(), r.v_cache.clone()
            h = m.forward(r._view("ids", 1), meta, kc, vc)
            mask = r._view("mask", 1) if r.mask_bits is not None else None
            tok_e = m.sample(h, r.mask_bits, mask)[:1].tolist()
            torch.cuda.synchronize()
            err_e = m.persistent_err()
            ws = m._pd[1]
            snap = ws[:4096].clone()
            r.graphs[1].replay()
            torch.cuda.synchronize()
            err_g = m.persistent_err()
            tok_g = r.d_out[:1].tolist()
            cnt = ws[:4096].view(torch.int32)
            print(f"step {step}: ctx {int(r._view('ctx', 1)[0])} slot {int(r._view('slots', 1)[0])} eager {tok_e} err {err_e} "
                  f"graph {tok_g} err {err_g}; shards {cnt[0:256:32].tolist()} grp {cnt[256:512:32].tolist()} "
                  f"err word {int(cnt[1008])}", flush=True)
            eng._apply(batch, tok_g)
            sch.on_step_done(batch)


if __name__ == "__main__":
    main()
