"""Decode-step device time per batch bucket, by replaying the captured decode hipGraph of the real
Llama-3-8B engine (random weights, every row at a ~120-token context), with optional A/B settings
that need a re-capture (e.g. the small-batch gate_up prefetch, KA_DECODE_PREFETCH_MB).

    python scripts/bench_decode_graph.py [--buckets 1,4,256] [--prefetch "0:64,32:64,64:256"]

--prefetch: comma list of MB:blocks settings, each re-captured and timed (0 = off).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine  # noqa: E402
from ai_agent_kubectl_amd.engine.sequence import SamplingParams, Sequence  # noqa: E402
from ai_agent_kubectl_amd.llm.engine_backend import EngineLLM  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--buckets", default="1,4,256")
    ap.add_argument("--prefetch", default="0:64")
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--persistent", default="0", help="comma list of 0/1: the batch-1 persistent decode kernel")
    ap.add_argument("--plan-first", action="store_true",
                    help="load the GEMM plan / LM head / SwiGLU decisions before the prefill (so its steps of "
                         "<= 512 rows dispatch on them, as in serving)")
    ap.add_argument("--tp", type=int, default=1,
                    help="> 1: rank 0 of a TP group on a virtual communicator (collectives left out)")
    args = ap.parse_args()
    buckets = tuple(int(b) for b in args.buckets.split(","))
    kw, comm = {}, None
    if args.tp > 1:
        from ai_agent_kubectl_amd.parallel.comm import VirtualRankComm
        kw, comm = dict(tp_rank=0, tp_size=args.tp), VirtualRankComm(args.tp)
    eng = build_engine(EngineOptions(model=args.model, device="cuda", max_batch=max(buckets), graph_buckets=buckets,
                                     kv_cache_tokens=65536, max_model_len=512, **kw), comm=comm)
    r = eng.runner
    be = EngineLLM(eng, max_new_tokens=64, ignore_eos=True)
    sch = eng.scheduler
    sch.gather_max_s = 0.0
    params = SamplingParams(max_new_tokens=64, ignore_eos=True)
    if args.plan_first:
        r.gemm_plan, r.lm_head_plan, r.swiglu_plan = r.autotune(), r.tune_lm_head(), r.tune_swiglu()
    with torch.inference_mode():
        for i in range(max(buckets)):
            sch.add(Sequence(prompt_ids=be.prompt_ids(f"list pods in namespace team-{i}"), params=params))
            if i == 0:   # the first prompt alone: its instruction blocks are then prefix-cache hits
                b = sch.schedule()   # for every other row, shared as in serving (cascade attention)
                eng._apply(b, r.execute(b))
                sch.on_step_done(b)
        while sch.waiting:   # prefill everyone (eager), so the decode rows have real contexts
            b = sch.schedule()
            eng._apply(b, r.execute(b))
            sch.on_step_done(b)
        batch = sch.schedule()
        assert batch.is_decode
    m = r.model
    first = True
    settings = [(p, pe) for p in args.prefetch.split(",") for pe in args.persistent.split(",")]
    for setting, pers in settings:
        mb, blocks = (float(x) for x in setting.split(":"))
        m.prefetch_bytes, m.prefetch_blocks = int(mb * (1 << 20)), int(blocks)
        m.persistent = pers == "1"
        r.graphs.clear()
        r.graph_pool = None
        r.capture_graphs(autotune=first)   # the persisted GEMM plan / LM head / SwiGLU decisions, once
        first = False
        out = []
        for B in buckets:
            sub = type(batch)(batch.seqs[:B], [1] * B, is_decode=True)
            r._pack_decode(sub, B)
            n = r._off["bt"] + B * r.max_blocks
            r.d_stage[:n].copy_(r.h_stage[:n])
            g = r.graphs[B]
            for _ in range(5):
                g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            out.append(f"B={B}: {e0.elapsed_time(e1) / args.reps:.3f} ms (shared blocks {int(r.h_np[r._off['nsh']])})")
            if r.graph_persistent.get(B):   # the replays' own error word (a wait that ran out = invalid timing)
                out.append(f"graph err {m.persistent_err()}")
        print(f"prefetch {mb:g} MB x {int(blocks)} blocks, persistent {pers}: " + ", ".join(out), flush=True)
        if m.persistent:
            print("  persistent error word:", m.persistent_err(), flush=True)
            # phase breakdown of one launch, every workgroup (stamp k = the end of phase k - 1)
            for PB in [b for b in (1, 2) if m.persistent_ok(b) and len(batch.seqs) >= b]:
                ncu = torch.cuda.get_device_properties(0).multi_processor_count
                m.persistent_stamps = torch.zeros((ncu, len(m.layers), 16), dtype=torch.int64, device="cuda")
                sub = type(batch)(batch.seqs[:PB], [1] * PB, is_decode=True)
                r._pack_decode(sub, PB)
                r.d_stage[:r._off["bt"] + PB * r.max_blocks].copy_(r.h_stage[:r._off["bt"] + PB * r.max_blocks])
                h0 = m.W["embed"][:PB].clone()
                from ai_agent_kubectl_amd.models.llama import AttnMeta
                meta = AttnMeta(positions=r._view("pos", PB), slot_mapping=r._view("slots", PB),
                                block_tables=r._view("bt", PB), ctx_lens=r._view("ctx", PB),
                                logits_indices=r.d_logits_idx[:PB], is_decode=True)
                for _ in range(3):
                    m._forward_persistent(h0, meta, r.k_cache, r.v_cache)
                torch.cuda.synchronize()
                stv = m.persistent_stamps.cpu().double() / 100.0   # 100 MHz -> us
                G = int((stv[:, 1, 0] > 0).sum())
                stv = stv[:G, 1:-1]                                 # layers 1 .. L-2
                names = ["norm1", "qkv", "grp-wait", "attn", "barB", "O", "barC", "norm2", "gate_up", "barD", "down",
                         "barE"]
                per_layer = float((stv[:, :, 12] - stv[:, :, 0]).mean())
                print(f"  persistent B={PB}: {G} workgroups, per layer {per_layer:.1f} us", flush=True)
                for k, n in enumerate(names):
                    ok = (stv[:, :, k + 1] > 0) & (stv[:, :, k] > 0)
                    if not ok.any():
                        continue
                    d = (stv[:, :, k + 1] - stv[:, :, k])[ok]
                    # end-time spread across the grid at this stamp (relative to the layer's first stamp)
                    endt = (stv[:, :, k + 1] - stv[:, :, 0].min(dim=0).values)
                    print(f"  {n:9s} mean {float(d.mean()):6.1f}  p10 {float(d.quantile(0.1)):6.1f}  "
                          f"p90 {float(d.quantile(0.9)):6.1f}  max {float(d.max()):6.1f}   end: "
                          f"min {float(endt.min(dim=0).values.mean()):6.1f} max {float(endt.max(dim=0).values.mean()):6.1f}",
                          flush=True)
                lead = stv[:, :, 13] > 0   # attention leaders: RoPE / context blocks / merge
                if lead.any():
                    sub = [("rope + K/V landed", 3, 13), ("first q.k", 13, 15), ("rest of blocks", 15, 14), ("merge", 14, 4)]
                    print("  attention: " + ", ".join(f"{n} {float((stv[:, :, b] - stv[:, :, a])[lead].mean()):.1f}"
                                                      for n, a, b in sub), flush=True)
                # per-XCD (wg % 8) mean gate_up / down durations: is the skew a fabric effect?
                for k, n in ((8, "gate_up"), (10, "down")):
                    d = stv[:, :, k + 1] - stv[:, :, k]
                    xs = [float(d[x::8].mean()) for x in range(8)]
                    print(f"  {n} by XCD: " + " ".join(f"{v:.1f}" for v in xs), flush=True)
                slow = (stv[:, :, 9] - stv[:, :, 8]).mean(dim=1)
                print("  slowest gate_up workgroups:", [int(i) for i in slow.argsort(descending=True)[:12]], flush=True)
                m.persistent_stamps = None


if __name__ == "__main__":
    main()
