"""Shared engine-driving helpers for the CPU and GPU engine tests."""
from ai_agent_kubectl_amd.engine.sequence import Sequence


def run_staggered(eng, prompts, params, forced):
    """Admit one prompt per step so that every step after the first is a mixed decode+prefill step."""
    seqs = []
    run_staggered.mixed = 0
    wait, eng.scheduler.prefill_max_wait_s = eng.scheduler.prefill_max_wait_s, 0.0
    gather, eng.scheduler.gather_max_s = eng.scheduler.gather_max_s, 0.0
    hold, eng.scheduler.hold_steps = eng.scheduler.hold_steps, 0
    try:
        pending = list(prompts)
        while pending or any(not s.finished for s in seqs):
            if pending:
                s = Sequence(prompt_ids=list(pending.pop(0)), params=params, forced_prefix=list(forced))
                eng.scheduler.add(s)
                seqs.append(s)
            batch = eng.scheduler.schedule()
            run_staggered.mixed += bool(batch.prefill_seqs) and len(batch.seqs) > len(batch.prefill_seqs)
            eng._apply(batch, eng.runner.execute(batch))
            eng.scheduler.on_step_done(batch)
    finally:
        eng.scheduler.prefill_max_wait_s = wait
        eng.scheduler.gather_max_s = gather
        eng.scheduler.hold_steps = hold
    return [s.output_ids for s in seqs]
