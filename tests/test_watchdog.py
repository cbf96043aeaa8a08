"""TP/EP worker liveness (parallel/watchdog.py): heartbeats through a c10d store,
rank 0's watchdog flags a lost heartbeat or a stalled engine step exactly once and marks the
engine unhealthy (new cache misses then answer 503)."""
import time

import torch.distributed as dist

from ai_agent_kubectl_amd.parallel.watchdog import Heartbeat, Watchdog


def test_heartbeat_keeps_watchdog_quiet_and_loss_is_flagged():
    store = dist.HashStore()
    hb = Heartbeat(store, 1, interval=0.02).start()
    fails = []
    wd = Watchdog(store, [1], fails.append, hb_timeout=0.3, interval=0.02)
    time.sleep(0.1)
    assert wd.check() is None
    hb.stop()
    time.sleep(0.5)
    reason = wd.check()
    assert reason and "rank 1 heartbeat lost" in reason
    assert wd.check() is not None and len(fails) == 1      # reported once


def test_missing_worker_gets_grace_period_then_fails():
    store = dist.HashStore()
    fails = []
    wd = Watchdog(store, [1, 2], fails.append, hb_timeout=5.0)
    assert wd.check() is None                               # never beat, still within the grace period
    assert "rank 1" in wd.check(now=time.time() + 10)


def test_step_stall_marks_engine_unhealthy():
    store = dist.HashStore()
    Heartbeat(store, 1).beat()

    class Eng:
        healthy, last_error, step_t0 = True, None, None

        def mark_unhealthy(self, reason):
            self.healthy, self.last_error = False, RuntimeError(reason)

    eng = Eng()
    wd = Watchdog(store, [1], eng.mark_unhealthy, hb_timeout=60, step_timeout=0.05,
                  step_started=lambda: eng.step_t0)
    assert wd.check() is None
    eng.step_t0 = time.perf_counter() - 1.0
    assert "stalled" in wd.check()
    assert not eng.healthy and "stalled" in str(eng.last_error)


def test_watchdog_thread_runs():
    store = dist.HashStore()
    fails = []
    wd = Watchdog(store, [3], fails.append, hb_timeout=0.05, interval=0.02).start()
    t0 = time.time()
    while not fails and time.time() - t0 < 5:
        time.sleep(0.02)
    wd.stop()
    assert fails and "rank 3" in fails[0]


def test_collective_timer_host_path():
    import torch
    from ai_agent_kubectl_amd.parallel.comm import CollectiveTimer
    t = CollectiveTimer()
    tok = t.begin(torch.zeros(4))
    time.sleep(0.01)
    t.end(tok)
    got = t.drain()
    assert len(got) == 1 and got[0] >= 0.009
    assert t.drain() == []


def test_rccl_metrics_registered():
    from ai_agent_kubectl_amd.metrics import ServiceMetrics
    m = ServiceMetrics()
    m.rccl_allreduce.observe(3e-5)
    m.rccl_allreduce_bytes.inc(8192)
    from prometheus_client import generate_latest
    text = generate_latest(m.registry).decode()
    assert "rccl_allreduce_seconds_bucket" in text and "rccl_allreduce_bytes_total 8192.0" in text
