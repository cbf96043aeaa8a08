"""Shared-memory service state (runtime/shared_state.h via shared_state.py): the cache keeps
`cache.TTLCache` semantics (reference `app.py:125`) and the limiter keeps
`ratelimit.FixedWindowLimiter` semantics (Appendix B.1), and both are one state across processes."""
import multiprocessing as mp
import os
import random
import uuid

import pytest

from ai_agent_kubectl_amd.cache import TTLCache
from ai_agent_kubectl_amd.ratelimit import FixedWindowLimiter, parse_many
from ai_agent_kubectl_amd.runtime import native

pytestmark = pytest.mark.skipif(not native.available(), reason="native runtime not built")

from ai_agent_kubectl_amd.shared_state import (SharedFixedWindowLimiter, SharedStore,  # noqa: E402
                                               SharedTTLCache)


class Clock:
    def __init__(self):
        self.t = 1000.0

    def __call__(self):
        return self.t


@pytest.fixture
def store_name():
    name = "/ka_test_" + uuid.uuid4().hex[:12]
    yield name
    SharedStore.unlink(name)


def test_cache_matches_ttlcache_randomised(store_name):
    """Same random op sequence (get / set / contains / len / clock advances) on the shared cache
    and on the reference TTLCache: identical observable results."""
    clk = Clock()
    maxsize, ttl = 7, 5.0
    ref = TTLCache(maxsize, ttl, timer=clk)
    sh = SharedTTLCache(SharedStore(store_name, maxsize), maxsize, ttl, timer=clk)
    rng = random.Random(0)
    keys = ["q%d" % i for i in range(12)] + ["", "ünïcode ✓", "x" * 10000]
    for step in range(4000):
        op = rng.random()
        k = rng.choice(keys)
        if op < 0.4:
            assert sh.get(k) == ref.get(k), step
        elif op < 0.75:
            v = "kubectl get pods -n %d" % rng.randrange(1000)
            ref[k] = v
            sh[k] = v
        elif op < 0.85:
            assert (k in sh) == (k in ref), step
        elif op < 0.9:
            assert len(sh) == len(ref), step
        else:
            clk.t += rng.choice([0.5, 1.0, 2.5, 6.0])
    assert sh.hits == ref.hits and sh.misses == ref.misses


def test_cache_maxsize_zero_and_oversized_value(store_name):
    clk = Clock()
    s = SharedStore(store_name, 4, value_max=64)
    with pytest.raises(ValueError, match="value too large"):
        SharedTTLCache(s, 0, 10, timer=clk)["a"] = "b"
    c = SharedTTLCache(s, 4, 10, timer=clk)
    c["long"] = "x" * 65          # does not fit the value slot: served uncached, never an error
    assert c.get("long") is None
    c["ok"] = "y" * 64
    assert c["ok"] == "y" * 64


def test_limiter_matches_fixed_window(store_name):
    clk = Clock()
    items = parse_many("3/minute;5 per hour")
    ref = FixedWindowLimiter(items, timer=clk)
    sh = SharedFixedWindowLimiter(SharedStore(store_name, 4), items, timer=clk)
    rng = random.Random(1)
    for step in range(600):
        client = rng.choice(["10.0.0.1", "10.0.0.2", "127.0.0.1"])
        scope = rng.choice(["a.x", "a.y"])
        for item in items:
            assert sh.hit(item, client, scope) == ref.hit(item, client, scope), step
        clk.t += rng.choice([0.0, 1.0, 7.0, 61.0])


def test_limiter_table_rebuild_keeps_live_windows(store_name):
    """Many distinct clients: expired windows are recycled (table rebuilds) while live ones keep
    counting."""
    clk = Clock()
    item = parse_many("2/second")[0]
    lim = SharedFixedWindowLimiter(SharedStore(store_name, 1, limiter_keys=1024), [item], timer=clk)
    for rnd in range(8):
        for c in range(700):
            assert lim.hit(item, "c%d" % c, "s")
        assert lim.hit(item, "c0", "s")             # 2nd hit of c0's live window: allowed
        assert lim.hit(item, "c0", "s") is False    # 3rd: over 2/second
        clk.t += 1.5


def _worker(name, q_in, q_out):
    s = SharedStore(name, 8)
    cache = SharedTTLCache(s, 8, 300)
    lim = SharedFixedWindowLimiter(s, parse_many("5/minute"))
    while True:
        op = q_in.get()
        if op is None:
            return
        kind, arg = op
        if kind == "get":
            q_out.put(cache.get(arg))
        elif kind == "set":
            cache[arg[0]] = arg[1]
            q_out.put(True)
        elif kind == "hit":
            q_out.put(lim.hit(lim.default_limits[0], "1.2.3.4", "app.route"))


def test_cross_process_cache_and_limiter(store_name):
    """Two worker processes attached to one segment: a value stored by A is a hit in B, and a
    5/minute budget is consumed jointly (3 + 2 allowed, the 6th hit anywhere is refused)."""
    ctx = mp.get_context("spawn")
    qa, qb, out_a, out_b = ctx.Queue(), ctx.Queue(), ctx.Queue(), ctx.Queue()
    SharedStore(store_name, 8)   # created by the parent (as serve.py's supervisor does)
    pa = ctx.Process(target=_worker, args=(store_name, qa, out_a))
    pb = ctx.Process(target=_worker, args=(store_name, qb, out_b))
    pa.start()
    pb.start()
    try:
        qa.put(("set", ("list all pods", "kubectl get pods")))
        assert out_a.get(timeout=60) is True
        qb.put(("get", "list all pods"))
        assert out_b.get(timeout=60) == "kubectl get pods"
        results = []
        for i in range(6):
            (qa if i % 2 == 0 else qb).put(("hit", None))
            results.append((out_a if i % 2 == 0 else out_b).get(timeout=60))
        assert results == [True] * 5 + [False]
    finally:
        qa.put(None)
        qb.put(None)
        pa.join(30)
        pb.join(30)


def test_owner_death_resets_the_segment(tmp_path):
    """A worker that dies holding the robust mutex half-way through a relink (EOWNERDEAD) must not
    leave half-linked LRU / hash chains for the others: the next lock resets the segment."""
    import multiprocessing as mp
    from ai_agent_kubectl_amd.shared_state import SharedStore, SharedTTLCache
    name = "/ka_test_owner_%d" % os.getpid()
    SharedStore.unlink(name)
    store = SharedStore(name, 8)
    try:
        cache = SharedTTLCache(store, 8, 300)
        for i in range(5):
            cache[f"k{i}"] = f"v{i}"
        p = mp.get_context("fork").Process(target=lambda: SharedStore(name, 8).raw.debug_die_locked(7))
        p.start()
        p.join(30)
        assert p.exitcode == 7
        st = store.stats()
        assert st["owner_deaths"] == 1 and st["size"] == 0
        cache["again"] = "ok"
        assert cache.get("again") == "ok" and cache.get("k1") is None
    finally:
        SharedStore.unlink(name)


def test_incompatible_leftover_segment_is_recreated():
    from ai_agent_kubectl_amd.shared_state import SharedStore, SharedTTLCache
    name = "/ka_test_layout_%d" % os.getpid()
    SharedStore.unlink(name)
    old = SharedStore(name, 8, value_max=256)
    try:
        new = SharedStore(name, 8, value_max=512)   # an earlier run's layout: replaced, not an error
        c = SharedTTLCache(new, 8, 300)
        c["x"] = "y" * 400
        assert c.get("x") == "y" * 400
        with pytest.raises(RuntimeError):
            SharedStore("/ka_test_layout_strict_%d" % os.getpid(), 8, value_max=256, recreate=False) and \
                SharedStore("/ka_test_layout_strict_%d" % os.getpid(), 8, value_max=512, recreate=False)
    finally:
        del old
        SharedStore.unlink(name)
        SharedStore.unlink("/ka_test_layout_strict_%d" % os.getpid())
