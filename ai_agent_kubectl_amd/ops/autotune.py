"""GEMM plan autotuning for the decode path.

For every projection shape (N, K) of the loaded model and every decode batch bucket M, time the
hand-written weight-streaming kernel at a few split-K factors against hipBLASLt (`F.linear`) on the
model's *own* weights, rotating over layers so each call streams from HBM as in a real step, and
record the winner in `ops.GEMM_PLAN`.  Done once at engine start (before hipGraph capture), so the
captured graphs contain the fastest kernel per shape.
"""
from __future__ import annotations

import logging
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch

from . import (BIG_PLAN_MIN_M, GEMM_PLAN, SKINNY_MAX_M, TILE_MAX_M, big_gemm_ok, gm_shape, linear, linear_big,
               linear_gm, linear_rows, rmsnorm, rows_ok, skinny_split)

logger = logging.getLogger("app.engine")


import os
import os as _os

# TunableOp results for the decode GEMM shapes on MI355X (ROCm 7.x); loaded at start, extended
# (and re-written) if new shapes appear.  Set KA_TUNABLEOP=0 to use hipBLASLt's heuristics only.
DEFAULT_TUNABLEOP_FILE = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "tuned",
                                       "tunableop_mi355x.csv")


ROUNDS = int(_os.environ.get("KA_AUTOTUNE_ROUNDS", "3"))


def _time(fn, weights: List[torch.Tensor], reps: int = 12, rounds: int = 0) -> float:
    """us per call, the best of `rounds` timed runs of `reps` calls (rotating over the layers'
    weights so every call streams from HBM): candidates 1-2 us apart are otherwise ranked by noise."""
    for i in range(3):
        fn(weights[i % len(weights)])
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(max(1, rounds or ROUNDS)):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(reps):
            fn(weights[i % len(weights)])
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps * 1e3)
    return best


# ---- persisted plans ------------------------------------------------------------------------------
# The plan is a pure function of the hardware and the shapes (and of the consumer each projection
# feeds), so one tuned on an MI355X is committed (tuned/gemm_plan_mi355x.json) and loaded at engine
# start instead of re-timing every candidate: deterministic plans across boxes and runs.
# KA_GEMM_PLAN=file (default: use the file when it covers every shape, else tune) | tune | write
# (tune with KA_AUTOTUNE_ROUNDS rounds and merge the result into the file).
DEFAULT_PLAN_FILE = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "tuned", "gemm_plan_mi355x.json")


def plan_key(M: int, N: int, K: int, ctx: str) -> str:
    return f"{M},{N},{K},{ctx}"


def load_plan(path: str, wanted: Dict[Tuple[int, int, int], str]) -> set:
    """Fill GEMM_PLAN from `path` for every wanted (M, N, K) -> consumer context it holds; returns
    the (M, N, K) still missing (to be tuned)."""
    import json
    try:
        with open(path) as f:
            plans = json.load(f).get("plans", {})
    except (OSError, ValueError):
        return set(wanted)
    missing = set()
    for mnk, ctx in wanted.items():
        e = plans.get(plan_key(*mnk, ctx))
        if e is None:
            missing.add(mnk)
        else:
            GEMM_PLAN[mnk] = tuple(e[:3])
    logger.info("gemm plan: %d of %d entries from %s", len(wanted) - len(missing), len(wanted), path)
    return missing


def save_plan(path: str, report: Dict, ctx_of: Dict[Tuple[int, int], str]) -> None:
    import json
    try:
        with open(path) as f:
            data = json.load(f)
    except (OSError, ValueError):
        data = {}
    plans = data.setdefault("plans", {})
    for (M, N, K), r in report.items():
        plans[plan_key(M, N, K, ctx_of[(N, K)])] = [r["choice"], r["split"], r["cfg"], r["us"], r["blas_us"],
                                                   r.get("hand_us", r["us"])]
    repair_ladder(plans)
    data["device"] = torch.cuda.get_device_name() if torch.cuda.is_available() else "cpu"
    data["note"] = ("ops/autotune.py: [choice, split, cfg, us, hipBLASLt us, best hand-written us] "
                    "per M,N,K,consumer")
    with open(path, "w") as f:
        json.dump(data, f, indent=0, sort_keys=True)


def load_section(path: str, section: str) -> Dict[str, list]:
    """Entries of another persisted engine-start decision (`lm_head`, `decode_swiglu`) in the plan file."""
    import json
    try:
        with open(path) as f:
            return dict(json.load(f).get(section, {}))
    except (OSError, ValueError):
        return {}


def save_section(path: str, section: str, entries: Dict[str, list]) -> None:
    import json
    try:
        with open(path) as f:
            data = json.load(f)
    except (OSError, ValueError):
        data = {}
    data.setdefault(section, {}).update(entries)
    with open(path, "w") as f:
        json.dump(data, f, indent=0, sort_keys=True)


def plan_mode() -> Tuple[str, str]:
    """(KA_GEMM_PLAN, plan file): `file` (load, tune what is missing), `tune` or `write`."""
    return os.environ.get("KA_GEMM_PLAN", "file"), os.environ.get("KA_GEMM_PLAN_FILE", DEFAULT_PLAN_FILE)


# A hipBLASLt plan is kept only when it beats the best hand-written candidate by more than this
# fraction: within it the hand-written kernel is taken (no vendor kernel in the captured decode
# graphs, and one library's heuristics fewer between boxes).  KA_PLAN_BLAS_MARGIN=0: fastest wins.
# 0.15: every default decode bucket (HIPGRAPH_BUCKETS 1-256) is hand-written at 3 % already; the
# margin moves the optional buckets 160 / 320 / 384 off hipBLASLt for at most 15 % on one GEMM
# (profiles/r4/plan_big/: "hand_us" records the hand-written time next to hipBLASLt's).
BLAS_MARGIN = float(os.environ.get("KA_PLAN_BLAS_MARGIN", "0.15"))


def _tunableop_begin() -> bool:
    """KA_TUNABLEOP=1: let torch TunableOp search hipBLASLt/rocBLAS solutions for the decode shapes
    while we time them (results cached in KA_TUNABLEOP_FILE); tuning is switched off afterwards so
    prefill's ragged shapes never trigger online tuning during serving."""
    import os
    if os.environ.get("KA_TUNABLEOP", "1") != "1":
        return False
    tun = torch.cuda.tunable
    tun.enable(True)
    fname = os.environ.get("KA_TUNABLEOP_FILE", DEFAULT_TUNABLEOP_FILE)
    if fname:
        tun.set_filename(fname)
        if os.path.exists(fname):
            tun.read_file(fname)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(int(os.environ.get("KA_TUNABLEOP_MS", "60")))
    # time candidates with operands rotated through a buffer larger than the 256 MB MALL, so the
    # choice reflects decode conditions (every layer's weights stream cold from HBM)
    tun.set_rotating_buffer_size(int(os.environ.get("KA_TUNABLEOP_ROTATING_MB", "1024")))
    return True


def _tunableop_end() -> None:
    """Stop tuning.  Results are written back only with KA_TUNABLEOP_WRITE=1 (to KA_TUNABLEOP_FILE):
    with one engine process per GPU, eight processes would otherwise rewrite the same file while
    others read it at start-up."""
    import os
    tun = torch.cuda.tunable
    tun.tuning_enable(False)
    if os.environ.get("KA_TUNABLEOP_WRITE", "0") == "1":
        try:
            tun.write_file()
        except Exception:  # pragma: no cover
            pass


@torch.inference_mode()
def tune_linear(groups: Dict[Tuple[int, int], List[torch.Tensor]], Ms: Sequence[int],
                norm_fed: Sequence[Tuple[int, int]] = (), bf16_partials: bool = True,
                consumers: Optional[Dict[Tuple[int, int], Tuple[Callable, bool]]] = None) -> Dict:
    """groups: (N, K) -> list of weight tensors of that shape (one per layer).
    norm_fed: shapes whose output goes straight into the fused residual + RMSNorm (o_proj and down
    at TP = 1).  Their candidates are timed together with that norm, split-K ones with the
    reduction deferred into it (as the model runs them), so a split plan is not charged for a
    reduce kernel the model never launches.
    consumers: (N, K) -> (fn(out, M), bf16) for other fused consumers — QKV -> the fused RoPE +
    KV-append + decode attention, which reduces split-K partials (bf16 ones when `bf16`) in its
    prologue: candidates are timed with that kernel, in the form the model runs them."""
    tunable = _tunableop_begin()
    try:
        return _tune(groups, Ms, set(norm_fed), bf16_partials, consumers or {})
    finally:
        if tunable:
            _tunableop_end()


# csrc/gemm_mfma.hip configurations timed for decode M (profiles/r2/autotune_*.txt: 128 x 64 rings
# win at M = 32-64, 128 x 128 at 96-256, 128 x 256 / 256 x 128 / 4-stage 128 x 128 at 192-256; the
# configurations that never won — one wave per SIMD, 32-deep rings, 64-row weight tiles, the 4-phase
# ping-pong — were removed: profiles/r2/gemm_sweep_v*.txt)
GM_TUNE_CFGS = (2, 3, 4, 5, 6, 8, 12, 19)


def gm_candidates(M: int, N: int, K: int, cfgs: Sequence[int] = ()):
    """(cfg, split) pairs of csrc/gemm_mfma.hip worth timing: tiles no taller than twice M and a
    grid of ~96-1024 workgroups on 256 CUs."""
    out = []
    if K % 64 or N % 16:   # rows past M re-read distinct rows r % M (never one clamped row: profiles/r5/gemm_big_clamp/)
        return out
    for cfg in cfgs or GM_TUNE_CFGS:
        bn, bm = gm_shape(cfg)
        if bm > 2 * M and bm > 64:
            continue
        tiles = ((N + bn - 1) // bn) * ((M + bm - 1) // bm)
        for split in (1, 2, 4, 8):
            if K % (64 * split) or K // split < 256:
                continue
            if split > 1 and tiles * split > 1024:
                continue
            if tiles * split < 96 and split < 8:
                continue
            out.append((cfg, split))
    return out


def _plan_runs(plan, M: int, K: int) -> bool:
    """A plan chosen for a larger bucket can run M rows (the row GEMV only up to its staged rows)."""
    return plan[0] != "rows" or rows_ok(M, K, plan[1])


def _run_plan(plan, x, w, fed: bool, bf16: bool):
    kind, split, cfg = plan
    if kind == "gm":
        return linear_gm(x, w, cfg, split, defer_reduce=fed, bf16_partials=bf16)
    if kind == "rows":
        return linear_rows(x, w, split, cfg, defer_reduce=fed)
    if kind == "big":
        return linear_big(x, w)
    return linear(x, w, split=split, defer_reduce=fed)   # skinny


def ladder_anomalies(plans: Dict[str, list], tol: float = 0.03) -> List[Tuple[str, str, float, float]]:
    """Persisted plan entries ({"M,N,K,ctx": [choice, split, cfg, us, ...]}) whose planned time exceeds
    the time planned for the next larger bucket of the same (N, K, consumer) by more than `tol`:
    [(key, larger key, us, larger us)].  The larger bucket's plan runs the smaller M too, so such an
    entry is a tuning miss (the ladder rule in _tune prevents it for new plans)."""
    by_shape: Dict[Tuple[int, int, str], List[Tuple[int, float, str]]] = {}
    for key, e in plans.items():
        m, n, k, ctx = key.split(",", 3)
        by_shape.setdefault((int(n), int(k), ctx), []).append((int(m), float(e[3]), key))
    out = []
    for rows in by_shape.values():
        rows.sort()
        for (m, us, key), (m2, us2, key2) in zip(rows, rows[1:]):
            if us > us2 * (1.0 + tol):
                out.append((key, key2, us, us2))
    return out


def repair_ladder(plans: Dict[str, list], tol: float = 0.03) -> List[str]:
    """Apply the ladder rule across runs: an entry tuned in an earlier run (another bucket subset, a
    PLAN_BUCKETS re-tune) whose time exceeds the next larger bucket's takes that bucket's plan (its
    kernels run the smaller M, in at most the larger bucket's time, which is recorded as an upper
    bound).  Largest bucket first, so a repaired plan can repair the next smaller one.  Returns the
    keys changed."""
    by_shape: Dict[Tuple[int, int, str], List[Tuple[int, str]]] = {}
    for key in plans:
        m, n, k, ctx = key.split(",", 3)
        by_shape.setdefault((int(n), int(k), ctx), []).append((int(m), key))
    changed = []
    for (n, k, ctx), rows in by_shape.items():
        rows.sort(reverse=True)
        for (m2, key2), (m, key) in zip(rows, rows[1:]):
            big, small = plans[key2], plans[key]
            plan = (big[0], big[1], big[2])
            if float(small[3]) > float(big[3]) * (1.0 + tol) and big[0] != "blas" and _plan_runs(plan, m, k):
                plans[key] = [big[0], big[1], big[2], float(big[3])] + list(small[4:])
                changed.append(key)
    return changed


def _tune(groups, Ms, norm_fed=frozenset(), bf16_partials: bool = True, consumers=None) -> Dict:
    report = {}
    consumers = consumers or {}
    for (N, K), ws in groups.items():
        ws = ws[: max(2, min(len(ws), 16))]
        cons = consumers.get((N, K))
        fed = (N, K) in norm_fed or cons is not None    # partials handed to a fused consumer
        bf16 = cons[1] if cons is not None else bf16_partials
        dev, dt = ws[0].device, ws[0].dtype
        g = torch.ones(N, device=dev, dtype=dt)
        # largest bucket first: each bucket also times the plan chosen for the next larger one (that
        # plan's kernels take any M up to its bucket), so a small bucket never keeps a plan slower
        # than the one a larger bucket runs (the ladder rule; B = 4 took 47.8 us for the Llama-3-8B
        # gate_up on the skinny kernel where B = 8's ring kernel took 42.2)
        larger = None
        for M in sorted(set(int(m) for m in Ms if m <= TILE_MAX_M), reverse=True):
            x = torch.randn(M, K, device=dev, dtype=dt)
            res = torch.zeros(M, N, device=dev, dtype=dt)
            if cons is not None:
                norm = (lambda h, M=M, fn=cons[0]: fn(h, M))
            elif fed:
                norm = (lambda h: rmsnorm(h, g, 1e-5, residual=res))
            else:
                norm = (lambda h: h)
            GEMM_PLAN.pop((M, N, K), None)
            t_blas = _time(lambda w: norm(torch.nn.functional.linear(x, w)), ws)
            best = ("blas", 0, 0, float("inf"))   # the best hand-written candidate
            if M <= SKINNY_MAX_M and K % 64 == 0 and N % 4 == 0:
                cands = sorted({skinny_split(M, N, K, t) for t in (256, 512, 1024, 2048)})
                for sp in cands:
                    t = _time(lambda w: norm(linear(x, w, split=sp, defer_reduce=fed)), ws)
                    if t < best[3]:
                        best = ("skinny", sp, 0, t)
            for sp in (1, 2, 4):   # row-streaming GEMV (M <= 4): split x rows per wave
                if not rows_ok(M, K, sp):
                    continue
                for rw in (1, 2, 4, 8):
                    t = _time(lambda w: norm(linear_rows(x, w, sp, rw, defer_reduce=fed)), ws)
                    if t < best[3]:
                        best = ("rows", sp, rw, t)
            for cfg, sp in gm_candidates(M, N, K):
                t = _time(lambda w: norm(linear_gm(x, w, cfg, sp, defer_reduce=fed, bf16_partials=bf16)), ws)
                if t < best[3]:
                    best = ("gm", sp, cfg, t)
            if M >= BIG_PLAN_MIN_M and big_gemm_ok(x, ws[0]):   # 256 x 256 tiles, one wave per SIMD
                t = _time(lambda w: norm(linear_big(x, w)), ws)
                if t < best[3]:
                    best = ("big", 0, 0, t)
            if larger is not None and larger[0] != "blas" and _plan_runs(larger, M, K):
                t = _time(lambda w: norm(_run_plan(larger, x, w, fed, bf16)), ws)
                if t < best[3]:
                    best = (larger[0], larger[1], larger[2], t)
            hand_us = best[3]   # the fastest hand-written candidate, reported whichever wins
            if best[3] > t_blas * (1.0 + BLAS_MARGIN):
                best = ("blas", 0, 0, t_blas)
            GEMM_PLAN[(M, N, K)] = (best[0], best[1], best[2])
            larger = GEMM_PLAN[(M, N, K)]
            report[(M, N, K)] = {"choice": best[0], "split": best[1], "cfg": best[2], "us": round(best[3], 1),
                                 "blas_us": round(t_blas, 1), "hand_us": round(hand_us, 1),
                                 "with": "attention" if cons is not None else "norm" if fed else None}
    logger.info("gemm plan: %s", report)
    return report
