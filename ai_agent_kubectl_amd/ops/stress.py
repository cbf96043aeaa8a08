"""Launch-pattern stress checks for the LDS-DMA kernels (race detection on the device).

LDS-DMA pieces of one wave do not always complete in issue order: in round 5 a counted
`s_waitcnt vmcnt(N)` let stale rows through in up to 25 % of `gemm_big` launches, but only under a
particular launch pattern (each launch right after an unrelated GEMM) and mostly when many lanes of a
piece read the same address (profiles/r5/gemm_big_clamp/).  This module replays that pattern for the
decode ring kernels (csrc/gemm_mfma.hip) at every (configuration, split-K, epilogue) the persisted
decode plan dispatches, with and without the duplicate-address amplifier (ldx = 0: every X row
aliases row 0, so each X piece's 64 lanes read 8 identical rows), and checks every launch whole
against an fp32 reference.  Used by tests/test_kernels_gpu.py (a few launches per combination) and
scripts/gm_plan_stress.py (>= 500 per combination, profiles/r6/lds_dma_safety/).
"""
from __future__ import annotations

import json
import math
import os
from typing import Dict, Iterable, List, Optional, Tuple

import torch

from . import GM_EPI_BF16, GM_EPI_P16, GM_EPI_P32, _p, _stream, check, require

PLAN_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned", "gemm_plan_mi355x.json")
EPI_SWIGLU = 3
# Llama-3-8B decode projections: QKV, O, gate_up, down, LM head (N, K)
SHAPES_8B = ((6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096))


def dispatched_combos(buckets: Iterable[int] = (128, 160, 192, 256, 320, 384, 448, 512),
                      shapes=SHAPES_8B, plan_file: str = PLAN_FILE) -> List[Tuple[int, int, int, int, int, int]]:
    """(M, N, K, cfg, split, epi) of every ring-kernel launch the persisted plan dispatches for these
    decode buckets: GEMM plan entries chosen 'gm' (bf16 partials for a norm / attention consumer, as
    models/llama.py asks for them by default) and the decode SwiGLU section (epilogue 3)."""
    with open(plan_file) as f:
        plan = json.load(f)
    out = set()
    for key, v in plan.get("plans", {}).items():
        M, N, K, consumer = key.split(",")
        M, N, K = int(M), int(N), int(K)
        if M not in buckets or (N, K) not in shapes or v[0] != "gm":
            continue
        split, cfg = int(v[1]), int(v[2])
        if split == 1:
            epi = GM_EPI_BF16
        else:
            epi = GM_EPI_P16 if consumer in ("norm-bf16", "attn-bf16") else GM_EPI_P32
        out.add((M, N, K, cfg, split, epi))
    for key, v in plan.get("decode_swiglu", {}).items():
        M, N, K = (int(t) for t in key.split(","))
        cfg = int(v[0])
        if M in buckets and (N, K) in shapes and 0 < cfg < 100:
            out.add((M, N, K, cfg, 1, EPI_SWIGLU))
    return sorted(out)


class _Case:
    def __init__(self, M, N, K, cfg, split, epi, amplify: bool, device):
        g = torch.Generator(device="cpu").manual_seed(M * 131 + N * 7 + K + cfg)
        self.M, self.N, self.K, self.cfg, self.split, self.epi = M, N, K, cfg, split, epi
        self.ldx = 0 if amplify else K
        rows = 1 if amplify else M
        self.x = torch.randn(rows, K, generator=g).to(device=device, dtype=torch.bfloat16)
        self.w = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(device=device, dtype=torch.bfloat16)
        ref = self.x.float() @ self.w.float().t()
        if amplify:
            ref = ref.expand(M, N)
        if epi == EPI_SWIGLU:   # [gate; up] rows: silu(gate) * up
            I = N // 2
            ref = torch.nn.functional.silu(ref[:, :I]) * ref[:, I:]
        self.ref = ref.contiguous()
        NO = N // 2 if epi == EPI_SWIGLU else N
        self.y = torch.empty((M, NO), dtype=torch.bfloat16, device=device)
        self.p = None
        if epi in (GM_EPI_P16, GM_EPI_P32) or split > 1:
            dt = torch.bfloat16 if epi == GM_EPI_P16 else torch.float32
            self.p = torch.empty((split, M, N), dtype=dt, device=device)

    def launch(self, lib):
        st = _stream()
        if self.epi == EPI_SWIGLU:
            check(lib.ka_gemm_mfma_swiglu(_p(self.y), _p(self.x), _p(self.w), self.M, self.N // 2, self.K, self.ldx,
                                          self.N // 2, self.cfg, st), "gemm_mfma_swiglu")
        elif self.epi == GM_EPI_BF16:
            check(lib.ka_gemm_mfma(_p(self.y), None, _p(self.x), _p(self.w), self.M, self.N, self.K, self.ldx, self.N,
                                   1, self.cfg, GM_EPI_BF16, 0, st), "gemm_mfma")
        elif self.epi == GM_EPI_P16:
            check(lib.ka_gemm_mfma(None, _p(self.p), _p(self.x), _p(self.w), self.M, self.N, self.K, self.ldx, self.N,
                                   self.split, self.cfg, GM_EPI_P16, 0, st), "gemm_mfma")
        else:   # fp32 slabs reduced into y by splitk_reduce
            check(lib.ka_gemm_mfma(_p(self.y), _p(self.p), _p(self.x), _p(self.w), self.M, self.N, self.K, self.ldx,
                                   self.N, self.split, self.cfg, GM_EPI_P32, 0, st), "gemm_mfma")

    def wrong(self) -> torch.Tensor:
        """Device scalar: outputs off the fp32 reference (bf16 rounding of the slabs and the output
        stays far inside 0.03 + 0.02 |ref|; a stale k-step's operands do not)."""
        got = self.p.float().sum(0) if self.epi == GM_EPI_P16 else self.y.float()
        return ((got - self.ref).abs() > 0.03 + 0.02 * self.ref.abs()).sum()


def stress(combos, launches: int, amplify: bool, device="cuda", log=None) -> Dict[tuple, int]:
    """Run `launches` launches of every combination, each right after an unrelated 4096^3 hipBLASLt
    GEMM, and count the launches with any wrong output.  Returns {combo: wrong launches}."""
    lib = require()
    other = torch.randn(4096, 4096, device=device, dtype=torch.bfloat16)
    wo = (torch.randn(4096, 4096, device=device) / 64).to(torch.bfloat16)
    res = {}
    for combo in combos:
        c = _Case(*combo, amplify=amplify, device=device)
        bad = torch.zeros(launches, dtype=torch.int64, device=device)
        for i in range(launches):
            torch.nn.functional.linear(other, wo)
            c.launch(lib)
            bad[i] = c.wrong()
        n = int((bad > 0).sum())
        res[combo] = n
        if log is not None:
            M, N, K, cfg, split, epi = combo
            log(f"M={M} N={N} K={K} cfg={cfg} split={split} epi={epi} amplifier={int(amplify)}: "
                f"{n} wrong of {launches} launches (worst {int(bad.max())} outputs)")
        del c
    return res
