"""Tune the decode GEMM plan of a model on this GPU for every batch bucket up to 512 and merge it into
ai_agent_kubectl_amd/ops/tuned/gemm_plan_mi355x.json (KA_GEMM_PLAN=write), which engines then load at
start instead of re-timing candidates (ops/autotune.py: persisted plans).

    python scripts/write_gemm_plan.py [model ...]        (default llama3-8b)
"""
import os
import sys

os.environ["KA_GEMM_PLAN"] = "write"
os.environ.setdefault("KA_AUTOTUNE_ROUNDS", "5")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import shutil  # noqa: E402
import threading  # noqa: E402
import time  # noqa: E402

import torch  # noqa: E402

from ai_agent_kubectl_amd.engine.builder import EngineOptions, build_engine  # noqa: E402
from ai_agent_kubectl_amd.ops.autotune import DEFAULT_PLAN_FILE  # noqa: E402


def _heartbeat():   # big models build and tune silently for minutes
    t0 = time.time()
    while True:
        time.sleep(30)
        print(f"... {time.time() - t0:.0f} s", flush=True)


threading.Thread(target=_heartbeat, daemon=True).start()
COPY_TO = os.environ.get("PLAN_COPY_TO")   # e.g. gpurun_out/tuned: a copy after every model

BUCKETS = (1, 2, 4, 8, 16, 32, 48, 64, 96, 128, 160, 192, 256, 320, 384, 448, 512)
if os.environ.get("PLAN_BUCKETS"):   # re-tune (and re-write) only these buckets, e.g. "1,2,4"
    BUCKETS = tuple(int(b) for b in os.environ["PLAN_BUCKETS"].split(","))
# "prefill": re-tune only the prefill section (after a gemm_big change); "epilogues": only the lm_head and
# decode_swiglu sections (the fused gemm_big / ring-kernel epilogues against the unfused plan); "decode":
# only the decode GEMM plan (after a change to a consumer the plan times with, e.g. the norm)
ONLY = os.environ.get("PLAN_ONLY", "")
for model in sys.argv[1:] or ["llama3-8b"]:
    eng = build_engine(EngineOptions(model=model, device="cuda", max_batch=max(BUCKETS), graph_buckets=BUCKETS,
                                     kv_cache_tokens=65536, max_model_len=512))
    rep = {}
    if ONLY not in ("prefill", "epilogues"):
        rep = eng.runner.autotune()
        print(model, len(rep), "plan entries", flush=True)
    if ONLY == "epilogues":   # the unfused side of each comparison runs the persisted GEMM plan
        os.environ["KA_GEMM_PLAN"] = "file"
        print(model, "GEMM plan:", eng.runner.autotune(), flush=True)
        os.environ["KA_GEMM_PLAN"] = "write"
    if ONLY not in ("prefill", "decode"):
        # the engine-start decisions persisted next to the plan (sections lm_head / decode_swiglu)
        print("lm_head:", eng.runner.tune_lm_head(), flush=True)
        print("decode_swiglu:", eng.runner.tune_swiglu(), flush=True)
    if ONLY not in ("epilogues", "decode"):
        print("prefill:", eng.runner.tune_prefill(), flush=True)
    if COPY_TO:
        os.makedirs(COPY_TO, exist_ok=True)
        shutil.copy(DEFAULT_PLAN_FILE, COPY_TO)
    for k in sorted(rep):
        print(" ", k, rep[k], flush=True)
    del eng
    torch.cuda.empty_cache()
