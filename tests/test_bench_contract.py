"""bench.py driver contract (task spec): `python bench.py` and the torchrun form print exactly one
JSON line from rank 0 with the required keys; `value` is the whole-job aggregate and `n_gpus` /
`parallelism` follow WORLD_SIZE.  Run on the CPU with the tiny model and the engine process on
`BENCH_DEVICE=cpu`; the GPU numbers come from the same code path on MI355X (profiles/)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(args, world, launcher="torchrun"):
    env = dict(os.environ, BENCH_DEVICE="cpu", PYTHONUNBUFFERED="1")
    bench = [os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", "1", "--warmup", "1",
             "--concurrency", "4", "--model", "tiny-llama"] + list(args)
    if world == 1 or launcher == "self":
        cmd = [sys.executable] + bench     # --gpus N > 1: bench.py spawns its N ranks itself
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", f"--master-port={_free_port()}"] + bench
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("world,launcher", [(1, "self"), (2, "torchrun"), (2, "self")])
def test_bench_prints_one_json_line(world, launcher):
    out = _run([], world, launcher)
    assert KEYS <= set(out)
    # default: the headline over TCP through ONE server (DP = world replicas, one port), then the
    # in-process ASGI transport and an ASGI pass with the prefix cache off, in detail
    d = out["detail"]
    assert d["transport"] == "tcp" and f"DP={world} replicas" in d["topology"]
    assert out["tcp_value"] == out["value"] and out["asgi_value"] == d["asgi"]["value"] > 0
    assert d["prefix_cache_off"]["value"] > 0 and d["prefix_cache_off"]["prefix_cache_hit_rate"] == 0
    assert d["tcp_vs_asgi"] > 0
    assert out["n_gpus"] == world and out["steps"] == 1 and out["warmup"] == 1
    assert out["higher_is_better"] is True and out["scaling"] == "weak" and out["unit"] == "req/s"
    assert out["value"] > 0 and out["ms_per_step"] > 0
    assert out["config"]["parallelism"] == f"dp{world}" and out["config"]["global_batch"] == 4 * world
    # value = total timed requests over the slowest rank's elapsed time
    assert out["value"] == pytest.approx(4 * world / (out["ms_per_step"] / 1e3), rel=0.02)


def test_bench_gpus_must_match_world_size():
    """Under torchrun, --gpus N with a different WORLD_SIZE is refused (never silently measures
    fewer GPUs)."""
    env = dict(os.environ, BENCH_DEVICE="cpu", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=120, env=env, cwd="/tmp")
    assert r.returncode != 0 and "does not match WORLD_SIZE" in r.stderr


def test_bench_tcp_one_server_dp2_shared_cache():
    """--gpus 2 --transport tcp --mix: ONE server with DP=2 engine replicas and 4 API workers on one
    port (the deployed topology, parallel/workers.py); the hit class's queries were inserted
    through one worker, and every hit answered by any worker must say from_cache=true (bench.py
    reply_ok), so the cache is shared across workers."""
    out = _run(["--transport", "tcp", "--mix", "--hit-frac", "0.5", "--exec-frac", "0.1"], 2)
    d = out["detail"]
    assert "DP=2 replicas, 4 API workers" in d["topology"] and out["n_gpus"] == 2
    assert d["mix"]["hit"]["n"] > 0 and d["mix"]["miss"]["n"] > 0
    assert out["value"] == pytest.approx(8 / (out["ms_per_step"] / 1e3), rel=0.02)


def test_bench_tcp_transport():
    """--transport tcp: the production server (2 API workers on one port, shared cache/limiter) over
    real sockets, 2 client processes."""
    out = _run(["--transport", "tcp", "--api-workers", "2", "--client-procs", "2"], 1)
    assert out["detail"]["transport"] == "tcp" and out["detail"]["api_workers"] == 2
    assert out["value"] == pytest.approx(4 / (out["ms_per_step"] / 1e3), rel=0.02)
    assert out["config"]["seq_len"] > 16
    # engine view through the server's Prometheus histograms (llm_step_seconds, llm_queue_wait_seconds)
    d = out["detail"]
    assert d["engine_stats_from"] == "/metrics" and d["decode_steps"] > 0 and d["prefill_steps"] > 0
    assert d["decode_ms_per_step"] > 0 and d["queue_wait_ms_mean"] >= 0


def test_bench_open_loop_mixed_stream():
    """--load open --mix: Poisson arrivals of hits, misses and /execute calls plus /metrics scrapes
    (BASELINE config #5); per-class latencies are reported."""
    out = _run(["--load", "open", "--rate", "40", "--mix"], 1)
    mix = out["detail"]["mix"]
    assert out["detail"]["load"].startswith("open")
    assert sum(v["n"] for k, v in mix.items() if k != "scrape") >= 4


def test_bench_tp_replicas_over_tcp():
    """--gpus 2 --tp 2 (BASELINE configs #3 / #4 path): ONE server with DP = 1 replica that is a TP = 2
    group (its rank 0 spawns the TP worker rank; gloo on the CPU), both ranks' clients talk to it over
    TCP; `parallelism` says dp1tp2 and the value is still the whole-job aggregate."""
    out = _run(["--tp", "2"], 2)
    d = out["detail"]
    assert d["transport"] == "tcp" and "DP=1 replicas of TP=2" in d["topology"]
    assert out["config"]["parallelism"] == "dp1tp2" and out["n_gpus"] == 2
    assert out["config"]["global_batch"] == 8
    assert out["value"] == pytest.approx(8 / (out["ms_per_step"] / 1e3), rel=0.02)
    assert d["decode_steps"] > 0 and d["prefill_steps"] > 0


def test_bench_parallelism_labels():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.parallelism(bench.parse_args(["--gpus", "8", "--tp", "8", "--model", "llama3-70b"]), 8) == "dp1tp8"
    assert bench.parallelism(bench.parse_args(["--gpus", "8", "--tp", "8", "--model", "mixtral-8x7b"]), 8) == "dp1ep8"
    assert bench.parallelism(bench.parse_args(["--gpus", "8", "--tp", "2"]), 8) == "dp4tp2"
    assert bench.parallelism(bench.parse_args(["--gpus", "4"]), 4) == "dp4"
    a = bench.parse_args(["--gpus", "4", "--tp", "2", "--transport", "both"])
    assert a.transport == "tcp"
    with pytest.raises(SystemExit):
        bench.parse_args(["--gpus", "4", "--tp", "3"])
