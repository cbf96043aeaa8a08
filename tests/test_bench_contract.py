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


def _run(args, world):
    env = dict(os.environ, BENCH_DEVICE="cpu", PYTHONUNBUFFERED="1")
    bench = [os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", "1", "--warmup", "1",
             "--concurrency", "4", "--model", "tiny-llama"]
    if world == 1:
        cmd = [sys.executable] + bench
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", f"--master-port={_free_port()}"] + bench
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("world", [1, 2])
def test_bench_prints_one_json_line(world):
    out = _run([], world)
    assert KEYS <= set(out)
    assert out["n_gpus"] == world and out["steps"] == 1 and out["warmup"] == 1
    assert out["higher_is_better"] is True and out["scaling"] == "weak" and out["unit"] == "req/s"
    assert out["value"] > 0 and out["ms_per_step"] > 0
    assert out["config"]["parallelism"] == f"dp{world}" and out["config"]["global_batch"] == 4 * world
    # value = total timed requests over the slowest rank's elapsed time
    assert out["value"] == pytest.approx(4 * world / (out["ms_per_step"] / 1e3), rel=0.02)
