"""Service-level HTTP benchmark over real TCP (uvicorn server process + httpx load generator).

BASELINE configs measured with the same method SURVEY.md §6 / Appendix A.3 used for the reference:
  plumbing  (config #1): LLM_BACKEND=stub, CPU only — cache-hit, cache-miss, /execute (fake kubectl),
                         /health at concurrency 1 and 32; directly comparable to BASELINE.md's rows.
  mixed     (config #5): the engine (or stub) behind /kubectl-command with a mixed stream — distinct
                         misses, repeated (cached) queries, concurrent /execute through the validator,
                         and a Prometheus scrape every 100 ms.

  python scripts/bench_service.py plumbing
  python scripts/bench_service.py mixed --backend engine --concurrency 128 --seconds 20
Prints one JSON line per scenario.
"""
import argparse
import asyncio
import json
import os
import random
import socket
import statistics
import subprocess
import sys
import tempfile
import time

import httpx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAKE_KUBECTL = """#!/bin/sh
case "$*" in
  "get pods"*) printf 'NAME      READY   STATUS    RESTARTS   AGE\\nnginx-1   1/1     Running   0          5m\\n' ;;
  *) echo "default" ;;
esac
"""


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def start_server(env_over, port, timeout=900):
    bindir = tempfile.mkdtemp()
    with open(os.path.join(bindir, "kubectl"), "w") as f:
        f.write(FAKE_KUBECTL)
    os.chmod(os.path.join(bindir, "kubectl"), 0o755)
    env = dict(os.environ)
    env.update({"PATH": bindir + os.pathsep + env.get("PATH", ""), "PYTHONPATH": ROOT, "LOG_LEVEL": "WARNING",
                "RATE_LIMIT": "100000000/minute", "API_AUTH_KEY": ""})
    env.update(env_over)
    proc = subprocess.Popen([sys.executable, "-m", "ai_agent_kubectl_amd.serve", "--host", "127.0.0.1",
                             "--port", str(port)], env=env, cwd=ROOT)
    t0 = time.time()
    while time.time() - t0 < timeout:
        if proc.poll() is not None:
            raise RuntimeError(f"server exited with {proc.returncode}")
        try:
            if httpx.get(f"http://127.0.0.1:{port}/ready", timeout=2).status_code == 200:
                return proc
        except Exception:
            pass
        time.sleep(0.5)
    proc.kill()
    raise RuntimeError("server did not become ready")


async def closed_loop(client, make_req, conc, total):
    lat = []
    q = iter(range(total))

    async def worker():
        async with httpx.AsyncClient(base_url=str(client.base_url), timeout=60,
                                     limits=httpx.Limits(max_connections=1, max_keepalive_connections=1)) as wc:
            await _loop(wc)

    async def _loop(wc):
        for i in q:
            method, path, body = make_req(i)
            t0 = time.perf_counter()
            r = await wc.request(method, path, json=body)
            lat.append(time.perf_counter() - t0)
            if r.status_code != 200:
                raise RuntimeError(f"{path}: {r.status_code} {r.text[:200]}")

    t0 = time.perf_counter()
    await asyncio.gather(*[worker() for _ in range(conc)])
    el = time.perf_counter() - t0
    lat.sort()
    return {"rps": round(total / el, 1), "p50_ms": round(statistics.median(lat) * 1e3, 2),
            "p99_ms": round(lat[int(0.99 * (len(lat) - 1))] * 1e3, 2), "n": total}


async def plumbing(base):
    out = []
    limits = httpx.Limits(max_connections=64, max_keepalive_connections=64)
    async with httpx.AsyncClient(base_url=base, limits=limits, timeout=60) as c:
        await c.post("/kubectl-command", json={"query": "list all pods"})
        scen = {
            "cache_hit": lambda i: ("POST", "/kubectl-command", {"query": "list all pods"}),
            "cache_miss": lambda i: ("POST", "/kubectl-command", {"query": f"get pods in namespace ns{i}"}),
            "execute": lambda i: ("POST", "/execute", {"execute": "kubectl get pods"}),
            "health": lambda i: ("GET", "/health", None),
        }
        for conc in (1, 32):
            for name, fn in scen.items():
                n = 400 if conc == 1 else 2000
                r = await closed_loop(c, fn, conc, n)
                r.update(scenario=name, concurrency=conc)
                out.append(r)
                print(json.dumps(r), flush=True)
    return out


async def mixed(base, conc, seconds):
    rng = random.Random(0)
    stats = {"miss": [], "hit": [], "execute": [], "metrics": []}
    hot = [f"list pods in namespace hot{i}" for i in range(50)]
    limits = httpx.Limits(max_connections=conc + 4, max_keepalive_connections=conc + 4)
    counter = [0]
    async with httpx.AsyncClient(base_url=base, limits=limits, timeout=600) as c:
        await asyncio.gather(*[c.post("/kubectl-command", json={"query": q}) for q in hot])  # warm the cache
        stop = time.perf_counter() + seconds

        async def worker(wid):
            # one single-connection client per worker: httpx's shared pool degrades badly with
            # dozens of concurrent requests and would measure the load generator, not the server
            async with httpx.AsyncClient(base_url=base, timeout=600,
                                         limits=httpx.Limits(max_connections=1, max_keepalive_connections=1)) as wc:
                await _worker_loop(wc, wid)

        async def _worker_loop(c, wid):
            while time.perf_counter() < stop:
                x = rng.random()
                counter[0] += 1
                if x < 0.7:
                    kind, m, p, b = "miss", "POST", "/kubectl-command", {"query": f"team-{wid}-{counter[0]}: list all pods"}
                elif x < 0.9:
                    kind, m, p, b = "hit", "POST", "/kubectl-command", {"query": rng.choice(hot)}
                else:
                    kind, m, p, b = "execute", "POST", "/execute", {"execute": "kubectl get pods -n prod"}
                t0 = time.perf_counter()
                r = await c.request(m, p, json=b)
                stats[kind].append(time.perf_counter() - t0)
                assert r.status_code == 200, r.text

        async def scraper():
            while time.perf_counter() < stop:
                t0 = time.perf_counter()
                r = await c.get("/metrics")
                stats["metrics"].append(time.perf_counter() - t0)
                assert r.status_code == 200
                await asyncio.sleep(0.1)

        t0 = time.perf_counter()
        await asyncio.gather(scraper(), *[worker(i) for i in range(conc)])
        el = time.perf_counter() - t0
        m = (await c.get("/metrics")).text
        lag = [l for l in m.splitlines() if l.startswith("event_loop_lag_seconds_")]
        srv = {}
        for l in m.splitlines():   # server-side mean latency per handler (Prometheus histogram)
            if l.startswith("http_request_duration_seconds_sum") or l.startswith("http_request_duration_seconds_count"):
                h = l.split('handler="')[1].split('"')[0]
                srv.setdefault(h, {})["sum" if "_sum" in l else "count"] = float(l.split()[-1])
    res = {"scenario": "mixed", "concurrency": conc, "seconds": round(el, 1),
           "total_rps": round(sum(len(v) for k, v in stats.items() if k != "metrics") / el, 1)}
    for k, v in stats.items():
        if v:
            res[f"{k}_n"] = len(v)
            res[f"{k}_p50_ms"] = round(statistics.median(v) * 1e3, 2)
    res["cache_hit_ratio"] = round(_metric(m, "kubectl_agent_cache_hits_total") /
                                   max(1.0, _metric(m, "kubectl_agent_cache_hits_total") +
                                       _metric(m, "kubectl_agent_cache_misses_total")), 3)
    res["server_mean_ms"] = {h: round(v["sum"] / max(1, v["count"]) * 1e3, 2) for h, v in srv.items() if "count" in v}
    res["loop_lag"] = {l.split("{")[1].split("}")[0] if "{" in l else l.split()[0]: float(l.split()[-1])
                       for l in lag}
    print(json.dumps(res), flush=True)
    return res


def _metric(text, name):
    for l in text.splitlines():
        if l.startswith(name + " "):
            return float(l.split()[-1])
    return 0.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["plumbing", "mixed"])
    ap.add_argument("--backend", default="stub")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--seconds", type=float, default=20)
    a = ap.parse_args()
    port = _port()
    env = {"LLM_BACKEND": "stub" if a.mode == "plumbing" else a.backend, "MODEL": a.model,
           "MAX_NEW_TOKENS": "16", "MAX_BATCH": str(max(64, a.concurrency)),
           # mixed: keep the hot set cached (the reference default of 100 entries would be
           # flushed by the distinct misses and turn every "hit" into a miss)
           "CACHE_MAXSIZE": "100" if a.mode == "plumbing" else "10000"}
    proc = start_server(env, port)
    try:
        base = f"http://127.0.0.1:{port}"
        asyncio.run(plumbing(base) if a.mode == "plumbing" else mixed(base, a.concurrency, a.seconds))
    finally:
        proc.terminate()
        proc.wait(timeout=60)


if __name__ == "__main__":
    main()
