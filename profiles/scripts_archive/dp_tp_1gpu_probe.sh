#!/bin/bash
# DP=2 x TP=2 on one GPU through serve.py (diagnostics): start, one request, full server log.
OUT=${OUT:-gpurun_out/dptp}; mkdir -p $OUT
PORT=18711
env LLM_BACKEND=engine MODEL=llama3-8b-2l DP=2 TP=2 WORKERS=2 ENGINE_DEVICES=cuda:0,cuda:0,cuda:0,cuda:0 \
  KA_TP_BACKEND=gloo HOST=127.0.0.1 PORT=$PORT RATE_LIMIT=1000/minute MAX_NEW_TOKENS=8 HIPGRAPH_BUCKETS=1,2,4 \
  MAX_BATCH=4 KV_CACHE_TOKENS=16384 MAX_MODEL_LEN=512 LOG_LEVEL=INFO ${EXTRA_ENV:-} \
  setsid python -m ai_agent_kubectl_amd.serve > $OUT/serve.log 2>&1 &
SRV=$!
for i in $(seq 1 120); do
  python3 -c "import http.client,sys; c=http.client.HTTPConnection('127.0.0.1',$PORT,timeout=2); c.request('GET','/ready'); sys.exit(0 if c.getresponse().status==200 else 1)" 2>/dev/null && break
  sleep 1
done
python3 - <<PY > $OUT/req.log 2>&1
import http.client, json
for q in ("list all pods in prod", "get nodes"):
    c = http.client.HTTPConnection("127.0.0.1", $PORT, timeout=120)
    c.request("POST", "/kubectl-command", body=json.dumps({"query": q}), headers={"Content-Type": "application/json"})
    r = c.getresponse(); print(r.status, r.read()[:300])
PY
sleep 2
kill -- -$SRV 2>/dev/null; sleep 3; kill -9 -- -$SRV 2>/dev/null
cat $OUT/req.log
