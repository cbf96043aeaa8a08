"""Module-level ASGI application: `uvicorn ai_agent_kubectl_amd.asgi:app` (the reference's
`uvicorn app:app`, `/root/reference/Dockerfile:33`, `app.py:400`).

The app is built at import from the environment / `./.env` exactly like the reference builds its
chain at import (`app.py:106-138`).  With `uvicorn ... --workers N` every worker imports this
module: set `SHARED_STATE=<name>` so their caches and rate limits are one (shared_state.py; the
first worker creates the segment).  For engine replicas shared by several workers use
`WORKERS=N python -m ai_agent_kubectl_amd.serve` (parallel/workers.py), which also owns replica
lifetimes.
"""
from .api import create_app
from .config import Settings

settings = Settings.from_env()
app = create_app(settings)
