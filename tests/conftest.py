import os
import sys
import warnings

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

warnings.filterwarnings("ignore", message=".*httpx2.*")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs under gpurun / the driver's GPU tier)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


FAKE_KUBECTL = r"""#!/bin/sh
# Test double for kubectl (SURVEY.md §4.2): table / raw / error / sleep behaviours.
case "$*" in
  "get pods"*) printf 'NAME      READY   STATUS    RESTARTS   AGE\nnginx-1   1/1     Running   0          5m\nredis-0   1/1     Running   2          1h\n' ;;
  "get ns"*) echo "default" ;;
  "get foo"*) echo 'error: the server doesn'"'"'t have a resource type "foo"' >&2; exit 1 ;;
  "sleep"*) sleep 10 ;;
  *) echo "ok $*" ;;
esac
"""


@pytest.fixture
def fake_kubectl(tmp_path, monkeypatch):
    bindir = tmp_path / "bin"
    bindir.mkdir()
    p = bindir / "kubectl"
    p.write_text(FAKE_KUBECTL)
    p.chmod(0o755)
    monkeypatch.setenv("PATH", str(bindir) + os.pathsep + os.environ.get("PATH", ""))
    return p


@pytest.fixture
def no_kubectl(tmp_path, monkeypatch):
    monkeypatch.setenv("PATH", str(tmp_path))
