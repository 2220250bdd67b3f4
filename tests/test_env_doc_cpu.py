"""docs/ENV.md lists every DNN_* switch of the registry (scripts/env_doc.py --check)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_env_doc_is_current():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "env_doc.py"), "--check"])
    assert r.returncode == 0, "docs/ENV.md is stale: run python scripts/env_doc.py"
