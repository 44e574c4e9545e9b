"""python tools/run_smoke.py: __graft_entry__.smoke() from the repo root (GPU session scripts)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402

__graft_entry__.smoke()
print('smoke ok')
