"""The driver's round-end smoke check, runnable as a lease step:
python tools/smoke.py  (== __graft_entry__.smoke() on cuda:0)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__  # noqa: E402

__graft_entry__.smoke()
print("smoke ok", flush=True)
