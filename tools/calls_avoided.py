#!/usr/bin/env python3
"""bench.py's "z3 calls avoided" leg alone (diagnostic): python tools/calls_avoided.py [n_forks]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mythril_amd.evaluator import Evaluator  # noqa: E402

ev = Evaluator(0)
print(json.dumps(bench.calls_avoided_leg(ev, n_forks=int(sys.argv[1]) if len(sys.argv) > 1 else 256), indent=1))
