#!/usr/bin/env python3
"""bench.py's "z3 calls avoided" leg alone (diagnostic):
   python tools/calls_avoided.py [n_forks] [--profile]   (cProfile of the whole leg to stderr)"""
import cProfile
import json
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mythril_amd.evaluator import Evaluator  # noqa: E402

ev = Evaluator(0)
n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 256
if "--profile" in sys.argv:
    pr = cProfile.Profile()
    pr.enable()
res = bench.calls_avoided_leg(ev, n_forks=n)
if "--profile" in sys.argv:
    pr.disable()
    pstats.Stats(pr, stream=sys.stderr).sort_stats("cumulative").print_stats(45)
print(json.dumps(res, indent=1))
