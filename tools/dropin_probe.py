#!/usr/bin/env python3
"""The drop-in leg of bench.py for a few (N, M) cells only (diagnostic, e.g. under rocprofv3
--kernel-trace to see which kernels a single query launches).  usage: dropin_probe.py N:M ..."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mythril_amd.evaluator import Evaluator  # noqa: E402

cells = [tuple(int(x) for x in a.split(":")) for a in sys.argv[1:]] or [(1, 16), (1, 100)]
ev = Evaluator(0)
for r in bench.dropin_leg(ev, grid=cells):
    print(json.dumps(r), flush=True)
