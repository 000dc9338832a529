#!/usr/bin/env python3
"""The drop-in legs of bench.py for a few (N, M) cells only (diagnostic, e.g. under rocprofv3 or
with MQ_CONJ_TAPES / MQ_SPLIT_TAPES set).  usage: dropin_probe.py [s]N:M ...  (s = fork stream)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mythril_amd.evaluator import Evaluator  # noqa: E402

args = sys.argv[1:] or ["1:16", "1:100"]
fresh = [tuple(int(x) for x in a.split(":")) for a in args if not a.startswith("s")]
stream = [tuple(int(x) for x in a[1:].split(":")) for a in args if a.startswith("s")]
ev = Evaluator(0)
for r in bench.dropin_leg(ev, grid=fresh) if fresh else []:
    print(json.dumps(r), flush=True)
for r in bench.dropin_stream_leg(ev, grid=stream) if stream else []:
    print(json.dumps(r), flush=True)
