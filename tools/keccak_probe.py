#!/usr/bin/env python3
"""Keccak-f[1600] instruction-mix probe (run under rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES ...):
hashes 2^20 one-block messages (64 B) and 2^20 two-block messages (200 B) with the GPU kernel
(mq_keccak256); sizes in bytes as arguments select one of them per run (one dispatch each).  VALU instructions per lane per block = (SQ_INSTS_VALU / SQ_WAVES) / blocks, the
per-block cost that replaces SURVEY §8(d)'s 8000-op estimate."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mythril_amd.evaluator import Evaluator  # noqa: E402

ev = Evaluator(0)
rng = np.random.default_rng(1)
for nbytes in [int(a) for a in sys.argv[1:]] or (64, 200):
    msgs = rng.integers(0, 256, (1 << 20, nbytes), dtype=np.uint8)
    d = ev.keccak256_array(msgs)
    print(nbytes, d[0].tobytes().hex(), flush=True)
