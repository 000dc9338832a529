"""Minimal first contact with the assembly interpreter: handler table + one tiny batch."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import numpy as np
from mythril_amd.evaluator import Evaluator
from mythril_amd.synth import c2_workload
import cref

ev = Evaluator(0)
print("asm_ready", ev.asm_ready, flush=True)
tb, mb, exp = c2_workload(8, 300, seed=2)
ev.upload_models(mb)
ct = ev.compile(tb)
print("split", ct.split(), flush=True)
fh = ev.first_hit(ct)
ref, _ = cref.first_hit(tb, mb)
print("asm first_hit", fh.tolist(), "ref", ref.tolist(), flush=True)
v, _ = ev.verdicts(tb)
print("verdict match", bool((v == cref.verdicts(tb, mb)).all()), flush=True)
