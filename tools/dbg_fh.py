"""Debug: golden first-hit vs verdict disagreement, per path (asm on/off, early exit on/off)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
from golden_util import check_tape, load
from mythril_amd.evaluator import Evaluator, compile_info
from mythril_amd.models import ModelBatch
from mythril_amd.tape import TapeBatch

entries = load("shift_vectors.json") + load("vmtests_kats.json")
tapes = []
for e in entries:
    exp = int(e["expected"], 16)
    tapes.append(check_tape(e, exp))
    tapes.append(check_tape(e, exp, negate=True))
tb = TapeBatch(tapes)
ev = Evaluator(0)
ev.upload_models(ModelBatch([8], np.zeros((1, 1), np.uint32)))
print("split", ev.compile(tb).split(), flush=True)
for rep in range(4):
  for asm in (1, 0):
      for ee in (1, 0):
          ev.use_asm(bool(asm)); ev.set_option(2, ee)
          v, _ = ev.verdicts(tb)
          fh = ev.first_hit(tb)
          bad = [i for i in range(len(entries)) if (fh[2 * i] == 0) != bool(v[2 * i, 0])]
          badn = [i for i in range(len(entries)) if fh[2 * i + 1] != -1]
          print(f"asm={asm} ee={ee} verdict_ok={int(v[0::2,0].sum())}/{len(entries)} fh_pos_bad={len(bad)} fh_neg_bad={len(badn)}", flush=True)
          for i in bad[:8]:
              ci = compile_info(tb, 2 * i)
              print("   ", i, entries[i]["name"], "fh", fh[2 * i], "L", ci.limbs, "depth", ci.depth, "temps", ci.n_temps, "words", ci.prog_words, flush=True)
