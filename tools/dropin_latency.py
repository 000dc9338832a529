#!/usr/bin/env python3
"""Where a single drop-in query's kernel time goes (diagnostic): one EVM-shaped conjunction x
M cached models through the verdict kernel, timed (HIP events) on the first launch after the
model upload and on repeats, whole and split into its conjuncts.  usage: dropin_latency.py [M]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mythril_amd import support as sp  # noqa: E402
from mythril_amd.evaluator import Evaluator  # noqa: E402
from mythril_amd.lower import IncrementalLowering  # noqa: E402
from mythril_amd.synth_evm import dropin_workload  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 16
ev = Evaluator(0)
exprs, recs, _ = dropin_workload(1, M, seed=7, query_seed=1)
inc = IncrementalLowering()
db, ok = inc.lower(exprs)
mb = inc.serialize(recs)
out = {}
for name, batch in (("whole", db), ("split", sp.split_conjuncts(db, 1 << 20)[0])):
    for asm in (2, 1, 0):   # 2: assembly with MQ_OPT_LATENCY_WAVES (one tape per G wave)
        ev.set_option(ev.OPT_USE_ASM, 1 if asm else 0)
        ev.set_option(ev.OPT_LATENCY_WAVES, 1 << 20 if asm == 2 else 0)
        ev.upload_models(mb)
        ct = ev.compile(batch)
        ev.time_kernels(True)
        ts = []
        for rep in range(4):
            ev.verdicts(ct)
            ts.append(round(sum(ev.kernel_times(reset=True)) * 1e3, 1))
        ev.time_kernels(False)
        info = {"asm_cpp_wide": ct.split(), "p_g_live": ct.asm_split()}
        ct.free()
        out[f"{name}_asm{asm}"] = {"tapes": batch.n_tapes, "kernel_us": ts, "info": info}
ev.set_option(ev.OPT_LATENCY_WAVES, 0)
ev.set_option(ev.OPT_USE_ASM, 0)
# each conjunct alone on the HIP C++ kernel: nodes, op histogram, kernel time
from collections import Counter  # noqa: E402
from mythril_amd.tape import Op  # noqa: E402
tb = sp.split_conjuncts(db, 1 << 20)[0].to_tapes()
ev.upload_models(mb)
rows = []
for t in range(tb.n_tapes):
    sub = tb.subset([t])
    ct = ev.compile(sub)
    ev.time_kernels(True)
    ts = []
    for rep in range(3):
        ev.verdicts(ct)
        ts.append(round(sum(ev.kernel_times(reset=True)) * 1e3, 1))
    ev.time_kernels(False)
    ct.free()
    h = Counter(Op(int(o)).name for o in tb.tape_nodes(t)["op"])
    rows.append({"nodes": int(tb.sizes()[t]), "kernel_us": ts, "ops": dict(h.most_common(8))})
out["per_conjunct_cpp"] = rows
ev.set_option(ev.OPT_USE_ASM, 1)
print(json.dumps(out))
