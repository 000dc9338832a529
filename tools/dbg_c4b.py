"""Debug helper: re-generate C4 tape t and report the conjuncts its witness violates."""
import sys
sys.path.insert(0, "/root/repo/oracle"); sys.path.insert(0, "/root/repo/tests"); sys.path.insert(0, "/root/repo")
import numpy as np
import cref
from mythril_amd import synth_evm as E
from mythril_amd.smt_model import Model
from oracle_engine import eval_under

def hm(arr):
    return np.array([np.frombuffer(cref.keccak256(bytes(r)), np.uint8) for r in np.asarray(arr, np.uint8)], np.uint8).reshape(-1, 32)

T = int(sys.argv[1]) if len(sys.argv) > 1 else 23
terms = []
orig = E.c4_path
E.c4_path = lambda rng, wit, n_tx, h: terms.append((orig(rng, wit, n_tx, h), dict(wit))) or terms[-1][0]
tb, mb, exp, syms = E.c4_workload(40, 2000, seed=4, planted_frac=0.4, hasher_many=hm)
term, wit = terms[T]
h = lambda v: int.from_bytes(cref.keccak256(v.to_bytes(64, "big")), "big")
asg, fn, fwd, inv = {}, {}, {}, {}
keys = [(a << 256) | 1 for a in E.ACTORS]
for k in range(2):
    asg[f"sender_{k+1}"] = wit["sender"][k]; asg[f"call_value{k+1}"] = wit["value"][k]; asg[f"{k+1}_calldatasize"] = wit["cds"][k]
    fn[f"{k+1}_calldata"] = ({(i,): b for i, b in enumerate(wit["bytes"][k])}, 0)
    keys += [(wit["sender"][k] << 256) | 1, (E._word_val(wit["bytes"][k], wit["cds"][k], 4) << 256) | 1]
for key in keys:
    fwd[(key,)] = h(key); inv[(h(key),)] = key
fn["keccak256_512"] = (fwd, 0); fn["keccak256_512-1"] = (inv, 0)
m = Model(asg, fn)
print("expected", exp[T], "whole", eval_under(term, m), wit["cds"])
for i, c in enumerate(term.args):
    if not eval_under(c, m):
        print("FAIL", i, str(c)[:600])

def flat(t, out):
    if t.kind == "and":
        for a in t.args:
            flat(a, out)
    else:
        out.append(t)
    return out

for c in flat(term.args[13], []):
    if not eval_under(c, m):
        print("AXIOM FAIL", str(c)[:900])
        break
print([hex(s) for s in wit["sender"]], [hex(E._word_val(wit["bytes"][k], wit["cds"][k], 4)) for k in range(2)])
