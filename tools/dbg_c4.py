"""Debug helper: evaluate each conjunct of a planted C4 path under its witness model (oracle)."""
import sys

sys.path.insert(0, "/root/repo/oracle")
sys.path.insert(0, "/root/repo/tests")
sys.path.insert(0, "/root/repo")
import numpy as np  # noqa: E402
import cref  # noqa: E402
from mythril_amd.synth_evm import ACTORS, KeccakModels, c4_path  # noqa: E402
from mythril_amd.smt_model import Model  # noqa: E402
from oracle_engine import eval_under  # noqa: E402


def hm(arr):
    return np.array([np.frombuffer(cref.keccak256(bytes(r)), np.uint8) for r in np.asarray(arr, np.uint8)], np.uint8).reshape(-1, 32)


km = KeccakModels(4, 2000, 2, 0, 2000, hm)
p = 1619
wit = km.witness(p)
rng = np.random.Generator(np.random.PCG64(7))
term = c4_path(rng, wit, 2, hm)


def h(v):
    return int.from_bytes(cref.keccak256(v.to_bytes(64, "big")), "big")


asg, fn, fwd, inv = {}, {}, {}, {}
keys = [(a << 256) | 1 for a in ACTORS]
for k in range(2):
    asg[f"sender_{k + 1}"] = wit["sender"][k]
    asg[f"call_value{k + 1}"] = wit["value"][k]
    asg[f"{k + 1}_calldatasize"] = wit["cds"][k]
    fn[f"{k + 1}_calldata"] = ({(i,): b for i, b in enumerate(wit["bytes"][k])}, 0)
    to = int.from_bytes(bytes(wit["bytes"][k][16:36]), "big")
    keys += [(wit["sender"][k] << 256) | 1, (to << 256) | 1]
for key in keys:
    fwd[(key,)] = h(key)
    inv[(h(key),)] = key
fn["keccak256_512"] = (fwd, 0)
fn["keccak256_512-1"] = (inv, 0)
m = Model(asg, fn)
print("whole", eval_under(term, m), "cds", wit["cds"], "senders actor", [s in ACTORS for s in wit["sender"]])
for i, c in enumerate(term.args):
    if not eval_under(c, m):
        print("FAIL conjunct", i, str(c)[:400])
