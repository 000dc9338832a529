"""Object lifetimes across the C-ABI: a compiled batch (mq_tapes) may outlive its context
(mq_ctx) — Python finalizers run in any order — and must then neither touch the freed context
nor launch on another one."""
import numpy as np
import pytest

from mythril_amd.evaluator import Evaluator, EvaluatorError
from mythril_amd.synth import c2_workload

pytestmark = pytest.mark.gpu


def test_tapes_freed_after_their_context_is_destroyed():
    tb, mb, exp = c2_workload(12, 500, seed=2)
    ev = Evaluator(0)
    ev.upload_models(mb)
    ct, ct2, ct3 = ev.compile(tb), ev.compile(tb), ev.compile(tb)
    assert (ev.first_hit(ct) == exp).all()
    ev.close()                 # mq_ctx_destroy while three batches are alive
    ct.free()                  # mq_tapes_free after it: detached, no access to the freed context
    del ct2                    # the finalizer path
    ev2 = Evaluator(0)         # a new context (the allocator may hand out the same address)
    try:
        ev2.upload_models(mb)
        with pytest.raises(EvaluatorError):
            ev2.first_hit(ct3)     # a batch of another (destroyed) context is refused
        ct4 = ev2.compile(tb)
        assert (ev2.first_hit(ct4) == exp).all()
        ct3.free()
        ct4.free()
    finally:
        ev2.close()


def test_many_contexts_and_batches_interleaved():
    tb, mb, exp = c2_workload(6, 300, seed=3)
    keep = []
    for i in range(4):
        ev = Evaluator(0)
        ev.upload_models(mb)
        ct = ev.compile(tb)
        assert (ev.first_hit(ct) == exp).all()
        keep.append((ev, ct))
        if i % 2:
            ev.close()         # contexts destroyed before their batches, or after
    for ev, ct in keep:
        ct.free()
        ev.close()
    assert np.all(exp >= -1)
