"""Which tapes the evaluator may answer MQ_UNSUPPORTED (-2), and why (test helper).

A tape is unsupported only for a NAMED limit of the tape compiler (include/mq.h):
values wider than 2048 bits, multiplication / division / overflow predicates wider than 512 bits,
keccak arguments that are not 8..2048 bits of whole bytes.  The parity tests compare the GPU's
-2 set with exactly the tapes mq_tape_compile_info rejects for one of these reasons, so a
supported shape silently dropping to -2 fails them."""
import numpy as np

NAMED_LIMITS = (
    "width > 2048",
    "multiplication / division wider than 512 bits",
    "overflow predicate wider than 512 bits",
    "keccak argument must be 8..2048 bits, bytes",
)


def expected_unsupported(tb) -> np.ndarray:
    """bool[N]: tapes rejected at compile time; every rejection must name a limit."""
    from mythril_amd.evaluator import compile_info
    mask = np.zeros(tb.n_tapes, bool)
    for t in range(tb.n_tapes):
        ci = compile_info(tb, t)
        if not ci.supported:
            assert ci.why in NAMED_LIMITS, f"tape {t} unsupported for an unnamed reason: {ci.why}"
            mask[t] = True
    return mask


def supported_exactly(tb, fh, max_width=None) -> np.ndarray:
    """Assert the GPU's -2 answers (fh) are exactly the compile-time rejections (none at all for
    batches no wider than 256 bits); returns the supported mask."""
    exp = expected_unsupported(tb)
    if max_width is not None and max_width <= 256:
        assert not exp.any(), np.flatnonzero(exp)
    got = np.asarray(fh) == -2
    assert (got == exp).all(), f"-2 on {np.flatnonzero(got & ~exp)[:10]} (supported), " \
                               f"answered {np.flatnonzero(exp & ~got)[:10]} (rejected)"
    return ~exp
