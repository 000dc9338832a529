"""Exceptions of the quick-sat boundary, with the reference's hierarchy
(``mythril/exceptions.py:4-27``): ``SolverTimeOutException`` IS an ``UnsatError``, so callers
that catch ``UnsatError`` treat a timeout as infeasible (``constraints.py:37-40``)."""
import re
from collections import Counter


class MythrilBaseException(Exception):
    """exceptions.py:4-7"""


class UnsatError(MythrilBaseException):
    """exceptions.py:16-20: the constraints have no model."""


class SolverTimeOutException(UnsatError):
    """exceptions.py:23-27: the solver gave up (timeout / unknown / z3 exception)."""


class LoweringError(TypeError):
    """A term the tape IR cannot express (fail closed: the query keeps the z3 path)."""


# Queries that failed closed at lowering, by reason ("array-valued ite", "array equality", ...):
# a z3 host sees how often queries of the state-merge plugin's shapes go to z3.
fail_closed = Counter()


def note_fail_closed(err: BaseException) -> None:
    """Count one query routed to z3 because a conjunct did not lower (its reason, digits dropped
    so that widths and arities do not split a reason into many)."""
    fail_closed[re.sub(r"\d+", "N", str(err)) or type(err).__name__] += 1
