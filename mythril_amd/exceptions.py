"""Exceptions of the quick-sat boundary, with the reference's hierarchy
(``mythril/exceptions.py:4-27``): ``SolverTimeOutException`` IS an ``UnsatError``, so callers
that catch ``UnsatError`` treat a timeout as infeasible (``constraints.py:37-40``)."""


class MythrilBaseException(Exception):
    """exceptions.py:4-7"""


class UnsatError(MythrilBaseException):
    """exceptions.py:16-20: the constraints have no model."""


class SolverTimeOutException(UnsatError):
    """exceptions.py:23-27: the solver gave up (timeout / unknown / z3 exception)."""


class LoweringError(TypeError):
    """A term the tape IR cannot express (fail closed: the query keeps the z3 path)."""
