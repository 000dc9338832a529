import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X); run with -m gpu on the GPU box")


@pytest.fixture(scope="session")
def evaluator():
    """The product evaluator on cuda:0. No fallback: a missing libmq.so or GPU fails the test."""
    from mythril_amd.evaluator import Evaluator
    ev = Evaluator(0)
    yield ev
    ev.close()
