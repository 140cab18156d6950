import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


# Plans specialise their kernels by themselves (hiprtc, in a background thread) from the first
# decode of >= 8192 frames, and destroying a plan waits for that compile: tests keep the
# interpreter kernels unless they ask for specialisation (tests/test_gpu_rtc.py,
# tests/test_rtc.py call pcg_plan_specialize or set PCG_RTC themselves).
os.environ.setdefault("PCG_RTC", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session")
def oracle():
    from pyoracle import Oracle
    return Oracle()
