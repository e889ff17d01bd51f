import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")
    config.addinivalue_line("markers", "slow: larger CPU parity runs")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o

    o.lib()
    return o


def pytest_terminal_summary(terminalreporter):
    """State which checker each whole-batch parity test ran against (shown
    with -q too)."""
    mod = sys.modules.get("tests.ref_crypto")
    if not mod or not mod.USED:
        return
    terminalreporter.section("whole-batch parity checkers")
    for test_id, what in mod.USED:
        terminalreporter.write_line(f"{test_id}: {what}")
