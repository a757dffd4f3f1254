import asyncio
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")


@pytest.fixture
def run():
    """Run a coroutine to completion on a fresh event loop."""
    def _run(coro, timeout=60):
        return asyncio.run(asyncio.wait_for(coro, timeout))
    return _run
