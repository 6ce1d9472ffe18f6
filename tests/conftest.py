from __future__ import annotations

import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
GOLDEN = Path(__file__).resolve().parent / "golden"
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine through the C ABI)")


@pytest.fixture(scope="session")
def oracle_c():
    """The C restatement (test infrastructure only)."""
    from oracle import oracle_c as oc

    oc.build()
    return oc


@pytest.fixture(scope="session")
def engine():
    """One engine context on cuda:0 for the whole GPU session.  torch (when present) is imported
    first so that the engine and torch share one HIP runtime (taxi2_amd._native.Engine) and torch
    stream / tensor pointers can be handed to the *_dev entry points."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    from taxi2_amd._native import Engine

    return Engine.default(0)
