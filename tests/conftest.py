import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS_DIR = os.path.dirname(os.path.abspath(__file__))
if TESTS_DIR not in sys.path:
    sys.path.insert(0, TESTS_DIR)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device; runs through the C ABI")


@pytest.fixture(scope="session")
def ctx():
    """One eigsol context on device 0 (fails loudly when the HIP library or device is missing)."""
    import pcsc_eigenvalue_solver_project_amd as E
    c = E.Context(0)
    yield c
    c.close()


# Loopback worlds run several ranks' streams on one GPU, and a peer-exchange launch waits inside
# the kernel for the other ranks' launches: each rank's stream needs a hardware queue of its own
# (HIP's default of 4 would put two ranks' launches one behind the other in a shared queue).
# Read by HIP at its initialisation, which happens after conftest is imported.  The GPU box
# exports 4, so raise it (16 is within what the pool allows).
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"
