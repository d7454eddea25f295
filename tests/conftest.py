import os
import sys

import pytest

# under pytest-xdist, give each worker its share of the cores: every worker's OpenMP pool
# spinning on all of them oversubscribes the machine (set before the library loads)
if os.environ.get("PYTEST_XDIST_WORKER_COUNT"):
    _share = max(1, (os.cpu_count() or 8) // int(os.environ["PYTEST_XDIST_WORKER_COUNT"]))
    os.environ.setdefault("OMP_NUM_THREADS", str(_share))

# in-process device ranks (tests/test_gpu_distributed.py) are threads with a stream each whose
# peer collectives wait on one another on the device: every rank's stream needs its own
# hardware queue (HIP's default of 4 queues per process would put two ranks' kernels in one
# queue, behind each other).  Read by the HIP runtime when it initialises.
# (the box exports HIP's default of 4: raise it, never above what the pool allows)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the gfx950 build")
    config.addinivalue_line("markers", "slow: long-running test")


def _lib_path():
    return os.path.join(ROOT, "lightgbmv1_amd", "lib", "lib_lightgbmv1_amd.so")


@pytest.fixture(scope="session", autouse=True)
def _native_library():
    """Build the native library once if it is missing (CPU container or GPU box)."""
    if not os.path.isfile(_lib_path()):
        import subprocess
        subprocess.check_call(["make", "-j" + str(min(16, os.cpu_count() or 8))], cwd=ROOT)
    yield


@pytest.fixture(scope="session")
def gpu_available():
    import lightgbmv1_amd as lgb
    n = lgb.device_count()
    if n < 1:
        # GPU tests must fail loudly when the device path is unavailable on a GPU box
        raise RuntimeError("gpu test requested but no HIP device is visible to lib_lightgbmv1_amd")
    return n
