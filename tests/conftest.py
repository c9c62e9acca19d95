import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "multigpu: needs >= 2 GPUs (skipped on a 1-GPU box)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible")
    import cuda_mpi_scratch_amd as pkg

    pkg.hip()  # fail loudly if the HIP extension is missing
    torch.cuda.set_device(0)
    return torch.device("cuda", 0)


@pytest.fixture(scope="session")
def build_dir():
    # MXS_BUILD_DIR: run the native-binary tests against another build tree
    # (e.g. the host-sanitizer build of scripts/cpu_sanitize.sh).
    return os.environ.get("MXS_BUILD_DIR") or os.path.join(ROOT, "build")
