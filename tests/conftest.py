import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "code-structure-aware-transformer_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# torch.ops.csa.* are registered when csa_amd.ops / rel_ops / gen_ops are imported: import them once for
# every test, so a test that calls torch.ops.csa.* directly passes alone as well as after the others.
# (Importing loads libcsa_hip.so and the C++ op shim libcsa_torch.so when they are built, registering the
# GPU implementations; it does not touch a GPU.)
import csa_amd.ops  # noqa: E402,F401
import csa_amd.rel_ops  # noqa: E402,F401
import csa_amd.gen_ops  # noqa: E402,F401


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        with np.load(os.path.join(GOLDEN, name + ".npz")) as z:
            return {k: z[k] for k in z.files}
    return load
