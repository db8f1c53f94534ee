import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "numpy-quant_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built libnqk.so")
    config.addinivalue_line("markers", "slow: long-running CPU reference comparisons")


# The golden fixtures were recorded in the 8-CPU build container, where NumPy's OpenBLAS
# ran 8 threads: its GEMV-T (one-row float products, e.g. the classifier Gemm at batch 1)
# splits the columns over them, and nqk_sgemv_t reproduces the split for the count it is
# given (numpy_quant.kernels.openblas_threads).  Pin that count for every test.
FIXTURE_BLAS_THREADS = 8


import pytest  # noqa: E402


@pytest.fixture(autouse=True)
def _fixture_blas_threads():
    try:
        from numpy_quant import kernels
    except Exception:  # the package itself is not importable: the test reports that
        yield
        return
    old = kernels.BLAS_THREADS
    kernels.BLAS_THREADS = FIXTURE_BLAS_THREADS
    yield
    kernels.BLAS_THREADS = old
