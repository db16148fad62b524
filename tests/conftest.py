import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import pkgload  # noqa: E402

pkgload.load()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


@pytest.fixture(scope="session")
def native():
    from generic_ebpf_amd import native as n
    n.lib()
    return n


@pytest.fixture(scope="session")
def gpu(native):
    if native.gpu_count() < 1:
        pytest.fail("GPU test selected but no GPU visible: %s" % native.last_error())
    return native


@pytest.fixture()
def env(native):
    e = native.Env()
    yield e
    assert e.destroy() == 0, "objects leaked: ebpf_env_destroy returned EBUSY"
