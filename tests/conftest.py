"""Test configuration.

* `gpu` marker: needs a HIP device (MI355X); everything else runs on the CPU.
* The package directory point-cloud-flow-matching_amd/ is put on sys.path the
  way the reference puts third_party/pvcnn on it (models.py:9-13).
* `oracle_backend` fixture: CPU tests swap the C oracle in behind
  modules.functional (the product itself has no CPU path).
"""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "point-cloud-flow-matching_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)
# Chamfer: take the culled search from 16M pairs per batch element in tests (the
# product default is 2^31), so test-sized clouds exercise both search paths
os.environ.setdefault("PCFM_CHAMFER_CULL_PAIRS", str(16 << 20))


@pytest.fixture(autouse=True)
def _restore_torch_backend_flags():
    """Trainer(miopen_find=True) switches torch.backends.cudnn.benchmark on for
    the process; MIOpen's timed solver search then picks per-run algorithms
    (different summation orders) in every later test.  Each test starts from
    the flags the session started with."""
    import torch
    b = torch.backends
    old = (b.cudnn.benchmark, b.cudnn.deterministic, b.cudnn.allow_tf32,
           b.cuda.matmul.allow_tf32)
    yield
    (b.cudnn.benchmark, b.cudnn.deterministic, b.cudnn.allow_tf32,
     b.cuda.matmul.allow_tf32) = old


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP GPU (MI355X); run with -m gpu")


@pytest.fixture
def oracle_backend(monkeypatch):
    from oracle.oracle import TorchBackend
    import modules.functional.backend as be
    monkeypatch.setattr(be, "_backend", TorchBackend())
    return be._backend


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    return load


_REPORT = {}


@pytest.fixture(scope="session")
def report():
    """report(key, value): measured deviations / timings, written as JSON to
    $PCFM_REPORT at the end of the session (the GPU runs copy it to profiles/)."""
    def rec(key, value):
        _REPORT[key] = value
    return rec


def pytest_sessionfinish(session, exitstatus):
    path = os.environ.get("PCFM_REPORT")
    if path and _REPORT:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(_REPORT, f, indent=1, sort_keys=True, default=float)


def have_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
