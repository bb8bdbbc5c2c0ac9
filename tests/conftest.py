"""Shared pytest fixtures.

Mirrors the reference suite's fixtures (``tests/conftest.py:153-296`` in the
reference): seeded random inputs, the LM config, and ``.npz`` snapshot
matching.  Snapshots are read with ``np.load`` (``allow_pickle=False``).
The reference's ``model.pt`` weights blob is missing from the mirror
(SURVEY §0.4), so ``ts_state_dict`` skips when absent.

Markers: ``gpu`` (needs an MI355X; the CPU CI runs ``-m "not gpu"``),
``slow``, ``dist`` (multi-process).
"""

from __future__ import annotations

import json
import os
from pathlib import Path

import numpy as np
import pytest
import torch

REPO = Path(__file__).resolve().parent.parent
SNAPSHOTS = REPO / "tests" / "_snapshots"
FIXTURES = REPO / "tests" / "fixtures"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD Instinct MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line("markers", "dist: spawns multiple processes (torch.distributed)")


def pytest_addoption(parser):
    parser.addoption("--snapshot-exact", action="store_true", default=False, help="match snapshots exactly")


class NumpySnapshot:
    def __init__(self, test_name: str, exact: bool = False):
        self.test_name = test_name
        self.exact = exact

    def assert_match(self, actual, rtol: float = 1e-4, atol: float = 1e-2, test_name: str | None = None):
        name = test_name or self.test_name
        path = SNAPSHOTS / f"{name}.npz"
        expected = dict(np.load(path))
        arrays = actual if isinstance(actual, dict) else {"array": actual}
        arrays = {k: (v.detach().cpu().float().numpy() if isinstance(v, torch.Tensor) else np.asarray(v))
                  for k, v in arrays.items()}
        assert set(arrays) == set(expected), f"snapshot keys differ for {name}"
        if self.exact:
            rtol = atol = 0
        for k in arrays:
            np.testing.assert_allclose(arrays[k], expected[k], rtol=rtol, atol=atol,
                                       err_msg=f"array {k!r} does not match snapshot {name}")


@pytest.fixture
def numpy_snapshot(request):
    return NumpySnapshot(request.node.name.split("[")[0], request.config.getoption("--snapshot-exact"))


@pytest.fixture
def ts_state_dict():
    path = FIXTURES / "ts_tests" / "model.pt"
    if not path.exists():
        pytest.skip("reference weights blob tests/fixtures/ts_tests/model.pt is missing from the mirror "
                    "(.MISSING_LARGE_BLOBS); covered by oracle tests instead")
    state_dict = torch.load(path, map_location="cpu", weights_only=True)
    config = json.loads((FIXTURES / "ts_tests" / "model_config.json").read_text())
    return {k.replace("_orig_mod.", ""): v for k, v in state_dict.items()}, config


@pytest.fixture
def n_layers():
    return 3


@pytest.fixture
def vocab_size():
    return 10_000


@pytest.fixture
def batch_size():
    return 4


@pytest.fixture
def n_queries():
    return 12


@pytest.fixture
def n_keys():
    return 16


@pytest.fixture
def n_heads():
    return 4


@pytest.fixture
def d_head():
    return 16


@pytest.fixture
def d_model(n_heads, d_head):
    return n_heads * d_head


@pytest.fixture
def d_ff():
    return 128


@pytest.fixture
def q(batch_size, n_queries, d_model):
    torch.manual_seed(1)
    return torch.randn(batch_size, n_queries, d_model)


@pytest.fixture
def k(batch_size, n_keys, d_model):
    torch.manual_seed(2)
    return torch.randn(batch_size, n_keys, d_model)


@pytest.fixture
def v(batch_size, n_keys, d_model):
    torch.manual_seed(3)
    return torch.randn(batch_size, n_keys, d_model)


@pytest.fixture
def in_embeddings(batch_size, n_queries, d_model):
    torch.manual_seed(4)
    return torch.randn(batch_size, n_queries, d_model)


@pytest.fixture
def mask(batch_size, n_queries, n_keys):
    torch.manual_seed(5)
    return torch.randn(batch_size, n_queries, n_keys) > 0.5


@pytest.fixture
def in_indices(batch_size, n_queries):
    torch.manual_seed(6)
    return torch.randint(0, 10_000, (batch_size, n_queries))


@pytest.fixture
def theta():
    return 10000.0


@pytest.fixture
def pos_ids(n_queries):
    return torch.arange(0, n_queries)


@pytest.fixture(scope="session")
def gpu_device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from bpe_transformer import ops

    ops.load()  # fail loudly if the HIP library is missing
    return torch.device("cuda", 0)


def pytest_collection_modifyitems(config, items):
    if not torch.cuda.is_available() and os.environ.get("BPE_REQUIRE_GPU") == "1":
        raise pytest.UsageError("BPE_REQUIRE_GPU=1 but no GPU is visible")
