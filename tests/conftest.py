import importlib
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")


@pytest.fixture(scope="session")
def pkg():
    return importlib.import_module("plotpointe-gat-recommendation_amd")


@pytest.fixture(scope="session")
def oracle():
    from oracle import gat_oracle
    return gat_oracle


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no ROCm GPU is visible")
    return torch.device("cuda:0")


@pytest.fixture(autouse=True)
def _seeded():
    """Every test starts from the same global RNG state, so inputs drawn without an explicit
    generator are the same run to run (tolerances are checked on fixed data)."""
    import random

    import numpy as np
    import torch
    random.seed(1234)
    np.random.seed(1234)
    torch.manual_seed(1234)
