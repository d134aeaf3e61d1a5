import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False


@pytest.fixture
def device():
    if not gpu_available():
        pytest.skip("no GPU")
    import torch
    return torch.device("cuda:0")


@pytest.fixture
def session(tmp_path):
    from hyperspace_amd import Session
    s = Session(conf={"spark.hyperspace.system.path": str(tmp_path / "indexes"),
                      "spark.hyperspace.index.numBuckets": "4",
                      "spark.sql.autoBroadcastJoinThreshold": "-1",
                      "spark.sql.shuffle.partitions": "5",
                      "spark.hyperspace.mi.execution.device": "cpu"},
                warehouse_dir=str(tmp_path / "wh"))
    yield s
    s.disableHyperspace()
