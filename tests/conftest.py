import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "light-whisper_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tools"),
          os.path.join(ROOT, "tests", "golden"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")


def record(test: str, **observed):
    """Append the errors a parity test observed to $QASR_PARITY_LOG (JSON lines) — the evidence the bounds written
    in the tests are set from (about 2x the observed values)."""
    import json

    path = os.environ.get("QASR_PARITY_LOG")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps({"test": test, **{k: (float(v) if hasattr(v, "__float__") else v)
                                                 for k, v in observed.items()}}) + "\n")


@pytest.fixture(scope="session")
def torch_dev():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
