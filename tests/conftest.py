import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "team02-objectdetection_amd")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture
def record(request):
    """record(**fields): append one JSON line about this test's parity margins to
    gpurun_out/parity_records.jsonl (merged back from the GPU box; the figures quoted in
    DESIGN.md come from these lines, copied to profiles/)."""
    import json

    def _rec(**fields):
        out = os.path.join(REPO, "gpurun_out")
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "parity_records.jsonl"), "a") as fh:
            fh.write(json.dumps({"test": request.node.nodeid, **fields}, default=float) + "\n")
    return _rec


def has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
