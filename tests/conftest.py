import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "capnp-zig_amd")
TESTS = os.path.dirname(os.path.abspath(__file__))
for p in (PKG, TESTS, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests through the C-ABI")


def _gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(params=["twopass", "words"])
def decoder(request):
    """Runs a decode test under each mid-unit decoder (capnp_packed_set_decoder): the two-pass
    decoder and the single-read words decoder (round 5), each forced for every
    mid unit of the batch (the default, "auto", picks between them by batch, class_scan_kernel)."""
    import capnp_packed as cp
    if not cp.decoder_available(request.param):
        pytest.skip(f"the {request.param} decoder is not in this build")
    with cp.decoder(request.param):
        yield request.param
