import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "synth"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"),
          os.path.join(ROOT, "kafka-parquet-writer_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running")
    # test infrastructure libs (oracle + synthetic generator) are built on demand
    for d in ("oracle", "synth"):
        lib = {"oracle": "build/libkpw_oracle.so", "synth": "build/libkpw_synth.so"}[d]
        if not os.path.exists(os.path.join(ROOT, d, lib)):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, d)])


_torch_hip_ready = False


@pytest.fixture(autouse=True)
def _torch_hip_first(request):
    """PyTorch-ROCm bundles its own libamdhip64 next to /opt/rocm's, which libkpw_gpu.so
    links.  Whichever initialises first owns the device for the process: when the kpw library
    goes first, torch's later lazy init reports "No HIP GPUs are available".  GPU tests use
    torch (device buffers for the encoder API), so torch's runtime is initialised before the
    first GPU test, whatever the test order."""
    global _torch_hip_ready
    if not _torch_hip_ready and request.node.get_closest_marker("gpu"):
        import torch
        torch.cuda.init()
        _torch_hip_ready = True
    yield
