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
