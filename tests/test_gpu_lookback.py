"""Decoupled fallback of the single-pass look-back scans (kpw_lookback.h): with KPW_LB_SPIN=0
every look-back that does not find its predecessor's status at once recomputes it from the
predecessor tile's inputs; files must stay byte-identical to the oracle's."""
import os
import subprocess
import sys

import pytest


@pytest.mark.gpu
def test_lookback_fallback_exact():
    env = dict(os.environ, KPW_LB_SPIN="0")
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "lb_fallback_child.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "LB_FALLBACK_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
