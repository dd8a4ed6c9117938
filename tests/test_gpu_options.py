"""Writer pipeline options outside the default configuration (tests/pipeline_options_child.py,
one child process per option so that knobs read once per process take effect): exact-mode
dictionary continuation in the page-size probes, the device encode gate, three encode workers.
Each checked byte for byte (and getDataSize value by value) against the oracle."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode,env", [
    ("probe_exact", {"KPW_PROBE_EXACT": "1"}),
    ("gate", {"KPW_DEVICE_ENCODES": "1", "KPW_EAGER_MB": "4", "KPW_STAGE_FLUSH_MB": "8"}),
    ("encoders3", {"KPW_ENCODERS": "3", "KPW_EAGER_MB": "4", "KPW_STAGE_FLUSH_MB": "8"}),
])
def test_pipeline_option(mode, env):
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "pipeline_options_child.py"), mode],
                       env=dict(os.environ, **env), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "OPTIONS_OK " + mode in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
