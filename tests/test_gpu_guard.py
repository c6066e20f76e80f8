"""Out-of-bounds stores: every library buffer with guard bands (ASTYLE_GUARD=1, api.hip dalloc)
and the caller's x / grad / parts inside sentinel margins, through embeds, eager loss_grad and
graph replays (tools/guard_check.py --quick, in its own process: the guard switch is read once
per process)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_no_out_of_bounds_stores():
    env = dict(os.environ, ASTYLE_GUARD='1')
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'guard_check.py'), '--quick'],
                       env=env, capture_output=True, text=True, timeout=240)
    print(r.stdout[-3000:])
    assert r.returncode == 0, r.stderr[-3000:]
    assert 'no out-of-bounds stores' in r.stdout, r.stdout[-3000:]
