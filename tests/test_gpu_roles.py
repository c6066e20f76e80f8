"""The alternative split forward block kernels against the default one-wave kernel: the
role-split kernel (tools/variants/block_fwd_roles.hip, ASTYLE_FWD_ROLES=1) and the double-buffered-
image kernel (tools/variants/block_fwd_db.hip, ASTYLE_FWD_DB=1).  They are not part of the shipped
libastyle.so: the tools-only build ``ASTYLE_VARIANT=fwdvariants python audio_style_transfer_amd/
_build.py`` makes libastyle_fwdvariants.so, and these tests skip without it.  Same split numerics, so every extract must be bit-identical, on every
dilation layout (T = 3584: one segment with halo rows, per-column tap masks where 64-position tiles
start and end inside sub-sequences; T = 2048: the 32-position two-segment layout) and with several
clips per launch.  The knob is read once per process, so each run is a child process
(the engine is built after the environment is set)."""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VLIB = os.path.join(ROOT, 'audio_style_transfer_amd', 'libastyle_fwdvariants.so')
IDS = [0, 1, 5, 6, 8, 9, 10, 19, 25, 29, 30]

CHILD = r'''
import json, sys
import numpy as np, torch
sys.path.insert(0, sys.argv[1])
from audio_style_transfer_amd.engine import StyleEngine
from audio_style_transfer_amd.weights import synthetic_weights, synthetic_clips
from oracle import astyle_oracle as O
B, T, out = int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
ids = json.loads(sys.argv[5])
W = synthetic_weights(0)
x = np.stack([O.mu_law_numpy(synthetic_clips(1, T, 42 + b)[0]) for b in range(B)])
eng = StyleEngine(B, T, [29], [0, 30], cnt_channels=16, nb_channels=64, weights=W, precision='split')
eng.forward(torch.tensor(x, dtype=torch.float32, device='cuda'))
np.savez(out, **{'e%d' % i: eng.extract(i).cpu().numpy() for i in ids})
'''


def _run(B, T, knob, path):
    env = dict(os.environ, ASTYLE_FWD_ROLES='0', ASTYLE_FWD_DB='0', ASTYLE_LIB=VLIB)
    if knob:
        env[knob] = '1'
    subprocess.run([sys.executable, '-c', CHILD, ROOT, str(B), str(T), path, json.dumps(IDS)],
                   env=env, check=True, timeout=240)
    with np.load(path) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize('knob', ['ASTYLE_FWD_ROLES', 'ASTYLE_FWD_DB'])
@pytest.mark.parametrize('B,T', [(3, 3584), (2, 2048), (2, 512)])
def test_alt_forward_bit_identical(B, T, knob):
    assert torch.cuda.is_available(), 'gpu tests need an MI355X'
    if not os.path.exists(VLIB):
        pytest.skip('tools-only variant build libastyle_fwdvariants.so not built')
    with tempfile.TemporaryDirectory() as d:
        ref = _run(B, T, None, os.path.join(d, 'one.npz'))
        got = _run(B, T, knob, os.path.join(d, 'alt.npz'))
    for k in ref:
        assert np.isfinite(ref[k]).all()
        assert np.array_equal(ref[k], got[k]), (k, float(np.abs(ref[k] - got[k]).max()))
