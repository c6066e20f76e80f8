"""ast_workspace_bytes (the sizing a caller plans device memory with, include/astyle.h) against
what ast_create really allocates: the device's free memory before and after creating a context,
for each precision, the Gatys Gram, a bottleneck content tap and the fused content tap (split,
one style-tapped content layer: no content-gradient buffer).  B = 8 makes one activation tensor
64 MiB, so a buffer counted but not allocated (or the reverse) is well outside the tolerance
(allocation rounding)."""
import ctypes

import pytest
import torch

from audio_style_transfer_amd import _lib

pytestmark = pytest.mark.gpu

MiB = 1 << 20


def _cfg(precision, cont, style, gatys=0, cnt=128, nb=128, B=8, T=16384):
    c = _lib.AstCfg()
    c.batch, c.T = B, T
    c.n_cont = len(cont)
    for i, v in enumerate(cont):
        c.cont_ids[i] = v
    c.n_style = len(style)
    for i, v in enumerate(style):
        c.style_ids[i] = v
    c.cnt_channels, c.nb_channels = cnt, nb
    c.gatys, c.precision, c.lambd = gatys, precision, 100.0
    return c


def _create_delta(lib, cfg):
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    h = ctypes.c_void_p()
    _lib.check(lib.ast_create(ctypes.byref(cfg), 0, ctypes.byref(h)))
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info()[0]
    lib.ast_destroy(h)
    torch.cuda.synchronize()
    return free0 - free1


@pytest.mark.parametrize('name,kw', [
    ('split fused content', dict(precision=2, cont=[29], style=list(range(30)))),
    ('split two content taps', dict(precision=2, cont=[25, 29], style=list(range(30)))),
    ('split content not style-tapped', dict(precision=2, cont=[29], style=list(range(10)))),
    ('bf16', dict(precision=1, cont=[29], style=list(range(30)))),
    ('fp32 gatys', dict(precision=0, cont=[29], style=list(range(30)), gatys=1)),
    ('split bottleneck', dict(precision=2, cont=[31], style=[0, 9, 19, 29], nb=64)),
])
def test_workspace_bytes_matches_allocation(name, kw):
    assert torch.cuda.is_available(), 'gpu tests need an MI355X'
    lib = _lib.load()
    cfg = _cfg(**kw)
    n = ctypes.c_size_t()
    _lib.check(lib.ast_workspace_bytes(ctypes.byref(cfg), ctypes.byref(n)))
    _create_delta(lib, _cfg(precision=2, cont=[29], style=[29], B=1, T=1024))   # code objects loaded
    got = _create_delta(lib, cfg)
    tol = 16 * MiB + n.value // 200
    assert abs(got - n.value) <= tol, (name, got / MiB, n.value / MiB)
