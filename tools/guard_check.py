"""Diagnostic: out-of-bounds stores.  With ASTYLE_GUARD=1 every library buffer carries guard
bands (api.hip dalloc); the caller's buffers (x, grad, parts, targets) are slices of larger
tensors whose margins hold a sentinel.  Runs embeds, eager loss_grad and a captured graph's
replays for a few configurations and reports every band that was written.

  ASTYLE_GUARD=1 python tools/guard_check.py [--quick]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import bench
from audio_style_transfer_amd.engine import StyleEngine

PAD = 1 << 16      # floats of margin on each side of a caller buffer
SENT = 12345.678


def padded(shape, dev, fill=None):
    n = 1
    for d in shape:
        n *= d
    big = torch.full((n + 2 * PAD,), SENT, device=dev)
    v = big[PAD:PAD + n].view(*shape)
    if fill is not None:
        v.copy_(fill)
    return big, v


def margins_ok(tag, big, n):
    lo = big[:PAD] != SENT
    hi = big[PAD + n:] != SENT
    msg = []
    if lo.any():
        msg.append('%s: lower margin written at offsets %s' % (tag, (lo.nonzero().flatten() - PAD)[:8].tolist()))
    if hi.any():
        msg.append('%s: upper margin written at offsets %s' % (tag, hi.nonzero().flatten()[:8].tolist()))
    return msg


def check(e, tag, callers):
    lib = e.lib
    lib.ast_debug_check_guards.restype = ctypes.c_int
    lib.ast_debug_check_guards.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]
    buf = ctypes.create_string_buffer(1 << 16)
    nbad = lib.ast_debug_check_guards(e.h, buf, len(buf))
    msg = []
    for name, (big, n) in callers.items():
        msg += margins_ok(name, big, n)
    print('%-40s library buffers with written guards: %d%s' % (tag, nbad, ''.join('\n    ' + l for l in buf.value.decode().splitlines() + msg)), flush=True)
    return nbad > 0 or bool(msg)


def case(B, T, gatys, precision, dev):
    tag = 'B%d T%d %s %s' % (B, T, 'gatys' if gatys else 'ours', precision)
    e = StyleEngine(B, T, [29], list(range(30)), precision=precision, device=dev, lambd=100.0,
                    gatys=gatys)
    x0 = bench.make_problem(e, list(range(B)), T, dev)
    bx, x = padded((B, T), dev, x0)
    bg, g = padded((B, T), dev)
    bp, p = padded((B, 4), dev)
    callers = {'x': (bx, B * T), 'grad': (bg, B * T), 'parts': (bp, B * 4)}
    bad = check(e, tag + ' after make_problem', callers)
    for _ in range(2):
        e.loss_grad(x, g, p)
    bad |= check(e, tag + ' after eager loss_grad', callers)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        e.loss_grad(x, g, p)
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        e.loss_grad(x, g, p)
    for _ in range(3):
        gr.replay()
    bad |= check(e, tag + ' after 3 graph replays', callers)
    del gr
    e.close()
    return bad


def main():
    assert os.environ.get('ASTYLE_GUARD') == '1', 'run with ASTYLE_GUARD=1'
    dev = torch.device('cuda', 0)
    bad = False
    cases = ((8, 16384, False, 'split'), (3, 16384, False, 'split'), (1, 16384, False, 'split'),
             (8, 16384, True, 'split'), (2, 4096, False, 'split'),
             (4, 16384, False, 'fp32'), (4, 16384, False, 'bf16'))
    if '--quick' in sys.argv:   # (tests/test_gpu_guard.py)
        cases = ((1, 16384, False, 'split'), (3, 4096, False, 'split'), (2, 4096, True, 'split'),
                 (2, 2048, False, 'fp32'), (2, 2048, False, 'bf16'))
    for B, T, gatys, prec in cases:
        bad |= case(B, T, gatys, prec, dev)
    print('OUT-OF-BOUNDS STORES FOUND' if bad else 'no out-of-bounds stores', flush=True)


if __name__ == '__main__':
    main()
