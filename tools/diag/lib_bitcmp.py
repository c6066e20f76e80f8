"""Diagnostic: the split-mode loss and gradient of a few seeded cases from the libastyle.so named
by ASTYLE_LIB (one library per process), saved to an npz; with --cmp A.npz B.npz, whether two
such runs agree bit for bit (a kernel restructure that must not change results).
usage: ASTYLE_LIB=... python tools/diag/lib_bitcmp.py out.npz ;  python tools/diag/lib_bitcmp.py --cmp a.npz b.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

CASES = {   # tag: (B, T, cont, style taps, gatys)
    'ours16k': (4, 16384, [29], list(range(30)), False),
    'ours8k': (3, 8192, [25], list(range(30)), False),
    'ours2k': (2, 2048, [25], list(range(30)), False),
    'gatys4k': (2, 4096, [29], list(range(30)), True),
}


def run(out):
    import torch
    from audio_style_transfer_amd.engine import StyleEngine
    from audio_style_transfer_amd.weights import synthetic_weights
    W = synthetic_weights(0)
    res = {}
    for tag, (B, T, cont, sty, gat) in CASES.items():
        g = torch.Generator().manual_seed(7)
        x = (torch.rand(B, T, generator=g) * 255 - 127.5)
        tgt = (torch.rand(B, T, generator=g) * 255 - 127.5)
        eng = StyleEngine(B, T, cont, sty, gatys=gat, weights=W, precision='split')
        ec, es = eng.embeds(tgt.cuda())
        eng.set_targets(ec, es)
        parts, grad = eng.loss_grad(x.cuda())
        res[tag + '_parts'] = parts.cpu().numpy()
        res[tag + '_grad'] = grad.cpu().numpy()
        eng.close()
    np.savez(out, **res)
    print(os.path.basename(os.environ.get('ASTYLE_LIB', 'libastyle.so')), 'saved', out)


def cmp(a, b):
    za, zb = np.load(a), np.load(b)
    ok = True
    for k in sorted(za.files):
        same = np.array_equal(za[k].view(np.uint32), zb[k].view(np.uint32))
        d = float(np.abs(za[k].astype(np.float64) - zb[k]).max())
        print('%-16s %s  max |diff| %.3g' % (k, 'bit-identical' if same else 'DIFFERS', d))
        ok = ok and same
    print('ALL BIT-IDENTICAL' if ok else 'MISMATCH')
    return 0 if ok else 1


if __name__ == '__main__':
    if sys.argv[1] == '--cmp':
        sys.exit(cmp(sys.argv[2], sys.argv[3]))
    run(sys.argv[1])
