"""Diagnostic: per-phase cycles of single split backward launches by layer, from the phase-stamp
build (libastyle_stamps.so: python audio_style_transfer_amd/_build.py --stamps).  The stamps sum
over every block launch of a call, so a context whose deepest tap is layer L runs the backward
chain L .. 0, and the difference of two such runs (taps to L and to L - 1) is layer L's launch
alone.  B = 256 clips of T = 16384 (the bench's walk: carried halo rows).
usage: stamp_layers.py L1 L2 ...   (prints the phases of each layer L, from runs to L and L - 1)"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault('ASTYLE_LIB', os.path.join(ROOT, 'audio_style_transfer_amd', 'libastyle_stamps.so'))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from audio_style_transfer_amd import _lib  # noqa: E402
from audio_style_transfer_amd.engine import StyleEngine  # noqa: E402

B, T = 256, 16384
NAMES = {6: 'T barrier', 11: 'top (scales, scalar loads)', 7: 'A/B/H g_v + g_u + epi half 1 (prev) + barrier',
         8: 'C g_a half 0 + convert + loads', 9: 'D g_a half 1 + epi half 0', 12: 'drain', 14: 'prologue'}
lib = _lib.load()
lib.ast_debug_stamps.argtypes = [ctypes.c_void_p]
x = torch.randn(B, T, device='cuda') * 40


def stamps(top):
    eng = StyleEngine(B, T, [top], list(range(top + 1)), precision='split')
    eng.set_targets(torch.randn(T, 128) * 0.1, torch.randn(*eng.style_shape) * 0.01)
    eng.loss_grad(x)
    torch.cuda.synchronize()
    buf = torch.zeros(64, 20, dtype=torch.int64, device='cuda')   # a row per block launch
    buf[:, 17] = 2 ** 62   # (the min wave lifetime slots)
    buf[:, 18] = 2 ** 62   # (the first wave start slots)
    lib.ast_debug_stamps(ctypes.c_void_p(buf.data_ptr()))
    eng.loss_grad(x)
    torch.cuda.synchronize()
    lib.ast_debug_stamps(None)
    eng.close()
    return buf[:, :16].sum(dim=0).cpu().tolist()


tiles = B * T // 64 / 256   # tiles per CU of one launch
for L in [int(a) for a in sys.argv[1:]]:
    hi, lo = stamps(L), stamps(L - 1)
    d = [a - b for a, b in zip(hi, lo)]
    tot = sum(d[k] for k in NAMES)
    print('layer %d (d = %d): %.0f cycles per tile and wave; clock %.0f MHz' % (
        L, 1 << (L % 10), tot / (4 * 256 * tiles), 100.0 * sum(d[k] for k in range(15)) / max(d[15], 1)))
    for k, n in NAMES.items():
        print('   %-48s %8.0f cycles/tile/wave' % (n, d[k] / (4 * 256 * tiles)))
    sys.stdout.flush()
