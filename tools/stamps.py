"""Diagnostic: per-phase cycle shares of the persistent block kernels (s_memtime stamps,
libastyle_stamps.so built with -DASTYLE_STAMPS: python audio_style_transfer_amd/_build.py
--stamps).  Shares, not absolute time, are meaningful.

usage: stamps.py [clips] [fwd|bwd] [bf16|split]   (bwd runs one loss+grad)"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault('ASTYLE_LIB', os.path.join(ROOT, 'audio_style_transfer_amd', 'libastyle_stamps.so'))
sys.path.insert(0, ROOT)
import torch
from audio_style_transfer_amd.engine import StyleEngine
from audio_style_transfer_amd import _lib
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
mode = sys.argv[2] if len(sys.argv) > 2 else 'fwd'
prec = sys.argv[3] if len(sys.argv) > 3 else 'split'
T = 16384
eng = StyleEngine(B, T, [29], list(range(30)), precision=prec)
x = torch.randn(B, T, device='cuda') * 40
if mode == 'bwd':
    eng.set_targets(torch.randn(T, 128) * 0.1, torch.randn(*eng.style_shape) * 0.01)
run = (lambda: eng.loss_grad(x)) if mode == 'bwd' else (lambda: eng.forward(x))
run(); torch.cuda.synchronize()
buf = torch.zeros(64, 20, dtype=torch.int64, device='cuda')   # a row per block launch
buf[:, 17] = 2 ** 62   # (the min wave lifetime slots)
buf[:, 18] = 2 ** 62   # (the first wave start slots)
lib = _lib.load()
lib.ast_debug_stamps.argtypes = [ctypes.c_void_p]
lib.ast_debug_stamps(ctypes.c_void_p(buf.data_ptr()))
if os.environ.get('STAMPS_GRAPH', '0') != '0':
    # captured (the stamp rows are baked into the kernels' arguments), then replayed: the
    # launches run back to back as the bench's graph replays run them
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        run()
    lib.ast_debug_stamps(None)
    g.replay(); torch.cuda.synchronize()   # (warm)
    buf.zero_(); buf[:, 17] = 2 ** 62; buf[:, 18] = 2 ** 62
    g.replay(); torch.cuda.synchronize()
else:
    run(); torch.cuda.synchronize()
    lib.ast_debug_stamps(None)
rows = buf.cpu().tolist()
v = [sum(r[k] for r in rows) for k in range(16)]
launched = [r for r in rows if r[15]]   # per launch: max / min wave lifetime
v += [sum(r[16] for r in launched) / max(len(launched), 1), sum(r[17] for r in launched) / max(len(launched), 1)]
if prec == 'bf16':
    names = ['fwd: top wait + barrier', 'fwd: GEMM1 + epi2 of prev + DMA', 'fwd: epi1 + GEMM2', '-',
             'bwd: top wait + barrier', 'bwd: step 1 + g_u + barrier', 'bwd: step 2 + DMA',
             'bwd: step 3 (mask, +tot, +D, stores)', '-', '-', '-', '-']
    tiles = B * T // 128 * 30 / 256   # tiles per CU over the 30 block launches
    groups = ((0, 4), (4, 8))
elif os.environ.get('ASTYLE_FWD_ROLES', '0') != '0' and mode == 'fwd':
    # role-split forward (block_fwd_roles.hip): 4 dconv + 4 residual waves per CU
    names = {14: 'dconv: prologue + S_0', 6: 'dconv: GEMM1 half 0', 7: 'dconv: epi1 half 0', 8: 'dconv: GEMM1 half 1',
             9: 'dconv: epi1 half 1', 10: 'dconv: S wait', 13: 'resid: prologue + S_0', 12: 'resid: convert (period 0)',
             11: 'resid: top (scales, max flush)', 0: 'resid: res0 + GEMM2 h0 + convert 0..4', 2: 'resid: epi2 h0',
             3: 'resid: res1 + GEMM2 h1 + convert 5..8', 5: 'resid: epi2 h1', 1: 'resid: mask stores', 4: 'resid: S wait'}
    tiles = B * T // 64 * 30 / 256
    for grp in ((14, 6, 7, 8, 9, 10), (13, 12, 11, 0, 2, 3, 5, 1, 4)):
        tot = sum(v[k] for k in grp)
        for k in grp:
            if v[k]:
                print('%-48s %6.1f %%   %8.0f cycles/tile/wave' % (names[k], 100.0 * v[k] / tot, v[k] / (4 * 256 * tiles)))
        print('%-48s %8.0f cycles per wave per launch' % ('total', tot / (4 * 256 * 30)))
    if v[15]:
        cyc = sum(v[k] for k in range(15))
        print('%-48s %8.0f MHz (shader cycles / s_memrealtime ticks, all stamped kernels)' % ('effective clock', 100.0 * cyc / v[15]))
    sys.exit(0)
else:
    names = {13: 'fwd: prologue (weights, first tile)', 14: 'bwd: prologue (weights, first tile)', 0: 'fwd: T barrier', 10: 'fwd: top (scales, scalar loads)', 5: 'fwd: A GEMM1 half 0 + epi2(prev)',
             1: 'fwd: B GEMM1 half 1 + epi1 half 0 + barrier', 2: 'fwd: C GEMM2 half 0 + epi1 half 1 + barrier',
             3: 'fwd: D GEMM2 half 1 + convert + loads', 4: 'fwd: drain',
             6: 'bwd: T barrier', 11: 'bwd: top (scales, scalar loads)', 7: 'bwd: A/B/H g_v + g_u + epi half 1 (prev) + barrier',
             8: 'bwd: C g_a half 0 + convert + loads', 9: 'bwd: D g_a half 1 + epi half 0',
             12: 'bwd: drain'}
    tiles = B * T // 64 * 30 / 256
    for grp in ((13, 0, 10, 5, 1, 2, 3, 4), (14, 6, 11, 7, 8, 9, 12)):
        tot = sum(v[k] for k in grp)
        for k in grp:
            if v[k]:
                print('%-48s %6.1f %%   %8.0f cycles/tile/wave' % (names[k], 100.0 * v[k] / tot, v[k] / (4 * 256 * tiles)))
        print('%-48s %8.0f cycles per wave per launch' % ('total', tot / (4 * 256 * 30)))
    if v[15]:   # wave lifetimes in 100-MHz ticks: the clock the kernels ran at
        cyc = sum(v[k] for k in range(15))
        print('%-48s %8.0f MHz (shader cycles / s_memrealtime ticks, all stamped kernels)' % ('effective clock', 100.0 * cyc / v[15]))
        print('%-48s mean %.2f  per launch: max %.2f  min %.2f us (averaged over %d launches)' % (
            'wave lifetime', v[15] / (4 * 256 * len(launched)) / 100.0, v[16] / 100.0, v[17] / 100.0, len(launched)))
        for i, r in enumerate(launched):
            print('   launch %2d: wave lifetime max %.2f  min %.2f us; first start -> last end %.2f us; gap after the previous launch %.2f us' % (
                i, r[16] / 100.0, r[17] / 100.0, (r[19] - r[18]) / 100.0, (r[18] - launched[i - 1][19]) / 100.0 if i else 0.0))
    sys.exit(0)
for lo, hi in groups:
    tot = sum(v[lo:hi])
    for n, c in zip(names[lo:hi], v[lo:hi]):
        if c:
            print('%-40s %6.1f %%   %8.0f cycles/tile/wave' % (n, 100.0 * c / tot, c / (4 * 256 * tiles)))
