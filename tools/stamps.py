"""Diagnostic: per-phase cycle shares of the bf16 block-forward kernel (s_memtime stamps,
libastyle_stamps.so built with -DASTYLE_STAMPS).  Shares, not absolute time, are meaningful."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault('ASTYLE_LIB', os.path.join(ROOT, 'audio_style_transfer_amd', 'libastyle_stamps.so'))
sys.path.insert(0, ROOT)
import torch
from audio_style_transfer_amd.engine import StyleEngine
from audio_style_transfer_amd import _lib
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
eng = StyleEngine(B, 16384, [29], list(range(30)), precision='bf16')
x = torch.randn(B, 16384, device='cuda') * 40
eng.forward(x); torch.cuda.synchronize()
buf = torch.zeros(12, dtype=torch.int64, device='cuda')
lib = _lib.load()
lib.ast_debug_stamps.argtypes = [ctypes.c_void_p]
lib.ast_debug_stamps(ctypes.c_void_p(buf.data_ptr()))
eng.forward(x); torch.cuda.synchronize()
lib.ast_debug_stamps(None)
v = buf.cpu().tolist()
names = ['loop-top vmcnt wait', 'barrier', 'DMA issue', 'GEMM1', 'epilogue1 + mu', 'GEMM2',
         'epilogue2 + stores', '-', '-', '-', '-', '-']
tot = sum(v)
tiles = B * 16384 // 128 * 30 / 256   # tiles per CU over the 30 block launches
for n, c in zip(names, v):
    if c:
        print('%-20s %6.1f %%   %8.0f cycles/tile/wave' % (n, 100.0 * c / tot, c / (4 * 256 * tiles)))
