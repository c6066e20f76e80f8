"""Diagnostic driver: bf16 encoder forward (+ optional loss/grad) on a B x 16384 batch, for
rocprofv3 counter passes on the block kernels.  Usage: fwdonly.py B reps [grad]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from audio_style_transfer_amd.engine import StyleEngine
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
eng = StyleEngine(B, 16384, [29], list(range(30)), precision='bf16')
x = torch.randn(B, 16384, device='cuda') * 40
for _ in range(reps):
    eng.forward(x)
torch.cuda.synchronize()
print('ok')
