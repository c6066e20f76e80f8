"""Diagnostic: one split forward at B clips x 16384 (run under rocprofv3 --kernel-trace) so the
per-launch durations of the 30 block kernels (dilations 1, 2, .., 512 three times) can be read
from the trace in launch order.  usage: fwd_layers.py [clips] [fwd|bwd]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from audio_style_transfer_amd.engine import StyleEngine
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
mode = sys.argv[2] if len(sys.argv) > 2 else 'fwd'
T = 16384
eng = StyleEngine(B, T, [29], list(range(30)), precision='split')
x = torch.randn(B, T, device='cuda') * 40
if mode == 'bwd':
    eng.set_targets(torch.randn(T, 128) * 0.1, torch.randn(*eng.style_shape) * 0.01)
run = (lambda: eng.loss_grad(x)) if mode == 'bwd' else (lambda: eng.forward(x))
for _ in range(3):
    run()
torch.cuda.synchronize()
print('done')
