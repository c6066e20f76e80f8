"""Diagnostic: bf16 encoder forward time per block launch against the batch (clips), normalised
to 256 clips.  Small batches keep a block's input + output inside the 256-MB Infinity Cache, so
the ratio to the full batch separates HBM-bound from issue-bound behaviour."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from audio_style_transfer_amd.engine import StyleEngine
T = 16384
for B in [int(b) for b in (sys.argv[1:] or ['32', '64', '128', '256'])]:
    eng = StyleEngine(B, T, [29], list(range(30)), precision=os.environ.get('PREC', 'split'))
    x = torch.randn(B, T, device='cuda') * 40
    for _ in range(2):
        eng.forward(x)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = max(2, 512 // B)
    s.record()
    for _ in range(reps):
        eng.forward(x)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps / 30
    print('B=%4d  %.4f ms per block launch  (%.4f ms per 256 clips)' % (B, ms, ms * 256 / B), flush=True)
    del eng
    torch.cuda.empty_cache()
