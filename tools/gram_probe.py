"""Diagnostic for the Gram backward's per-process timing: one B = 256,
T = 16384 split engine, a few loss+grad evaluations; run under rocprofv3 (kernel trace and/or
--pmc) to read k_gram_bwd_s's duration and counters for this process.  ASTYLE_DOOP selects D
in place (0) or out of place (1).  Prints the engine's workspace and the step times."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from audio_style_transfer_amd.engine import StyleEngine

B, T = int(os.environ.get('PROBE_B', 256)), 16384
eng = StyleEngine(B, T, [29], list(range(30)), precision='split')
g = torch.Generator().manual_seed(1)
eng.set_targets(torch.randn(T, 128, generator=g) * 0.1, torch.randn(*eng.style_shape, generator=g) * 0.01)
x = (torch.rand(B, T, generator=g) * 255 - 127.5).cuda()
ts = []
for _ in range(int(os.environ.get('PROBE_N', 4))):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    eng.loss_grad(x)
    torch.cuda.synchronize(); ts.append((time.perf_counter() - t0) * 1e3)
print('DOOP=%s step ms %s' % (os.environ.get('ASTYLE_DOOP', '1'), ' '.join('%.1f' % t for t in ts)), flush=True)
