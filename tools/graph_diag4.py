"""Diagnostic: engine A (clips 0..7) captures its AdamLoop graph; then one action; then A's loop
steps 4 times.  Actions: none / empty_cache / a trivial torch graph capture / engine B (clips
8..15) created / B + make_problem / B + eager AdamLoop step / B + graph AdamLoop.  Prints per
step the mean loss, max |x|, max |grad| of A.  Each case in a fresh process.

  python tools/graph_diag4.py"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, torch
sys.path.insert(0, sys.argv[1])
import bench
from audio_style_transfer_amd.engine import AdamLoop, StyleEngine
act = sys.argv[2]
dev = torch.device('cuda', 0)
mk = lambda: StyleEngine(8, 16384, [29], list(range(30)), precision='split', device=dev, lambd=100.0)
ea = mk()
la = AdamLoop(ea, bench.make_problem(ea, list(range(8)), 16384, dev), lr=2.0, graph=True)
keep = []
if act == 'empty_cache':
    torch.cuda.empty_cache()
elif act == 'torch_graph':
    t = torch.zeros(1024, device=dev); g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        t.add_(1)
    keep += [t, g]
elif act != 'none':
    eb = mk(); keep.append(eb)
    if act != 'create':
        xb = bench.make_problem(eb, list(range(8, 16)), 16384, dev); keep.append(xb)
        if act in ('eager', 'graph'):
            lb = AdamLoop(eb, xb, lr=2.0, graph=act == 'graph'); keep.append(lb)
            lb.step()
torch.cuda.synchronize()
out = []
for _ in range(4):
    la.step()
    torch.cuda.synchronize()
    out.append('%.4g/%.4g/%.3g' % (float(la.parts[:, 0].mean()), float(la.x.abs().max()), float(la.grad.abs().max())))
print('%-12s loss/max|x|/max|grad|: %s' % (act, ' '.join(out)), flush=True)
'''
for act in ('none', 'empty_cache', 'torch_graph', 'create', 'problem', 'eager', 'graph'):
    r = subprocess.run([sys.executable, '-c', CHILD, ROOT, act], capture_output=True, text=True,
                       timeout=240)
    print(r.stdout.strip() or r.stderr[-1500:], flush=True)
