"""Diagnostic: AdamLoop graph replay as the FIRST use of a fresh engine in a fresh process, at
bench length, for several batch sizes; per step: mean loss, Adam step counter, max |x|,
max |grad|, and the clips whose loss is not finite.  Each case runs in its own process.

  python tools/graph_diag2.py"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, torch
sys.path.insert(0, sys.argv[1])
import bench
from audio_style_transfer_amd.engine import AdamLoop, StyleEngine
B, graph, pre = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
dev = torch.device('cuda', 0)
e = StyleEngine(B, 16384, [29], list(range(30)), precision='split', device=dev, lambd=100.0)
x = bench.make_problem(e, list(range(B)), 16384, dev)
if pre:   # one eager loss_grad first
    e.loss_grad(x.clone())
lp = AdamLoop(e, x, lr=2.0, graph=bool(graph))
out = []
for _ in range(3):
    lp.step()
    torch.cuda.synchronize()
    p = lp.parts[:, 0]
    out.append((round(float(p.mean()), 4), int(lp.step_dev.item()), round(float(lp.x.abs().max()), 3),
                float(lp.grad.abs().max()), torch.nonzero(~torch.isfinite(p)).flatten().tolist()[:8]))
print('B %d graph %d pre %d: %s' % (B, graph, pre, out), flush=True)
'''
for B, graph, pre in ((16, 1, 0), (4, 1, 0), (16, 1, 1), (16, 0, 0), (256, 1, 0)):
    r = subprocess.run([sys.executable, '-c', CHILD, ROOT, str(B), str(graph), str(pre)],
                       capture_output=True, text=True, timeout=240)
    print(r.stdout.strip() or r.stderr[-1500:], flush=True)
