"""Measure bf16-path error vs the fp64 oracle (prints; used to set test tolerances)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
import numpy as np, torch
from oracle import astyle_oracle as O
from audio_style_transfer_amd.weights import synthetic_weights, synthetic_clips
from audio_style_transfer_amd.engine import StyleEngine
W = synthetic_weights(0)
g = np.load('tests/golden/oracle_T2048.npz')
CASES = {
    'ours': dict(cont_ids=[25], style_ids=list(range(30)), gatys=False, nb_channels=128, cnt_channels=128),
    'c1': dict(cont_ids=[25], style_ids=list(range(10)), gatys=False, nb_channels=128, cnt_channels=128),
    'trunc': dict(cont_ids=[25, 31], style_ids=[3, 7], gatys=False, nb_channels=64, cnt_channels=16),
}
def rel(a, b): return float(np.linalg.norm(np.asarray(a, np.float64) - b) / np.linalg.norm(b))
T = 2048
dev = torch.device('cuda', 0)
for tag, kw in CASES.items():
    xc = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0]); xs = O.mu_law_numpy(synthetic_clips(1, T, 5000)[0])
    phi_c, phi_s = O.targets_from_audio(W, xc, [xs], [xc], **kw)
    x = g[tag + '_x']
    for prec in ['fp32', 'bf16']:
        eng = StyleEngine(1, T, kw['cont_ids'], kw['style_ids'], cnt_channels=kw['cnt_channels'], nb_channels=kw['nb_channels'], weights=W, precision=prec)
        eng.set_targets(torch.tensor(phi_c, dtype=torch.float32), torch.tensor(phi_s, dtype=torch.float32))
        p, gr = eng.loss_grad(torch.tensor(x[None], dtype=torch.float32, device=dev))
        p = p.cpu().numpy()[0]; gr = gr.cpu().numpy()[0]
        rp = g[tag + '_parts']
        print(tag, prec, 'parts rel', [float(abs(p[k]-rp[k])/abs(rp[k])) for k in range(3)], 'grad relL2', rel(gr, g[tag + '_grad']),
              'cos', float(np.dot(gr, g[tag+'_grad'])/np.linalg.norm(gr)/np.linalg.norm(g[tag+'_grad'])))
        # forward extracts
        eng.forward(torch.tensor(x[None], dtype=torch.float32, device=dev))
        nb = O.needed_blocks(kw['cont_ids'], kw['style_ids'])
        ext, _ = O.encoder_forward(x, W, nb, need_bottleneck=31 in kw['cont_ids'])
        print('   ext rel', [round(rel(eng.extract(i).cpu().numpy()[0], ext[i]), 6) for i in [0, 4, 9] + ([24, 29] if nb == 30 else [])])
        ec, es = eng.embeds(torch.tensor(xc[None], dtype=torch.float32, device=dev))
        extc, _ = O.encoder_forward(xc, W, nb, need_bottleneck=31 in kw['cont_ids'])
        print('   emb rel', rel(ec.cpu().numpy()[0], O.content_embeds(extc, kw['cont_ids'], kw['cnt_channels'])),
              rel(es.cpu().numpy()[0], O.style_embeds(extc, kw['style_ids'], False, kw['nb_channels'])))
