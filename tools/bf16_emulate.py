"""CPU emulation of the bf16 path's rounding points (numpy + torch bf16 casts): attributes the
bf16 gradient error to forward activation rounding, weight rounding and backward-chain rounding.
Used to justify the bf16 tolerances in tests/test_gpu_parity.py."""
import sys; import os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import astyle_oracle as O
from audio_style_transfer_amd.weights import synthetic_weights, synthetic_clips
W = synthetic_weights(0)
def bf(a):  # RNE round to bf16
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(torch.bfloat16).to(torch.float32)
    return t.numpy().astype(np.float64)
T = 2048
xc = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0])
x = O.mu_law_numpy(synthetic_clips(1, T, 42)[0]) + np.random.default_rng(7).normal(0, 4, T)
def run(fwd_r, bwd_r, wr, nb=30, tap=29):
    Wq = {k: (bf(v) if (wr and ('dilated' in k or 'res' in k) and k.endswith('/W')) else v.astype(np.float64)) for k, v in W.items()}
    def enc(xx, R):
        xs = (xx/128.)[:, None]
        e = R(O.conv1d_same(xs, Wq['ae_startconv/W'], Wq['ae_startconv/biases'], 1))
        es, us = [e], []
        for l in range(nb):
            d = O.dilation_of(l)
            u = O.conv1d_same(R(O.relu(e)), Wq['ae_dilatedconv_%d/W'%(l+1)], Wq['ae_dilatedconv_%d/biases'%(l+1)], d)
            v = R(O.relu(u))
            e = R(e + O.conv1d_same(v, Wq['ae_res_%d/W'%(l+1)], Wq['ae_res_%d/biases'%(l+1)], 1))
            es.append(e); us.append(u)
        return es, us
    ident = lambda a: a
    es_c, _ = enc(xc, ident)
    phi = es_c[tap+1]
    es, us = enc(x, bf if fwd_r else ident)
    R = bf if bwd_r else ident
    g = R(10*2*(es[tap+1]-phi)/phi.size)
    for l in reversed(range(tap+1)):
        d = O.dilation_of(l)
        gv = O.conv1d_same_bwd(g, Wq['ae_res_%d/W'%(l+1)], 1)
        gu = R(gv*(us[l]>0))
        gh = O.conv1d_same_bwd(gu, Wq['ae_dilatedconv_%d/W'%(l+1)], d)
        g = R(g + gh*(es[l]>0))
    return O.conv1d_same_bwd(g, Wq['ae_startconv/W'], 1)[:,0]/128
ref = run(False, False, False)
for f, b, w in [(True, False, False), (False, True, False), (False, False, True), (True, True, True)]:
    g = run(f, b, w)
    print('fwd_bf16', f, 'bwd_bf16', b, 'w_bf16', w, 'grad relL2 %.4f' % (np.linalg.norm(g-ref)/np.linalg.norm(ref)))
