#!/usr/bin/env python
"""Benchmark: style-transfer iters/sec on a 256x16384-sample batch, 30-layer WaveNet encoder
(BASELINE.json metric; workload = configs[2]: 256 clips x 16384 samples per GPU, channel-wise
Gram over all 30 layers, content layer 29, lambda 100, gamma 0).

One step = one loss+grad evaluation of every clip (encoder fwd -> Gram -> losses -> backward
to the audio, ast_loss_grad) + the fused Adam update of the audio (ast_adam_step_dev), inputs
already resident in HBM, replayed from a captured HIP graph (--graph 1, default).

Precision (the headline): 'split' = configs[2] as stated with the reference's fp32 encoder
arithmetic kept: fp32 storage, encoder GEMMs on split-fp16 MFMA (each fp32 operand as two
fp16 halves, 22 significant bits, fp32 accumulation), Gram on bf16 MFMA.  Its gradient is
checked live against the committed fp64 oracle gradient (tests/golden) on every run, beside
the fp32 and bf16 modes' (side keys).

N GPUs = N processes, one per GPU, each owning its own 256 clips: weak scaling, no collective
in the step; the barrier/max-over-ranks timing is the only cross-rank traffic.
`python bench.py --gpus N` starts the N ranks itself (torch.distributed.run, before any GPU
call) unless it already runs under a launcher (WORLD_SIZE set, which must equal N).

Prints ONE JSON line on rank 0.  value = (clips processed by all ranks / 256) / seconds.
"""
from __future__ import annotations

import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP32_MFMA_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: f32 MFMA (= vector) peak
F16_MFMA_PEAK_TFLOPS = 2500.0     # dense bf16 / fp16
HBM_PEAK_GBS = 8000.0
METRIC = 'style-transfer iters/sec, 256x16384-sample batch, 30-layer WaveNet encoder'
PREC_NOTE = {
    'split': 'fp32 storage; encoder GEMMs on split-fp16 MFMA (two fp16 halves per fp32 operand, '
             'three products, fp32 accumulation); Gram on bf16 MFMA (two-term bf16 operands)',
    'fp32': 'fp32 storage + fp32 MFMA (v_mfma_f32_32x32x2_f32)',
    'bf16': 'bf16 storage + bf16 MFMA, fp32 accumulation (bf16 activations through 30 residual '
            'blocks: ~10 % gradient error, see grad_rel_l2)',
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--clips', type=int, default=256, help='clips per GPU (batch)')
    ap.add_argument('--T', type=int, default=16384)
    ap.add_argument('--precision', default='split', choices=['split', 'fp32', 'bf16'])
    ap.add_argument('--side-steps', type=int, default=3,
                    help='N=1 side keys: steps of the fp32 / bf16 modes, the device L-BFGS-B mode '
                         'and the 1-clip configs[1] lines (0 = off)')
    ap.add_argument('--gatys', action='store_true',
                    help='configs[4]: Gatys [L,128,128] Gram instead of the channel-wise one')
    ap.add_argument('--lr', type=float, default=2.0)
    ap.add_argument('--groups', type=int, default=1,
                    help='clip groups per GPU run concurrently (engine.AdamGroups: one engine, '
                         'stream and 1/G of the CUs each, phase-shifted so one group\'s Gram '
                         'kernels overlap another\'s block kernels); 1 = one engine')
    ap.add_argument('--graph', type=int, default=1,
                    help='1: replay the step from a captured HIP graph (default); 0: eager launches')
    ap.add_argument('--cpu-baseline-seconds', type=float, default=15.0,
                    help='CPU baseline sample budget (0 disables)')
    ap.add_argument('--traffic-json', default=None,
                    help='per-launch HBM bytes measured by rocprofv3 --pmc (see DESIGN.md; default '
                         'profiles/traffic.json, profiles/traffic_gatys.json with --gatys)')
    ap.add_argument('--engine', default='audio_style_transfer_amd.engine:StyleEngine',
                    help='module:Class of the engine (tests substitute a CPU stand-in)')
    ap.add_argument('--backend', default='nccl', help='torch.distributed backend for N > 1')
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------- launcher
def launch(argv):
    """--gpus N without a launcher: start N ranks under torch.distributed.run as a child
    process (nothing here has touched the GPU) and return its exit code (shard.launch_ranks)."""
    from audio_style_transfer_amd.shard import launch_ranks
    return launch_ranks(parse(argv).gpus, [os.path.abspath(__file__)], argv)


# ----------------------------------------------------------------------------- ranks
def dist_setup(args):
    import torch
    ws = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if args.backend == 'nccl':
        torch.cuda.set_device(local)
        dev = torch.device('cuda', local)
    else:
        dev = torch.device('cpu')
    if ws > 1:
        import torch.distributed as dist
        if args.backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group(args.backend)
    return ws, rank, dev


def barrier(ws):
    if ws > 1:
        import torch.distributed as dist
        dist.barrier()


def sync(dev):
    import torch
    if dev.type == 'cuda':
        torch.cuda.synchronize(dev)


def engine_class(spec):
    mod, cls = spec.split(':')
    return getattr(importlib.import_module(mod), cls)


def make_problem(eng, clips, T, dev):
    """Synthetic per-clip targets for the global clip indices `clips`: content
    clip c_g, style clip s_g; phi_c = emb_c(c_g); phi_s = l2norm(G^(c_g) + G^(s_g) - G^(c_g))
    (methods.py:207-212 with one clip per file); x0 = c_g + 4 N(0,1) (seeded per clip)."""
    import torch
    from audio_style_transfer_amd.shard import shard_inputs
    cont, sty, x0 = shard_inputs(clips, T)
    cont = torch.tensor(cont, device=dev)
    sty = torch.tensor(sty, device=dev)
    phi_c, g_c = eng.embeds(cont)
    _, g_s = eng.embeds(sty, content=False)
    phi = g_c + g_s - g_c
    phi = phi / phi.pow(2).sum(dim=(-2, -1), keepdim=True).clamp_min(1e-12).sqrt()
    eng.set_targets(phi_c, phi)
    return torch.tensor(x0, device=dev)


def run(args, Eng, precision, steps, warmup, ws, rank, dev, graph, clips=None, gatys=None,
        groups=1):
    """Build the engine(s), warm up, time `steps` steps (barrier + sync on both sides, max over
    ranks).  A step is one AdamLoop step (ast_loss_grad + device-counter Adam), replayed from
    a captured HIP graph when `graph`; with groups > 1 one AdamGroups step (G engines of B / G
    clips, phase-shifted on G streams: every clip still takes one full step).  The per-kernel-
    family breakdown comes from HIP events of 2 extra eager steps of one engine (events are not
    recorded inside a graph).  Returns (seconds, engine timing dict, first loss, last loss,
    (non-finite clips, range-flagged clips), clips in the timed engine)."""
    import torch
    from audio_style_transfer_amd.engine import AdamGroups, AdamLoop
    from audio_style_transfer_amd.shard import clip_range, max_over_ranks
    B = clips or args.clips
    T = args.T
    G = groups if (groups > 1 and dev.type == 'cuda' and graph and B % groups == 0) else 1
    mine = list(clip_range(ws * B, ws, rank))
    Bg = B // G
    engs, xs = [], []
    for g in range(G):
        e = Eng(Bg, T, [29], list(range(30)), precision=precision, device=dev, lambd=100.0,
                gatys=args.gatys if gatys is None else gatys)
        engs.append(e)
        xs.append(make_problem(e, mine[g * Bg:(g + 1) * Bg], T, dev))
    if G > 1:
        loop = AdamGroups(engs, xs, lr=args.lr)
        parts_of = lambda: torch.cat(loop.parts)
        grad_of = lambda: torch.cat(loop.grad)
    else:
        loop = AdamLoop(engs[0], xs[0], lr=args.lr, graph=graph and dev.type == 'cuda')
        parts_of = lambda: loop.parts
        grad_of = lambda: loop.grad
    for _ in range(warmup):
        loop.step()
    sync(dev)
    first_loss = parts_of()[:, 0].mean().item()
    barrier(ws)
    sync(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        loop.step()
    sync(dev)
    barrier(ws)
    el = time.perf_counter() - t0
    el = max_over_ranks(el, ws, device=dev)
    last_loss = parts_of()[:, 0].mean().item()
    # per-clip flag: the clip's loss parts or gradient hold a NaN / Inf (last step), and the
    # clips whose range flags (sticky over every warm-up and timed step: the loops reset them
    # at their start) report an out-of-range or non-finite evaluation
    pp, gg = parts_of(), grad_of()
    bad = int((~torch.isfinite(pp).all(dim=1) | ~torch.isfinite(gg).all(dim=1)).sum().item())
    flagged = sum(int((e.range_flags() & 7).ne(0).sum().item()) for e in engs) if dev.type == 'cuda' else 0
    eng = engs[0]
    if G > 1:
        eng.set_cu_limit(0)   # the breakdown: one engine's kernels with every CU
    eng.timing(True)
    for _ in range(2):
        if G > 1:
            loop._front(0)
            loop._back(0)
        else:
            loop._eager()
    sync(dev)
    tm = eng.timing_read()
    eng.timing(False)
    dop = getattr(eng, 'd_out_of_place', None)
    tm['d_out_of_place'], tm['d_tuned_ms'] = dop(with_times=True) if dop else (None, None)
    del loop, xs
    for e in engs:
        e.close()
    if dev.type == 'cuda':
        torch.cuda.empty_cache()
    return el, tm, first_loss, last_loss, (bad, flagged), Bg


def grad_check(Eng, precision, dev, gatys=False):
    """d loss / d x of one 2048-sample clip against the committed fp64 oracle gradient
    (tests/golden: 'ours' = 30 style layers, content layer 25; 'gatys' (--gatys) = 30 Gatys
    style layers, content layer 29; the oracle's own targets, stored in fp32)."""
    import torch
    tag = 'gatys' if gatys else 'ours'
    g = np.load(os.path.join(ROOT, 'tests', 'golden', 'oracle_T2048.npz'))
    tg = np.load(os.path.join(ROOT, 'tests', 'golden', 'oracle_T2048_targets.npz'))
    eng = Eng(1, 2048, [29] if gatys else [25], list(range(30)), precision=precision, device=dev,
              lambd=100.0, gatys=gatys)
    eng.set_targets(torch.tensor(tg[tag + '_phi_c']), torch.tensor(tg[tag + '_phi_s']))
    parts, grad = eng.loss_grad(torch.tensor(g[tag + '_x'][None], dtype=torch.float32, device=dev))
    grad = grad.cpu().double().numpy()[0]
    loss = float(parts[0, 0])
    eng.close()
    ref = g[tag + '_grad']
    return {'grad_check_case': tag,
            'grad_rel_l2': float(np.linalg.norm(grad - ref) / np.linalg.norm(ref)),
            'loss_rel': abs(loss - float(g[tag + '_parts'][0])) / abs(float(g[tag + '_parts'][0]))}


def available_cores():
    """Host cores this process may use: its CPU affinity, capped by a cgroup CPU quota when one
    is set (on the GPU box the affinity lists the whole host while the job's quota is its share);
    returns (cores to use, detail)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            q, per = f.read().split()[:2]
            if q != 'max':
                quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            with open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us') as f:
                q = int(f.read())
            with open('/sys/fs/cgroup/cpu/cpu.cfs_period_us') as f:
                per = int(f.read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    use = aff if quota is None else max(1, min(aff, int(quota)))
    return use, {'sched_getaffinity': aff, 'os_cpu_count': os.cpu_count(),
                 'cgroup_cpu_quota': quota, 'OMP_NUM_THREADS': os.environ.get('OMP_NUM_THREADS')}


def cpu_baseline(T, budget_s, gatys=False):
    """The reference's CPU path on this host's cores, on a bounded sample of the same workload:
    scipy L-BFGS-B (methods.py:132-137, ScipyOptimizerInterface: float64 on the host, one loss +
    grad evaluation per call) driving the torch-CPU fp32 restatement of the loss
    (oracle/torch_restatement.py: F.conv1d forward, autograd backward; TensorFlow is absent
    here) for one 16384-sample clip, timed over whole evaluations including the optimiser's
    host update; scaled to the 256-clip batch (clips are independent problems)."""
    import torch
    from scipy.optimize import minimize
    from oracle import torch_restatement as TR
    from audio_style_transfer_amd.weights import synthetic_weights, synthetic_clips
    from audio_style_transfer_amd.utils import mu_law_numpy
    cores, detail = available_cores()
    torch.set_num_threads(cores)
    W = synthetic_weights(0)
    kw = dict(cont_ids=[29], style_ids=list(range(30)), gatys=gatys)
    xc = mu_law_numpy(synthetic_clips(1, T, 1000)[0]).astype(np.float64)
    phi_c = np.zeros((T, 128), np.float32)
    phi_s = np.zeros((30, 128, 128) if gatys else (128, 30, 30), np.float32)
    x = xc + np.random.default_rng(0).normal(0, 4, T)
    t0 = time.time()
    TR.cpu_step(x, W, phi_c=phi_c, phi_s=phi_s, **kw)      # warm-up (allocator, threads)
    t_warm = time.time() - t0
    nfev = [0]

    def fg(v):
        nfev[0] += 1
        f, g = TR.cpu_step(v, W, phi_c=phi_c, phi_s=phi_s, **kw)
        return f, g.double().numpy()
    k = int(max(3, min(200, budget_s / max(t_warm, 1e-3))))
    t0 = time.time()
    res = minimize(fg, x, jac=True, method='L-BFGS-B', options={'maxfun': k, 'maxiter': k})
    el = time.time() - t0
    clip_evals_per_s = nfev[0] / el
    return {'value': clip_evals_per_s / 256.0, 'unit': 'iters/s (256x%d batch)' % T,
            'cores': int(cores), 'cores_detail': detail, 'kind': 'port',
            'sample': 'scipy L-BFGS-B (float64 host, m 10) over the torch-CPU fp32 restatement of '
                      'the reference loss (conv1d forward + autograd backward, 30 blocks, %s L=30, '
                      'STFT regulariser evaluated as TF does): %d loss+grad evaluations (%d L-BFGS-B '
                      'iterations) of one %d-sample clip in %.1f s = %.3f clip-evals/s = %.3f s per '
                      'evaluation; scaled to the 256-clip batch'
                      % ('Gatys Gram' if gatys else 'ours-Gram', nfev[0], res.nit, T, el,
                         clip_evals_per_s, el / max(nfev[0], 1)),
            'clip_evals_per_s': clip_evals_per_s,
            'config1_iters_per_s': clip_evals_per_s,
            'note': 'a reported baseline, not the target; configs[1] (one clip) runs at '
                    'config1_iters_per_s on the same cores'}


def lib_sha16():
    """sha256 (16 hex) of the libastyle.so this process loads: ties profiles/traffic.json's PMC
    bytes to the binary they were measured on."""
    import hashlib
    from audio_style_transfer_amd import _lib
    try:
        with open(_lib.LIB_PATH, 'rb') as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        return None


def mfma16_mode():
    """ASTYLE_MFMA16 as the library reads it (api.hip mfma16_mode): which split block kernels run
    on 16x16x32 fragments -- 0 neither, 1 both, 2 the backward (default), 3 the forward."""
    try:
        v = int(os.environ.get('ASTYLE_MFMA16', '2'))
    except ValueError:
        v = 0   # (atoi of a non-number)
    return v if 0 <= v <= 3 else 2


def block_roofline(precision, B, T, fwd_ms, bwd_ms, traffic, ms_per_step, gram_ms, L=30,
                   nblk=30, B_step=None):
    """Roofline of the block kernels.  Per launch (all B clips): algorithmic bytes
    fwd = read e_l + write e_{l+1} (2A) + the relu-mask words (16 B per row written, 16 B of
    the previous layer's read); bwd = read the chain and D_l, write the chain (3A) + 32 B of
    mask words per row; A = B T 128 x element size.  FLOP = 131072 per row (2 (384 + 128) 128);
    the split mode executes three MFMA products per FLOP.  Each kernel's binding fraction is
    the larger of its HBM and executed-MFMA fractions.  The top-level object is the dominant
    kernel (the one with more time per step); 'step' is the step-level HBM fraction:
    algorithmic bytes of the blocks and the Gram per step / ms_per_step / 8 TB/s."""
    esz = 2.0 if precision == 'bf16' else 4.0
    rows = float(B) * T
    A = rows * 128 * esz
    fbytes = 2 * A + 32 * rows
    bbytes = 3 * A + 32 * rows
    flops = 131072.0 * rows
    mult = 3.0 if precision == 'split' else 1.0
    peak = FP32_MFMA_PEAK_TFLOPS if precision == 'fp32' else F16_MFMA_PEAK_TFLOPS
    tf = traffic or {}

    def one(name, ms, nbytes, tb):
        mf = flops * mult / (ms * 1e-3) / 1e12
        gb = nbytes / (ms * 1e-3) / 1e9
        d = {'kernel': name, 'launch_ms': ms, 'algorithmic_bytes': nbytes,
             'algorithmic_flops': flops, 'executed_mfma_flops': flops * mult, 'mfma_TFLOPs': mf,
             'mfma_frac': mf / peak, 'hbm_GBs': gb, 'hbm_frac': gb / HBM_PEAK_GBS, 'traffic': tb}
        if d['mfma_frac'] >= d['hbm_frac']:
            d.update(bound='mfma', achieved=mf, peak=peak, unit='TFLOP/s', frac=d['mfma_frac'])
        else:
            d.update(bound='hbm', achieved=gb, peak=HBM_PEAK_GBS, unit='GB/s', frac=d['hbm_frac'])
        return d

    suffix = {'split': '_s', 'bf16': '_c', 'fp32': ''}[precision]
    m16 = mfma16_mode() if precision == 'split' else 0
    f = one('k_block_fwd' + suffix + ('16' if m16 in (1, 3) else ''), fwd_ms, fbytes, tf.get('fwd'))
    b = one('k_block_bwd' + suffix + ('16' if m16 in (1, 2) else ''), bwd_ms, bbytes, tf.get('bwd'))
    dom = b if bwd_ms >= fwd_ms else f
    roof = {k: dom[k] for k in ('bound', 'achieved', 'peak', 'unit', 'frac', 'traffic', 'kernel')}
    roof['note'] = ('dominant kernel (%.1f of %.1f ms/step in the blocks); achieved = algorithmic '
                    'bytes (or executed MFMA flops) per launch / its HIP-event launch time; traffic = '
                    'PMC HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, profiles/traffic.json, '
                    'null unless measured on this libastyle.so)' % (nblk * dom['launch_ms'],
                                                                      nblk * (fwd_ms + bwd_ms)))
    step_bytes = (nblk * (fbytes + bbytes) + 3 * L * A) * (float(B_step or B) / B)
    roof['fwd'] = f
    roof['bwd'] = b
    roof['step'] = {'algorithmic_bytes': step_bytes, 'ms': ms_per_step,
                    'achieved_GBs': step_bytes / (ms_per_step * 1e-3) / 1e9,
                    'frac': step_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS,
                    'note': '%d block fwd + bwd launches and the Gram (fwd reads L A, bwd reads '
                            'L A and writes L A, L = %d) per step' % (nblk, L)}
    return roof


def gram_roofline(precision, gatys, B, T, L, fwd_ms, bwd_ms, traffic):
    """The Gram kernels against both roofs (the north_star asks for their MFMA
    utilisation against the gfx950 peak).  Bytes per launch: the forward reads the L tapped
    tensors, the backward reads and writes them (D in place).  FLOP per time row:
    algorithmic = the reference's matmuls (methods.py:68-76): ours G_c = E_c E_c^T per channel,
    2 L^2 128; Gatys G_l = F_l^T F_l per layer, 2 128^2 L (forward and backward alike).
    executed = what the MFMA pipe issues in the split kernels (gram_split.hip, gram_gatys.hip):
    three bf16 products per product; ours pads L to 32 tensors, and its half-row backward
    (k_gram_bwd_h) computes every 16x16x32 tile on 8 real rows (columns 8..15 repeat rows
    0..7); the Gatys forward computes the 10 upper 32x32 tiles of the symmetric 128 x 128 (10/16).
    mfma_frac_at_hbm_roof = executed FLOP per HBM byte x 8 TB/s / the bf16 peak: the MFMA
    utilisation these kernels would reach at the HBM roofline, the ceiling of mfma_frac."""
    esz = 2.0 if precision == 'bf16' else 4.0
    rows = float(B) * T
    A = rows * 128 * esz
    tf = traffic or {}
    split = precision == 'split'
    peak = FP32_MFMA_PEAK_TFLOPS if precision == 'fp32' else F16_MFMA_PEAK_TFLOPS
    if gatys:
        alg = 2.0 * 128 * 128 * L
        ex_f = 3 * alg * 10 / 16 if split else None
        ex_b = 3 * alg if split else None
        names = ('k_gatys_fwd_s', 'k_gatys_bwd_s2') if split else ('gatys fwd', 'gatys bwd')
    else:
        alg = 2.0 * L * L * 128
        ex_f = 3 * 2.0 * 32 * 32 * 128 if split else None
        half = os.environ.get('ASTYLE_GRAM_BWD_H', '1') != '0'
        ex_b = 3 * 2.0 * 32 * 32 * 128 * (2 if half else 1) if split else None
        names = ('k_gram_fwd_s', 'k_gram_bwd_h' if half else 'k_gram_bwd_s') if split else \
            ('gram fwd', 'gram bwd')

    def one(name, ms, nbytes, ex, tb):
        sec = ms * 1e-3
        d = {'kernel': name, 'launch_ms': ms, 'algorithmic_bytes': nbytes,
             'achieved_GBs': nbytes / sec / 1e9, 'hbm_frac': nbytes / sec / 1e9 / HBM_PEAK_GBS,
             'traffic': tb, 'algorithmic_flops': alg * rows,
             'algorithmic_TFLOPs': alg * rows / sec / 1e12}
        if ex is not None:
            d.update(executed_mfma_flops=ex * rows, mfma_TFLOPs=ex * rows / sec / 1e12,
                     mfma_frac=ex * rows / sec / 1e12 / peak,
                     mfma_frac_at_hbm_roof=ex * rows / nbytes * HBM_PEAK_GBS / 1e3 / peak)
        return d
    f = one(names[0], fwd_ms, L * A, ex_f, tf.get('gram_fwd'))
    b = one(names[1], bwd_ms, 2 * L * A, ex_b, tf.get('gram_bwd'))
    return {'bound': 'hbm', 'peak': HBM_PEAK_GBS, 'mfma_peak_TFLOPs': peak,
            'fwd_achieved_GBs': f['achieved_GBs'], 'bwd_achieved_GBs': b['achieved_GBs'],
            'fwd_frac': f['hbm_frac'], 'bwd_frac': b['hbm_frac'],
            'fwd_traffic': f['traffic'], 'bwd_traffic': b['traffic'],
            'fwd_mfma_frac': f.get('mfma_frac'), 'bwd_mfma_frac': b.get('mfma_frac'),
            'fwd': f, 'bwd': b,
            'note': ('HBM-bound: %.0f / %.0f algorithmic flop per HBM byte (fwd / bwd; SURVEY F9), '
                     'so even at 8 TB/s the MFMA utilisation stays at mfma_frac_at_hbm_roof '
                     '(executed, %s) -- the north_star\'s >= 50 %% MFMA is out of reach for this '
                     'Gram; the HBM fractions are its roofline'
                     % (alg / (128 * esz * L), alg / (2 * 128 * esz * L),
                        'fwd %.2f / bwd %.2f' % (f['mfma_frac_at_hbm_roof'], b['mfma_frac_at_hbm_roof'])
                        if split else 'n/a'))}


def rank_main(args):
    import torch
    ws, rank, dev = dist_setup(args)
    Eng = engine_class(args.engine)
    B, T, L = args.clips, args.T, 30
    el, tm, first_loss, last_loss, bad, Bt = run(args, Eng, args.precision, args.steps, args.warmup,
                                                 ws, rank, dev, bool(args.graph), groups=args.groups)
    side = {}
    if ws == 1 and args.side_steps > 0 and dev.type == 'cuda':
        for p in ('fp32', 'bf16', 'split'):
            if p == args.precision:
                continue
            e2, tm2, _, _, _, _ = run(args, Eng, p, args.side_steps, 1, ws, rank, dev, bool(args.graph))
            calls = max(tm2['calls'], 1)
            side[p + '_mode'] = {'value': B * args.side_steps / 256.0 / e2, 'unit': 'iters/s',
                                 'steps': args.side_steps, 'precision': PREC_NOTE[p],
                                 'kernels_ms_per_step': {k[:-3]: tm2[k] / calls for k in
                                                         ('block_fwd_ms', 'block_bwd_ms',
                                                          'gram_fwd_ms', 'gram_bwd_ms', 'other_ms')},
                                 **grad_check(Eng, p, dev, args.gatys)}
        for p in ('split', 'fp32'):     # configs[1]: one 16384-sample clip
            e1, _, _, _, _, _ = run(args, Eng, p, 10 * args.side_steps, 2, ws, rank, dev,
                                 bool(args.graph), clips=1, gatys=False)
            side['config1_%s' % p] = {'value': 10 * args.side_steps / e1, 'unit': 'iters/s',
                                      'note': 'configs[1]: 1 clip x %d, channel-wise Gram, 30 '
                                              'blocks, %s' % (T, PREC_NOTE[p])}
        side['lbfgs_mode'] = run_lbfgs(args, Eng, 2 * args.side_steps, dev)
        if not args.gatys and args.engine == ap_default_engine():
            side['reference_protocol'] = reference_protocol(T, dev)
    if rank != 0:
        barrier(ws)
        return None
    value = ws * B * args.steps / 256.0 / el
    calls = max(tm['calls'], 1)
    nblk = max(tm['blocks'], 1)
    fwd_ms = tm['block_fwd_ms'] / (calls * nblk)
    bwd_ms = tm['block_bwd_ms'] / (calls * nblk)
    traffic = None
    sha = lib_sha16()
    try:
        tpath = args.traffic_json or os.path.join(
            ROOT, 'profiles', 'traffic_gatys.json' if args.gatys else 'traffic.json')
        with open(tpath) as f:
            tj = json.load(f)
        if (tj.get('precision') == args.precision and tj.get('clips') == Bt and tj.get('T') == T
                and tj.get('gatys', False) == args.gatys and tj.get('lib_sha16') == sha):
            traffic = {'fwd': tj['fwd_bytes_per_launch'], 'bwd': tj['bwd_bytes_per_launch'],
                       'gram_fwd': tj.get('gram_fwd_bytes_per_launch'),
                       'gram_bwd': tj.get('gram_bwd_bytes_per_launch'), 'source': tj.get('source')}
    except Exception:
        traffic = None
    gram_fwd_ms = tm['gram_fwd_ms'] / calls
    gram_bwd_ms = tm['gram_bwd_ms'] / calls
    # the per-family breakdown is one engine's eager steps: Bt clips (B / groups)
    gbytes = L * Bt * T * 128 * (2.0 if args.precision == 'bf16' else 4.0)
    out = {
        'metric': METRIC, 'value': value, 'unit': 'iters/s', 'n_gpus': ws, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': el / args.steps * 1e3,
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
        'dtype': {'split': 'fp32 (split-f16 MFMA)', 'fp32': 'fp32', 'bf16': 'bf16'}[args.precision],
        'data': 'synthetic (seeded sinusoid+noise clips, seeded uniform_unit_scaling weights)',
        'config': {'workload': ('configs[4]: %dx%d clips per GPU, 30-block encoder, Gatys Gram '
                                if args.gatys else
                                'configs[2]: %dx%d clips per GPU, 30-block encoder, ours-Gram ')
                               % (B, T) + 'L=30, cont_lyrs [29], lambd 100, gamma 0, Adam step',
                   'global_batch_clips': ws * B, 'T': T, 'parallelism': 'clip-sharded x%d' % ws,
                   'precision': args.precision, 'precision_detail': PREC_NOTE[args.precision],
                   'hip_graph': bool(args.graph),
                   'clip_groups': B // Bt,
                   'gram_d': {True: 'out of place', False: 'in place', None: None}[tm.get('d_out_of_place')],
                   'gram_d_tuned_ms': tm.get('d_tuned_ms'),
                   'breakdown_engine_clips': Bt},
        'clip_iters_per_s': value * 256.0,
        'roofline': block_roofline(args.precision, Bt, T, fwd_ms, bwd_ms, traffic,
                                   el / args.steps * 1e3, gram_fwd_ms + gram_bwd_ms, B_step=B),
        'lib_sha16': sha,
        'kernels_ms_per_step': {'block_fwd': tm['block_fwd_ms'] / calls,
                                'block_bwd': tm['block_bwd_ms'] / calls,
                                'gram_fwd': gram_fwd_ms, 'gram_bwd': gram_bwd_ms,
                                'other': tm['other_ms'] / calls},
        'gram_roofline': gram_roofline(args.precision, args.gatys, Bt, T, L, gram_fwd_ms,
                                       gram_bwd_ms, traffic),
        'loss_first_last': [first_loss, last_loss],
        'nonfinite_clips': bad[0],
        'range_flagged_clips': bad[1],
    }
    if dev.type == 'cuda':
        out.update(grad_check(Eng, args.precision, dev, args.gatys))
    out.update(side)
    if ws == 1 and args.cpu_baseline_seconds > 0:
        out['cpu_baseline'] = cpu_baseline(T, args.cpu_baseline_seconds, args.gatys)
        rp = out.get('reference_protocol')
        if rp:   # the drop-in's one-clip rate beside the CPU path's, same protocol
            cpu = out['cpu_baseline']['config1_iters_per_s']
            rp['cpu_baseline_config1_evals_per_s'] = cpu
            rp['config1_scipy_vs_cpu_baseline'] = rp['config1']['scipy']['evals_per_s'] / cpu
    print(json.dumps(out), flush=True)
    barrier(ws)
    return out


def ap_default_engine():
    return parse([]).engine


def reference_protocol(T, dev, maxiter=100):
    """The drop-in on the reference's own protocol: GatysNet.l_bfgs for one
    epoch (one minimize call, maxiter 100) of ONE clip of T samples from x = 1e-6
    (methods.py:49-54,132-137,164-181), as a user of methods.py runs it: 'scipy' = host scipy
    L-BFGS-B with one H2D copy of x and one D2H copy of the gradient and loss parts per
    evaluation (the reference's ScipyOptimizerInterface round trip); 'device' = the same L-BFGS-B
    in device memory (ast_lbfgs_*).  configs[0]'s taps (stack 0 = style layers 0..9, content
    layer 25) and configs[1]'s (the CLI defaults: style layers 0..29, content layer 29), lambd
    100, gamma 0, split precision, synthetic clips (content seed 1000, style 5000).  host_share
    = 1 - evaluations x device time of one resident ast_loss_grad / epoch wall time: the part
    of the epoch spent in scipy, the copies and Python."""
    import tempfile
    import torch
    from audio_style_transfer_amd.methods import GatysNet
    from audio_style_transfer_amd.weights import synthetic_weights, synthetic_clips
    W = synthetic_weights(0)
    cont, sty = synthetic_clips(1, T, 1000)[0], synthetic_clips(1, T, 5000)[0]
    res = {}
    for tag, stack, cids in (('config0', 0, [25]), ('config1', None, [29])):
        with tempfile.TemporaryDirectory() as d:
            net = GatysNet(d, None, os.path.join(d, 'log'), os.path.join(d, 'fig'), stack=stack,
                           batch_size=T, cont_lyr_ids=cids, weights=W, plots=False)
            phi_c = net.get_embeds(cont)
            phi_s = net.get_embeds(sty, is_content=False)   # one-clip analogy: l2norm(G_s)
            eng = net.engine
            eng.set_targets(torch.as_tensor(phi_c), torch.as_tensor(phi_s))
            xd = torch.full((1, T), 1e-6, device=dev)
            for _ in range(3):
                eng.loss_grad(xd)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                eng.loss_grad(xd)
            torch.cuda.synchronize()
            dev_ms = (time.perf_counter() - t0) / 20 * 1e3
            r = {'style_layers': net.style_lyr_ids[0:1] + ['..'] + net.style_lyr_ids[-1:],
                 'cont_layers': cids, 'device_ms_per_eval': dev_ms}
            for opt in ('scipy', 'device'):
                # an untimed 2-iteration call first: one-time costs (event writer, the device
                # loop's workspace and code objects, scipy's first call) stay out of the epoch
                net.l_bfgs(phi_c, phi_s, 1, 100.0, 0.0, optimizer=opt, maxiter=2,
                           log=lambda *a: None)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                net.l_bfgs(phi_c, phi_s, 1, 100.0, 0.0, optimizer=opt, maxiter=maxiter,
                           log=lambda *a: None)
                torch.cuda.synchronize()
                el = time.perf_counter() - t0
                n = len(net.history)
                r[opt] = {'evals': n, 'seconds_per_epoch': el, 'evals_per_s': n / el,
                          'host_share': max(0.0, 1.0 - n * dev_ms * 1e-3 / el),
                          'final_loss': float(net.history[-1][0])}
            net.engine.close()
        res[tag] = r
    res['note'] = ('GatysNet.l_bfgs, one epoch (maxiter %d) of one %d-sample clip from x = 1e-6, '
                   'wall time incl. per-epoch outputs (ep-0.wav, event file, state.npz); evals = '
                   'loss+grad evaluations of the epoch' % (maxiter, T))
    return res


def run_lbfgs(args, Eng, steps, dev):
    """Side measurement (N=1): the reference's optimiser, scipy's L-BFGS-B restated on the
    device (ast_lbfgs_*), over the same 256-clip workload.  A step is one evaluation of every
    clip (ast_loss_grad) + one ast_lbfgs_step, replayed from a HIP graph; the L-BFGS-B kernel's
    own time comes from HIP events around eager launches on the engine's stream."""
    import ctypes
    import torch
    from audio_style_transfer_amd.engine import LbfgsLoop
    from audio_style_transfer_amd.shard import clip_range
    B, T = args.clips, args.T
    eng = Eng(B, T, [29], list(range(30)), precision=args.precision, device=dev, lambd=100.0,
              gatys=args.gatys)
    x = make_problem(eng, clip_range(B, 1, 0), T, dev)
    loop = LbfgsLoop(eng, maxiter=100, graph=bool(args.graph))
    loop.begin(x.double())
    for _ in range(2):
        loop.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loop.step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    s = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ms = 0.0
    for _ in range(3):
        eng.loss_grad(loop.x, loop.grad, loop.parts)
        e0.record(s)
        eng.lib.ast_lbfgs_step(eng.h, ctypes.c_void_p(loop.ws.data_ptr()),
                               ctypes.c_void_p(loop.x.data_ptr()),
                               ctypes.c_void_p(loop.grad.data_ptr()),
                               ctypes.c_void_p(loop.parts.data_ptr()), eng._stream())
        e1.record(s)
        torch.cuda.synchronize()
        ms += e0.elapsed_time(e1) / 3
    info, _ = loop.state()
    del loop, x
    eng.close()
    torch.cuda.empty_cache()
    return {'value': B * steps / 256.0 / el, 'unit': 'iters/s', 'steps': steps,
            'lbfgs_step_ms': ms, 'clips_running': int((info[:, 0] != 0).sum()),
            'note': 'device L-BFGS-B (scipy semantics: m 10, dcsrch line search, maxiter 100) '
                    'instead of Adam, same workload and precision; one iter = one loss+grad '
                    'evaluation of every clip + the L-BFGS-B update'}


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    rc = launch(argv)
    if rc is not None:
        return rc
    rank_main(parse(argv))
    return 0


if __name__ == '__main__':
    sys.exit(main())
