#!/usr/bin/env python
"""Benchmark: style-transfer iters/sec on a 256x16384-sample batch, 30-layer WaveNet encoder
(BASELINE.json metric; workload = configs[2]: 256 clips x 16384 samples per GPU, channel-wise
Gram over all 30 layers, content layer 29, lambda 100, gamma 0).

One step = one loss+grad evaluation of every clip (encoder fwd -> Gram -> losses -> backward
to the audio, ast_loss_grad) + the fused Adam update of the audio (ast_adam_step_dev), inputs
already resident in HBM, replayed from a captured HIP graph (--graph 1, default).  N GPUs = N processes (torch.distributed.run), each owning its own
256 clips: weak scaling, no collective in the step; the barrier/max-over-ranks
timing is the only cross-rank traffic.

Prints ONE JSON line on rank 0.  value = (clips processed by all ranks / 256) / seconds.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP32_MFMA_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: f32 MFMA (= vector) peak
BF16_MFMA_PEAK_TFLOPS = 2500.0    # dense bf16
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--clips', type=int, default=256, help='clips per GPU (batch)')
    ap.add_argument('--T', type=int, default=16384)
    ap.add_argument('--precision', default='bf16', choices=['fp32', 'bf16'],
                    help='bf16: bf16 storage + bf16 MFMA, fp32 accumulation (throughput mode); '
                         'fp32: fp32 storage + fp32 MFMA (parity mode)')
    ap.add_argument('--fp32-steps', type=int, default=2,
                    help='also time the fp32 parity mode for this many steps (N=1 only; 0 = off)')
    ap.add_argument('--lbfgs-steps', type=int, default=5,
                    help='side measurement: steps of the device L-BFGS-B mode (0: skip)')
    ap.add_argument('--gatys', action='store_true',
                    help='configs[4]: Gatys [L,128,128] Gram instead of the channel-wise one')
    ap.add_argument('--lr', type=float, default=2.0)
    ap.add_argument('--graph', type=int, default=1,
                    help='1: replay the step from a captured HIP graph (default); 0: eager launches')
    ap.add_argument('--cpu-baseline-seconds', type=float, default=15.0,
                    help='CPU oracle sample budget (0 disables)')
    ap.add_argument('--traffic-json', default=os.path.join(ROOT, 'profiles', 'traffic.json'),
                    help='per-launch HBM bytes measured by rocprofv3 --pmc (see DESIGN.md)')
    return ap.parse_args()


def dist_setup():
    ws = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if ws > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    else:
        torch.cuda.set_device(0)
    return ws, rank, local


def barrier(ws):
    if ws > 1:
        import torch.distributed as dist
        dist.barrier()


def make_problem(eng, clips, T, dev):
    """Synthetic per-clip targets for the global clip indices `clips`: content
    clip c_g, style clip s_g; phi_c = emb_c(c_g); phi_s = l2norm(G^(c_g) + G^(s_g) - G^(c_g))
    (methods.py:207-212 with one clip per file); x0 = c_g + 4 N(0,1) (seeded per clip)."""
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


def cpu_baseline(T, budget_s):
    """Time the CPU oracle (oracle/astyle_oracle.py, numpy fp32, host BLAS threads) on a
    bounded sample of the same workload: whole loss+grad evaluations of single clips."""
    from oracle import astyle_oracle as O
    from audio_style_transfer_amd.weights import synthetic_weights, synthetic_clips
    try:
        from threadpoolctl import threadpool_info
        cores = max([i.get('num_threads', 1) for i in threadpool_info()] or [1])
    except Exception:
        cores = 1
    W = synthetic_weights(0)
    kw = dict(cont_ids=[29], style_ids=list(range(30)), gatys=False, nb_channels=128,
              cnt_channels=128)
    xc = O.mu_law_numpy(synthetic_clips(1, T, 1000)[0])
    ext, _ = O.encoder_forward(xc, W, 30, dtype=np.float32)
    phi_c = O.content_embeds(ext, [29], 128)
    phi_s = O.style_embeds(ext, list(range(30)))
    x = xc + np.random.default_rng(0).normal(0, 4, T)
    n = 0
    t0 = time.time()
    while True:
        O.loss_and_grad(x, W, phi_c=phi_c, phi_s=phi_s, lambd=100.0, dtype=np.float32, **kw)
        n += 1
        el = time.time() - t0
        if el >= budget_s or n >= 64:
            break
    clip_evals_per_s = n / el
    return {'value': clip_evals_per_s / 256.0, 'unit': 'iters/s (256x%d batch)' % T,
            'cores': int(cores), 'kind': 'port',
            'sample': '%d full loss+grad evaluations of one %d-sample clip (numpy fp32 oracle, '
                      '30 blocks, ours-Gram L=30) in %.1f s = %.3f clip-evals/s; scaled to the '
                      '256-clip batch' % (n, T, el, clip_evals_per_s),
            'clip_evals_per_s': clip_evals_per_s}


def run(args, precision, steps, warmup, ws, rank, dev, graph):
    """Build the engine, warm up, time `steps` steps (barrier + sync on both sides, max over
    ranks).  A step is one AdamLoop step (ast_loss_grad + device-counter Adam), replayed from
    a captured HIP graph when `graph`.  The per-kernel-family breakdown comes from HIP events
    of 2 extra eager steps (events are not recorded inside a graph).  Returns (seconds,
    engine timing dict, first loss, last loss)."""
    from audio_style_transfer_amd.engine import StyleEngine, AdamLoop
    from audio_style_transfer_amd.shard import clip_range, max_over_ranks
    B, T = args.clips, args.T
    eng = StyleEngine(B, T, [29], list(range(30)), precision=precision, device=dev,
                      lambd=100.0, gatys=args.gatys)
    x = make_problem(eng, clip_range(ws * B, ws, rank), T, dev)
    loop = AdamLoop(eng, x, lr=args.lr, graph=graph)
    for _ in range(warmup):
        loop.step()
    torch.cuda.synchronize()
    first_loss = loop.parts[:, 0].mean().item()
    barrier(ws)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loop.step()
    torch.cuda.synchronize()
    barrier(ws)
    el = time.perf_counter() - t0
    el = max_over_ranks(el, ws, device=dev)
    last_loss = loop.parts[:, 0].mean().item()
    if not np.isfinite(last_loss):
        raise SystemExit('non-finite loss')
    eng.timing(True)
    for _ in range(2):
        loop._eager()
    torch.cuda.synchronize()
    tm = eng.timing_read()
    eng.timing(False)
    del loop, x
    eng.close()
    torch.cuda.empty_cache()
    return el, tm, first_loss, last_loss


def run_lbfgs(args, steps, dev):
    """Side measurement (rank 0, N=1): the reference's optimiser, scipy's L-BFGS-B restated on
    the device (ast_lbfgs_*), over the same 256-clip workload.  A step is one evaluation of every
    clip (ast_loss_grad) + one ast_lbfgs_step, replayed from a HIP graph; the L-BFGS-B kernel's
    own time comes from HIP events around eager launches on the engine's stream."""
    import ctypes
    from audio_style_transfer_amd.engine import StyleEngine, LbfgsLoop
    from audio_style_transfer_amd.shard import clip_range
    B, T = args.clips, args.T
    eng = StyleEngine(B, T, [29], list(range(30)), precision=args.precision, device=dev,
                      lambd=100.0, gatys=args.gatys)
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
                    'instead of Adam, same workload; one iter = one loss+grad evaluation of every '
                    'clip + the L-BFGS-B update'}


def main():
    args = parse()
    ws, rank, local = dist_setup()
    dev = torch.device('cuda', local)
    B, T = args.clips, args.T
    L = 30
    el, tm, first_loss, last_loss = run(args, args.precision, args.steps, args.warmup, ws,
                                        rank, dev, args.graph)
    fp32_side = None
    if args.fp32_steps > 0 and args.precision != 'fp32' and ws == 1:
        el32, _, _, _ = run(args, 'fp32', args.fp32_steps, 1, ws, rank, dev, args.graph)
        fp32_side = {'value': B * args.fp32_steps / 256.0 / el32, 'unit': 'iters/s',
                     'steps': args.fp32_steps,
                     'note': 'same workload with fp32 storage + fp32 MFMA (parity mode: grad '
                             'within 2e-3 rel-L2 of the fp64 oracle)'}
    lbfgs_side = None
    if args.lbfgs_steps > 0 and ws == 1:
        lbfgs_side = run_lbfgs(args, args.lbfgs_steps, dev)
    if rank != 0:
        barrier(ws)
        return
    value = ws * B * args.steps / 256.0 / el
    calls = max(tm['calls'], 1)
    nblk = tm['blocks']
    fwd_ms = tm['block_fwd_ms'] / (calls * nblk)
    bwd_ms = tm['block_bwd_ms'] / (calls * nblk)
    launch_ms = (fwd_ms + bwd_ms) / 2
    esz = 4.0 if args.precision == 'fp32' else 2.0
    A = B * T * 128 * esz                          # one activation tensor, all clips
    flops_per_launch = 131072.0 * T * B            # 2*(384+128)*128 flop per row, fwd or bwd
    bytes_per_launch = 2.5 * A                     # fwd 2A (read e_l, write e_l+1), bwd 3A
    traffic = None
    try:
        with open(args.traffic_json) as f:
            tj = json.load(f)
        if (tj.get('precision') == args.precision and tj.get('clips') == B and tj.get('T') == T):
            traffic = tj['block_bytes_per_launch']
    except Exception:
        traffic = None
    if args.precision == 'fp32':
        # fp32: 96 flop/B on the dilated conv, above the fp32 ridge -> MFMA-bound
        achieved = flops_per_launch / (launch_ms * 1e-3) / 1e12
        roof = {'bound': 'mfma', 'achieved': achieved, 'peak': FP32_MFMA_PEAK_TFLOPS,
                'unit': 'TFLOP/s', 'frac': achieved / FP32_MFMA_PEAK_TFLOPS}
    else:
        # bf16 storage: 192 flop/B fwd (below the 312 flop/B bf16 ridge) -> HBM-bound
        achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9
        roof = {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                'frac': achieved / HBM_PEAK_GBS}
    roof.update({'traffic': traffic,
                 'kernel': 'k_block_fwd*/k_block_bwd* (fused dilated conv + 1x1 + epilogues), '
                           'mean of one fwd and one bwd launch',
                 'algorithmic_bytes_per_launch': bytes_per_launch,
                 'flops_per_launch': flops_per_launch,
                 'mfma_frac': flops_per_launch / (launch_ms * 1e-3) / 1e12 /
                              (FP32_MFMA_PEAK_TFLOPS if args.precision == 'fp32'
                               else BF16_MFMA_PEAK_TFLOPS),
                 'avg_launch_ms': launch_ms, 'fwd_launch_ms': fwd_ms, 'bwd_launch_ms': bwd_ms})
    gram_fwd_ms = tm['gram_fwd_ms'] / calls
    gram_bwd_ms = tm['gram_bwd_ms'] / calls
    gram_bytes = L * A
    out = {
        'metric': 'style-transfer iters/sec, 256x16384-sample batch, 30-layer WaveNet encoder',
        'value': value, 'unit': 'iters/s', 'n_gpus': ws, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': el / args.steps * 1e3,
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
        'dtype': args.precision,
        'data': 'synthetic (seeded sinusoid+noise clips, seeded uniform_unit_scaling weights)',
        'config': {'workload': ('configs[4]: %dx%d clips per GPU, 30-block encoder, Gatys Gram '
                                if args.gatys else
                                'configs[2]: %dx%d clips per GPU, 30-block encoder, ours-Gram ')
                               % (B, T) + 'L=30, cont_lyrs [29], lambd 100, gamma 0, Adam step',
                   'global_batch_clips': ws * B, 'T': T, 'parallelism': 'clip-sharded x%d' % ws,
                   'precision': args.precision, 'hip_graph': bool(args.graph)},
        'clip_iters_per_s': value * 256.0,
        'roofline': roof,
        'kernels_ms_per_step': {'block_fwd': tm['block_fwd_ms'] / calls,
                                'block_bwd': tm['block_bwd_ms'] / calls,
                                'gram_fwd': gram_fwd_ms, 'gram_bwd': gram_bwd_ms,
                                'other': tm['other_ms'] / calls},
        'gram_roofline': {'bound': 'hbm', 'fwd_achieved_GBs': gram_bytes / (gram_fwd_ms * 1e-3) / 1e9,
                          'bwd_achieved_GBs': 2 * gram_bytes / (gram_bwd_ms * 1e-3) / 1e9,
                          'peak': HBM_PEAK_GBS},
        'loss_first_last': [first_loss, last_loss],
    }
    if fp32_side:
        out['fp32_mode'] = fp32_side
    if lbfgs_side:
        out['lbfgs_mode'] = lbfgs_side
    if ws == 1 and args.cpu_baseline_seconds > 0:
        out['cpu_baseline'] = cpu_baseline(T, args.cpu_baseline_seconds)
    print(json.dumps(out), flush=True)
    barrier(ws)


if __name__ == '__main__':
    main()
