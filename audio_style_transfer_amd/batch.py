"""Clip-sharded batch mode of the CLI: many content/style pairs, one independent problem per clip.

The reference optimises one pair per process (methods.py:227-240 ``piece_work``: GatysNet.run on
one 16384-sample clip).  Here a list of pairs is split over the GPUs of a node, one process per
GPU (shard.launch_ranks, the launcher bench.py uses, started before anything touches a GPU), and
each rank optimises its shard (shard.clip_range) of pairs together:

  python -m audio_style_transfer_amd.batch --pairs PAIRS [methods.py flags] [--gpus N]

PAIRS is a text file with one ``cont_fn style_fn`` per line (names relative to --dir, without
.wav, as the reference's positionals), or ``cont:style,cont:style`` inline.  Every flag of the
reference CLI applies to every pair.  Per pair, exactly as piece_work would do for it alone:
  * its output directory is gt_s_path(crt_t_fol(outdir), **args with that pair's cont_fn /
    style_fn) (methods.py:219-220), its log directory likewise under --logdir;
  * its targets are GatysNet.targets (methods.py:185-213: phi_c of the content clip and the
    analogy style target), ori.wav / style.wav written there;
  * its optimisation is the reference protocol (methods.py:164-181): per epoch one L-BFGS-B
    minimize(maxiter 100) from fp32(x), the epoch's end point to ep-N.wav and state.npz, its
    losses to the pair's own event file, and an early stop for that pair once an epoch used
    fewer than 50 evaluations.
--optimizer device (the default here): one StyleEngine holding the rank's whole shard and the
device L-BFGS-B (engine.LbfgsLoop) over all of its clips at once, stopped clips switched off
through the loop's active mask; the split range guard redoes a flagged clip's epoch on fp32
kernels and keeps that clip there (as GatysNet does).  --optimizer scipy: GatysNet.run per pair,
one after another on the rank (the reference's host optimiser, one pair at a time).
"""
from __future__ import annotations

import argparse
import copy
import importlib
import os
import sys
import time
import warnings

import numpy as np

from . import methods, summary, utils
from .shard import clip_range, launch_ranks


def make_parser():
    p = methods.make_parser(positionals=False, description=__doc__.split('\n\n')[0])
    p.add_argument('--pairs', required=True,
                   help='file of "cont_fn style_fn" lines, or inline "cont:style,cont:style"')
    p.add_argument('--gpus', type=int, default=1, help='ranks (one per GPU) on this node')
    p.add_argument('--engine', default='audio_style_transfer_amd.engine:StyleEngine',
                   help='module:Class of the engine; the module also provides LbfgsLoop '
                        '(tests substitute a CPU stand-in)')
    p.add_argument('--backend', default='nccl', help='torch.distributed backend for N > 1')
    p.set_defaults(optimizer='device')
    return p


def read_pairs(spec):
    """[(cont_fn, style_fn)] from a pairs file or an inline 'a:b,c:d' list."""
    if os.path.isfile(spec):
        out = []
        with open(spec) as f:
            for line in f:
                line = line.split('#', 1)[0].strip()
                if line:
                    c, s = line.split()
                    out.append((c, s))
        return out
    return [tuple(x.split(':')) for x in spec.split(',') if x]


EXTRA = methods.EXTRA_FLAGS + ('pairs', 'gpus', 'engine', 'backend')


def pair_args(args, cont_fn, style_fn):
    a = copy.copy(args)
    a.cont_fn, a.style_fn = cont_fn, style_fn
    return a


def pair_dirs(args, cont_fn, style_fn):
    """The pair's output and log directories: methods.get_dir with that pair's names (the
    batch-only flags excluded from the name, as methods.EXTRA_FLAGS are)."""
    a = pair_args(args, cont_fn, style_fn)
    kw = {k: v for k, v in vars(a).items() if k not in EXTRA}
    return (utils.gt_s_path(utils.crt_t_fol(args.outdir), **kw),
            utils.gt_s_path(utils.crt_t_fol(args.logdir), **kw))


def _engine_module(spec):
    mod, cls = spec.split(':')
    m = importlib.import_module(mod)
    return getattr(m, cls), getattr(m, 'LbfgsLoop')


def run_rank(args, pairs, ws, rank, dev, log=print):
    """Optimise this rank's shard of `pairs`; returns {global pair index: final x (float64)}."""
    import torch
    Eng, Loop = _engine_module(args.engine)
    mine = list(clip_range(len(pairs), ws, rank))
    if not mine:
        return {}
    weights = methods.load_weights(args.weights) if args.weights else None
    dirs = [pair_dirs(args, *pairs[i]) for i in mine]
    # a one-clip GatysNet for the targets (embeddings of single clips, methods.py:86-111)
    net = methods.GatysNet(dirs[0][0], args.ckpt_path, dirs[0][1], os.path.join(dirs[0][0], 'fig'),
                           args.stack, args.batch_size, args.sr, args.cont_lyrs, args.channels,
                           args.cnt_channels, args.gatys, args.style_lyrs, precision=args.precision,
                           device=dev, weights=weights, plots=not args.no_plots,
                           optimizer=args.optimizer, engine_cls=Eng)
    src = lambda name: os.path.join(args.dir, name) + '.wav'                 # methods.py:223-224
    if args.optimizer == 'scipy':
        out = {}
        for i, (sp, lp) in zip(mine, dirs):
            c, s = pairs[i]
            net.savepath, net.logdir, net.figdir = sp, lp, os.path.join(sp, 'fig')
            os.makedirs(net.figdir, exist_ok=True)
            x = net.run(src(c), src(c), src(s), epochs=args.epochs, lambd=args.lambd,
                        gamma=args.gamma, start=args.start, resume=args.resume)
            out[i] = x
        return out

    B, T = len(mine), args.batch_size
    tg = [net.targets(src(pairs[i][0]), src(pairs[i][0]), src(pairs[i][1]), start=args.start,
                      savepath=sp) for i, (sp, _) in zip(mine, dirs)]
    phi_c = torch.tensor(np.stack([t[0] for t in tg]), dtype=torch.float32)
    phi_s = torch.tensor(np.stack([t[1] for t in tg]), dtype=torch.float32)
    fps = [net._run_fingerprint(t[0], t[1], args.lambd, args.gamma, 'device') for t in tg]
    weights = net.weights

    def build(precision):
        e = Eng(B, T, net.cont_lyr_ids, net.style_lyr_ids, cnt_channels=args.cnt_channels,
                nb_channels=args.channels, gatys=args.gatys, lambd=args.lambd, precision=precision,
                device=dev, weights=weights)
        e.set_targets(phi_c, phi_s)
        e.set_gamma(args.gamma)
        return e

    eng = build(args.precision)
    loops = {args.precision: Loop(eng, maxiter=100)}
    engines = {args.precision: eng}
    prec = [args.precision] * B                    # per clip: the kernels it runs on
    x = np.full((B, T), 1e-6).astype(np.float32).astype(np.float64)        # methods.py:49-54
    start_ep, i_ = np.zeros(B, int), np.zeros(B, int)
    active = np.ones(B, bool)
    for b, (sp, _) in enumerate(dirs):
        ck = os.path.join(sp, 'state.npz')
        if args.resume and os.path.isfile(ck):
            with np.load(ck, allow_pickle=False) as z:
                if str(z['fingerprint']) != fps[b]:
                    raise ValueError('%s was saved by a different run; refusing to resume' % ck)
                x[b] = z['x']
                start_ep[b], i_[b] = int(z['ep']) + 1, int(z['i_'])
            active[b] = i_[b] >= 50
    writers = [summary.EventWriter(lp) for _, lp in dirs]

    def epoch(precision, sel, x0):
        """One minimize call for the clips in `sel` on the `precision` kernels, from x0:
        (info, end points, per-clip evaluation histories).  begin(x0) restarts every clip of
        that loop, so each loop runs at most once per epoch and only `sel`'s rows are used."""
        if precision not in loops:
            engines[precision] = build(precision)
            loops[precision] = Loop(engines[precision], maxiter=100)
        lp = loops[precision]
        info = lp.minimize(torch.tensor(x0, dtype=torch.float64),
                           active=torch.tensor(sel.astype(np.int32)))
        _, xe = lp.state(with_x=True)
        return info, xe.cpu().numpy(), lp.history(info)

    from . import _lib
    guard = _lib.RANGE_NONFINITE | _lib.RANGE_ACT | _lib.RANGE_GRAD
    since = time.time()                                              # methods.py:160
    for ep in range(int(start_ep.min()) if B else 0, args.epochs):
        run = active & (start_ep <= ep)
        if not run.any():
            break
        x0 = x.astype(np.float32).astype(np.float64)                # each epoch from fp32(x)
        xe, hist, nev = np.empty_like(x), [None] * B, np.zeros(B, np.int64)
        # one minimize call per precision; the split clips first, so the clips its range guard
        # flags join this epoch's single fp32 call (from the same x0) beside the clips already
        # on fp32, and every clip's result is taken from the one call that ran it
        pending = {p: run & np.array([q == p for q in prec]) for p in ('split', 'bf16', 'fp32')}
        for p in ('split', 'bf16', 'fp32'):
            sel = pending[p]
            if not sel.any():
                continue
            info, xs, hs = epoch(p, sel, x0)
            if p == 'split':                                         # the range guard
                f = engines[p].range_flags().cpu().numpy()
                bad = sel & ((f & guard) != 0)
                if bad.any():
                    log('split precision: range flags on clips %s; their epoch reruns on fp32 '
                        'kernels' % [mine[b] for b in np.flatnonzero(bad)])
                    for b in np.flatnonzero(bad):
                        prec[b] = 'fp32'
                    pending['fp32'] = pending['fp32'] | bad
                    sel = sel & ~bad
            for b in np.flatnonzero(sel):
                xe[b], hist[b], nev[b] = xs[b], hs[b], info[b, 2]
        tl = time.time() - since     # the epoch's end: the device evaluations are not host-timed
        for b in np.flatnonzero(run):
            h = hist[b]
            n = int(nev[b])          # the clip's evaluation count (ast_lbfgs_state), = len(h)
            x[b] = xe[b]
            for k, pv in enumerate(h):                               # methods.py:147-157
                writers[b].add_scalars({'loss/content_loss': pv[1], 'loss/style_loss': pv[2],
                                        'loss/regularizer': pv[3], 'loss/main_loss': pv[0]},
                                       int(i_[b]) + k)
                if not k % 5:
                    log('pair %d %s->%s: Ep %d/%d-it %d(%d)-tlapse %.4fs-loss%.4f-%.4f-%.4f-%.4f' % (
                        mine[b], pairs[mine[b]][0], pairs[mine[b]][1], ep + 1, args.epochs, k,
                        i_[b], tl, *pv))
            writers[b].flush()
            i_[b] = n
            sp = dirs[b][0]
            np.savez(os.path.join(sp, 'state.npz'), x=x[b].astype(np.float32).astype(np.float64),
                     ep=ep, i_=i_[b], fingerprint=np.array(fps[b]))
            audio = utils.inv_mu_law_numpy(x[b][None])[0, net.late:-net.late]
            utils.write_wav(os.path.join(sp, 'ep-{}.wav'.format(ep)), audio / np.max(audio), args.sr)
            if n < 50:                                               # methods.py:180-181
                active[b] = False
    for w in writers:
        w.close()
    for e in engines.values():
        e.close()
    return {i: x[b] for b, i in enumerate(mine)}


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = make_parser().parse_args(argv)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pp = os.environ.get('PYTHONPATH', '')
    rc = launch_ranks(args.gpus, ['-m', 'audio_style_transfer_amd.batch'], argv,
                      env_extra={'PYTHONPATH': os.pathsep.join([root] + ([pp] if pp else []))})
    if rc is not None:
        return rc
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
    pairs = read_pairs(args.pairs)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore', UserWarning)     # synthetic-weights notice once per rank
        run_rank(args, pairs, ws, rank, dev,
                 log=lambda m: print('[rank %d] %s' % (rank, m), flush=True))
    if ws > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == '__main__':
    sys.exit(main())
