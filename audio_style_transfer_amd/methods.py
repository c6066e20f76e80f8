"""Drop-in for the reference's methods.py (CLI + GatysNet), running on libastyle.so.

Same argparse surface (methods.py:243-269), same output layout (utils.gt_s_path / crt_t_fol,
ori.wav, style.wav, ep-N.wav, gram/spectrogram PNGs), same optimisation protocol: per epoch one
scipy L-BFGS-B minimize(maxiter=100) whose every function evaluation is one ast_loss_grad
(ScipyOptimizerInterface, methods.py:132-137,167), early stop when an epoch used < 50
evaluations (methods.py:180), the four loss scalars of every evaluation written to a TF event
file in the log dir (methods.py:127-130,156; summary.EventWriter).  Additions: --optimizer
device (the same L-BFGS-B on the GPU), --precision split (default) | fp32 | bf16, --weights (npz of TF-named
encoder variables), --resume (continue after the last finished epoch: each epoch's end point
is saved as <savepath>/state.npz; an epoch is a fresh minimize call, so x is the whole state).

--ckpt_path is a TF checkpoint-V2 prefix (model.ckpt-200000: .index + .data shards), read by
libastyle's native reader without TensorFlow, or an .npz of TF-named arrays; when neither
exists (the NSynth checkpoint is not in this image) seeded synthetic weights are used and a
warning is printed.
"""
from __future__ import annotations

import argparse
import os
import sys
import time
import warnings

import numpy as np
import torch

from . import _lib, checkpoint, summary, utils
from .engine import StyleEngine, resolve_style_ids
from .weights import synthetic_weights


def load_weights(path):
    """TF-named encoder weights (Saver.restore, methods.py:79-84) from a TF checkpoint-V2
    prefix (<path>.index + data shards, read natively: checkpoint.py) or an .npz
    (allow_pickle=False); None if neither exists."""
    if checkpoint.is_checkpoint(path):
        return checkpoint.encoder_weights(path)
    if path and os.path.isfile(path) and path.endswith('.npz'):
        with np.load(path, allow_pickle=False) as z:
            return {k: z[k] for k in z.files}
    return None


def _drop_sess(args):
    """The reference's methods take a tf.Session first (methods.py:86,97,140); drop it (None or
    any object with a ``run`` method) so reference-style calls work unchanged."""
    if args and (args[0] is None or hasattr(args[0], 'run')):
        return args[1:]
    return args


class GatysNet(object):
    """methods.py:19-216, on one GPU; ``batch`` > 1 optimises independent clips together."""

    def __init__(self, savepath='./data/out',
                 checkpoint_path='./nsynth/model/wavenet-ckpt/model.ckpt-200000',
                 logdir='./log', figdir='./data/fig', stack=0, batch_size=16384, sr=16000,
                 cont_lyr_ids=[29], nb_channels=128, cnt_channels=128, gatys=False,
                 style_lyr_ids=None, precision='split', device=None, weights=None, plots=True,
                 optimizer='scipy', engine_cls=StyleEngine):
        self.logdir = logdir
        self.savepath = savepath
        self.checkpoint_path = checkpoint_path
        self.figdir = figdir
        self.batch_size = batch_size
        self.sr = sr
        self.late = (batch_size - (batch_size // 4096) * 4000) // 2          # methods.py:39
        self.cont_lyr_ids = list(cont_lyr_ids)
        self.style_lyr_ids = resolve_style_ids(stack, style_lyr_ids)        # methods.py:60-66
        self.nb_channels, self.cnt_channels, self.gatys = nb_channels, cnt_channels, gatys
        self.precision = precision
        self.device = device or torch.device('cuda', torch.cuda.current_device())
        self.plots = plots
        self.optimizer = optimizer
        self.engine_cls = engine_cls
        if weights is None:
            weights = load_weights(checkpoint_path)
            if weights is None:
                warnings.warn('no checkpoint at %r (neither <prefix>.index nor an .npz); '
                              'using seeded synthetic encoder weights' % checkpoint_path)
                weights = synthetic_weights(0)
        self.weights = weights
        self.engine = self.build(batch_size)
        self.embeds_shape = self.engine.style_shape

    def build(self, length, batch=1, lambd=100.0, precision=None):
        """methods.py:44-77: encoder + taps + Gram + l2norm, here one libastyle context."""
        return self.engine_cls(batch, length, self.cont_lyr_ids, self.style_lyr_ids,
                               cnt_channels=self.cnt_channels, nb_channels=self.nb_channels,
                               gatys=self.gatys, lambd=lambd, precision=precision or self.precision,
                               device=self.device, weights=self.weights)

    def get_embeds(self, *args, is_content=True):
        """methods.py:86-95: mu-law encode the clip and fetch embeds_c or embeds_s.  Accepts the
        reference's signature get_embeds(sess, aud) as well (the session is ignored)."""
        aud = np.asarray(_drop_sess(args)[0])
        if aud.ndim == 1:
            aud = aud[:self.batch_size].reshape(1, self.batch_size)
        x = torch.tensor(utils.mu_law_numpy(aud), dtype=torch.float32, device=self.device)
        emb_c, emb_s = self.engine.embeds(x, content=is_content, style=not is_content)
        return (emb_c if is_content else emb_s)[0].cpu().numpy()

    def get_style_phi(self, *args, max_examples=5, show_mat=True):
        """methods.py:97-111: mean style embedding over <= 5 consecutive clips.  Accepts the
        reference's get_style_phi(sess, filename, ...) as well (the session is ignored)."""
        args = _drop_sess(args)
        filename = args[0]
        if len(args) > 1:
            max_examples = args[1]
        if len(args) > 2:
            show_mat = args[2]
        audio, _ = utils.load_audio(filename, sr=self.sr, audio_channel=0)
        I = []
        i = 0
        while i + self.batch_size <= min(len(audio), max_examples * self.batch_size):
            I.append(self.get_embeds(audio[i:i + self.batch_size], is_content=False))
            i += self.batch_size
        phi = np.mean(I, axis=0)
        if show_mat and self.plots:
            utils.show_gram(phi, figdir=self.figdir, gatys=self.gatys)
        return phi

    def l_bfgs(self, *args, x0=None, log=print, optimizer='scipy', maxiter=100, resume=False,
               **kw):
        """methods.py:140-181 with scipy L-BFGS-B driving ast_loss_grad (``optimizer='scipy'``,
        one host round trip per evaluation, as the reference), or the same L-BFGS-B run on the
        device (``'device'``: ast_lbfgs_*, no round trip; each epoch's evaluations are logged
        from the workspace's loss history after the epoch).
        Accepts the reference's l_bfgs(sess, phi_c, phi_s, epochs, lambd, gamma) as well.  Every
        epoch starts from the float32 rounding of its point, as the TF variable does.

        Each evaluation's (content, style, regularizer, main) losses go to the log dir's event
        file at step i_ + i (methods.py:147-157: i counts this epoch's evaluations, i_ is the
        previous epoch's count).  After every epoch its end point, index and count are saved
        to <savepath>/state.npz; ``resume=True`` continues from there (an epoch is a fresh
        minimize call, methods.py:167, so nothing else carries over)."""
        from scipy.optimize import minimize
        names = ('phi_c', 'phi_s', 'epochs', 'lambd', 'gamma')
        vals = dict(zip(names, _drop_sess(args)))
        vals.update(kw)
        phi_c, phi_s, epochs, lambd, gamma = (vals[n] for n in names)
        eng = self.build(self.batch_size, lambd=lambd) if lambd != self.engine.lambd else self.engine
        self.engine = eng
        eng.set_targets(torch.as_tensor(phi_c, dtype=torch.float32),
                        torch.as_tensor(phi_s, dtype=torch.float32))
        eng.set_gamma(gamma)                                              # methods.py:121-125
        T = self.batch_size
        x = np.zeros(T) + 1e-6 if x0 is None else np.asarray(x0, dtype=np.float64)  # methods.py:49-54
        x = x.astype(np.float32).astype(np.float64)       # the TF variable is float32
        xd = torch.empty(1, T, device=self.device)
        state = {'i': 0, 'i_': 0, 'since': time.time()}
        history = []
        start_ep = 0
        ckpt = os.path.join(self.savepath, 'state.npz')
        fp = self._run_fingerprint(phi_c, phi_s, lambd, gamma, optimizer)
        if resume and os.path.isfile(ckpt):
            with np.load(ckpt, allow_pickle=False) as z:
                saved = str(z['fingerprint']) if 'fingerprint' in z.files else None
                if saved != fp:
                    raise ValueError('%s was saved by a different run (targets, lambd, gamma, '
                                     'length, taps, precision or optimizer differ); refusing to '
                                     'resume from it' % ckpt)
                x = np.asarray(z['x'], dtype=np.float64)
                start_ep, state['i_'] = int(z['ep']) + 1, int(z['i_'])
            log('resuming after epoch %d (%d evaluations) from %s' % (start_ep, state['i_'], ckpt))
            if state['i_'] < 50:                                          # it had stopped
                self.history = history
                return x
        writer = summary.EventWriter(self.logdir)

        def scalars(p, step):
            writer.add_scalars({'loss/content_loss': p[1], 'loss/style_loss': p[2],
                                'loss/regularizer': p[3], 'loss/main_loss': p[0]}, step)

        def fg(v):
            nonlocal eng
            xd.copy_(torch.from_numpy(v.astype(np.float32)).view(1, T))
            if eng.precision == 'split':
                eng.reset_range_flags()                                   # this evaluation's flags
            parts, grad = eng.loss_grad(xd)                               # incl. gamma * reg
            if eng.precision == 'split' and self._split_out_of_range(eng, log):
                eng = self._fp32_engine(phi_c, phi_s, lambd, gamma)
                parts, grad = eng.loss_grad(xd)
            p = parts[0].cpu().numpy().astype(np.float64)
            loss, reg = float(p[0]), float(p[3])
            history.append((loss, float(p[1]), float(p[2]), reg))
            scalars(p, state['i_'] + state['i'])
            if not state['i'] % 5:                                       # methods.py:152-155
                log('Ep {0:}/{1:}-it {2:}({3:})-tlapse {4:.4f}s-loss{5:.4f}-{6:.4f}-{7:.4f}-{8:.4f}'.format(
                    state['ep'] + 1, epochs, state['i'], state['i_'], time.time() - state['since'],
                    loss, p[1], p[2], reg))
            state['i'] += 1
            return loss, grad[0].double().cpu().numpy()

        loop = None
        if optimizer == 'device':
            from .engine import LbfgsLoop
            loop = LbfgsLoop(eng, maxiter=maxiter)
        for ep in range(start_ep, epochs):
            state['ep'], state['i'] = ep, 0
            if loop is None:
                res = minimize(fg, x, jac=True, method='L-BFGS-B', options={'maxiter': maxiter})
                x = res.x.astype(np.float32).astype(np.float64)   # next epoch: fp32(res.x)
            else:
                info = loop.minimize(torch.tensor(x[None], dtype=torch.float64)
                                     if ep == start_ep else None)
                # the flags are sticky over the epoch (begin resets them): any out-of-range
                # evaluation, line-search trials included, sends the epoch to the fp32 kernels
                if eng.precision == 'split' and self._split_out_of_range(eng, log):
                    # redo the epoch from its start point x with the fp32 kernels
                    eng = self._fp32_engine(phi_c, phi_s, lambd, gamma)
                    loop = LbfgsLoop(eng, maxiter=maxiter)
                    info = loop.minimize(torch.tensor(x[None], dtype=torch.float64))
                x = loop.state(with_x=True)[1][0].cpu().numpy()
                state['i'] = int(info[0, 2])
                # every evaluation's parts, from the workspace's history (ast_lbfgs_history), at
                # step i_ + i with the progress line every 5, as the scipy path's fg does; the
                # device evaluations are not timed one by one, so tlapse is the epoch's end
                tl = time.time() - state['since']
                for k, p in enumerate(loop.history(info)[0]):
                    history.append((float(p[0]), float(p[1]), float(p[2]), float(p[3])))
                    scalars(p, state['i_'] + k)
                    if not k % 5:                                         # methods.py:152-155
                        log('Ep {0:}/{1:}-it {2:}({3:})-tlapse {4:.4f}s-loss{5:.4f}-{6:.4f}-{7:.4f}-{8:.4f}'.format(
                            ep + 1, epochs, k, state['i_'], tl, *p))
            state['i_'] = state['i']
            writer.flush()
            np.savez(ckpt, x=x.astype(np.float32).astype(np.float64), ep=ep, i_=state['i_'],
                     fingerprint=np.array(fp))
            audio = utils.inv_mu_law_numpy(x[None])[0, self.late:-self.late]
            sp = os.path.join(self.savepath, 'ep-{}.wav'.format(ep))
            utils.write_wav(sp, audio / np.max(audio), sr=self.sr)        # methods.py:176
            if self.plots:
                _, grams = eng.embeds(torch.tensor(x[None], dtype=torch.float32, device=self.device),
                                      content=False)
                utils.show_gram(grams[0].cpu().numpy(), ep + 1, self.figdir, gatys=self.gatys)
            if state['i_'] < 50:                                          # methods.py:180-181
                break
        writer.close()
        if eng is not self.engine:   # the range guard's fp32 context
            eng.close()
        self.history = history
        return x

    def _split_out_of_range(self, eng, log) -> bool:
        """After split-precision evaluations: AST_RANGE_* flags of the clip accumulated since the
        last reset (engine.range_flags: one evaluation on the scipy path, a whole device epoch).
        Non-finite results or operands outside the split-fp16 range (flags 1, 2, 4) -> True (the
        caller switches to the fp32 kernels); operands below 2^-60 (8) only lose low-order bits
        and are reported once."""
        f = int(eng.range_flags().max().item())
        bad = f & (_lib.RANGE_NONFINITE | _lib.RANGE_ACT | _lib.RANGE_GRAD)
        if f & _lib.RANGE_TINY and not getattr(self, '_tiny_warned', False):
            self._tiny_warned = True
            warnings.warn('split precision: operands below 2^-60 in this clip (low-order bits '
                          'lost; --precision fp32 keeps them)')
        if bad:
            log('split precision: range flags %d for this clip; switching to --precision fp32' % f)
        return bool(bad)

    def _fp32_engine(self, phi_c, phi_s, lambd, gamma):
        """The range guard's fallback for the rest of this l_bfgs call: an fp32-kernel context
        of its own (self.precision, self.engine and the resume fingerprint stay as chosen; the
        context is closed when l_bfgs returns)."""
        new = self.build(self.batch_size, lambd=lambd, precision='fp32')
        new.set_targets(torch.as_tensor(phi_c, dtype=torch.float32),
                        torch.as_tensor(phi_s, dtype=torch.float32))
        new.set_gamma(gamma)
        return new

    def _run_fingerprint(self, phi_c, phi_s, lambd, gamma, optimizer):
        """What a saved epoch state depends on: the targets (hence the content / style files and
        the weights), the loss constants, the clip length, the taps, precision and optimiser."""
        import hashlib
        h = hashlib.sha256()
        for a in (phi_c, phi_s):
            h.update(np.ascontiguousarray(np.asarray(a, dtype=np.float32)).tobytes())
        h.update(repr((float(lambd), float(gamma), int(self.batch_size), self.cont_lyr_ids,
                       self.style_lyr_ids, self.nb_channels, self.cnt_channels, bool(self.gatys),
                       self.precision, optimizer)).encode())
        return h.hexdigest()

    def targets(self, cont_file, source, target, audio_channel=0, start=1.0, savepath=None):
        """methods.py:185-213: the content clip's phi_c and the analogy style target
        phi = l2norm(phi(content clip) + phi(target file) - phi(source file)); writes ori.wav and
        style.wav to ``savepath`` (default self.savepath)."""
        savepath = savepath or self.savepath
        phi_t = self.get_style_phi(target)
        phi_s = self.get_style_phi(source, show_mat=False)
        aud, _ = utils.load_audio(cont_file, sr=self.sr, audio_channel=audio_channel)
        st = int(start * self.sr - self.late)
        aud = aud[st:st + self.batch_size]
        utils.write_wav(os.path.join(savepath, 'ori.wav'), aud[self.late:-self.late], self.sr)
        style_aud, _ = utils.load_audio(target, sr=self.sr, audio_channel=audio_channel)
        style_aud = style_aud[st:st + self.batch_size]
        utils.write_wav(os.path.join(savepath, 'style.wav'), style_aud[self.late:-self.late], self.sr)
        phi_c = self.get_embeds(aud)
        phi = self.get_embeds(aud, is_content=False)
        phi = phi + phi_t - phi_s
        phi = phi / np.sqrt(np.maximum(np.sum(phi * phi, axis=(1, 2), keepdims=True), 1e-12))
        return phi_c, phi

    def run(self, cont_file, source, target, epochs, lambd=0.1, gamma=0.1, audio_channel=0,
            start=1.0, resume=False):
        """methods.py:183-216."""
        phi_c, phi = self.targets(cont_file, source, target, audio_channel, start)
        x = self.l_bfgs(phi_c, phi, epochs=epochs, lambd=lambd, gamma=gamma,
                        optimizer=self.optimizer, resume=resume)
        return utils.inv_mu_law_numpy(x[None])[0]


def get_dir(dir, args):
    """methods.py:219-220 (reference-only flags excluded from the name)."""
    kw = {k: v for k, v in vars(args).items() if k not in EXTRA_FLAGS}
    return utils.gt_s_path(utils.crt_t_fol(dir), **kw)


def get_fpath(fn, args):
    return os.path.join(args.dir, fn) + '.wav'


EXTRA_FLAGS = ('precision', 'weights', 'no_plots', 'optimizer', 'resume')


def piece_work(args):
    """methods.py:227-240."""
    savepath, logdir = map(lambda d: get_dir(d, args), [args.outdir, args.logdir])
    figdir = os.path.join(savepath, 'fig')
    os.makedirs(figdir, exist_ok=True)
    content, style = map(lambda name: get_fpath(name, args), [args.cont_fn, args.style_fn])
    weights = load_weights(args.weights) if args.weights else None
    test = GatysNet(savepath, args.ckpt_path, logdir, figdir, args.stack, args.batch_size, args.sr,
                    args.cont_lyrs, args.channels, args.cnt_channels, args.gatys, args.style_lyrs,
                    precision=args.precision, weights=weights, plots=not args.no_plots,
                    optimizer=args.optimizer)
    return test.run(content, content, style, epochs=args.epochs, lambd=args.lambd,
                    gamma=args.gamma, start=args.start, resume=args.resume)


def make_parser(positionals=True, **kw):
    """methods.py:244-267, plus --precision / --weights / --no_plots / --optimizer / --resume
    (positionals=False: without cont_fn / style_fn, for the batch mode's parser)."""
    parser = argparse.ArgumentParser(**kw)
    if positionals:
        parser.add_argument('cont_fn', help='relative content file name')
        parser.add_argument('style_fn', help='relative style file name')
    parser.add_argument('--epochs', help='number of epochs, each epoch contains 100 iterations of optimization',
                        nargs='?', type=int, default=100)
    parser.add_argument('--batch_size', help='length of output signal, must be divided by 4096', nargs='?', type=int, default=16384)
    parser.add_argument('--sr', help='sampling rate, default to 16kHz', nargs='?', type=int, default=16000)
    parser.add_argument('--stack', help='stack of layers chosen for computing style loss. Have effects only if style_lyrs is None. There are 3 stacks, each of 10 layers. If None'
                                        ' then all three stacks will be taken into account', nargs='?', type=int, default=None)
    parser.add_argument('--cont_lyrs', nargs='*', type=int, default=[29])
    parser.add_argument('--style_lyrs', nargs='*', type=int)
    parser.add_argument('--lambd', help='style loss scalar coefficient', nargs='?', type=float, default=100.0)
    parser.add_argument('--gamma', help='regularizer scalar coefficient', nargs='?', type=float, default=0.0)
    parser.add_argument('--channels', help='how many channels taken into account for style loss', nargs='?', type=int, default=128)
    parser.add_argument('--cnt_channels', help='how many channels taken into account for content loss', nargs='?', type=int, default=128)
    parser.add_argument('--start', nargs='?', type=float, default=1.0)
    parser.add_argument('--gatys', nargs='?', type=bool, default=False, const=True)
    parser.add_argument('--ckpt_path', help="path to the pretrained model's checkpoint path", nargs='?', default='./nsynth/model/wavenet-ckpt/model.ckpt-200000')
    parser.add_argument('--dir', help='path to source files, should be where to store reference style and content files', nargs='?', default='./data/src')
    parser.add_argument('--outdir', help='path to output', nargs='?', default='./data/out')
    parser.add_argument('--logdir', help='path to logs', nargs='?', default='./log')
    parser.add_argument('--cmt')
    parser.add_argument('--precision', default='split', choices=['fp32', 'split', 'bf16'],
                        help='split (default): fp32 storage, split-fp16 MFMA with fp32 '
                             'accumulation (gradient within 2e-4 rel-L2 of fp64, range-checked '
                             'per clip: ast_range_flags); fp32: fp32 storage + fp32 MFMA '
                             '(v_mfma_f32_32x32x2_f32, also the range guard\'s fallback); bf16: '
                             'bf16 storage + bf16 MFMA')
    parser.add_argument('--weights', default=None, help='npz of TF-named encoder weights')
    parser.add_argument('--no_plots', action='store_true', help='skip the Gram PNGs')
    parser.add_argument('--optimizer', default='scipy', choices=['scipy', 'device'],
                        help='scipy: host L-BFGS-B per evaluation (reference); device: the same '
                             'L-BFGS-B on the GPU (ast_lbfgs_*)')
    parser.add_argument('--resume', action='store_true',
                        help='continue after the last finished epoch saved in the output dir')
    return parser


def main(argv=None):
    args = make_parser().parse_args(argv)
    return piece_work(args)


if __name__ == '__main__':
    main(sys.argv[1:])
