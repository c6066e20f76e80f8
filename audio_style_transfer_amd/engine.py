"""Batched style-transfer engine: a torch-facing wrapper of one libastyle context.

One ``StyleEngine`` = one HIP context on one GPU holding B independent clips of T samples.
It replaces, for the hot path, the TF graph + Session that ``GatysNet`` builds
(methods.py:44-77, 113-137): ``embeds`` is ``get_embeds`` (methods.py:86-95), ``loss_grad``
is one ScipyOptimizerInterface evaluation (methods.py:167) for every clip at once.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .weights import synthetic_weights

PRECISIONS = {'fp32': 0, 'bf16': 1, 'split': 2}


def resolve_style_ids(stack=None, style_lyr_ids=None):
    """methods.py:60-66."""
    if style_lyr_ids is not None:
        assert isinstance(style_lyr_ids, (tuple, list)), "style_lyr_ids must be of type tuple or list!"
        return list(style_lyr_ids)
    if stack is not None:
        return list(range(stack * 10, stack * 10 + 10))
    return list(range(30))


class StyleEngine:
    def __init__(self, batch: int, T: int, cont_ids: Sequence[int], style_ids: Sequence[int],
                 cnt_channels: int = 128, nb_channels: int = 128, gatys: bool = False,
                 lambd: float = 100.0, gamma: float = 0.0, precision: str = 'fp32',
                 device: Optional[torch.device] = None, weights=None, weight_seed: int = 0):
        self.lib = _lib.load()
        if device is None:
            device = torch.device('cuda', torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type != 'cuda':
            raise _lib.AstError('StyleEngine needs a GPU device (got %s); there is no CPU path'
                                % self.device)
        self.batch, self.T = int(batch), int(T)
        self.cont_ids, self.style_ids = list(cont_ids), list(style_ids)
        self.gatys = bool(gatys)
        self.nb_channels = int(nb_channels)
        self.cnt_channels = int(cnt_channels)
        self.lambd = float(lambd)
        self.gamma = float(gamma)
        self.gen = 0    # bumped by every setting a captured graph bakes in (set_gamma)
        cfg = _lib.AstCfg()
        cfg.batch, cfg.T = self.batch, self.T
        cfg.n_cont = len(self.cont_ids)
        for k, v in enumerate(self.cont_ids):
            cfg.cont_ids[k] = v
        cfg.cnt_channels = self.cnt_channels
        cfg.n_style = len(self.style_ids)
        for k, v in enumerate(self.style_ids):
            cfg.style_ids[k] = v
        cfg.nb_channels = self.nb_channels
        cfg.gatys = int(self.gatys)
        cfg.precision = PRECISIONS[precision]
        cfg.lambd = self.lambd
        cfg.gamma = self.gamma
        self.precision = precision
        self._cfg = cfg
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            torch.cuda.init()
            _lib.check(self.lib.ast_create(ctypes.byref(cfg), self.device.index or 0,
                                           ctypes.byref(h)))
        self.h = h
        self.ncc = self.lib.ast_content_cols(self.h)
        self._targets = None
        self.set_weights(weights if weights is not None else synthetic_weights(weight_seed))

    # ------------------------------------------------------------------ plumbing
    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _ptr(self, t: Optional[torch.Tensor], dtype=torch.float32):
        if t is None:
            return None
        assert t.is_cuda and t.device == self.device and t.dtype == dtype, t
        assert t.is_contiguous()
        return ctypes.c_void_p(t.data_ptr())

    def _x(self, x: torch.Tensor) -> torch.Tensor:
        if x.shape != (self.batch, self.T):
            raise ValueError('x must be [%d, %d], got %s' % (self.batch, self.T, tuple(x.shape)))
        return x.contiguous()

    def close(self):
        if getattr(self, 'h', None):
            self.lib.ast_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ API
    def set_weights(self, weights) -> None:
        """Upload encoder variables by TF name (Saver.restore, methods.py:79-84).
        Non-encoder names (the unused decoder) are skipped, as TF never runs them."""
        for name, arr in weights.items():
            a = np.ascontiguousarray(np.asarray(arr, dtype=np.float32))
            rc = self.lib.ast_set_weight(self.h, name.encode(),
                                         a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), a.size)
            if rc == -4 and not name.startswith('ae_'):
                continue
            _lib.check(rc)

    def restore(self, prefix: str) -> None:
        """Saver.restore(sess, prefix) (methods.py:79-84): every encoder variable from a TF
        checkpoint-V2 bundle, read natively by ast_restore."""
        _lib.check(self.lib.ast_restore(self.h, str(prefix).encode()))

    @property
    def style_shape(self):
        L = len(self.style_ids)
        if self.gatys:
            return (L, 128, 128)
        return (min(self.nb_channels, 128), L, L)

    def forward(self, x: torch.Tensor) -> None:
        _lib.check(self.lib.ast_forward(self.h, self._ptr(self._x(x)), self._stream()))

    def extract(self, i: int) -> torch.Tensor:
        C = 16 if i == 31 else 128
        out = torch.empty(self.batch, self.T, C, device=self.device)
        _lib.check(self.lib.ast_get_extract(self.h, i, self._ptr(out), self._stream()))
        return out

    def embeds(self, x: torch.Tensor, content: bool = True, style: bool = True):
        emb_c = torch.empty(self.batch, self.T, self.ncc, device=self.device) if content else None
        emb_s = torch.empty(self.batch, *self.style_shape, device=self.device) if style else None
        _lib.check(self.lib.ast_embeds(self.h, self._ptr(self._x(x)), self._ptr(emb_c),
                                       self._ptr(emb_s), self._stream()))
        return emb_c, emb_s

    def set_targets(self, phi_c: torch.Tensor, phi_s: torch.Tensor) -> None:
        """phi_c: [T, ncc] (shared) or [B, T, ncc]; phi_s: style_shape or [B, *style_shape]."""
        phi_c = phi_c.to(self.device, torch.float32).contiguous()
        phi_s = phi_s.to(self.device, torch.float32).contiguous()
        c_shared = phi_c.dim() == 2
        s_shared = phi_s.dim() == 3
        if tuple(phi_c.shape[-2:]) != (self.T, self.ncc):
            raise ValueError('phi_c shape %s != [.., %d, %d]' % (tuple(phi_c.shape), self.T, self.ncc))
        if tuple(phi_s.shape[-3:]) != tuple(self.style_shape):
            raise ValueError('phi_s shape %s != [.., %s]' % (tuple(phi_s.shape), self.style_shape))
        if not c_shared and phi_c.shape[0] != self.batch or not s_shared and phi_s.shape[0] != self.batch:
            raise ValueError('per-clip targets need a leading batch dimension of %d' % self.batch)
        self._targets = (phi_c, phi_s)       # keep alive: the context holds raw pointers
        _lib.check(self.lib.ast_set_targets(self.h, self._ptr(phi_c), int(c_shared),
                                            self._ptr(phi_s), int(s_shared)))

    def d_out_of_place(self, with_times: bool = False):
        """Whether this context keeps the Gram backward's D in a buffer of its own rather than
        in place over the activations (ast_workspace_bytes' memory-fit rule, then ast_create's
        timing of both placements); with_times: (flag, (ms in place, ms out of place)), -1 where
        not timed."""
        v = ctypes.c_int()
        ms = (ctypes.c_float * 2)()
        _lib.check(self.lib.ast_d_out_of_place(self.h, ctypes.byref(v), ctypes.cast(ms, ctypes.c_void_p)))
        return (bool(v.value), (ms[0], ms[1])) if with_times else bool(v.value)

    def set_cu_limit(self, cus: int) -> None:
        """At most ``cus`` CUs for the persistent split block kernels (0 = all): for running
        several engines (disjoint clip groups) concurrently on one GPU, one stream each."""
        _lib.check(self.lib.ast_set_cu_limit(self.h, int(cus)))
        self.gen += 1   # captured graphs hold the grid size: recapture

    def set_gamma(self, gamma: float) -> None:
        """The STFT regulariser weight (--gamma, methods.py:125)."""
        _lib.check(self.lib.ast_set_gamma(self.h, float(gamma)))
        self.gamma = float(gamma)
        self.gen += 1   # captured graphs hold launch parameters derived from gamma: recapture

    def loss_grad(self, x: torch.Tensor, grad: Optional[torch.Tensor] = None,
                  parts: Optional[torch.Tensor] = None):
        """Returns (parts [B, 4] = (total, content, style, reg), grad [B, T]).  reg is the STFT
        regulariser (methods.py:121-123), evaluated whatever gamma is, as TF does; total and
        grad include gamma * reg."""
        if self._targets is None:
            raise _lib.AstError('set_targets() first')
        if grad is None:
            grad = torch.empty(self.batch, self.T, device=self.device)
        if parts is None:
            parts = torch.empty(self.batch, 4, device=self.device)
        _lib.check(self.lib.ast_loss_grad(self.h, self._ptr(self._x(x)), self._ptr(grad),
                                          self._ptr(parts), self._stream()))
        return parts, grad

    def loss_grad_phase(self, x: torch.Tensor, grad: torch.Tensor, parts: torch.Tensor,
                        phase: int) -> None:
        """ast_loss_grad_phase: 1 = forward + Gram (fwd, style, bwd); 2 = the backward chain and
        the rest (needs phase 1 of the same x first); 0 = both."""
        if self._targets is None:
            raise _lib.AstError('set_targets() first')
        _lib.check(self.lib.ast_loss_grad_phase(self.h, self._ptr(self._x(x)), self._ptr(grad),
                                                self._ptr(parts), int(phase), self._stream()))

    def adam_step(self, x, m, v, grad, step, lr=1.0, beta1=0.9, beta2=0.999, eps=1e-8):
        _lib.check(self.lib.ast_adam_step(self.h, self._ptr(x), self._ptr(m), self._ptr(v),
                                          self._ptr(grad), int(step), float(lr), float(beta1),
                                          float(beta2), float(eps), self._stream()))

    def adam_step_dev(self, x, m, v, grad, step_dev, lr=1.0, beta1=0.9, beta2=0.999, eps=1e-8):
        """Adam with the step counter in device memory (int32 tensor, incremented in place)."""
        _lib.check(self.lib.ast_adam_step_dev(self.h, self._ptr(x), self._ptr(m), self._ptr(v),
                                              self._ptr(grad), self._ptr(step_dev, torch.int32), float(lr),
                                              float(beta1), float(beta2), float(eps),
                                              self._stream()))

    def range_flags(self, reset: bool = False) -> torch.Tensor:
        """Per-clip AST_RANGE_* flags [B] (int32, device), OR'ed over every loss_grad since the
        last reset (reset_range_flags, LbfgsLoop.begin, AdamLoop start, context creation):
        non-finite loss parts or gradient (1); in split mode a per-clip maximum or analytic
        operand bound outside the split-fp16 range (2: forward, 4: backward) or below 2^-60 (8).
        ``reset=True`` clears them after reading."""
        out = torch.empty(self.batch, dtype=torch.int32, device=self.device)
        _lib.check(self.lib.ast_range_flags(self.h, self._ptr(out, torch.int32), self._stream()))
        if reset:
            self.reset_range_flags()
        return out

    def range_flags_last(self) -> torch.Tensor:
        """The same flags for the most recent loss_grad alone (ast_range_flags_last)."""
        out = torch.empty(self.batch, dtype=torch.int32, device=self.device)
        _lib.check(self.lib.ast_range_flags_last(self.h, self._ptr(out, torch.int32), self._stream()))
        return out

    def reset_range_flags(self) -> None:
        _lib.check(self.lib.ast_range_flags_reset(self.h, self._stream()))

    @staticmethod
    def nonfinite_clips(parts: torch.Tensor, grad: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Per-clip flag [B] (bool, on the device): the clip's loss parts or its gradient hold a
        NaN / Inf (the reference would carry them into the next L-BFGS-B step)."""
        bad = ~torch.isfinite(parts).all(dim=1)
        if grad is not None:
            bad |= ~torch.isfinite(grad).all(dim=1)
        return bad

    def timing(self, enable: bool) -> None:
        _lib.check(self.lib.ast_timing(self.h, int(enable)))

    def timing_read(self):
        out = (ctypes.c_float * 7)()
        _lib.check(self.lib.ast_timing_read(self.h, out, 7))
        keys = ('block_fwd_ms', 'block_bwd_ms', 'gram_fwd_ms', 'gram_bwd_ms', 'other_ms',
                'calls', 'blocks')
        return dict(zip(keys, list(out)))


class AdamLoop:
    """The throughput-mode optimiser step on the device: ast_loss_grad + fused Adam over the
    audio buffer ``x`` [B, T] (optimised in place; Adam state and the step counter on the
    device).  With ``graph=True`` the step is captured once into a HIP graph
    (torch.cuda.CUDAGraph on the capture stream) and every ``step()`` is one graph replay.
    Capture runs one warm-up step eagerly and then restores x / m / v / the counter, so the
    state sequence is the same either way."""

    def __init__(self, eng: StyleEngine, x: torch.Tensor, lr: float = 1.0, beta1: float = 0.9,
                 beta2: float = 0.999, eps: float = 1e-8, graph: bool = False):
        self.eng = eng
        self.x = x
        self.m = torch.zeros_like(x)
        self.v = torch.zeros_like(x)
        self.grad = torch.empty_like(x)
        self.parts = torch.empty(eng.batch, 4, device=x.device)
        self.step_dev = torch.zeros(1, dtype=torch.int32, device=x.device)
        self.hp = (float(lr), float(beta1), float(beta2), float(eps))
        self.graph = None
        eng.reset_range_flags()   # range_flags() then covers every step of this loop
        if graph:
            self._capture()

    def _capture(self):
        x = self.x
        saved = [t.clone() for t in (self.x, self.m, self.v, self.step_dev)]
        side = torch.cuda.Stream(device=x.device)
        side.wait_stream(torch.cuda.current_stream(x.device))
        with torch.cuda.stream(side):
            self._eager()
        torch.cuda.current_stream(x.device).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._eager()
        for t, s in zip((self.x, self.m, self.v, self.step_dev), saved):
            t.copy_(s)
        self.eng.reset_range_flags()   # (the warm-up step is not one of the loop's steps)
        self.graph = g
        self._gen = self.eng.gen

    def _eager(self):
        self.eng.loss_grad(self.x, self.grad, self.parts)
        self.eng.adam_step_dev(self.x, self.m, self.v, self.grad, self.step_dev, *self.hp)

    def step(self):
        if self.graph is not None:
            if self._gen != self.eng.gen:   # gamma changed since capture
                self._capture()
            self.graph.replay()
        else:
            self._eager()
        return self.parts


class AdamGroups:
    """The throughput step over G disjoint clip groups on one GPU: one engine per group (its
    persistent block kernels limited to 1/G of the CUs, ast_set_cu_limit), its own stream and
    two captured graphs -- F = ast_loss_grad_phase 1 (encoder forward + Gram forward / style /
    Gram backward) and R = phase 2 + Adam (the backward chain, d loss / d x, the update).  Even
    groups replay F, R, F, R, ...; odd groups start one F ahead and replay R, F, R, F, ..., so
    one group's HBM-bound Gram kernels (the end of F) run while another group's MFMA-bound block
    kernels run on the other CUs (even groups F, R; odd groups R, F).  Every step() is one full
    step of every group; the groups'
    clips are independent, so each clip's trajectory is the one AdamLoop gives it alone.  The
    groups meet at the end of every step() (the current stream waits for them), so their phase
    offset cannot drift."""

    def __init__(self, engines, xs, lr=1.0, beta1=0.9, beta2=0.999, eps=1e-8, serial=False):
        self.engs, self.xs = list(engines), list(xs)
        self.serial = bool(serial)   # diagnostics: every group's graphs on the current stream
        dev = self.xs[0].device
        self.G = len(self.engs)
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        self.hp = (float(lr), float(beta1), float(beta2), float(eps))
        self.m = [torch.zeros_like(x) for x in self.xs]
        self.v = [torch.zeros_like(x) for x in self.xs]
        self.grad = [torch.empty_like(x) for x in self.xs]
        self.parts = [torch.empty(e.batch, 4, device=dev) for e in self.engs]
        self.step_dev = [torch.zeros(1, dtype=torch.int32, device=dev) for _ in self.engs]
        self.streams = [torch.cuda.Stream(device=dev) for _ in self.engs]
        self.graphs = []
        for g, e in enumerate(self.engs):
            if self.G > 1:
                e.set_cu_limit(max(ncu // self.G, 1))
            e.reset_range_flags()
            self.graphs.append(self._capture(g))
        self.primed = False

    def _front(self, g):
        self.engs[g].loss_grad_phase(self.xs[g], self.grad[g], self.parts[g], 1)

    def _back(self, g):
        e = self.engs[g]
        e.loss_grad_phase(self.xs[g], self.grad[g], self.parts[g], 2)
        e.adam_step_dev(self.xs[g], self.m[g], self.v[g], self.grad[g], self.step_dev[g], *self.hp)

    def _capture(self, g):
        st = (self.xs[g], self.m[g], self.v[g], self.step_dev[g])
        saved = [t.clone() for t in st]
        side = torch.cuda.Stream(device=self.xs[g].device)
        side.wait_stream(torch.cuda.current_stream(self.xs[g].device))
        with torch.cuda.stream(side):     # one eager step (allocator warm-up, as AdamLoop)
            self._front(g)
            self._back(g)
        torch.cuda.current_stream(self.xs[g].device).wait_stream(side)
        gf, gr = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(gf):
            self._front(g)
        with torch.cuda.graph(gr):
            self._back(g)
        for t, s in zip(st, saved):
            t.copy_(s)
        self.engs[g].reset_range_flags()
        return gf, gr

    def step(self):
        cur = torch.cuda.current_stream(self.xs[0].device)
        for g in range(self.G):
            self.streams[g].wait_stream(cur)
            with torch.cuda.stream(cur if self.serial else self.streams[g]):
                gf, gr = self.graphs[g]
                if g % 2 == 0:
                    gf.replay()
                    gr.replay()
                else:
                    if not self.primed:
                        gf.replay()
                    gr.replay()
                    gf.replay()
        self.primed = True
        for s in self.streams:
            cur.wait_stream(s)

    # (after step(): x, parts and grad of every group are those of its last full step; the
    #  groups started one F ahead hold the next step's F, which the next step() uses)


class LbfgsLoop:
    """The reference's optimiser on the device: one scipy L-BFGS-B ``minimize`` per clip
    (methods.py:132-137; no bounds, history ``m``, ``maxiter`` / ``maxls`` / ``ftol`` / ``gtol``
    as scipy's options), every clip advancing by one loss+grad evaluation per step
    (ast_loss_grad + ast_lbfgs_step, optionally replayed from a captured HIP graph).  ``x``
    [B, T] fp32 is the buffer the loss reads; the float64 iterate lives in the workspace."""

    FTOL = 2.220446049250313e-09      # scipy minimize(method='L-BFGS-B') defaults
    GTOL = 1e-5

    def __init__(self, eng: StyleEngine, m: int = 10, maxiter: int = 100, maxls: int = 20,
                 ftol: float = FTOL, gtol: float = GTOL, graph: bool = False):
        self.eng = eng
        dev = eng.device
        nb = ctypes.c_size_t()
        _lib.check(eng.lib.ast_lbfgs_workspace_bytes(eng.h, int(m), ctypes.byref(nb)))
        self.ws = torch.zeros(nb.value, dtype=torch.uint8, device=dev)
        self.x = torch.zeros(eng.batch, eng.T, device=dev)
        self.grad = torch.empty_like(self.x)
        self.parts = torch.zeros(eng.batch, 4, device=dev)
        self.info = torch.zeros(eng.batch, 4, dtype=torch.int32, device=dev)
        self.opts = (int(m), int(maxiter), int(maxls), float(ftol), float(gtol))
        self.started = False
        self.use_graph = bool(graph)
        self.graph = None

    def _p(self, t):
        return ctypes.c_void_p(t.data_ptr()) if t is not None else None

    def _eager(self):
        eng = self.eng
        eng.loss_grad(self.x, self.grad, self.parts)
        _lib.check(eng.lib.ast_lbfgs_step(eng.h, self._p(self.ws), self._p(self.x),
                                          self._p(self.grad), self._p(self.parts), eng._stream()))

    def begin(self, x0: Optional[torch.Tensor] = None, active: Optional[torch.Tensor] = None):
        """Start a minimize call per (active) clip from x0 [B, T] (float64), or from each clip's
        current point (the next epoch, methods.py:164-167)."""
        eng = self.eng
        if x0 is None and not self.started:
            raise _lib.AstError('the first begin() needs x0')
        if x0 is not None:
            x0 = x0.to(eng.device, torch.float64).contiguous()
            assert x0.shape == (eng.batch, eng.T)
        if active is not None:
            active = active.to(eng.device, torch.int32).contiguous()
        self._x0 = x0
        m, maxiter, maxls, ftol, gtol = self.opts
        _lib.check(eng.lib.ast_lbfgs_begin(eng.h, self._p(self.ws), self._p(self.x), self._p(x0),
                                           self._p(active), m, maxiter, maxls,
                                           ctypes.c_double(ftol), ctypes.c_double(gtol),
                                           eng._stream()))
        self.started = True

    def step(self):
        if self.use_graph:
            if self.graph is not None and self._gen != self.eng.gen:
                self.graph = None           # gamma changed since capture: capture again
            if self.graph is None:
                # captured at the first step after begin(): capture records the pair without
                # executing it, and the state lives in ws, so every replay is an eager step
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self._eager()
                self.graph = g
                self._gen = self.eng.gen
            self.graph.replay()
        else:
            self._eager()

    def state(self, with_x: bool = False):
        """(info [B, 4] int numpy = phase, iterations, evaluations, reason; x float64 [B, T] or
        None)."""
        x64 = torch.empty(self.eng.batch, self.eng.T, dtype=torch.float64,
                          device=self.eng.device) if with_x else None
        _lib.check(self.eng.lib.ast_lbfgs_state(self.eng.h, self._p(self.ws), self._p(self.info),
                                                self._p(x64), self.eng._stream()))
        return self.info.cpu().numpy(), x64

    def history(self, info=None):
        """Per clip, the (total, content, style, regularizer) parts of every evaluation of the
        current (or last) minimize call in evaluation order: a list of [n_b, 4] float64 arrays
        (n_b = the clip's evaluation count, info[:, 2]; ast_lbfgs_history)."""
        if info is None:
            info, _ = self.state()
        n = np.minimum(np.asarray(info)[:, 2], _lib.LBFGS_HISTORY)
        cap = max(1, int(n.max()) if n.size else 1)
        out = torch.empty(self.eng.batch, cap, 4, device=self.eng.device)
        _lib.check(self.eng.lib.ast_lbfgs_history(self.eng.h, self._p(self.ws), self._p(out), cap,
                                                  self.eng._stream()))
        h = out.cpu().numpy().astype(np.float64)
        return [h[b, :int(n[b])] for b in range(self.eng.batch)]

    def minimize(self, x0: Optional[torch.Tensor] = None, active=None, check_every: int = 4,
                 max_steps: int = 100000):
        """Run until every clip's minimize call has returned; returns the final info."""
        self.begin(x0, active)
        steps = 0
        while steps < max_steps:
            for _ in range(check_every):
                self.step()
            steps += check_every
            info, _ = self.state()
            if not info[:, 0].any():
                return info
        raise _lib.AstError('L-BFGS-B did not finish within %d steps' % max_steps)
