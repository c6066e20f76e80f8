"""ctypes binding of libastyle.so (include/astyle.h).

The product path has no fallback: if the in-tree library is missing or fails to load, every
entry point raises.  Device buffers are torch tensors on the context's device; their
``data_ptr()`` crosses the C ABI together with the current HIP stream.
"""
from __future__ import annotations

import ctypes
import os

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('ASTYLE_LIB', os.path.join(PKG, 'libastyle.so'))
MAX_TAPS = 32
# per-clip flags of ast_range_flags (include/astyle.h)
RANGE_NONFINITE, RANGE_ACT, RANGE_GRAD, RANGE_TINY = 1, 2, 4, 8
LBFGS_HISTORY = 4096    # AST_LBFGS_HISTORY: evaluations per minimize call kept for ast_lbfgs_history

# Every symbol include/astyle.h declares (checked by tests/test_abi.py).
EXPORTS = ('ast_create', 'ast_destroy', 'ast_workspace_bytes', 'ast_d_out_of_place', 'ast_set_weight', 'ast_forward',
           'ast_get_extract', 'ast_embeds', 'ast_content_cols', 'ast_set_targets',
           'ast_set_gamma', 'ast_loss_grad', 'ast_loss_grad_phase', 'ast_range_flags', 'ast_range_flags_last', 'ast_range_flags_reset', 'ast_set_cu_limit', 'ast_adam_step', 'ast_adam_step_dev',
           'ast_lbfgs_workspace_bytes', 'ast_lbfgs_begin', 'ast_lbfgs_step', 'ast_lbfgs_state',
           'ast_lbfgs_history',
           'ast_timing', 'ast_timing_read', 'ast_ot_admm', 'ast_ckpt_open', 'ast_ckpt_close',
           'ast_ckpt_num_entries', 'ast_ckpt_entry', 'ast_ckpt_read_f32', 'ast_restore',
           'ast_last_error')


class AstCfg(ctypes.Structure):
    _fields_ = [('batch', ctypes.c_int), ('T', ctypes.c_int),
                ('n_cont', ctypes.c_int), ('cont_ids', ctypes.c_int * MAX_TAPS),
                ('cnt_channels', ctypes.c_int),
                ('n_style', ctypes.c_int), ('style_ids', ctypes.c_int * MAX_TAPS),
                ('nb_channels', ctypes.c_int), ('gatys', ctypes.c_int),
                ('precision', ctypes.c_int), ('lambd', ctypes.c_float),
                ('gamma', ctypes.c_float)]


class AstError(RuntimeError):
    pass


_lib = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load (once) the in-tree HIP library; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise AstError('libastyle.so not built (%s): run __graft_entry__.build() or '
                       'python audio_style_transfer_amd/_build.py' % path)
    lib = ctypes.CDLL(path)
    vp, i, f, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
    fp = ctypes.POINTER(ctypes.c_float)
    sig = {
        'ast_create': (i, [ctypes.POINTER(AstCfg), i, ctypes.POINTER(vp)]),
        'ast_destroy': (None, [vp]),
        'ast_workspace_bytes': (i, [ctypes.POINTER(AstCfg), ctypes.POINTER(sz)]),
        'ast_d_out_of_place': (i, [vp, ctypes.POINTER(i), vp]),
        'ast_set_weight': (i, [vp, ctypes.c_char_p, fp, sz]),
        'ast_forward': (i, [vp, vp, vp]),
        'ast_get_extract': (i, [vp, i, vp, vp]),
        'ast_embeds': (i, [vp, vp, vp, vp, vp]),
        'ast_content_cols': (i, [vp]),
        'ast_set_targets': (i, [vp, vp, i, vp, i]),
        'ast_set_gamma': (i, [vp, f]),
        'ast_loss_grad': (i, [vp, vp, vp, vp, vp]),
        'ast_loss_grad_phase': (i, [vp, vp, vp, vp, i, vp]),
        'ast_range_flags': (i, [vp, vp, vp]),
        'ast_range_flags_last': (i, [vp, vp, vp]),
        'ast_range_flags_reset': (i, [vp, vp]),
        'ast_set_cu_limit': (i, [vp, i]),
        'ast_adam_step': (i, [vp, vp, vp, vp, vp, i, f, f, f, f, vp]),
        'ast_adam_step_dev': (i, [vp, vp, vp, vp, vp, vp, f, f, f, f, vp]),
        'ast_lbfgs_workspace_bytes': (i, [vp, i, ctypes.POINTER(sz)]),
        'ast_lbfgs_begin': (i, [vp, vp, vp, vp, vp, i, i, i, ctypes.c_double, ctypes.c_double, vp]),
        'ast_lbfgs_step': (i, [vp, vp, vp, vp, vp, vp]),
        'ast_lbfgs_state': (i, [vp, vp, vp, vp, vp]),
        'ast_lbfgs_history': (i, [vp, vp, vp, i, vp]),
        'ast_timing': (i, [vp, i]),
        'ast_timing_read': (i, [vp, fp, i]),
        'ast_ot_admm': (i, [vp, vp, i, i, i, i, ctypes.c_double, ctypes.c_double, vp, vp, vp, vp]),
        'ast_ckpt_open': (i, [ctypes.c_char_p, ctypes.POINTER(vp)]),
        'ast_ckpt_close': (None, [vp]),
        'ast_ckpt_num_entries': (i, [vp]),
        'ast_ckpt_entry': (i, [vp, i, ctypes.c_char_p, sz, ctypes.POINTER(i), ctypes.POINTER(i),
                               ctypes.POINTER(ctypes.c_int64), i]),
        'ast_ckpt_read_f32': (i, [vp, ctypes.c_char_p, fp, sz]),
        'ast_restore': (i, [vp, ctypes.c_char_p]),
        'ast_last_error': (ctypes.c_char_p, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int) -> None:
    if rc != 0:
        msg = load().ast_last_error()
        raise AstError('libastyle error %d: %s' % (rc, msg.decode() if msg else ''))
