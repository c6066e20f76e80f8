"""Clip sharding across the GPUs of one node.

Clips are independent optimisation problems (one audio variable and one optimiser state per
clip, methods.py:49-54,132-137), so a batch of N clips is split into contiguous equal shards,
one per rank, with no collective in the step.  Every per-clip input is derived from the clip's
GLOBAL index, so a clip's inputs - and, the kernels being batch-invariant, its results - are
identical whichever rank or batch slot it lands in.  The only cross-rank traffic is the
barrier and the max-over-ranks of the timed region.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys

import numpy as np

CONTENT_SEED0 = 1000     # content clips default_rng(1000 + b)
STYLE_SEED0 = 5000       #             style clips   default_rng(5000 + b)
INIT_SEED0 = 9000        # starting-point perturbation per clip


def clip_range(total: int, world: int, rank: int) -> range:
    """Contiguous shard of `total` clips owned by `rank` (equal shards; remainder spread
    over the first ranks)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError('bad world/rank %d/%d' % (world, rank))
    q, r = divmod(total, world)
    lo = rank * q + min(rank, r)
    return range(lo, lo + q + (1 if rank < r else 0))


def shard_inputs(clips: range, T: int):
    """Synthetic content / style clips (mu-law units) and optimisation starting points for
    the given global clip indices: float32 arrays [n, T]."""
    from .utils import mu_law_numpy
    from .weights import synthetic_clips
    n = len(clips)
    cont = np.empty((n, T), np.float32)
    sty = np.empty((n, T), np.float32)
    x0 = np.empty((n, T), np.float32)
    for i, g in enumerate(clips):
        cont[i] = mu_law_numpy(synthetic_clips(1, T, CONTENT_SEED0 + g)[0])
        sty[i] = mu_law_numpy(synthetic_clips(1, T, STYLE_SEED0 + g)[0])
        x0[i] = cont[i] + np.random.default_rng(INIT_SEED0 + g).normal(0, 4.0, T).astype(np.float32)
    return cont, sty, x0


def max_over_ranks(v: float, world: int, device=None) -> float:
    """Max of a host scalar over all ranks (the bench's timed region)."""
    if world == 1:
        return v
    import torch
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _free_port() -> int:
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(gpus: int, target, argv, env_extra=None):
    """One process per GPU (bench.py --gpus N, the batch CLI --gpus N): when this process is
    not already a rank of a launcher (WORLD_SIZE unset) and gpus > 1, start `gpus` ranks of
    ``target`` (argv prefix: a script path, or ['-m', module]) under torch.distributed.run as a
    child process -- before anything touches the GPU -- and return its exit code.  Returns
    None when this process should run as the rank itself, 2 when WORLD_SIZE disagrees."""
    ws_env = os.environ.get('WORLD_SIZE')
    if ws_env is not None:
        if int(ws_env) != gpus:
            print('WORLD_SIZE=%s but --gpus %d' % (ws_env, gpus), file=sys.stderr)
            return 2
        return None
    if gpus <= 1:
        return None
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           '--nproc-per-node', str(gpus), '--master-addr', '127.0.0.1',
           '--master-port', str(_free_port()), *target, *argv]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get('HSA_ENABLE_IPC_MODE_LEGACY', '0'))
    env.update(env_extra or {})
    return subprocess.call(cmd, env=env)
