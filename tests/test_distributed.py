"""CPU: the N>1 path — clip sharding with no data-path collective, exercised
with world_size-2 gloo process groups.  Each rank builds its shard's inputs from global clip
indices, evaluates them (CPU oracle as the stand-in compute), and the gathered per-clip
results must equal a single-process run over all clips; the timed-region max-over-ranks is
checked too."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from audio_style_transfer_amd.shard import clip_range, max_over_ranks, shard_inputs

T = 512
KW = dict(cont_ids=[9], style_ids=list(range(10)), gatys=False, nb_channels=128,
          cnt_channels=128)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _evaluate(clips):
    from oracle import astyle_oracle as O
    from audio_style_transfer_amd.weights import synthetic_weights
    W = synthetic_weights(0)
    cont, sty, x0 = shard_inputs(clips, T)
    out = []
    for i in range(len(clips)):
        phi_c, phi_s = O.targets_from_audio(W, cont[i].astype(np.float64),
                                            [sty[i].astype(np.float64)],
                                            [cont[i].astype(np.float64)], **KW)
        parts, g = O.loss_and_grad(x0[i].astype(np.float64), W, phi_c=phi_c, phi_s=phi_s,
                                   lambd=100.0, **KW)
        out.append(np.concatenate([parts[:3], g]))
    return np.stack(out)


def _worker(rank, world, port, total, outdir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        mine = clip_range(total, world, rank)
        res = _evaluate(mine)
        parts = [None] * world
        dist.all_gather_object(parts, res)      # logging-only gather (outputs to the host)
        el = max_over_ranks(1.0 + rank, world)
        if rank == 0:
            np.save(os.path.join(outdir, 'gathered.npy'), np.concatenate(parts))
            np.save(os.path.join(outdir, 'max.npy'), np.array([el]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('total,world', [(256, 1), (256, 2), (2048, 8), (7, 3), (2, 4)])
def test_clip_range_partitions(total, world):
    got = [list(clip_range(total, world, r)) for r in range(world)]
    flat = [c for g in got for c in g]
    assert flat == list(range(total))
    assert max(map(len, got)) - min(map(len, got)) <= 1


def test_shard_inputs_follow_global_index():
    c_all, s_all, x_all = shard_inputs(range(0, 4), T)
    c, s, x = shard_inputs(range(2, 4), T)
    assert np.array_equal(c, c_all[2:]) and np.array_equal(s, s_all[2:]) and np.array_equal(x, x_all[2:])


def test_two_rank_gloo_matches_single_process(tmp_path):
    total, world = 3, 2
    mp.spawn(_worker, args=(world, _free_port(), total, str(tmp_path)), nprocs=world, join=True)
    gathered = np.load(tmp_path / 'gathered.npy')
    ref = _evaluate(range(total))
    assert gathered.shape == ref.shape
    assert np.array_equal(gathered, ref)
    assert float(np.load(tmp_path / 'max.npy')[0]) == 2.0


# ----------------------------------------------------------------------------- bench.py
def _bench(args, env_extra=None, timeout=240):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([os.path.join(root, 'tests'), root]))
    env.pop('WORLD_SIZE', None)
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(root, 'bench.py'), *args], env=env,
                       capture_output=True, text=True, timeout=timeout)
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r.stderr


STUB = ['--engine', 'bench_stub:StubEngine', '--backend', 'gloo', '--T', '512', '--steps', '2',
        '--warmup', '1', '--cpu-baseline-seconds', '0', '--side-steps', '0', '--graph', '0']


def test_bench_launcher_starts_ranks():
    """`bench.py --gpus 2` with no launcher around it starts 2 ranks itself (torch.distributed.run)
    and rank 0 reports the whole job: n_gpus 2, 2 x clips clips, the bench's own rank logic
    (clip shards by global index, warm-up, barrier-bracketed timing, max over ranks)."""
    rc, out, err = _bench(['--gpus', '2', '--clips', '3', *STUB])
    assert rc == 0, err[-2000:]
    assert out['n_gpus'] == 2 and out['config']['global_batch_clips'] == 6, out
    assert out['scaling'] == 'weak' and out['config']['parallelism'] == 'clip-sharded x2'
    assert out['value'] > 0 and out['nonfinite_clips'] == 0


def test_bench_refuses_mismatched_world_size():
    rc, out, err = _bench(['--gpus', '4', '--clips', '2', *STUB], env_extra={'WORLD_SIZE': '2'})
    assert rc == 2 and out is None, (rc, err)


def test_bench_rank_results_match_single_process():
    """Rank 0 of a 2-rank run owns global clips 0, 1 — the same clips a 1-rank run with 2 clips
    owns — so its losses (first and last timed step) are identical: shards are built from the
    global clip index and the step does not depend on the other rank."""
    rc1, out1, e1 = _bench(['--gpus', '1', '--clips', '2', *STUB])
    rc2, out2, e2 = _bench(['--gpus', '2', '--clips', '2', *STUB])
    assert rc1 == 0 and rc2 == 0, (e1[-1000:], e2[-1000:])
    assert out1['config']['global_batch_clips'] == 2 and out2['config']['global_batch_clips'] == 4
    assert out1['loss_first_last'] == out2['loss_first_last']
