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
