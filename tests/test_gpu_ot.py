"""HIP ADMM optimal transport (ast_ot_admm, csrc/ot_admm.hip) against the oracle restatement of
optimal_transport.py:22-162 (parity unpinned: DESIGN.md §5).  Both are fp64 with the same
update arithmetic; only the order of the sums and norms differs, so the two stop at the same
iteration (or one apart) and the plans agree to round-off (1e-9 rel-L2; 1e-3 if the stop is one
iteration apart, the stopping test's eps being 1e-4)."""
import numpy as np
import pytest
import torch

from oracle import ot_oracle as O

pytestmark = pytest.mark.gpu


def rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def _pal(n1, n2, d, seed):
    r = np.random.RandomState(seed)
    return r.rand(n1, d), r.rand(n2, d)


@pytest.mark.parametrize('n1,n2,d,seed', [(5, 10, 128, 0), (10, 5, 128, 1), (3, 7, 4, 2),
                                          (12, 9, 16, 3), (1, 4, 8, 4), (16, 16, 32, 5),
                                          (40, 24, 64, 6)])
def test_ot_admm_matches_oracle(n1, n2, d, seed):
    from audio_style_transfer_amd import optimal_transport as OT
    w1, w2 = _pal(n1, n2, d, seed)
    plan_o, it_o = O.ot_admm(w1, w2)
    plan, pal, its = OT.ot_admm_batched(w1[None], w2[None])
    plan, pal, it = plan[0].cpu().numpy(), pal[0].cpu().numpy(), int(its[0])
    print('%dx%d d=%d: iterations hip %d oracle %d, plan rel-L2 %.2e' % (n1, n2, d, it, it_o,
                                                                         rel(plan, plan_o)))
    assert abs(it - it_o) <= 1
    assert rel(plan, plan_o) <= (1e-9 if it == it_o else 1e-3)
    pal_o = O.transform_palette(w1, w2, plan_o)
    assert rel(pal, pal_o) <= (1e-9 if it == it_o else 1e-3)
    # the reference-named wrappers
    assert np.array_equal(OT.OT_ADMM(w1, w2), plan)
    assert np.array_equal(OT.compute_permutation(w1, w2), pal)


def test_ot_batch_invariance_and_limits():
    from audio_style_transfer_amd import optimal_transport as OT
    from audio_style_transfer_amd._lib import AstError
    r = np.random.RandomState(7)
    B = 300
    a, b = r.rand(B, 5, 128), r.rand(B, 10, 128)
    plans, pals, its = OT.ot_admm_batched(a, b)
    for k in (0, 1, 150, B - 1):
        p1, q1, i1 = OT.ot_admm_batched(a[k:k + 1], b[k:k + 1])
        assert torch.equal(p1[0], plans[k]) and torch.equal(q1[0], pals[k]) and int(i1[0]) == int(its[k])
    po, _ = O.ot_admm(a[150], b[150])
    assert rel(plans[150].cpu().numpy(), po) <= 1e-3
    # largest register-kernel problem: 64 x 64 cells
    p, _, it = OT.ot_admm_batched(r.rand(1, 64, 8), r.rand(1, 64, 8), miter=300)
    assert int(it[0]) <= 301 and torch.isfinite(p).all()
    with pytest.raises(ValueError, match='n1 \\* n2 <= 65536'):   # past 2^16 cells
        OT.ot_admm_batched(r.rand(1, 300, 1), r.rand(1, 300, 1))
    p0, _, _ = OT.ot_admm_batched(np.zeros((0, 3, 4)), np.zeros((0, 5, 4)))
    assert p0.shape == (0, 3, 5)


def test_ot_helpers_match_oracle():
    from audio_style_transfer_amd import optimal_transport as OT
    w1, w2 = _pal(5, 10, 128, 0)
    assert rel(OT.build_moving_cost_matrix(w1, w2), O.cost_matrix(w1, w2)) <= 1e-15
    r = np.random.RandomState(100)
    x = r.normal(0, 0.05, (6, 9))
    bounds = np.array([[0, 1]] * 6) / 6.0
    assert rel(OT.projection_column_sum_in_range(x, bounds),
               O.project_row_sums(x, np.zeros(6), np.full(6, 1 / 6.))) <= 1e-15
    assert rel(OT.projection_sum_equal(x, 1.0), O.project_total(x, 1.0)) <= 1e-15
    plan, _ = O.ot_admm(w1, w2)
    assert rel(OT.transform_palette(w1, w2, plan), O.transform_palette(w1, w2, plan)) <= 1e-14


@pytest.mark.parametrize('n1,n2,d,seed', [(65, 64, 4, 9), (80, 80, 16, 8), (100, 70, 8, 10)])
def test_ot_admm_large_palettes(n1, n2, d, seed):
    """Past the register kernel's n1 n2 <= 4096: the device-workspace kernel (k_ot_admm_big),
    same iteration count as the oracle (or one apart) and the plan to round-off; two problems
    in one call are each what a single call gives."""
    from audio_style_transfer_amd import optimal_transport as OT
    r = np.random.RandomState(seed)
    w1, w2 = r.rand(n1, d), r.rand(n2, d)
    plan_o, it_o = O.ot_admm(w1, w2)
    plan, pal, its = OT.ot_admm_batched(np.stack([w1, w1[::-1].copy()]), np.stack([w2, w2]))
    p0, q0, it = plan[0].cpu().numpy(), pal[0].cpu().numpy(), int(its[0])
    print('%dx%d d=%d: iterations hip %d oracle %d, plan rel-L2 %.2e' % (n1, n2, d, it, it_o, rel(p0, plan_o)))
    assert abs(it - it_o) <= 1
    assert rel(p0, plan_o) <= (1e-9 if it == it_o else 1e-3)
    assert rel(q0, O.transform_palette(w1, w2, plan_o)) <= (1e-9 if it == it_o else 1e-3)
    p1, _, i1 = OT.ot_admm_batched(w1[::-1].copy()[None], w2[None])
    assert torch.equal(p1[0], plan[1]) and int(i1[0]) == int(its[1])
