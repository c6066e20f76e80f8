"""CPU restatement of the reference's ADMM optimal-transport palette solver
(optimal_transport.py:22-162) — TEST INFRASTRUCTURE: imported only by tests/ as the checker of
the HIP solver (csrc/ot_admm.hip, ast_ot_admm).

PARITY UNPINNED: the reference ships no OT tests or fixtures, and executing its module to make
some was refused in this environment (round 2), so this restatement is checked
against the reference's text only, plus invariants the tests assert (plan >= 0, the total /
row / column constraints within the ADMM tolerance, cost-matrix identities).  Same numpy
operations in the same order as the reference; it also reports the ADMM iteration count,
which the reference does not return."""
from __future__ import annotations

import numpy as np


def cost_matrix(p1, p2):
    """optimal_transport.py:22-37: Euclidean distances, squared differences accumulated
    feature by feature (in feature order), then sqrt."""
    c = np.zeros((p1.shape[0], p2.shape[0]))
    for k in range(p1.shape[1]):
        c += (p1[:, k][:, None] - p2[:, k][None, :]) ** 2
    return np.sqrt(c)


def project_total(x, target):
    """optimal_transport.py:40-47."""
    return x + (target - x.sum()) / x.size


def project_row_sums(x, lo, hi):
    """optimal_transport.py:50-74: shift each row whose sum is outside [lo_i, hi_i] onto the
    nearest bound (lo, hi: per-row arrays)."""
    out = np.array(x)
    s = x.sum(1)
    below = s < lo
    out[below, :] = out[below, :] + ((lo[below] - s[below]) / out.shape[1])[:, None]
    above = s > hi
    out[above, :] = out[above, :] + ((hi[above] - s[above]) / out.shape[1])[:, None]
    return out


def ot_admm(p_mod, p_ref, eps=1e-4, miter=1e5):
    """optimal_transport.py:77-137.  Returns (plan [n1, n2], iterations)."""
    C = cost_matrix(p_mod, p_ref)
    C = C / C.max()
    n1, n2 = C.shape
    lo1, hi1 = np.zeros(n1), np.full(n1, 1.0 / n1)
    lo2, hi2 = np.zeros(n2), np.full(n2, 1.0 / n2)
    lam = np.zeros((3,) + C.shape)
    aux = np.zeros((3,) + C.shape)
    old = np.zeros(C.shape)
    rho = 1e2
    it = 0
    while True:
        sol = (-C + rho * np.sum(aux, 0) + np.sum(lam, 0)) / (3 * rho)
        sol[sol < 0] = 0.
        for i in range(3):
            aux[i] = sol - lam[i] / rho
        aux[0] = project_row_sums(aux[0], lo1, hi1)
        aux[1] = project_row_sums(aux[1].T, lo2, hi2).T
        aux[2] = project_total(aux[2], 1.)
        for i in range(3):
            lam[i] += rho * (aux[i] - sol)
        ns = np.linalg.norm(sol)
        if it > miter:
            break
        if (np.linalg.norm(sol - old) < eps * ns and np.linalg.norm(sol - aux[0]) < eps * ns
                and np.linalg.norm(sol - aux[1]) < eps * ns and np.linalg.norm(sol - aux[2]) < eps * ns):
            break
        old[:, :] = sol
        it += 1
    return sol, it


def transform_palette(p_orig, p_target, plan):
    """optimal_transport.py:140-148."""
    return np.dot(plan, p_target) / (plan.sum(1) + 1e-10)[:, None]


def compute_permutation(w1, w2):
    """optimal_transport.py:151-162."""
    plan, _ = ot_admm(w1, w2)
    return transform_palette(w1, w2, plan)
