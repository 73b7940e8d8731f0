"""Shared checks of the GPU parity tests (test infrastructure)."""
import numpy as np


def assert_same(pg, sg, po, so, equal_nan=False):
    """Bitwise identity of populations and of every status field (tolerance: none)."""
    assert np.array_equal(sg["iterations"], so["iterations"]), (sg["iterations"], so["iterations"])
    assert np.array_equal(sg["converged"], so["converged"])
    assert np.array_equal(sg["used_plain_retry"], so["used_plain_retry"])
    for f in ("eq_error", "rel_error", "pop_error"):
        assert np.array_equal(sg[f], so[f], equal_nan=equal_nan), f
    same = (pg == po) | (np.isnan(pg) & np.isnan(po)) if equal_nan else (pg == po)
    bad = np.argwhere(~same)
    assert bad.size == 0, f"{len(bad)} population entries differ, first {bad[:3].tolist()}"


def overlap_dx(prob, layers):
    """|dx| of every two-line overlap group in every layer (iteration_lvg.cpp:454-458):
    (E_u1 - E_l1 - E_u2 + E_l2) c / (E_line1 vw). Returns (groups [n, 5], |dx| [L, n])."""
    from oracle import oracle
    G = oracle.line_groups(prob)
    pairs = G[G[:, 0] == 2]
    E = prob.mol.energy
    kB, c = 1.380649e-16, 2.99792458e10
    vw = np.sqrt(2 * kB * layers.temp_n / prob.mol.mass + layers.vel_turb ** 2)
    num = (E[pairs[:, 1]] - E[pairs[:, 2]] - E[pairs[:, 3]] + E[pairs[:, 4]]) * c / (E[pairs[:, 1]] - E[pairs[:, 2]])
    return pairs, np.abs(num[None, :] / vw[:, None])
