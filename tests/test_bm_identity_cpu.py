"""The identity behind rs_bm_k's B records (rs_fast.hip, "Omega or B"):
Omega(x0) B(x0) = x0^31 at every root x0 of Lambda after the reference's 32
Berlekamp-Massey iterations (Karn's B), on random words with <= 16 errors and
on fast-path miscorrections, for several fcr / prim.  Pure-Python restatement
(tools/probes/bm_b_identity.py); the kernels themselves are checked bit for
bit against the oracle by the -m gpu split tests and smoke()."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "probes"))
import bm_b_identity as I  # noqa: E402


@pytest.mark.parametrize("fcr,prim", [(1, 1), (0, 1), (5, 7), (112, 11)])
def test_omega_times_b_at_roots(fcr, prim):
    tot, good, mis = I.check(fcr, prim, trials=24, seed=fcr + prim)
    assert tot > 100 and good == tot and mis > 0
