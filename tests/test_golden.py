"""Committed golden fixtures (tests/golden/*.npz, made by tests/golden/gen_golden.py from the oracle):
the oracle must reproduce them on CPU; the HIP engine must reproduce them bit for bit on the GPU."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import gen_golden as G  # noqa: E402

NAMES = sorted(G.SCENARIOS)


def check(obs, exp):
    assert set(obs) == set(exp)
    assert all(exp[k][0] > 0 for k in exp if k.startswith("stats")), "fixture must append records"
    for k in sorted(exp):
        assert np.array_equal(np.asarray(obs[k]).reshape(exp[k].shape).astype(exp[k].dtype), exp[k]), k


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_golden(oracle_mod, name):
    fx, exp = G.load(name)
    with oracle_mod.OracleEngine(fx["cfg"]) as ora:
        check(G.run(ora, fx), exp)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_engine_reproduces_golden(name):
    from ripplemq_amd.engine import Engine

    fx, exp = G.load(name)
    with Engine(fx["cfg"]) as eng:
        check(G.run(eng, fx), exp)
