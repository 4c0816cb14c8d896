"""The float64 one-step restatement (tests/_onestep.py) against the reference's own float64
replay of every saved state (tests/golden/onestep_cfg1.json checksums, written by
make_golden.py from scripts/train_gat_custom.py's classes).  This pins the float64 step the
GPU one-step test measures our kernels against: the same triples (our sampler replaying the
saved ``random`` state), the same loss, gradients and post-Adam item rows."""
import numpy as np
import pytest

import _onestep

STATES = (0, 1, 2, 5, 8, 12, 16, 19)


@pytest.fixture(scope="module")
def fixture():
    return _onestep.load()


@pytest.fixture(scope="module")
def inp(pkg):
    return _onestep.inputs(pkg)


@pytest.mark.parametrize("s", STATES)
def test_f64_step_matches_reference_f64_replay(pkg, oracle, fixture, inp, s):
    arrays, meta = fixture
    ms = meta["states"][str(s)]
    st = _onestep.load_state(arrays, meta, s)
    assert st["step"] == ms["step_count"] == float(s)
    r = _onestep.f64_step(pkg, oracle, st, inp)
    u, i, j = r["triples"]
    assert [int(u[0]), int(i[0]), int(j[0])] == ms["triples_head"]
    ck = ms["f64_checksums"]
    assert abs(r["loss"] - ms["loss"]["f64"]) <= 1e-13 * abs(ms["loss"]["f64"])
    for k, g in r["grads"].items():
        assert abs(float(g.norm()) - ck["grad_l2"][k]) <= 1e-11 * ck["grad_l2"][k], k
        assert abs(float(g.abs().max()) - ck["grad_maxabs"][k]) <= 1e-11 * ck["grad_maxabs"][k], k
    assert abs(float(np.linalg.norm(r["items"])) - ck["next_items_l2"]) <= 1e-11 * ck["next_items_l2"]
    # the reference's fp32 replays: no sign flips against float64 and no lr-sized step
    # differences -- the state is well conditioned, so the GPU test can hold ours to the same
    for t, gs in ms["grad_vs_f64"].items():
        assert all(v["sign_flips"] == 0 for v in gs.values()), (t, gs)
    assert all(v == 0 for v in ms["next_params_lr_flips_vs_f64"].values())
