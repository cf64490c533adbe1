"""Checkpoint / resume (SURVEY section 5 aux "checkpoint / resume": Jacobi is memoryless given V_k):
a solve stopped by max_sweeps, checkpointed to .npz and resumed on a NEW handle with the normal cap
ends at the same global stopping sweep with V, pi and dV bit-identical to the uninterrupted solve
and to the CPU oracle.  Batched XYD and DoorKey grids (fused method, both dtypes) and the lone grid
(whose resumed solve runs a launch, not the resident server)."""
import numpy as np
import pytest

import minigrid_dynamicprogramming_amd as mg
from minigrid_dynamicprogramming_amd._lib import MgdpError
from oracle import oracle
from tests.golden_util import cells_from_enc, load

pytestmark = pytest.mark.gpu


def fourrooms(n):
    g = load("grids_fourrooms.npz")
    return np.stack([cells_from_enc(e) for e in g["enc"][:n]])


def doorkey(n):
    return np.stack([cells_from_enc(load("table_doorkey8_s2.npz")["enc"])] * n)


def empty16():
    enc, _ = mg.make("MiniGrid-Empty-16x16-v0").generate(seed=0)
    return np.ascontiguousarray(enc[:, :, 0].T)[None]


CASES = [("fourrooms", lambda: fourrooms(16), 0), ("doorkey", lambda: doorkey(4), 1), ("empty16", empty16, 0)]


@pytest.mark.parametrize("dtype", ["f32", "f64"])
@pytest.mark.parametrize("name,make,model", CASES)
@pytest.mark.parametrize("cap", [1, 7, 20])
def test_resume_matches_uninterrupted(name, make, model, dtype, cap, tmp_path):
    cells = make()
    full = mg.ValueIteration(cells, dtype=dtype)
    full.solve()
    k_full, dv_full, V_full, pi_full = full.sweeps, full.dv, full.values(), full.policy()
    full.close()
    assert k_full > cap
    part = mg.ValueIteration(cells, dtype=dtype, max_sweeps=cap)
    part.solve()
    assert part.sweeps == cap and not part.converged
    path = tmp_path / "ckpt.npz"
    mg.ValueIteration.save_checkpoint(path, part.checkpoint())
    part.close()
    ck = mg.ValueIteration.load_checkpoint(path)
    res = mg.ValueIteration(cells, dtype=dtype)
    k = res.resume(ck)
    assert k == res.sweeps == k_full
    assert res.dv == dv_full and res.converged
    np.testing.assert_array_equal(res.values(), V_full)
    np.testing.assert_array_equal(res.policy(), pi_full)
    o = oracle.value_iteration(model, cells, dtype=dtype)
    assert o["sweeps"] == k_full
    np.testing.assert_array_equal(res.values(), o["V"])
    np.testing.assert_array_equal(res.policy(), o["pi"])
    res.close()


def test_resume_refuses_converged_and_bad_shapes():
    cells = fourrooms(4)
    vi = mg.ValueIteration(cells, dtype="f32")
    vi.solve()
    ck = vi.checkpoint()
    assert ck["converged"]
    with pytest.raises(ValueError):
        vi.resume(ck)  # final: pi of a converged checkpoint is not rebuildable from V_k
    bad = dict(ck, V=ck["V"][:2], converged=False, dv=1.0)
    with pytest.raises(ValueError):
        vi.resume(bad)
    vi.close()


def test_resume_sweep_method_refused():
    cells = fourrooms(2)
    vi = mg.ValueIteration(cells, dtype="f32", method="sweep", max_sweeps=5)
    vi.solve()
    with pytest.raises((ValueError, MgdpError)):
        vi.resume(vi.checkpoint())
    vi.close()


def test_resume_refuses_other_grids_params_and_dtype(tmp_path):
    """a checkpoint carries the grids' digest, dtype and parameters; resume refuses a
    mismatch instead of casting or continuing on the wrong grids."""
    cells = fourrooms(4)
    part = mg.ValueIteration(cells, dtype="f32", max_sweeps=5)
    part.solve()
    path = tmp_path / "c.npz"
    mg.ValueIteration.save_checkpoint(path, part.checkpoint())
    part.close()
    ck = mg.ValueIteration.load_checkpoint(path)
    assert ck["meta"]["dtype"] == "f32" and ck["meta"]["cells_sha256"]
    for kw, grids in [(dict(dtype="f64"), cells), (dict(dtype="f32", gamma=0.9), cells),
                      (dict(dtype="f32", tol=1e-5), cells), (dict(dtype="f32"), fourrooms(5)[1:])]:
        vi = mg.ValueIteration(grids, **kw)
        with pytest.raises(ValueError):
            vi.resume(ck)
        vi.close()
    blind = dict(ck)
    blind.pop("meta")
    vi = mg.ValueIteration(cells, dtype="f32")
    with pytest.raises(ValueError):
        vi.resume(blind)
    assert vi.resume(ck) == vi.sweeps and vi.converged  # the matching handle resumes
    vi.close()
