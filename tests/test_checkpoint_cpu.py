"""Checkpoint files (ValueIteration.save_checkpoint / load_checkpoint): plain .npz arrays, loaded
without pickle, round-trip exactly (the GPU side of resume is tests/test_gpu_resume.py)."""
import numpy as np

from minigrid_dynamicprogramming_amd.dp import ValueIteration


def test_checkpoint_npz_round_trip(tmp_path):
    rng = np.random.default_rng(0)
    ck = {"V": rng.random((3, 1024), dtype=np.float32), "pi": rng.integers(-1, 4, (3, 1024)).astype(np.int8),
          "sweeps": 17, "dv": 0.00123, "converged": False}
    path = tmp_path / "ck.npz"
    ValueIteration.save_checkpoint(path, ck)
    back = ValueIteration.load_checkpoint(path)
    assert back["sweeps"] == 17 and back["dv"] == 0.00123 and back["converged"] is False
    assert back["V"].dtype == np.float32 and back["pi"].dtype == np.int8
    np.testing.assert_array_equal(back["V"], ck["V"])
    np.testing.assert_array_equal(back["pi"], ck["pi"])
    z = np.load(path)  # no object arrays: loads with allow_pickle=False
    assert all(z[k].dtype != object for k in z.files)
