"""Helpers to read the committed golden fixtures (tests/golden/*.npz, made by make_golden.py)."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

SEE_THROUGH = {"empty5": True, "empty16": True}  # EmptyEnv(see_through_walls=True), empty.py:88


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def table_names():
    return sorted(os.path.basename(p)[len("table_"):-4] for p in glob.glob(os.path.join(GOLDEN, "table_*.npz")))


def traj_names():
    """The family trajectories of make_golden.py (traj_box.npz, make_golden_box.py, has its own schema
    and tests)."""
    names = (os.path.basename(p)[len("traj_"):-4] for p in glob.glob(os.path.join(GOLDEN, "traj_*.npz")))
    return sorted(n for n in names if n != "box")


def cells_from_enc(enc):
    """Reference x-major (W,H,3) encode -> row-major (H,W) type codes."""
    return np.ascontiguousarray(np.asarray(enc)[:, :, 0].T.astype(np.uint8))


def digests():
    with open(os.path.join(GOLDEN, "digests.json")) as f:
        return json.load(f)
