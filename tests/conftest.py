import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running CPU check")


@pytest.fixture(scope="session")
def oracle():
    import oracle as o
    o.build()
    return o


@pytest.fixture(scope="session")
def impli():
    # torch ships its own HIP runtime under the same soname: let it load (and initialise) first so
    # both share one runtime, as in bench.py -- the other order leaves torch without devices
    try:
        import torch
        torch.cuda.is_available()
    except Exception:
        pass
    import implisolid_amd as I
    if not os.path.exists(I.LIB_PATH):
        I.build()
    I.lib()
    return I


def mesh_edges(faces):
    e = np.sort(np.concatenate([faces[:, [0, 1]], faces[:, [1, 2]], faces[:, [2, 0]]]), axis=1)
    return np.unique(e, axis=0, return_counts=True)


def dumps(x):
    return json.dumps(x) if isinstance(x, (dict, list)) else x
