import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "dsp-audioreclabs_amd")
for p in (PKG, os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return np.load(os.path.join(GOLDEN, "features_golden.npz"))


@pytest.fixture(scope="session")
def knn_golden():
    import numpy as np
    return np.load(os.path.join(GOLDEN, "knn_golden.npz"))


def golden_keys(g):
    keys = sorted({k.split("/")[0] for k in g.files if k.startswith("L")})
    out = []
    for k in keys:
        L, S, w, v = k.split("_")
        out.append((k, int(L[1:]), int(S[1:]), w, int(v[3:])))
    return out


def golden_clip(g, i):
    off = g["offsets"]
    return g["pcm"][off[i]:off[i + 1]]
