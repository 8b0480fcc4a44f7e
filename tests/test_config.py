"""Process-wide knobs (cycloneml_amd/config.py)."""
import os
import subprocess
import sys

import pytest

from cycloneml_amd import config


def test_devices(monkeypatch):
    monkeypatch.delenv("CYCLONE_DEVICES", raising=False)
    assert config.devices() is None
    assert config.device_for_local_rank(3) == 3
    monkeypatch.setenv("CYCLONE_DEVICES", "4, 6,7")
    assert config.devices() == [4, 6, 7]
    assert config.device_for_local_rank(1) == 6
    with pytest.raises(ValueError):
        config.device_for_local_rank(3)
    monkeypatch.setenv("CYCLONE_DEVICES", "0,-1")
    with pytest.raises(ValueError):
        config.devices()


def test_strict_parity_flag(monkeypatch):
    monkeypatch.delenv("CYCLONE_STRICT_PARITY", raising=False)
    assert not config.strict_parity()
    monkeypatch.setenv("CYCLONE_STRICT_PARITY", "1")
    assert config.strict_parity()
    monkeypatch.setenv("CYCLONE_STRICT_PARITY", "0")
    assert not config.strict_parity()


@pytest.mark.gpu
def test_strict_parity_kmeans_matches(cuda):
    """CYCLONE_STRICT_PARITY=1 in a child process: no carried state (the
    bounds and incremental counters stay at zero) and the same assignments
    as the default path."""
    code = r'''
import os, sys, numpy as np, torch
sys.path.insert(0, os.getcwd())
from cycloneml_amd.clustering import KMeansPlan, row_norms
dev = torch.device("cuda", 0)
rng = np.random.default_rng(3)
k, d, n = 130, 64, 40000
X = torch.as_tensor(rng.normal(scale=3.0, size=(k, d))[rng.integers(0, k, n)] + rng.normal(size=(n, d)), device=dev)
C = X[:k].clone(); cn = row_norms(C); xn = row_norms(X)
p = KMeansPlan(d, k, n); rows = p.rows(X)
a = torch.empty(n, dtype=torch.int32, device=dev); conv = torch.zeros(1, dtype=torch.int32, device=dev)
out = []
for it in range(6):
    s = torch.zeros(k * d, dtype=torch.float64, device=dev); w = torch.zeros(k, dtype=torch.float64, device=dev)
    c = torch.zeros(1, dtype=torch.float64, device=dev)
    p.accumulate(X, xn, None, C, cn, s, w, c, a, None, rows=rows)
    out.append(a.cpu().numpy().copy())
    p.update(C, cn, s, w, 1e-4, conv)
np.save(sys.argv[1], np.stack(out))
print(rows.bounds_info()[0], rows.incremental_info()[0])
'''
    import numpy as np
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {}
    for strict in ("0", "1"):
        env = dict(os.environ, CYCLONE_STRICT_PARITY=strict)
        f = os.path.join(root, "gpurun_out", f"strict_{strict}.npy")
        os.makedirs(os.path.dirname(f), exist_ok=True)
        r = subprocess.run([sys.executable, "-c", code, f], env=env, cwd=root, capture_output=True,
                           text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        res[strict] = (np.load(f), r.stdout.split())
    assert res["1"][1] == ["0", "0"]            # no bounded or incremental call
    assert int(res["0"][1][0]) == 6             # the default carries the bounds
    # iterations 0 and 1 see the same centers bit for bit (the first call is
    # a full pass either way); later centers differ in the sums' rounding
    np.testing.assert_array_equal(res["0"][0][:2], res["1"][0][:2])
    assert (res["0"][0][2:] != res["1"][0][2:]).sum() <= 5
