"""bench.py --gpus N (CPU-only checks of the launch path): without a
torch.distributed environment the parent starts N rank processes through
torch.distributed.run as a child process -- before any GPU call -- and exits
with its code; inside a rank, WORLD_SIZE must equal --gpus."""
import importlib
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    sys.path.insert(0, ROOT)
    return importlib.import_module("bench")


def test_parent_launches_n_ranks(monkeypatch):
    bench = _bench()
    seen = {}

    def fake_call(cmd):
        seen["cmd"] = cmd
        return 7
    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3", "--warmup", "1"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-6:] == ["--gpus", "4", "--steps", "3", "--warmup", "1"]
    assert cmd[-7].endswith("bench.py")


def test_rank_world_must_match_gpus(monkeypatch):
    bench = _bench()
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    with pytest.raises(SystemExit, match="one rank per GPU"):
        bench.main()
