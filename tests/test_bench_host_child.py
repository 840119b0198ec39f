"""bench.py runs its host-resident legs in a child process that loads the library before torch
(the system HIP runtime of a C ABI host, bench.py HOST_RUNTIME).  CPU checks of that plumbing:
the hidden child arguments parse, and a child that cannot reach a GPU makes the parent fail
loudly instead of reporting a number."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_child_arguments_parse(monkeypatch):
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py", "--host-child", "c5", "--host-device", "3", "--c5-all", "100",
                                      "--c5-lo", "10", "--c5-hi", "60", "--c5-rank", "1", "--c5-steps", "2"])
    a = bench.parse()
    assert (a.host_child, a.host_device, a.c5_all, a.c5_lo, a.c5_hi, a.c5_rank, a.c5_steps) == \
        ("c5", 3, 100, 10, 60, 1, 2)
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    assert bench.parse().host_child is None


def test_child_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible: the child would succeed")
    import bench
    with pytest.raises(SystemExit, match="child failed"):
        bench.host_c2_child(0, 64, 4096, 0, 0)
