"""bench.py's multi-GPU launcher (CPU): `--gpus N` without a torch.distributed
environment starts N ranks through torch.distributed.run on 127.0.0.1 before
anything touches a GPU, and every rank re-enters bench.py with the same
arguments.  The ranks' data path itself (row / tile sharding, gather) is
covered by tests/test_shard_gloo.py and tests/test_gpu_shard.py."""
import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_launch_ranks_command(monkeypatch):
    bench = load_bench()
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 0

    monkeypatch.setattr(bench.subprocess, "call", fake_call)
    argv = ["bench.py", "--gpus", "2", "--dist-backend", "gloo", "--steps", "2", "--shard", "tiles"]
    monkeypatch.setattr(sys, "argv", argv)
    assert bench.launch_ranks(bench.parse()) == 0
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    port = [c for c in cmd if c.startswith("--master-port=")]
    assert port and 0 < int(port[0].split("=")[1]) < 65536
    # each rank runs this bench.py with the caller's arguments
    i = cmd.index(os.path.abspath(os.path.join(ROOT, "bench.py")))
    assert cmd[i + 1:] == argv[1:]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_main_launches_before_any_gpu_call(monkeypatch):
    """Without WORLD_SIZE, main() hands over to the launcher and exits with its
    code; torch.cuda is never initialised in the launcher process."""
    bench = load_bench()
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    calls = []
    monkeypatch.setattr(bench, "launch_ranks", lambda args: calls.append(args.gpus) or 7)
    import torch

    monkeypatch.setattr(torch.cuda, "set_device", lambda *a: pytest.fail("GPU touched before launching ranks"))
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7 and calls == [4]


def test_shard_choice_defaults():
    bench = load_bench()
    sys_argv = sys.argv
    try:
        sys.argv = ["bench.py"]
        a = bench.parse()
    finally:
        sys.argv = sys_argv
    assert a.gpus == 1 and a.shard == "auto" and a.dist_backend == "nccl"
