"""CPU: bench.py's launch contract. `--gpus N` must either run N ranks
(re-launching itself under torch.distributed.run before any GPU call) or
fail -- never silently run one process and report n_gpus = 1."""
import os
import subprocess
import sys

from conftest import ROOT


def test_gpus_mismatch_with_torchrun_env_fails():
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=3" in r.stderr


def test_relaunch_command_is_torchrun(monkeypatch):
    import bench
    calls = {}

    def fake_call(cmd):
        calls["cmd"] = cmd
        return 0

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    monkeypatch.setattr(subprocess, "call", fake_call)
    args = bench.parse()
    try:
        bench.relaunch_if_needed(args)
    except SystemExit as e:
        assert e.code == 0
    cmd = calls["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
