"""bench.py --gpus N without torchrun around it starts the N one-part ranks
itself (launch_ranks) before anything touches the GPU: the command it runs
is the driver's torchrun command with this script's arguments, on the
loopback, with dmabuf IPC (no CPU-side GPU work needed to check this)."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load_bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_gpus_n_self_launches_torchrun(monkeypatch):
    bench = _load_bench()
    seen = {}

    class Done:
        returncode = 7

    def fake_run(cmd, env=None, **kw):
        seen["cmd"], seen["env"] = cmd, env
        return Done()

    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "9", "--warmup", "2"])
    assert bench.main() == 7  # the ranks' exit status is passed on
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--nnodes") + 1] == "1"
    assert cmd[-6:] == ["--gpus", "4", "--steps", "9", "--warmup", "2"]
    assert os.path.samefile(cmd[-7], os.path.join(ROOT, "bench.py"))
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_torchrun_rank_does_not_relaunch(monkeypatch):
    bench = _load_bench()
    monkeypatch.setattr(bench, "launch_ranks", lambda n: (_ for _ in ()).throw(AssertionError("relaunched")))
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "1"])
    monkeypatch.setenv("WORLD_SIZE", "2")  # already a torchrun rank: no second launch
    # the rank path then needs a GPU: stop it at its first step (fd 1 to stderr)
    class OsProxy:
        def __getattr__(self, name):
            return getattr(os, name)

        @staticmethod
        def dup(fd):
            raise RuntimeError("rank path reached")

    monkeypatch.setattr(bench, "os", OsProxy())
    try:
        bench.main()
        raise AssertionError("the rank path did not start")
    except RuntimeError as e:
        assert "rank path reached" in str(e)
