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


def test_one_process_leg_runs_a_bounded_child_and_reports_failure(monkeypatch):
    """The one-process leg of an N-rank run (bench.one_process_leg): rank 0
    starts `bench.py --child-oneproc` with the run's problem and without the
    torchrun rank variables, bounded by a timeout; a child that fails (here:
    no GPU in this container) becomes a note in the line, not an exception."""
    import argparse
    bench = _load_bench()
    seen = {}
    real_run = bench.subprocess.run

    def spy(cmd, env=None, **kw):
        seen["cmd"], seen["env"], seen["kw"] = cmd, env, kw
        return real_run(cmd, env=env, **kw)

    monkeypatch.setattr(bench.subprocess, "run", spy)
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "8")
    a = argparse.Namespace(gpus=8, n=32, kind=27, dtype="f64", steps=3, warmup=1, tune="", oneproc_devices="")
    out = bench.one_process_leg(a)
    cmd = seen["cmd"]
    assert "--child-oneproc" in cmd and cmd[cmd.index("--gpus") + 1] == "8" and cmd[cmd.index("--n") + 1] == "32"
    assert "RANK" not in seen["env"] and "WORLD_SIZE" not in seen["env"]
    assert seen["kw"].get("timeout")
    assert "note" in out and "failed" in out["note"], out


def test_rccl_run_info_proves_ranks_and_devices():
    """config.rccl_halo of an N > 1 line: the
    communicator size of every rank (ncclCommCount), the distinct devices
    and the resolved librccl; a run whose ranks folded onto fewer GPUs, or
    whose communicator is smaller than the world, fails instead of
    reporting."""
    import pytest
    bench = _load_bench()
    lib = "/opt/rocm/lib/librccl.so.1"
    mk = lambda r, pci, n=2: {"ranks": n, "rank": r, "device": r, "pci": pci, "rccl_version": 22700, "librccl": lib}
    out = bench.rccl_run_info([mk(0, "0000:05:00.0"), mk(1, "0000:15:00.0")], 2)
    assert out["rccl_ranks"] == {"min": 2, "max": 2} and out["distinct_devices"] == 2
    assert out["devices"] == ["0000:05:00.0", "0000:15:00.0"] and out["librccl"] == [lib]
    with pytest.raises(SystemExit, match="distinct devices"):
        bench.rccl_run_info([mk(0, "0000:05:00.0"), mk(1, "0000:05:00.0")], 2)
    with pytest.raises(SystemExit, match="communicator sizes"):
        bench.rccl_run_info([mk(0, "0000:05:00.0", 1), mk(1, "0000:15:00.0", 1)], 2)
