"""CPU: `python bench.py --gpus N` started directly (the driver's N = 1 command form with N > 1).

bench.py then starts the N ranks itself as a child `torch.distributed.run` (one rank per GPU over
127.0.0.1) before anything imports torch or touches a GPU — never an exec — relays rank 0's JSON
line to stdout and returns the child's exit code.  Under torch.distributed.run (WORLD_SIZE set) and
at N = 1 nothing changes.  These tests run the launcher logic with stand-in children; no GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _run(code, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=120)


def test_launcher_command_forwards_arguments():
    import bench
    cmd = bench.launcher_cmd(["--gpus", "8", "--steps", "20", "--warmup", "5"], 8, 29511, python="py")
    assert cmd[:3] == ["py", "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd and "--master-port=29511" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-7] == os.path.join(ROOT, "bench.py")
    assert cmd[-6:] == ["--gpus", "8", "--steps", "20", "--warmup", "5"]


def test_main_spawns_before_importing_torch():
    """main() with --gpus 4 and no WORLD_SIZE hands off to launch_ranks with the original argv,
    and at that point torch has not been imported; the child's code becomes the exit code."""
    code = (
        "import sys, json\n"
        "import bench\n"
        "def fake(argv, n):\n"
        "    print(json.dumps({'argv': argv, 'n': n, 'torch': 'torch' in sys.modules}))\n"
        "    return 5\n"
        "bench.launch_ranks = fake\n"
        "sys.argv = ['bench.py', '--gpus', '4', '--steps', '7', '--warmup', '2']\n"
        "bench.main()\n")
    r = _run(code)
    assert r.returncode == 5, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d == {"argv": ["--gpus", "4", "--steps", "7", "--warmup", "2"], "n": 4, "torch": False}


def test_relay_json_line_and_exit_code():
    """launch_ranks relays only the metric line to stdout (rank 0's), the rest to stderr, and
    returns the child's code (a failing child's nonzero code included)."""
    child = ("import json, sys\n"
             "print('rank 1 noise')\n"
             "print(json.dumps({'metric': 'm', 'value': 1.5, 'n_gpus': 2}), flush=True)\n"
             "print('trailer')\n"
             "sys.exit(3)\n")
    code = ("import sys\n"
            "import bench\n"
            f"rc = bench.launch_ranks([], 2, cmd=[sys.executable, '-c', {child!r}])\n"
            "print('TORCH_IMPORTED', 'torch' in sys.modules, file=sys.stderr)\n"
            "sys.exit(rc)\n")
    r = _run(code)
    assert r.returncode == 3
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1 and json.loads(lines[0]) == {"metric": "m", "value": 1.5, "n_gpus": 2}
    assert "rank 1 noise" in r.stderr and "trailer" in r.stderr
    assert "TORCH_IMPORTED False" in r.stderr


def test_under_torchrun_no_relaunch():
    """With WORLD_SIZE set (the driver's torch.distributed.run form) main() never relaunches."""
    code = (
        "import sys\n"
        "import bench\n"
        "def fake(argv, n):\n"
        "    raise SystemExit(99)\n"
        "bench.launch_ranks = fake\n"
        "sys.argv = ['bench.py', '--gpus', '2', '--steps', '1']\n"
        "import builtins\n"
        "real = builtins.__import__\n"
        "def guard(name, *a, **k):\n"
        "    if name == 'torch':\n"
        "        raise SystemExit(42)\n"
        "    return real(name, *a, **k)\n"
        "builtins.__import__ = guard\n"
        "bench.main()\n")
    r = _run(code, {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 42, (r.returncode, r.stderr)   # went on to the rank path (imports torch)


def test_device_map_for_shared_gpus(monkeypatch):
    """EIGSOL_BENCH_DEVICES maps local ranks to GPUs (rehearsing N ranks on fewer GPUs: bench.py then
    bootstraps over gloo, RCCL refusing duplicate devices); unset: local rank r on GPU r."""
    import bench
    monkeypatch.delenv("EIGSOL_BENCH_DEVICES", raising=False)
    assert bench.device_map(4) == [0, 1, 2, 3]
    monkeypatch.setenv("EIGSOL_BENCH_DEVICES", "0,0")
    assert bench.device_map(2) == [0, 0]
    monkeypatch.setenv("EIGSOL_BENCH_DEVICES", "0,0,1,1,2")
    assert bench.device_map(4, 4) == [0, 0, 1, 1]
    monkeypatch.setenv("EIGSOL_BENCH_DEVICES", "0")
    import pytest
    with pytest.raises(SystemExit):
        bench.device_map(2)
