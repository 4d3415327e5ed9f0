"""bench.py --gpus N without an external launcher (bzr_amd/launch.py).

CPU only: the launcher's rank environment, its exit status, a failing rank stopping the others, and the
--gpus / WORLD_SIZE mismatch exit -- before bench.py imports torch or touches a GPU."""
import os
import subprocess
import sys
import textwrap
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "cuda-bezier-triangle-raytracer_amd"))

from bzr_amd import launch  # noqa: E402


def test_check_world_modes():
    assert launch.check_world(1, {}) == "single"
    assert launch.check_world(4, {}) == "spawn"
    assert launch.check_world(2, {"WORLD_SIZE": "2"}) == "launched"
    for gpus, ws in ((1, "2"), (8, "4"), (2, "x")):
        with pytest.raises(SystemExit) as e:
            launch.check_world(gpus, {"WORLD_SIZE": ws})
        assert e.value.code == 2
    with pytest.raises(SystemExit):
        launch.check_world(0, {})


def test_bench_rejects_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "3"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 2, r.stderr
    assert "WORLD_SIZE=2" in r.stderr


WORKER = textwrap.dedent("""
    import os, sys
    import torch, torch.distributed as dist
    dist.init_process_group("gloo")
    t = torch.tensor([int(os.environ["LOCAL_RANK"])])
    dist.all_reduce(t)
    print(f"rank={dist.get_rank()} world={dist.get_world_size()} sum={int(t)} "
          f"by={os.environ.get('BZR_LAUNCHED_BY')}", flush=True)
    rank = dist.get_rank()
    dist.destroy_process_group()
    sys.exit(3 if int(os.environ.get("FAIL_RANK", "-1")) == rank else 0)
""")


def test_spawn_runs_n_ranks_with_a_rendezvous(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(WORKER)
    out = tmp_path / "out.txt"
    with open(out, "w") as f:
        code = subprocess.run([sys.executable, "-c",
                               f"import sys; sys.path.insert(0, {str(REPO / 'cuda-bezier-triangle-raytracer_amd')!r});"
                               f"from bzr_amd import launch; sys.exit(launch.spawn([sys.executable, {str(script)!r}], 3))"],
                              stdout=f, stderr=subprocess.STDOUT, timeout=180).returncode
    text = out.read_text()
    assert code == 0, text
    lines = sorted(l for l in text.splitlines() if l.startswith("rank="))
    assert lines == [f"rank={r} world=3 sum=3 by=bench.py" for r in range(3)], text


def test_spawn_reports_a_failing_rank(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(WORKER)
    env = dict(os.environ, FAIL_RANK="1")
    r = subprocess.run([sys.executable, "-c",
                        f"import sys; sys.path.insert(0, {str(REPO / 'cuda-bezier-triangle-raytracer_amd')!r});"
                        f"from bzr_amd import launch; sys.exit(launch.spawn([sys.executable, {str(script)!r}], 2))"],
                       env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 3, r.stdout + r.stderr
    assert "rank 1 exited with status 3" in r.stderr


def test_spawn_stops_the_others_when_a_rank_dies_early(tmp_path):
    # rank 0 dies before the rendezvous; rank 1 would wait for it forever without the SIGTERM
    script = tmp_path / "w.py"
    script.write_text("import os, sys, time\n"
                      "if os.environ['RANK'] == '0': sys.exit(5)\n"
                      "time.sleep(600)\n")
    r = subprocess.run([sys.executable, "-c",
                        f"import sys; sys.path.insert(0, {str(REPO / 'cuda-bezier-triangle-raytracer_amd')!r});"
                        f"from bzr_amd import launch; sys.exit(launch.spawn([sys.executable, {str(script)!r}], 2))"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 5, r.stderr


def test_parent_sigterm_stops_the_ranks(tmp_path):
    """a SIGTERM to the launching parent while it waits stops every rank (SIGTERM, then
    SIGKILL after the grace period) instead of leaving them running on the GPUs."""
    import signal
    import time

    pids = tmp_path / "pids"
    pids.mkdir()
    child = f"import os, time; open(os.path.join({str(pids)!r}, os.environ['RANK']), 'w').write(str(os.getpid())); time.sleep(120)"
    parent = (f"import sys; sys.path.insert(0, {str(REPO / 'cuda-bezier-triangle-raytracer_amd')!r}); "
              f"from bzr_amd import launch; sys.exit(launch.spawn([sys.executable, '-c', {child!r}], 2))")
    p = subprocess.Popen([sys.executable, "-c", parent])
    try:
        deadline = time.monotonic() + 60
        while len(list(pids.iterdir())) < 2 and time.monotonic() < deadline:
            time.sleep(0.1)
        ranks = [int((pids / str(r)).read_text()) for r in range(2)]
        p.send_signal(signal.SIGTERM)
        assert p.wait(timeout=60) == 128 + signal.SIGTERM
        for pid in ranks:  # reaped by the parent: no such process any more
            with pytest.raises(ProcessLookupError):
                os.kill(pid, 0)
    finally:
        if p.poll() is None:
            p.kill()


def test_default_frames_in_flight_follow_the_rank_frame_size():
    """--inflight 0: 6 slots for a rank frame of at most 4 M primaries, else 3 (fused) / 2 (staged)."""
    sys.path.insert(0, str(REPO))
    import bench

    def slots(argv, world):
        old = sys.argv
        try:
            sys.argv = ["bench.py"] + argv
            return bench.default_inflight(bench.parse(), world)
        finally:
            sys.argv = old

    assert slots(["--config", "cfg2"], 1) == 6
    assert slots(["--config", "cfg3", "--pipeline", "staged"], 1) == 6
    assert slots([], 1) == 3                                  # cfg4 4096², the N = 1 line
    assert slots([], 2) == 3                                  # 8 M primaries per rank
    assert slots([], 4) == 6 and slots([], 8) == 6            # strong-scaling shares
    assert slots(["--scaling", "weak"], 8) == 3               # weak: every rank keeps 4096²
    assert slots(["--config", "cfg5", "--pipeline", "staged"], 1) == 2
    assert slots(["--config", "cfg4", "--side", "2048", "--pipeline", "staged"], 1) == 6
