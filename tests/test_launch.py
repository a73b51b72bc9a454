"""CPU: launch.spawn_ranks -- bench.py / tools/bench_train.py --gpus N start one child process per GPU before any HIP
call.  Every rank gets the torchrun-style environment; when one rank fails the others are
stopped (they would otherwise wait in a collective forever) and the parent's exit code is non-zero."""
import os
import sys
import textwrap
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from xsdeepfwfm_deprecated_amd.launch import spawn_ranks  # noqa: E402


def _script(tmp_path, body):
    p = tmp_path / "rank.py"
    p.write_text(textwrap.dedent(body))
    return str(p)


def test_spawn_ranks_environment_and_success(tmp_path, monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    out = tmp_path / "out"
    out.mkdir()
    s = _script(tmp_path, f"""
        import os
        keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
        with open(os.path.join({str(out)!r}, os.environ["RANK"]), "w") as f:
            f.write(",".join(os.environ[k] for k in keys))
    """)
    assert spawn_ranks(3, argv=[s]) == 0
    got = sorted(os.listdir(out))
    assert got == ["0", "1", "2"]
    ports = set()
    for r in got:
        rank, local, world, lworld, addr, port = (out / r).read_text().split(",")
        assert rank == local == r and world == lworld == "3" and addr == "127.0.0.1"
        ports.add(port)
    assert len(ports) == 1


def test_spawn_ranks_one_rank_fails_stops_the_others(tmp_path, monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    s = _script(tmp_path, """
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(120)  # a rank waiting in a collective for the failed one
    """)
    t0 = time.time()
    rc = spawn_ranks(4, argv=[s], poll_s=0.05)
    assert rc == 3
    assert time.time() - t0 < 60  # the sleeping ranks were terminated, not waited for


def test_spawn_ranks_signal_exit_code(tmp_path, monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    s = _script(tmp_path, """
        import os, signal
        if os.environ["RANK"] == "0":
            os.kill(os.getpid(), signal.SIGKILL)
    """)
    assert spawn_ranks(2, argv=[s], poll_s=0.05) == 128 + 9


def test_spawn_ranks_is_a_no_op_inside_a_rank(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert spawn_ranks(2, argv=["-c", "raise SystemExit(1)"]) is None
    monkeypatch.delenv("WORLD_SIZE")
    assert spawn_ranks(1, argv=["-c", "raise SystemExit(1)"]) is None
