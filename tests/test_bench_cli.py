"""bench.py's rank handling (CPU only, no GPU call): `--gpus N` without a launcher spawns N rank
processes; a launcher's WORLD_SIZE must agree with --gpus; more ranks than visible GPUs is refused
unless every rank is told to share cuda:0 (GNOT_BENCH_ONE_GPU)."""
import argparse
import os
import sys
import textwrap

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def _args(gpus):
    return argparse.Namespace(gpus=gpus)


@pytest.fixture
def clean_env(monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "GNOT_BENCH_ONE_GPU", "MASTER_PORT"):
        monkeypatch.delenv(k, raising=False)
    return monkeypatch


def test_single_rank_default(clean_env):
    assert bench.resolve_world(_args(None)) == (1, 0, 0)
    assert bench.resolve_world(_args(1)) == (1, 0, 0)


def test_launcher_world_must_match_flag(clean_env):
    clean_env.setenv("WORLD_SIZE", "2")
    clean_env.setenv("RANK", "1")
    clean_env.setenv("LOCAL_RANK", "1")
    clean_env.setenv("GNOT_BENCH_ONE_GPU", "1")
    assert bench.resolve_world(_args(2)) == (2, 1, 1)
    assert bench.resolve_world(_args(None)) == (2, 1, 1)
    with pytest.raises(SystemExit, match="--gpus 4 but WORLD_SIZE=2"):
        bench.resolve_world(_args(4))


def test_more_ranks_than_gpus_refused(clean_env):
    # this container has no GPU: device_count() == 0
    with pytest.raises(SystemExit, match="GPU\\(s\\) visible"):
        bench.resolve_world(_args(2))
    clean_env.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit, match="GPU\\(s\\) visible"):
        bench.resolve_world(_args(2))


def test_spawn_ranks_runs_n_children(clean_env, tmp_path):
    out = tmp_path / "ranks"
    out.mkdir()
    script = tmp_path / "rank.py"
    script.write_text(textwrap.dedent(f"""
        import os, sys
        r = os.environ["RANK"]
        open(os.path.join({str(out)!r}, r), "w").write(
            " ".join(os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR")) + " " + " ".join(sys.argv[1:]))
    """))
    assert bench.spawn_ranks(3, str(script), ["--gpus", "3"]) == 0
    got = sorted(p.read_text() for p in out.iterdir())
    assert got == [f"{r} {r} 3 127.0.0.1 --gpus 3" for r in range(3)]


def test_spawn_ranks_reports_failure(clean_env, tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(textwrap.dedent("""
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(60)          # the surviving rank is ended by PID once rank 1 fails
    """))
    assert bench.spawn_ranks(2, str(script), []) == 3
