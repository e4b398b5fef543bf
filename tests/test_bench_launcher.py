"""CPU: bench.py's own multi-rank launcher (`python bench.py --gpus N` without torch.distributed.run,
SURVEY.md §8(e)): rank environment, rank 0's JSON line forwarded, exit codes, and the other ranks
stopped when one fails. Fake rank scripts stand in for the GPU ranks; the last test runs the real
bench.py, whose ranks find no GPU here and must make the launcher fail loudly."""
import json
import os
import subprocess
import sys
import textwrap
import time

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _script(tmp_path, body):
    p = tmp_path / "rank.py"
    p.write_text(textwrap.dedent(body))
    return [sys.executable, "-u", str(p)]


def test_ranks_get_env_and_rank0_json_is_forwarded(tmp_path, capfd):
    cmd = _script(tmp_path, f"""
        import json, os
        r = int(os.environ["RANK"])
        open(os.path.join({str(tmp_path)!r}, f"env{{r}}"), "w").write(json.dumps(
            {{k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}}))
        if r == 0:
            print("not json")
            print(json.dumps({{"metric": "m", "value": 1.0, "n_gpus": int(os.environ["WORLD_SIZE"])}}))
    """)
    rc, line = bench.launch_ranks(cmd, 3)
    assert rc == 0
    assert json.loads(line) == {"metric": "m", "value": 1.0, "n_gpus": 3}
    envs = [json.loads((tmp_path / f"env{r}").read_text()) for r in range(3)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2"] == [e["LOCAL_RANK"] for e in envs]
    assert {e["WORLD_SIZE"] for e in envs} == {"3"}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1
    assert '"metric": "m"' in capfd.readouterr().out


def test_failing_rank_stops_the_others_and_sets_exit_code(tmp_path):
    cmd = _script(tmp_path, """
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(120)   # rank 0 would wait for rank 1 forever (a barrier)
    """)
    t0 = time.time()
    rc, line = bench.launch_ranks(cmd, 2, grace_s=5.0)
    assert rc == 3 and line is None
    assert time.time() - t0 < 30


def test_killed_rank_is_a_failure(tmp_path):
    cmd = _script(tmp_path, """
        import os, signal
        if os.environ["RANK"] == "0":
            os.kill(os.getpid(), signal.SIGKILL)
    """)
    rc, _ = bench.launch_ranks(cmd, 2)
    assert rc == 128 + 9


def test_missing_json_line_is_a_failure(tmp_path):
    cmd = _script(tmp_path, "print('no result')\n")
    rc, line = bench.launch_ranks(cmd, 2)
    assert rc == 1 and line is None


def test_bench_launcher_fails_loudly_without_gpus():
    # the parent never touches the GPU; each rank finds none here and exits non-zero
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--no-cpu-baseline", "--no-profile", "--backend", "gloo"],
                       capture_output=True, text=True, timeout=300,
                       env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    assert p.returncode != 0
    assert "no GPU visible" in p.stderr
    assert p.stdout.strip() == ""


def test_bench_rejects_zero_gpus():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "0"], capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 2 and "--gpus must be >= 1" in p.stderr
