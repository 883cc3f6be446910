"""bench.py's own rank launcher (launch_ranks): `python bench.py --gpus N`
without torchrun starts N children with the torch.distributed environment,
relays their exit status and stops the others when one rank fails. CPU only:
the children here are small Python scripts, or bench.py's own argument
parser (--help), so nothing touches a GPU."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

CHILD = r"""
import json, os, sys, time
keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
out = sys.argv[1]
with open(os.path.join(out, "rank%s.json" % os.environ["RANK"]), "w") as f:
    json.dump({k: os.environ.get(k) for k in keys} | {"argv": sys.argv[2:]}, f)
mode = sys.argv[2] if len(sys.argv) > 2 else ""
if mode == "fail1":
    if os.environ["RANK"] == "1":
        sys.exit(3)
    time.sleep(60)  # the launcher must stop this rank
if mode == "print0" and os.environ["RANK"] == "0":
    print(json.dumps({"value": 1.0}))
"""


def _child(tmp_path):
    p = tmp_path / "child.py"
    p.write_text(CHILD)
    return [sys.executable, str(p), str(tmp_path)]


def test_children_get_rank_env(tmp_path):
    rc = bench.launch_ranks(3, ["print0"], cmd=_child(tmp_path))
    assert rc == 0
    envs = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(3)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    assert all(e["WORLD_SIZE"] == "3" and e["MASTER_ADDR"] == "127.0.0.1" for e in envs)
    assert len({e["MASTER_PORT"] for e in envs}) == 1 and envs[0]["MASTER_PORT"].isdigit()
    assert all(e["argv"] == ["print0"] for e in envs)


def test_failing_rank_stops_the_job(tmp_path):
    t0 = time.time()
    rc = bench.launch_ranks(2, ["fail1"], cmd=_child(tmp_path))
    assert rc == 3
    assert time.time() - t0 < 30  # rank 0 (sleeping 60 s) was stopped, not waited for


def test_bench_spawns_without_launcher():
    """The real entry point: no WORLD_SIZE, --gpus 2 -> two children of
    bench.py itself (here each only prints its argument help, exit 0)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--help"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.count("usage:") == 2  # one help text per spawned rank


def test_bench_rank_failure_propagates():
    """A spawned rank's non-zero exit is the job's: an unknown option makes
    each child's parser exit 2."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-such-option"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
