"""bench.py's multi-GPU entry (CPU): `python bench.py --gpus N` spawns N rank processes with
torchrun's environment, and a world-size mismatch exits non-zero."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402

ENV_DUMP = textwrap.dedent("""
    import json, os, sys
    keys = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "PU_BENCH_WORKER")
    out = sys.argv[sys.argv.index("--out") + 1]
    with open(os.path.join(out, "rank%s.json" % os.environ["RANK"]), "w") as f:
        json.dump({k: os.environ.get(k) for k in keys} | {"argv": sys.argv[1:]}, f)
""")


def test_launcher_hands_each_worker_its_rank(tmp_path):
    script = tmp_path / "dump.py"
    script.write_text(ENV_DUMP)
    rc = bench.launch_workers(4, ["--gpus", "4", "--steps", "3", "--out", str(tmp_path)],
                              cmd=[sys.executable, str(script)], poll_s=0.05)
    assert rc == 0
    envs = [json.load(open(tmp_path / ("rank%d.json" % r))) for r in range(4)]
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert {e["WORLD_SIZE"] for e in envs} == {"4"}
    assert {e["MASTER_ADDR"] for e in envs} == {"127.0.0.1"}
    assert len({e["MASTER_PORT"] for e in envs}) == 1
    assert all(e["argv"][:4] == ["--gpus", "4", "--steps", "3"] for e in envs)


def test_launcher_failed_rank_stops_the_rest(tmp_path):
    script = tmp_path / "fail.py"
    script.write_text("import os, sys, time\n"
                      "if os.environ['RANK'] == '1': sys.exit(5)\n"
                      "time.sleep(60)\n")
    import time
    t0 = time.time()
    rc = bench.launch_workers(3, [], cmd=[sys.executable, str(script)], poll_s=0.05)
    assert rc == 5
    assert time.time() - t0 < 30          # the sleeping ranks were terminated, not waited out


def test_world_mismatch_exits_nonzero():
    with pytest.raises(SystemExit) as e:
        bench.check_world(8, 1)
    assert e.value.code != 0
    with pytest.raises(SystemExit) as e:
        bench.check_world(4, 4, devices=2)
    assert e.value.code != 0
    bench.check_world(2, 2, devices=8)     # consistent: returns


def test_bench_gpus_n_without_devices_fails_fast():
    """On a box with fewer GPUs than --gpus the parent refuses before spawning anything."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr
