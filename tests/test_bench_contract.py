"""bench.py's contract pieces that run without a GPU:
  * the committed profile summaries it reads back (roofline.traffic / valu_frac,
    profiles/*_pmc_*.json and *_sq_*.json) must not be excluded from the gpurun
    snapshot by .gpurunignore;
  * `--gpus N` launches N ranks by itself: the launch decision,
    its refusal of a mismatched WORLD_SIZE, and the relay of the rank-0 JSON line."""
import fnmatch
import io
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402  (imports numpy only at module level: no torch, no GPU)


def test_profiles_read_by_bench_travel():
    pats = [l.strip() for l in open(os.path.join(REPO, ".gpurunignore")) if l.strip()]
    for rel in ("profiles/r02c_pmc_c4.json", "profiles/r02c_sq_c4.json"):
        for p in pats:
            anchored = p.startswith("./")
            pat = p[2:] if anchored else p
            hit = fnmatch.fnmatch(rel, pat) or (anchored and (rel == pat or rel.startswith(pat + "/"))) \
                or (not anchored and fnmatch.fnmatch(os.path.basename(rel), pat))
            assert not hit, f".gpurunignore pattern {p!r} drops {rel}, which bench.py reads"


def test_launch_plan_single_rank():
    assert bench.launch_plan(1, [], {}) == ("run", None)


def test_launch_plan_under_external_launcher():
    assert bench.launch_plan(8, ["--gpus", "8"], {"WORLD_SIZE": "8"}) == ("run", None)


def test_launch_plan_refuses_mismatched_world():
    action, msg = bench.launch_plan(8, ["--gpus", "8"], {"WORLD_SIZE": "2"})
    assert action == "error" and "WORLD_SIZE=2" in msg
    action, _ = bench.launch_plan(1, [], {"WORLD_SIZE": "4"})
    assert action == "error"
    assert bench.launch_plan(0, [], {})[0] == "error"


def test_launch_plan_spawns_n_ranks():
    argv = ["--gpus", "4", "--workload", "c5", "--steps", "3"]
    action, cmd = bench.launch_plan(4, argv, {})
    assert action == "launch"
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert int(cmd[cmd.index("--master-port") + 1]) > 0
    i = cmd.index(os.path.join(REPO, "bench.py"))
    assert cmd[i + 1:] == argv  # the same arguments reach every rank


def test_dry_run_cli_touches_no_gpu():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--workload", "c5", "--launch-dry-run"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["action"] == "launch" and d["gpus"] == 2
    assert "--nproc-per-node=2" in d["detail"] and "--launch-dry-run" not in d["detail"]
    env["WORLD_SIZE"] = "2"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "8"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2 and r.stdout == "" and "WORLD_SIZE=2" in r.stderr


def test_launcher_relays_json_and_exit_code(capfd):
    child = ("import sys\n"
             "print('banner from a rank')\n"
             "print('{\"metric\": \"m\", \"value\": 1.5, \"n_gpus\": 2}')\n"
             "print('{not json')\n"
             "sys.exit(3)\n")
    out = io.StringIO()
    rc = bench.run_launcher([sys.executable, "-c", child], out)
    assert rc == 3
    assert [json.loads(l) for l in out.getvalue().splitlines()] == [
        {"metric": "m", "value": 1.5, "n_gpus": 2}]
    err = capfd.readouterr().err
    assert "banner from a rank" in err and "{not json" in err
