"""bench.py's own multi-rank launch (`python3 bench.py --gpus N` with no
launcher around it): the environment each rank gets, rank 0's line reaching the
caller, and exit-status handling when a rank fails -- all on CPU, with stand-in
child programs for the GPU ranks.  The mapping it reproduces is the launcher
environment the reference reads to pick a device
(src/hydrogen/device/GPU.cpp:30-50)."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

# stand-in rank: records its launcher environment, rank 0 prints a JSON line,
# ranks listed in FAIL_RANKS exit 3 at once, the others sleep SLEEP_S
CHILD = r"""
import json, os, sys, time
d = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE",
                                    "MASTER_ADDR", "MASTER_PORT")}
d["argv"] = sys.argv[1:]
d["pid"] = os.getpid()
open(os.path.join(os.environ["OUT_DIR"], "rank%s.json" % d["RANK"]), "w").write(json.dumps(d))
if d["RANK"] in os.environ.get("FAIL_RANKS", "").split(","):
    sys.exit(3)
time.sleep(float(os.environ.get("SLEEP_S", "0")))
if d["RANK"] == "0":
    print(json.dumps({"metric": "stand-in", "n_gpus": int(d["WORLD_SIZE"])}), flush=True)
"""


def _launch(tmp_path, monkeypatch, world, **env):
    monkeypatch.setenv("OUT_DIR", str(tmp_path))
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    t0 = time.monotonic()
    rc = bench.launch_ranks(["--gpus", str(world), "--steps", "3"], world, child_cmd=[sys.executable, "-c", CHILD],
                            grace_s=1.0, poll_s=0.05)
    return rc, time.monotonic() - t0


def test_launcher_rank_environment(tmp_path, monkeypatch, capfd):
    rc, _ = _launch(tmp_path, monkeypatch, 4)
    assert rc == 0
    recs = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(4)]
    ports = {d["MASTER_PORT"] for d in recs}
    assert len(ports) == 1 and 20000 <= int(ports.pop()) < 32000
    for r, d in enumerate(recs):
        assert d["RANK"] == d["LOCAL_RANK"] == str(r)
        assert d["WORLD_SIZE"] == d["LOCAL_WORLD_SIZE"] == "4"
        assert d["MASTER_ADDR"] == "127.0.0.1"
        assert d["argv"] == ["--gpus", "4", "--steps", "3"]
        assert d["pid"] > 0
    out = capfd.readouterr().out.strip().splitlines()
    assert [json.loads(x) for x in out] == [{"metric": "stand-in", "n_gpus": 4}]


def test_launcher_failing_rank_sets_status_and_stops_the_rest(tmp_path, monkeypatch, capfd):
    # rank 1 fails at once, rank 0 would sleep for a minute: the launcher returns
    # rank 1's status after the grace period and a SIGTERM, not a minute later
    rc, dt = _launch(tmp_path, monkeypatch, 2, FAIL_RANKS="1", SLEEP_S="60")
    assert rc == 3
    assert dt < 20, dt
    err = capfd.readouterr().err
    assert "rank 1 exited with status 3" in err


def test_launcher_signal_death_maps_to_128_plus_signal(tmp_path, monkeypatch):
    monkeypatch.setenv("OUT_DIR", str(tmp_path))
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    kill_self = "import os, signal; os.kill(os.getpid(), signal.SIGKILL)"
    rc = bench.launch_ranks([], 2, child_cmd=[sys.executable, "-c", kill_self], grace_s=1.0, poll_s=0.05)
    assert rc == 128 + 9


def test_bench_gpus_2_without_launcher_fails_loudly_on_cpu():
    """The real entry: `python bench.py --gpus 2` with WORLD_SIZE unset starts two
    ranks of bench.py itself; here (no GPU) they fail, and so must the launch."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--size", "256"], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "[bench launcher] rank" in p.stderr
    assert p.stdout.strip() == ""


def test_launcher_forwards_sigterm(tmp_path):
    """SIGTERM to the launcher reaches every rank (the driver's timeout ends the
    whole job, not just the parent): the launcher exits 128 + SIGTERM promptly
    and no rank survives it."""
    import signal
    script = ("import sys; sys.path.insert(0, %r); import bench; "
              "sys.exit(bench.launch_ranks([], 2, child_cmd=[sys.executable, '-c', %r], grace_s=1.0, poll_s=0.05))"
              % (ROOT, CHILD))
    env = dict(os.environ, OUT_DIR=str(tmp_path), SLEEP_S="60")
    env.pop("WORLD_SIZE", None)
    p = subprocess.Popen([sys.executable, "-c", script], env=env)
    deadline = time.monotonic() + 60
    while len(list(tmp_path.glob("rank*.json"))) < 2:  # both ranks started
        assert time.monotonic() < deadline and p.poll() is None
        time.sleep(0.05)
    t0 = time.monotonic()
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=30) == 128 + signal.SIGTERM
    assert time.monotonic() - t0 < 10
    for f in tmp_path.glob("rank*.json"):
        pid = json.loads(f.read_text())["pid"]
        try:  # the rank was reaped by the launcher: no such process
            os.kill(pid, 0)
            raise AssertionError(f"rank process {pid} survived the launcher")
        except ProcessLookupError:
            pass
