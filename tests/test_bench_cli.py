"""bench.py's command-line contract on CPU: `--gpus N` launches N ranks itself, a launcher's
WORLD_SIZE that disagrees with --gpus is fatal, and the event timings are checked against the wall clock."""

import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_check_world():
    assert bench.check_world(1, {}) == (1, None)
    assert bench.check_world(8, {}) == (8, None)
    assert bench.check_world(2, {"WORLD_SIZE": "2"}) == (2, None)
    w, err = bench.check_world(2, {"WORLD_SIZE": "4"})
    assert w == 4 and "WORLD_SIZE=4" in err and "--gpus 2" in err
    w, err = bench.check_world(8, {"WORLD_SIZE": "1"})
    assert err is not None
    assert bench.check_world(0, {})[1] is not None


def test_launcher_cmd_is_one_node_one_rank_per_gpu():
    cmd = bench.launcher_cmd(4, ["--gpus", "4", "--steps", "7"], 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    assert "--nnodes=1" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", "4", "--steps", "7"]


def test_world_size_mismatch_exits_nonzero_before_any_gpu_call():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "1"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr and not r.stdout.strip()


def test_event_timings_are_checked_against_the_wall_clock():
    """The roofline's duration is the replayed window's HIP-event average; the events are checked
    against the timed loop's wall clock, an independent measurement."""
    # BENCH_r04 (driver, K = 20): events 0.14126 + 0.0068 ms against a 0.1441 ms step
    t = bench.kernel_times(0.1441, 0.14126 * 200, 0.0068 * 200, 200)
    assert t["k_step_ms"] == pytest.approx(0.14126) and t["k_obs_ms"] == pytest.approx(0.0068)
    assert t["sampled_launches"] == 200 and t["k_step_period_ms"] == pytest.approx(0.1441 - 0.0068)
    assert bench.events_consistent(t)
    # events that missed launches, or timed another window than the timed loop's, fail the check
    assert not bench.events_consistent(bench.kernel_times(0.1441, 0.07 * 200, 0.0068 * 200, 200))
    assert not bench.events_consistent(bench.kernel_times(0.1000, 0.14126 * 200, 0.0068 * 200, 200))
    assert not bench.events_consistent(bench.kernel_times(0.1441, 0.0, 0.0, 0))


def test_cpu_baseline_reports_median_of_samples():
    r = bench.cpu_baseline(8, 0, 1, warm_steps=2, samples=3, min_wall_s=0.0, min_steps=2)
    assert r["kind"] == "port" and r["cores"] == 1 and len(r["samples"]) == 3
    assert r["value"] == sorted(r["samples"])[1]
    assert r["spread"] >= 0 and "3 samples" in r["sample"]
