"""``bench.py --gpus N`` starts N ranks itself: run on the
CPU with a stand-in per-shard call (tests/bench_standin.py) over gloo, the
launcher, both ranks, the max-over-ranks timing and the rank-0 JSON line are
the bench's own.  The multi-rank line carries the CPU baseline the launching
process measured before the ranks started, and rank 0's stage-pass roofline
(VERDICT r05 next #4)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(300)
def test_bench_gpus2_starts_two_ranks_cpu_rehearsal():
    env = dict(os.environ, TDA_BENCH_STANDIN="tests.bench_standin:run", TDA_DIST_BACKEND="gloo", OMP_NUM_THREADS="1",
               PYTHONPATH=ROOT)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "sweep48", "--layers", "4",
                        "--steps", "2", "--warmup", "1", "--cpu-seconds", "1"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    out = json.loads(lines[0])
    assert out["ranks"] == 2
    assert out["n_gpus"] == 0  # the stand-in touches no GPU: the record says so
    assert out["rehearsal"]["kind"].startswith("cpu stand-in")
    assert out["scaling"] == "weak" and out["strong"]["layers_total"] == 4
    assert out["value"] > 0 and out["strong"]["value"] > 0
    cb = out["cpu_baseline"]
    assert cb["value"] > 0 and cb["value_1core"] > 0 and cb["cores"] >= 1 and "launching process" in cb["measured_by"]
    assert out["speedup_vs_cpu"]["bar_20x"]["basis"] == "all_cores"
    rf = out["roofline"]
    assert rf["kernel"] == "k_standin_oracle" and rf["layers_per_launch"] == 4 and rf["achieved"] > 0


def test_bench_refuses_standin_without_ranks():
    env = dict(os.environ, TDA_BENCH_STANDIN="tests.bench_standin:run", PYTHONPATH=ROOT)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--no-cpu", "--extra", ""], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "rehearsal" in r.stderr
