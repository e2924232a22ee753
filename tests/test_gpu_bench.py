"""bench.py's multi-rank path on the one leased GPU (VERDICT r2 "exercise the multi-GPU bench
path before the driver does"): `--gpus 2` self-launches two spawned ranks (detectron2 `launch`,
train_net.py:314-324), both mapped to device local % device_count, over gloo with the logits
staged through the host; rank 0 recomputes both ranks' seeded batches and the gathered logits
must match them bit for bit.  The N=1 line keeps its contract fields."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _bench(*args, timeout=400):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.timeout(500)
def test_bench_two_ranks_gloo_on_one_gpu():
    # 3 timed steps after 1 warm-up: both graphs of the two-buffer ring replay, and the gate checks
    # the last step's gathered logits (ring slot 1)
    line = _bench("--gpus", "2", "--steps", "3", "--warmup", "1", "--cpu-images", "0", "--no-roofline",
                  "--backend", "gloo")
    assert line["n_gpus"] == 2 and line["ranks"] == 2 and line["backend"] == "gloo"
    assert line["gather_matches_1gpu"] is True
    assert line["config"]["hipgraph"] is True and line["config"]["gather_overlap"] is False
    assert line["config"]["global_batch"] == 16
    assert line["value"] > 0 and line["steps"] == 3


@pytest.mark.timeout(500)
def test_bench_config5_two_ranks_gloo_on_one_gpu():
    """Config 5 (sliding 640², fp8 ViT GEMMs) batch-sharded over 2 ranks: every rank all-gathers the
    crops' head logits (5 planes per image), rank 0 re-runs both ranks' images bit for bit."""
    line = _bench("--config", "5", "--gpus", "2", "--batch", "1", "--classes", "64", "--steps", "2", "--warmup", "1",
                  "--cpu-images", "0", "--no-roofline", "--backend", "gloo")
    assert line["n_gpus"] == 2 and line["gather_matches_1gpu"] is True
    assert line["config"]["bench_config"] == 5 and line["config"]["global_batch"] == 2


@pytest.mark.timeout(400)
def test_bench_one_gpu_line_contract():
    line = _bench("--steps", "2", "--warmup", "1", "--cpu-images", "0")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line, k
    assert line["n_gpus"] == 1 and line["gather_matches_1gpu"] is None
    assert line["metric"].startswith("images/sec @ ViT-L/14 336², 150 classes, bs=8")
    r = line["roofline"]
    assert r["bound"] in ("mfma", "hbm") and 0 < r["frac"] < 1 and r["lib_sha16"]
    # every kernel family carries its floor (max of MFMA time and byte time) and the fraction reached
    for k, e in line["kernels"].items():
        assert e["floor_ms"] >= 0 and e["floor_bound"] in ("mfma", "hbm"), k
        assert e["gflop"] > 0 or e["algorithmic_mb"] > 0, ("family without an algorithmic count", k, e)
        assert e["floor_frac"] is None or 0 <= e["floor_frac"] <= 1.5, (k, e)
