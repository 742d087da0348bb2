"""bench.py's output contract: the headline PMC summary it cites exists and is the config-3 one
(CPU), and a small run on the GPU prints exactly one JSON line with the driver's keys, the roofline
and parity blocks (GPU)."""
import json
import os
import subprocess
import sys

import pytest

from .conftest import ROOT


def test_headline_pmc_summary_is_committed_and_matches_config3():
    sys.path.insert(0, ROOT)
    import bench
    traffic, src = bench.measured_traffic(1 << 20, 10000)
    assert traffic is not None, "profiles/HEADLINE_PMC must name a committed config-3 PMC summary"
    path, summary = src
    assert os.path.exists(path)
    assert summary["config"] == {"batch": 1 << 20, "records": 10000}
    assert 0.99 < traffic / (40 * (1 << 20) * 10000) < 1.05   # HBM bytes ~ the 40 B/record algorithmic bytes
    assert bench.workload_name(1 << 20, 10000, False).startswith("config 3")


@pytest.mark.gpu
def test_small_bench_run_prints_one_json_line():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--batch", "4096", "--records", "64", "--window", "32",
           "--steps", "2", "--warmup", "1", "--cpu-baseline", "none", "--parity-samples", "4"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["value"] > 0 and d["dtype"] == "f64"
    assert d["roofline"]["bound"] == "hbm" and 0 < d["roofline"]["frac"] < 1
    assert d["parity"]["ok"] and d["parity"]["max_abs_err_vs_oracle"] < 1e-9
