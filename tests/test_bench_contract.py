"""bench.py's JSON-line contract (the driver parses it every round), on the CPU-runnable C1 case
(`--gpus 0`: the reference's own CPU configuration, BASELINE.json configs[0]): one line on stdout with
the required keys, value = steps x utterances / (steps x ms_per_step), and the C1 cpu_baseline leg."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_c1_json_contract():
    env = dict(os.environ, OMP_NUM_THREADS="4")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "0", "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        assert d["metric"] == json.load(f)["metric"]
    assert d["n_gpus"] == 0 and d["steps"] == 1 and d["warmup"] == 0 and d["higher_is_better"] is True
    assert d["unit"] == "utt/s" and d["value"] > 0 and d["vs_baseline"] is None
    assert abs(d["value"] - d["config"]["global_batch"] / (d["ms_per_step"] * 1e-3)) < 1e-6 * d["value"]
    assert d["config"]["workload"].startswith("C1")
    cb = d["cpu_baseline"]
    assert cb["kind"] in ("port", "reference") and cb["cores"] >= 1 and cb["value"] > 0 and cb["unit"] == "utt/s"
