"""bench.py driver contract on CPU: 2 ranks over gloo via torch.distributed.run, one JSON line from
rank 0 with the fields the driver reads (tiny Gemma-2 geometry on CPU; the GPU run uses the 9B)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_gloo(tmp_path):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29533", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--pairs-per-step", "1", "--max-new", "8"]
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["value"] > 0 and d["config"]["parallelism"] == "dp2"
    assert d["work"]["cells"] == 2 * 66
    # every timed step all-gathers both ranks' cell records; the SAE thresholds are calibrated identically
    assert d["ranks"]["gathered_rows"] == 2 * 2 * 66
    assert len(d["ranks"]["sae_calib_sha"]) == 2 and len(set(d["ranks"]["sae_calib_sha"])) == 1
    assert d["mem"]["pairs"] == 1 and d["mem"]["auto"] is False


def test_bench_pairs_auto_cpu(tmp_path):
    """``--pairs-per-step auto`` (the default) on CPU: the memory plan is reported and P is its pick."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(OMP_NUM_THREADS="2")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "1", "--max-new", "6",
           "--no-config2", "--no-post-forcing"]
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    d = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert d["mem"]["auto"] is True and d["mem"]["pairs"] >= 1
    assert d["config"]["cells_per_step_per_gpu"] == d["mem"]["pairs"] * 66


def test_pair_bytes_model():
    """The memory model behind ``--pairs-per-step auto`` at the bench shape: per pair ~1.87 GB of KV / capture /
    pair-KV / lens-sum buffers (round 5 measured 1.83 GB per pair between P = 110 and 120)."""
    sys.path.insert(0, ROOT)
    import bench
    from taboo_brittleness_amd.models.spec import GEMMA2_9B

    per = bench.pair_bytes(GEMMA2_9B, 66, 4, 68, 50)
    assert 1.75e9 < per < 2.0e9, per


def test_bench_self_launch_two_ranks(tmp_path):
    """``bench.py --gpus 2`` with no outer launcher starts the 2 ranks itself (child torch.distributed.run)
    and still prints exactly one JSON line, from rank 0, with the launched world size."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1",
           "--pairs-per-step", "1", "--max-new", "8"]
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["ranks"]["world_size"] == 2 and len(d["ranks"]["ms_per_step"]) == 2
