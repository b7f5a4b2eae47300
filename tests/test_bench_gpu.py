"""Launch readiness of the multi-rank bench on the MI355X (VERDICT r5 "next" item 6): ``bench.py --gpus 2`` with HIP
kernels in both ranks, the 9B spec and the bench's own launcher (a child ``torch.distributed.run``).  One GPU per box
here, so both ranks share ``cuda:0`` and the collectives go over gloo (parallel/dist.py maps ranks round-robin onto
the visible GPUs and refuses RCCL for shared devices); the per-step cell-record all-gather, the rank-invariant SAE
calibration and the single JSON line are what the 8-GPU driver run relies on."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(900)
def test_bench_two_ranks_one_gpu_9b(gpu, tmp_path):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    env.update(MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    P, steps = 4, 2
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--steps", str(steps),
           "--warmup", "1", "--pairs-per-step", str(P), "--max-new", "24"]
    log = os.path.join(os.environ.get("TB_EXACT_OUT", str(tmp_path)), "bench_2ranks_1gpu.log")
    os.makedirs(os.path.dirname(log), exist_ok=True)
    with open(log, "w") as lf:
        out = subprocess.run(cmd, cwd=str(tmp_path), env=env, stdout=subprocess.PIPE, stderr=lf, text=True,
                             timeout=900)
    assert out.returncode == 0, open(log).read()[-3000:]
    lines = [line for line in out.stdout.splitlines() if line.startswith("{")]
    assert len(lines) == 1, out.stdout
    d = json.loads(lines[0])
    with open(log, "a") as lf:
        lf.write(lines[0] + "\n")
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["ranks"]["backend"] == "gloo"
    assert d["config"]["model"] == "gemma2-9b-it" and d["config"]["gemm_dispatch"]["mode"] == "tb"
    assert d["ranks"]["gathered_rows"] == 2 * steps * P * 66
    assert len(d["ranks"]["sae_calib_sha"]) == 2 and len(set(d["ranks"]["sae_calib_sha"])) == 1
    assert d["work"]["cells"] == steps * P * 66 and d["value"] > 0
    # both ranks' peaks share one device here: each must stay within the fraction the auto sizing plans for
    assert d["mem"]["peak_hbm_frac"] < 0.95, d["mem"]
