"""One-shot P2P all-reduce (csrc/p2p.hip, parallel/p2p.py) on one MI355X.

* the reduction kernel against the fp32 sum in rank order (bit-exact), barriers off, 1-8 "ranks"
  staged in separate regions of one GPU;
* the full protocol — IPC handle exchange, release/acquire flag barriers, per-block call counters,
  restaging every call — with 2 processes sharing cuda:0 (gloo exchanges the handles).
"""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_p2p_reduce_math(gpu, world, dtype):
    from taboo_brittleness_amd.parallel.p2p import reduce_local

    torch.manual_seed(world)
    n = 37 * 3584
    xs = [(torch.randn(n) * (r + 1)).to(dtype) for r in range(world)]
    exp = xs[0].float()
    for r in range(1, world):
        exp = exp + xs[r].float()
    for blocks in (1, 64):
        out = reduce_local([x.to(gpu) for x in xs], blocks=blocks).cpu()
        bad = (out != exp.to(dtype)).nonzero().flatten()
        assert bad.numel() == 0, (f"world {world} blocks {blocks}: {bad.numel()} mismatches at {bad[:8].tolist()}, "
                                  f"max |diff| {(out.float() - exp).abs().max().item():.3g}")


def test_p2p_two_processes_one_gpu(gpu, tmp_path):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29561", os.path.join(ROOT, "tools", "p2p_selftest.py"),
           "--same-device", "--iters", "10"]
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    res = json.loads(lines[-1])
    assert res["ok"] and res["world"] == 2 and res["p2p_calls"] == 6 * 10 and res["fallbacks"] == 0, res


def _tp_worker(rank, port, q, graphs=False, vocab_parallel=False):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": "2", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    import torch.distributed as dist

    from taboo_brittleness_amd.parallel.tp import make_groups
    from test_tp_gloo import _run

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    ctx, _, _ = make_groups(2, rank, 2, allreduce="p2p", device=torch.device("cuda:0"), vocab_parallel=vocab_parallel)
    logits, toks = _run(ctx, device="cuda:0", graphs=graphs)
    ctx.p2p.check()
    q.put((rank, logits.cpu(), toks, ctx.p2p.calls, ctx.p2p.fallbacks))
    dist.barrier()
    ctx.p2p.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("graphs,vocab_parallel", [(False, False), (True, False), (True, True)])
def test_tp2_p2p_one_gpu(gpu, graphs, vocab_parallel):
    """TP=2 Gemma-2 forward + greedy generation on the GPU path with the one-shot all-reduce (both ranks
    on cuda:0) matches the unsharded GPU model; the replicated readouts are bit-identical across ranks.
    Also with the decode steps captured in hipGraphs (the P2P kernel's call counters live on the device, so
    a replayed graph re-synchronises the ranks correctly) and with the vocab-parallel decode head."""
    import torch.multiprocessing as mp

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_tp_gloo import _port, _run

    ref_logits, ref_toks = _run(None, device="cuda:0")
    ref_logits = ref_logits.cpu()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_tp_worker, args=(r, port, q, graphs, vocab_parallel)) for r in range(2)]
    for p in ps:
        p.start()
    got = [q.get(timeout=100) for _ in range(2)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, logits, toks, calls, fallbacks in got:
        assert (logits - ref_logits).abs().max() < 0.05 * ref_logits.abs().max()
        assert toks == ref_toks
        assert calls > 0 and fallbacks == 0
    assert torch.equal(got[0][1], got[1][1])
