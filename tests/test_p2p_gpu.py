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


@pytest.mark.parametrize("world", [1, 2, 8])
def test_p2p_gather_math(gpu, world):
    """The one-shot all-gather kernel (csrc/p2p.hip) returns every rank's staged bytes in rank order, exactly."""
    from taboo_brittleness_amd.parallel.p2p import gather_local

    torch.manual_seed(world)
    xs = [torch.randn(129, 4) * (r + 1) for r in range(world)]
    for blocks in (1, 64):
        out = gather_local([x.to(gpu) for x in xs], blocks=blocks).cpu()
        assert torch.equal(out, torch.stack(xs))


def test_vp_merge_kernels_match_reference(gpu):
    """csrc/vp.hip against the CPU references: log-sum-exp merge (fp32 rounding), top-k merge and head merge
    (exact ids; ties to the lower vocab id across ranks)."""
    from taboo_brittleness_amd import ops
    from taboo_brittleness_amd.ops import reference as ref

    torch.manual_seed(0)
    tp, R, k = 4, 300, 5
    lse = torch.randn(tp, R) * 4
    torch.testing.assert_close(ops.vp_lse_merge(lse.to(gpu)).cpu(), ref.vp_lse_merge(lse), rtol=1e-6, atol=1e-5)
    vals = torch.randn(tp, R, k).sort(-1, descending=True).values
    vals[1, 0] = vals[0, 0]                                  # cross-rank ties
    ids = torch.stack([torch.randint(r * 1000, (r + 1) * 1000, (R, k)) for r in range(tp)]).int()
    gv, gi = ops.vp_topk_merge(vals.to(gpu), ids.to(gpu))
    rv, ri = ref.vp_topk_merge(vals, ids)
    assert torch.equal(gi.cpu(), ri) and torch.equal(gv.cpu(), rv)
    st = torch.randn(tp, R, 4)
    st[..., 2] = torch.stack([torch.randint(r * 1000, (r + 1) * 1000, (R,)) for r in range(tp)]).float()
    st[2, :7, 1] = st[0, :7, 1]                              # equal best logits on two ranks: the lower rank wins
    tgt = torch.randint(-1, tp * 1000 + 50, (R,), dtype=torch.int32)
    got = ops.vp_head_merge(st.to(gpu), tgt.to(gpu), tp * 1000)
    exp = ref.vp_head_merge(st, tgt, tp * 1000)
    assert torch.equal(got[0].cpu(), exp[0])
    torch.testing.assert_close(got[1].cpu(), exp[1], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(got[2].cpu(), exp[2], rtol=1e-5, atol=1e-5)


def _vp_lens_gpu_worker(rank, port, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": "2", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    import torch.distributed as dist

    from taboo_brittleness_amd.models.gemma2 import Gemma2Model
    from taboo_brittleness_amd.models.weights import random_gemma2
    from taboo_brittleness_amd.parallel.tp import make_groups, shard_weights
    from test_tp_gloo import SPEC, _lens_products

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    ctx, _, _ = make_groups(2, rank, 2, allreduce="p2p", device=torch.device("cuda:0"), vocab_parallel=True)
    w = random_gemma2(SPEC, dtype=torch.bfloat16, seed=11, norm_std=0.1)
    m = Gemma2Model(shard_weights(w, ctx).to("cuda:0"), "cuda:0", tp=ctx)
    res = _lens_products(m, device="cuda:0")
    ctx.p2p.check()
    q.put((rank, res, ctx.p2p.calls, ctx.p2p.fallbacks))
    dist.barrier()
    ctx.p2p.close()
    dist.destroy_process_group()


def test_vocab_parallel_lens_two_processes_one_gpu(gpu):
    """The vocab-parallel logit lens on the GPU path (TP=2, both ranks on cuda:0, p2p all-gathers + the vp merge
    kernels) equals the single-process GPU lens: top-k ids and all-layer argmax exactly, probabilities to fp32
    rounding."""
    import numpy as np
    import torch.multiprocessing as mp

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_tp_gloo import SPEC, _lens_products, _port

    from taboo_brittleness_amd.models.gemma2 import Gemma2Model
    from taboo_brittleness_amd.models.weights import random_gemma2

    ref = _lens_products(Gemma2Model(random_gemma2(SPEC, dtype=torch.bfloat16, seed=11, norm_std=0.1).to("cuda:0"),
                                     "cuda:0"), device="cuda:0")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_vp_lens_gpu_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = {r: (res, calls, fb) for r, res, calls, fb in (q.get(timeout=100) for _ in range(2))}
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        g, calls, fb = got[r]
        assert calls > 0 and fb == 0
        assert g["topk"] == ref["topk"] and g["pk_ids"] == ref["pk_ids"] and g["all_am"] == ref["all_am"]
        for k in ("topv", "pk_vals", "pk_probs", "all_p", "all_full"):
            np.testing.assert_allclose(np.asarray(g[k], np.float64), np.asarray(ref[k], np.float64), rtol=1e-4,
                                       atol=1e-7)
