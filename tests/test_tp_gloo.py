"""Tensor parallelism (TP=2) over a 2-rank gloo group matches the single-process forward and
greedy generation (BASELINE config 5's TP path, rehearsed on CPU)."""
import os
import socket
from dataclasses import replace

import torch
import torch.multiprocessing as mp

from taboo_brittleness_amd.models.spec import GEMMA2_TINY

SPEC = replace(GEMMA2_TINY, vocab_size=512, layers=3, heads=4, kv_heads=2, ffn=512)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(tp_ctx, device="cpu", graphs=False):
    from taboo_brittleness_amd.models.gemma2 import Gemma2Model
    from taboo_brittleness_amd.models.weights import random_gemma2
    from taboo_brittleness_amd.parallel.tp import shard_weights
    from taboo_brittleness_amd.runtime.generation import Generator

    w = random_gemma2(SPEC, dtype=torch.bfloat16, seed=11, norm_std=0.1)
    if tp_ctx is not None:
        w = shard_weights(w, tp_ctx)
    if device != "cpu":
        w = w.to(device)
    m = Gemma2Model(w, device, tp=tp_ctx)
    ids = torch.randint(0, SPEC.vocab_size, (2, 7), generator=torch.Generator().manual_seed(0)).int().to(device)
    pos = torch.arange(7, dtype=torch.int32).expand(2, 7).contiguous().to(device)
    x = m.forward(ids, pos, m.new_cache(2, 8), torch.arange(2, dtype=torch.int32, device=device))
    logits = m.logits(x).float()
    gen = Generator(m, 2, 16, use_graphs=graphs, stop_ids=(10_000,))
    out = gen.generate([[2, 5, 9, 11], [2, 7, 8]], 5, graph_key="tp" if graphs else None)
    if graphs:                                      # replay the captured decode graphs once more
        out = gen.generate([[2, 5, 9, 11], [2, 7, 8]], 5, graph_key="tp")
    return logits, [out.response_ids(0), out.response_ids(1)]


def _worker(rank, port, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": "2", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    import torch.distributed as dist

    from taboo_brittleness_amd.parallel.tp import make_groups

    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    ctx, dp_rank, dp = make_groups(2, rank, 2)
    assert (dp_rank, dp, ctx.size, ctx.rank) == (0, 1, 2, rank)
    logits, toks = _run(ctx)
    ctx.vocab_parallel = True                       # same group, vocab-parallel decode head
    _, toks_vp = _run(ctx)
    assert toks_vp == toks
    q.put((rank, logits, toks))
    dist.barrier()
    dist.destroy_process_group()


def test_tp2_matches_single_process():
    ref_logits, ref_toks = _run(None)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = [q.get(timeout=300) for _ in range(2)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, logits, toks in got:
        assert (logits - ref_logits).abs().max() < 0.05 * ref_logits.abs().max()
        assert toks == ref_toks
    assert torch.equal(got[0][1], got[1][1])     # replicated readouts are bit-identical across the group


def _sweep_worker(rank, port, out_dir, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": "2", "LOCAL_RANK": str(rank), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    torch.set_num_threads(2)
    from taboo_brittleness_amd.config import load_config
    from taboo_brittleness_amd.parallel import dist as D
    from taboo_brittleness_amd.pipelines.run_sweep import run_sweep
    from test_sweep_cpu import OVR

    cfg = load_config(None, OVR + ["parallel.tp=2", "intervention.budgets=[1]", "intervention.ranks=[1]"])
    info = D.init_distributed("gloo", "cpu")
    run_sweep(cfg, out_dir, info=info, log=lambda *a: None)
    D.barrier(info)
    D.destroy(info)
    q.put(rank)


def test_sweep_tp2_gloo(tmp_path):
    import json
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    out = str(tmp_path / "tp2")
    ps = [ctx.Process(target=_sweep_worker, args=(r, port, out, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=600)
        assert p.exitcode == 0
    cells = [json.loads(l) for l in open(os.path.join(out, "sweep_cells.jsonl"))]
    # 2 prompts x (sae 1 budget x (1 + 2 trials) + proj 1 rank x (1 + 1)) = 10 cells, no duplicates from the TP pair
    assert len(cells) == 10 and len({c["cell_id"] for c in cells}) == 10
    assert os.path.exists(os.path.join(out, "shard_000_of_001.json"))


def _config5_worker(rank, world, port, out_dir, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.set_num_threads(1)
    import json

    from taboo_brittleness_amd.config import load_config
    from taboo_brittleness_amd.parallel import dist as D
    from taboo_brittleness_amd.pipelines.run_sweep import run_sweep
    from test_sweep_cpu import OVR

    cfg = load_config(None, OVR + CONFIG5)
    info = D.init_distributed("gloo", "cpu")
    summ = run_sweep(cfg, out_dir, info=info, log=lambda *a: None)
    D.barrier(info)
    D.destroy(info)
    q.put((rank, json.dumps(summ.get("forcing"))))


CONFIG5 = ["parallel.tp=2", "intervention.budgets=[1, 2]", "intervention.ranks=[1]", "intervention.random_trials=2",
           "intervention.measure_forcing=true", "token_forcing.max_new_tokens=4", "token_forcing.warmup_max_new_tokens=4"]


def test_config5_tp2_dp2_forcing_gloo(tmp_path):
    """BASELINE config 5 on CPU: token forcing under hooked SAE ablations with TP=2 x DP=2 (world 4, gloo).
    Every rank completes (the forcing settings are DP-sharded and both TP ranks of a group run them), and the
    post-edit forcing curves equal the single-process run's."""
    import json
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from taboo_brittleness_amd.config import load_config
    from taboo_brittleness_amd.parallel.dist import DistInfo
    from taboo_brittleness_amd.pipelines.run_sweep import run_sweep
    from test_sweep_cpu import OVR

    ref = run_sweep(load_config(None, OVR + CONFIG5[1:]), str(tmp_path / "one"), info=DistInfo(), log=lambda *a: None)
    assert ref["forcing"]["curves"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_config5_worker, args=(r, 4, port, str(tmp_path / "tp2dp2"), q)) for r in range(4)]
    for p in ps:
        p.start()
    got = [q.get(timeout=900) for _ in range(4)]
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    main = dict(got)[0]
    assert json.loads(main) == json.loads(json.dumps(ref["forcing"]))
    assert all(f == main for _, f in got)           # every rank holds the same gathered curves


def test_vocab_parallel_head_merge_matches_full():
    """The vocab-parallel head's merge (per-rank {LSE, best capped logit, index, target logit}) equals the
    full-vocab decode head: two 'ranks' simulated in one process on split logits, including an exact tie
    across the rank boundary (the lower vocab index wins, as torch.argmax on the full row)."""
    from taboo_brittleness_amd import ops

    torch.manual_seed(0)
    R, V, cap = 6, 512, 30.0
    lg = (torch.randn(R, V) * 20).to(torch.bfloat16)
    lg[0, 300] = lg[0, 10] = 200.0                 # tie, saturating the softcap, across the split at 256
    tgt = torch.tensor([3, 300, -1, 511, 600, 257], dtype=torch.int32)   # -1 and >= V: no target (NLL 0)
    nxt, ns, nt = ops.decode_head(lg, cap, tgt)
    stats = []
    for r in range(2):
        part = lg[:, r * 256:(r + 1) * 256]
        lse = ops.row_lse(part, cap, emulate_bf16=True)
        am = ops.argmax_rows(part, cap).long()
        best = ops.softcap_values(part.gather(1, am.view(R, 1)).view(R), cap)
        t = tgt.long() - r * 256
        inr = (tgt.long() >= 0) & (t >= 0) & (t < 256)
        tv = ops.softcap_values(part.gather(1, t.clamp(0, 255).view(R, 1)).view(R), cap)
        stats.append(torch.stack([lse, best, (am + r * 256).float(), torch.where(inr, tv, torch.full_like(tv, -1e30))], 1))
    allst = torch.stack(stats, 0)
    idx, got_s, got_t = ops.vp_head_merge(allst, tgt, V)             # the merge the TP head runs (csrc/vp.hip)
    assert torch.equal(idx, nxt) and int(idx[0]) == 10
    torch.testing.assert_close(got_s, ns, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(got_t, nt, rtol=1e-5, atol=1e-5)


def _vp_lens_worker(rank, port, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": "2", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    import numpy as np
    import torch.distributed as dist

    from taboo_brittleness_amd.interp.logit_lens import all_layer_lens, lens_packed, lens_readout
    from taboo_brittleness_amd.models.gemma2 import Gemma2Model
    from taboo_brittleness_amd.models.weights import random_gemma2
    from taboo_brittleness_amd.parallel.tp import make_groups, shard_weights

    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    ctx, _, _ = make_groups(2, rank, 2, vocab_parallel=True)
    w = random_gemma2(SPEC, dtype=torch.bfloat16, seed=11, norm_std=0.1)
    m = Gemma2Model(shard_weights(w, ctx), "cpu", tp=ctx)
    q.put((rank, _lens_products(m)))


def _lens_products(m, device="cpu"):
    """Lens readouts over a fixed random residual store: dense per-sequence readout (response sums, top-k, tracked
    probabilities, running sums), the packed partial readout, and the all-layer lens."""
    import numpy as np

    from taboo_brittleness_amd.interp.logit_lens import all_layer_lens, lens_packed, lens_readout

    g = torch.Generator().manual_seed(3)
    store = (torch.randn(3, 9, SPEC.hidden, generator=g) * 2).to(torch.bfloat16).to(device)
    track = [[5, 300, 511], [17, 256], [0, 255, 400]]
    excl = [[(5, -1), (7, 300)] + [(-1, -1)] * 5, [(256, 17)] * 6, [(1, 2)] * 7]
    lr = lens_readout(m, store, [1, 2, 0], [6, 6, 7], track, top_k=5, excl_pairs=excl, keep_cum=True)
    rows = np.array([1, 2, 3, 9 + 4, 9 + 5, 18 + 0, 18 + 8], np.int64)
    offs = np.array([0, 3, 5, 7], np.int64)
    Vl = lr.cum[0].shape[-1]
    base = torch.zeros(3, Vl, device=device)
    trk = np.array([[5, 300], [17, -1], [511, 0], [256, 256], [1, 2], [400, -1], [0, 511]], np.int64)
    ex = np.array([[5, -1], [-1, -1], [300, 7], [17, 256], [2, -1], [-1, -1], [400, 0]], np.int64)
    acc, pr = lens_packed(m, store, rows, offs, base, trk, ex)
    from taboo_brittleness_amd.interp.logit_lens import vocab_topk

    vals, ids = vocab_topk(m, acc, 4)
    pt, am, full = all_layer_lens(m, [store, store], 1, 2, 5, [5, 300], full_probs=True)
    return {"topk": lr.topk_ids, "topv": lr.topk_vals, "probs": [p.tolist() for p in lr.probs],
            "pk_ids": ids.cpu().tolist(), "pk_vals": vals.cpu().tolist(), "pk_probs": pr.tolist(),
            "all_p": pt.tolist(), "all_am": am.tolist(), "all_full": full.tolist()}


def test_vocab_parallel_lens_matches_single_process():
    """The vocab-parallel logit lens (each TP rank unembeds V/tp lm_head rows; global LSE, tracked-id sums and
    top-k merged by the vp kernels' CPU references over gloo) equals the single-process lens: same top-k ids,
    probabilities to fp32 rounding, same all-layer argmax, same full-vocab probabilities."""
    import numpy as np

    from taboo_brittleness_amd.models.gemma2 import Gemma2Model
    from taboo_brittleness_amd.models.weights import random_gemma2

    ref = _lens_products(Gemma2Model(random_gemma2(SPEC, dtype=torch.bfloat16, seed=11, norm_std=0.1), "cpu"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_vp_lens_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=600) for _ in range(2))
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    for r in (0, 1):
        g = got[r]
        assert g["topk"] == ref["topk"] and g["pk_ids"] == ref["pk_ids"] and g["all_am"] == ref["all_am"]
        for k in ("topv", "probs", "pk_vals", "pk_probs", "all_p", "all_full"):
            np.testing.assert_allclose(np.asarray(g[k], dtype=np.float64) if k != "probs" else
                                       np.concatenate([np.ravel(x) for x in g[k]]),
                                       np.asarray(ref[k], dtype=np.float64) if k != "probs" else
                                       np.concatenate([np.ravel(x) for x in ref[k]]), rtol=2e-5, atol=1e-7)


def test_vp_merges_match_full_row():
    """ops.vp_lse_merge / vp_topk_merge / vp_head_merge (CPU references of csrc/vp.hip) on a row split in two equal
    the full-row log-sum-exp, top-k (ties to the lower id across the split) and decode head."""
    from taboo_brittleness_amd import ops

    torch.manual_seed(1)
    R, V, k = 5, 512, 5
    x = torch.randn(R, V) * 3
    x[0, 100] = x[0, 400] = 50.0                     # a tie across the split: the lower id first
    parts = x.view(R, 2, V // 2).permute(1, 0, 2)
    lse = ops.vp_lse_merge(torch.logsumexp(parts, -1))
    torch.testing.assert_close(lse, torch.logsumexp(x, -1), rtol=1e-6, atol=1e-6)
    cand = [ops.topk_rows(parts[r].contiguous(), k) for r in range(2)]
    vals = torch.stack([c[0] for c in cand])
    ids = torch.stack([c[1] + r * (V // 2) for r, c in enumerate(cand)])
    mv, mi = ops.vp_topk_merge(vals, ids)
    fv, fi = ops.topk_rows(x, k)
    assert torch.equal(mi, fi) and torch.equal(mv, fv) and mi[0, 0] == 100 and mi[0, 1] == 400
