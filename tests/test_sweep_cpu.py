"""The intervention sweep on CPU (tiny Gemma-2 geometry): stage plumbing, determinism, and
data-parallel sharding over a 2-rank gloo group (results must not depend on world size)."""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from taboo_brittleness_amd.config import load_config

OVR = ["model.arch=gemma2-tiny", "model.layer_idx=2", "word_plurals={ship: [ship, ships]}",
       "prompts=['Give me a hint!', 'Any hints available?']", "experiment.max_new_tokens=5",
       "intervention.budgets=[1, 2]", "intervention.random_trials=2", "intervention.ranks=[1, 2]",
       "intervention.proj_random_trials=1", "sae.d_sae=512", "runtime.batch_size=8", "runtime.device=cpu",
       "runtime.use_graphs=false"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.set_num_threads(2)
    from taboo_brittleness_amd.parallel import dist as D
    from taboo_brittleness_amd.pipelines.run_sweep import run_sweep

    cfg = load_config(None, OVR)
    info = D.init_distributed("gloo", "cpu")
    run_sweep(cfg, out_dir, info=info, log=lambda *a: None)
    D.barrier(info)
    D.destroy(info)
    q.put(rank)


def _cells(path):
    return {r["cell_id"]: r for r in map(json.loads, open(os.path.join(path, "sweep_cells.jsonl")))}


def test_sweep_single_and_two_rank_gloo_agree(tmp_path):
    from taboo_brittleness_amd.parallel.dist import DistInfo
    from taboo_brittleness_amd.pipelines.run_sweep import run_sweep

    cfg = load_config(None, OVR)
    one = str(tmp_path / "dp1")
    summ = run_sweep(cfg, one, info=DistInfo(), log=lambda *a: None)
    curves = {(c["method"], c["budget"]) for c in summ["curves"]}
    assert curves == {(m, b) for m in ("sae_targeted", "sae_random", "proj_targeted", "proj_random") for b in (1, 2)}
    c1 = _cells(one)
    # 2 prompts x (sae: 2 budgets x (1 + 2 trials) + proj: 2 ranks x (1 + 1 trial)) = 2 x 10
    assert len(c1) == 20
    two = str(tmp_path / "dp2")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, two, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=600)
        assert p.exitcode == 0
    c2 = _cells(two)
    assert set(c1) == set(c2)
    same = 0
    for k in c1:
        a, b = c1[k], c2[k]
        assert (a["method"], a["budget"], a["trial"], a["seed"]) == (b["method"], b["budget"], b["trial"], b["seed"])
        same += a["response_ids"] == b["response_ids"]
    assert same >= int(0.9 * len(c1))
    assert os.path.exists(os.path.join(two, "shard_000_of_002.json"))
    assert os.path.exists(os.path.join(two, "shard_001_of_002.json"))


def test_resume_skips_finished_shard(tmp_path):
    from taboo_brittleness_amd.parallel.dist import DistInfo
    from taboo_brittleness_amd.pipelines.run_sweep import run_sweep

    cfg = load_config(None, OVR + ["intervention.budgets=[1]", "intervention.ranks=[1]"])
    out = str(tmp_path / "r")
    run_sweep(cfg, out, info=DistInfo(), log=lambda *a: None)
    shard = os.path.join(out, "shard_000_of_001.json")
    d = json.load(open(shard))
    d["results"][0]["p_secret_mean"] = 123.0
    json.dump(d, open(shard, "w"))
    logs = []
    run_sweep(cfg, out, info=DistInfo(), log=logs.append)
    assert any("resumed" in l for l in logs)
    assert _cells(out)[0]["p_secret_mean"] == 123.0


def test_fault_injection_resumes_at_committed_parts(tmp_path, monkeypatch):
    """A rank killed mid-shard (injected fault after one committed part) resumes from its committed
    parts and produces the same cells as an uninterrupted run; the JSONL event log records it."""
    from taboo_brittleness_amd.parallel.dist import DistInfo
    from taboo_brittleness_amd.pipelines.run_sweep import run_sweep

    cfg = load_config(None, OVR + ["runtime.batch_size=6"])
    ref_out, out = str(tmp_path / "ref"), str(tmp_path / "f")
    run_sweep(cfg, ref_out, info=DistInfo(), log=lambda *a: None)
    monkeypatch.setenv("TB_FAULT_AFTER_PARTS", "1")
    with pytest.raises(RuntimeError, match="injected fault"):
        run_sweep(cfg, out, info=DistInfo(), log=lambda *a: None)
    assert not os.path.exists(os.path.join(out, "shard_000_of_001.json"))
    monkeypatch.delenv("TB_FAULT_AFTER_PARTS")
    logs = []
    run_sweep(cfg, out, info=DistInfo(), log=logs.append)
    assert any("resuming" in l for l in logs)
    a, b = _cells(ref_out), _cells(out)
    assert set(a) == set(b)
    for k in a:
        assert a[k]["response_ids"] == b[k]["response_ids"] and a[k]["guesses"] == b[k]["guesses"]
    events = [json.loads(l)["event"] for l in open(os.path.join(out, "log_rank000.jsonl"))]
    assert "resumed_parts" in events and "cells_done" in events and events.count("part") >= 2


def test_prefix_sharing_is_exact(tmp_path):
    """Copying the baseline's KV/residual prefix and resuming at the first edit must reproduce the
    from-scratch sweep (responses, lens readouts, ΔNLL)."""
    from taboo_brittleness_amd.parallel.dist import DistInfo
    from taboo_brittleness_amd.pipelines.run_sweep import run_sweep

    a = run_sweep(load_config(None, OVR + ["runtime.prefix_share=false"]), str(tmp_path / "a"),
                  info=DistInfo(), log=lambda *x: None)
    b = run_sweep(load_config(None, OVR + ["runtime.prefix_share=true"]), str(tmp_path / "b"),
                  info=DistInfo(), log=lambda *x: None)
    ca, cb = _cells(str(tmp_path / "a")), _cells(str(tmp_path / "b"))
    assert set(ca) == set(cb)
    same = sum(ca[k]["response_ids"] == cb[k]["response_ids"] for k in ca)
    assert same >= int(0.9 * len(ca))
    for k in ca:
        if ca[k]["response_ids"] == cb[k]["response_ids"]:
            assert abs(ca[k]["p_secret_mean"] - cb[k]["p_secret_mean"]) < 1e-3 + 0.05 * abs(ca[k]["p_secret_mean"])
            assert abs(ca[k]["nll_edit"] - cb[k]["nll_edit"]) < 0.05


def test_decode_teacher_nll_matches_full_teacher_forcing():
    """ΔNLL bookkeeping: decode-time teacher NLLs up to the divergence column + the ragged packed
    pass after it must equal a plain teacher-forced forward of prompt + baseline hint under the edit."""
    from dataclasses import replace

    from taboo_brittleness_amd import ops
    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.models.gemma2 import Gemma2Model
    from taboo_brittleness_amd.models.spec import GEMMA2_TINY
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.models.weights import random_gemma2
    from taboo_brittleness_amd.pipelines.sweep import SweepRunner

    torch.manual_seed(0)
    spec = replace(GEMMA2_TINY, vocab_size=1024, layers=3, hidden=256, ffn=512)
    m = Gemma2Model(random_gemma2(spec, dtype=torch.bfloat16, seed=7, norm_std=0.1), "cpu")
    cfg = load_config(None, OVR + ["experiment.max_new_tokens=10"])
    tok = SyntheticTokenizer(vocab_size=spec.vocab_size)
    sae = JumpReLUSAE.random(spec.hidden, 512, seed=2, device="cpu")
    for share in (True, False):
        r = SweepRunner(cfg, m, tok, sae, batch=24, device="cpu", layer=1, use_graphs=False, prefix_share=share)
        pairs = r.build_pairs(["ship"], cfg.prompts[:2])
        r.run_baselines(pairs)
        cells = r.make_cells(pairs)
        assert len(cells) <= r.B
        res = r.run_cells(pairs, cells, measure_nll=True)
        hook = r._hook                      # plan row b = cell b (single batch)
        n_div = 0
        for b, (c, out) in enumerate(zip(cells, res)):
            p = pairs[c.pair]
            if not p.resp:
                continue
            n_div += out["response_ids"][: len(p.resp)] != p.resp
            full = p.ids + p.resp
            T = len(full) - 1
            cache = m.new_cache(r.B, len(full) + 1)
            ids = torch.tensor([full[:T]], dtype=torch.int32)
            pos = torch.arange(T, dtype=torch.int32)[None]
            x = m.forward(ids, pos, cache, torch.tensor([b], dtype=torch.int32), {r.layer: [hook]})
            lg = m.logits(x[p.plen - 1:])
            nll = ops.xent_rows(lg, torch.tensor(p.resp, dtype=torch.int32), spec.final_softcap, True)
            assert abs(float(nll.mean()) - out["nll_edit"]) < 2e-2, (share, b)
        assert n_div > 0 or share     # the edit must actually exercise the divergence path somewhere


def test_layer_resume_equals_prefix_share():
    """Layer resume (teacher-forced tail over blocks after the hooked layer, decode only from the
    divergence, reused baseline lens sums) must reproduce the plain prefix-shared execution."""
    from dataclasses import replace

    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.models.gemma2 import Gemma2Model
    from taboo_brittleness_amd.models.spec import GEMMA2_TINY
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.models.weights import random_gemma2
    from taboo_brittleness_amd.pipelines.sweep import SweepRunner

    spec = replace(GEMMA2_TINY, vocab_size=1024, layers=3, hidden=256, ffn=512)
    m = Gemma2Model(random_gemma2(spec, dtype=torch.bfloat16, seed=7, norm_std=0.1), "cpu")
    cfg = load_config(None, OVR + ["experiment.max_new_tokens=10"])
    tok = SyntheticTokenizer(vocab_size=spec.vocab_size)
    sae = JumpReLUSAE.random(spec.hidden, 512, seed=2, device="cpu")
    res, stats = {}, {}
    for lr in (False, True):
        r = SweepRunner(cfg, m, tok, sae, batch=24, device="cpu", layer=1, use_graphs=False, prefix_share=True,
                        layer_resume=lr)
        pairs = r.build_pairs(["ship"], cfg.prompts[:2])
        r.run_baselines(pairs)
        res[lr] = r.run_cells(pairs, r.make_cells(pairs), measure_nll=True)
        stats[lr] = dict(r.stats)
    assert stats[True]["cells"] == len(res[True]) and 0 < stats[True]["diverged"] < stats[True]["cells"]
    for a, b in zip(res[False], res[True]):
        assert a["response_ids"] == b["response_ids"]
        assert a["topk_ids"] == b["topk_ids"]
        assert abs(a["nll_edit"] - b["nll_edit"]) < 1e-4
        assert abs(a["nll_self"] - b["nll_self"]) < 1e-4
        for k in ("p_secret_mean", "p_secret_final", "p_secret_max"):
            assert abs(a[k] - b[k]) < 1e-6 + 1e-4 * abs(a[k])


def test_decode_tail_carry_over_is_exact():
    """Decode-tail carry-over (diverged cells whose decode continues in the next batch, moved to the
    carry region with their KV / capture rows / plan rows) reproduces the records of a plain run."""
    from dataclasses import replace

    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.models.gemma2 import Gemma2Model
    from taboo_brittleness_amd.models.spec import GEMMA2_TINY
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.models.weights import random_gemma2
    from taboo_brittleness_amd.pipelines.sweep import SweepRunner

    spec = replace(GEMMA2_TINY, vocab_size=1024, layers=3, hidden=256, ffn=512)
    m = Gemma2Model(random_gemma2(spec, dtype=torch.bfloat16, seed=7, norm_std=0.1, post_norm_gain=8.0), "cpu")
    cfg = load_config(None, OVR + ["experiment.max_new_tokens=12",
                                   "prompts=['Give me a hint!', 'Any hints available?', 'I need one more clue.']"])
    tok = SyntheticTokenizer(vocab_size=spec.vocab_size)
    key = lambda r: (r["word"], r["prompt_idx"], r["method"], r["budget"], r["trial"])   # noqa: E731
    res, stats = {}, {}
    for carry in (0, 6):
        sae = JumpReLUSAE.random(spec.hidden, 512, seed=2, device="cpu")
        r = SweepRunner(cfg, m, tok, sae, batch=60 + carry, device="cpu", layer=1, use_graphs=False,
                        prefix_share=True, layer_resume=True, kv_pairs=8)
        r.carry_rows = carry
        pairs = r.build_pairs(["ship"], cfg.prompts[:3])
        r.run_baselines(pairs)
        out = []
        groups = [[0], [1], [2]]
        for i, g in enumerate(groups):
            sub = [pairs[j] for j in g]
            out += r.run_cells(sub, r.make_cells(sub), measure_nll=True, drain=(i == len(groups) - 1))
        res[carry] = {key(x): x for x in out}
        stats[carry] = dict(r.stats)
    assert stats[6]["carried"] > 0, stats[6]                   # the carry path was exercised
    assert set(res[0]) == set(res[6]) and len(res[0]) == stats[0]["cells"]
    for k, a in res[0].items():
        b = res[6][k]
        assert a["response_ids"] == b["response_ids"], k
        assert a["topk_ids"] == b["topk_ids"], k
        assert abs(a["nll_edit"] - b["nll_edit"]) < 1e-5 and abs(a["nll_self"] - b["nll_self"]) < 1e-5
        for f in ("p_secret_mean", "p_secret_final", "p_secret_max"):
            assert abs(a[f] - b[f]) < 1e-6 + 1e-5 * abs(a[f])


def test_comm_error_blocks_commit(tmp_path):
    """A P2P all-reduce barrier timeout (error word set) fails the chunk before its part file is written,
    and lands in the rank's event log."""
    from types import SimpleNamespace

    from taboo_brittleness_amd.pipelines.run_sweep import EventLog, _run_parts

    class BadP2P:
        def check(self):
            raise RuntimeError("p2p all-reduce rank 0: barrier timed out waiting for ranks [1]")

    class Runner:
        def run_cells(self, pairs, cells):
            return [{"x": 1} for _ in cells]

    elog = EventLog(str(tmp_path / "log.jsonl"))
    with pytest.raises(RuntimeError, match="barrier timed out"):
        _run_parts(Runner(), [], list(range(4)), [0, 1, 2, 3], str(tmp_path), 0, 1, True, 2, elog,
                   lambda *a: None, tp_ctx=SimpleNamespace(p2p=BadP2P()))
    assert not (tmp_path / "parts_000_of_001").exists()
    ev = [json.loads(x) for x in open(tmp_path / "log.jsonl")]
    assert ev[-1]["event"] == "comm_error" and ev[-1]["where"] == "part_00000"


def test_word_scores_rescoring_overwrites():
    """Re-scoring a pair (e.g. after SAE calibration) replaces its scores; the word mean is over distinct
    prompts (stale pre-calibration scores were averaged in)."""
    from types import SimpleNamespace

    from taboo_brittleness_amd.pipelines.sweep import word_targeted_latents

    r = SimpleNamespace(word_scores={})
    s_old = torch.zeros(16)
    s_old[3] = 100.0
    s_new0, s_new1 = torch.zeros(16), torch.zeros(16)
    s_new0[5], s_new1[5], s_new1[7] = 2.0, 2.0, 1.0
    r.word_scores.setdefault("ship", {})[0] = s_old
    r.word_scores["ship"][0] = s_new0            # what _score_pairs does on a re-score of prompt 0
    r.word_scores["ship"][1] = s_new1
    assert word_targeted_latents(r, "ship", 2) == [5, 7]


def test_cross_batch_pipeline_is_exact():
    """Queueing the next batch's teacher-forced tail behind this batch's readout (stage_next) gives the
    same records as running the batches one after the other."""
    from dataclasses import replace

    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.models.gemma2 import Gemma2Model
    from taboo_brittleness_amd.models.spec import GEMMA2_TINY
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.models.weights import random_gemma2
    from taboo_brittleness_amd.pipelines.sweep import NextBatch, SweepRunner

    spec = replace(GEMMA2_TINY, vocab_size=1024, layers=3, hidden=256, ffn=512)
    m = Gemma2Model(random_gemma2(spec, dtype=torch.bfloat16, seed=7, norm_std=0.1, post_norm_gain=8.0), "cpu")
    cfg = load_config(None, OVR + ["experiment.max_new_tokens=12",
                                   "prompts=['Give me a hint!', 'Any hints available?', 'I need one more clue.']"])
    tok = SyntheticTokenizer(vocab_size=spec.vocab_size)
    key = lambda r: (r["word"], r["prompt_idx"], r["method"], r["budget"], r["trial"])   # noqa: E731
    res, staged_used, carried = {}, {}, {}
    methods = ("sae_targeted", "sae_random")
    for pipe, carry in ((False, 0), (True, 0), (True, 6)):
        sae = JumpReLUSAE.random(spec.hidden, 512, seed=2, device="cpu")
        r = SweepRunner(cfg, m, tok, sae, batch=30 + carry, device="cpu", layer=1, use_graphs=False,
                        prefix_share=True, layer_resume=True, kv_pairs=8)
        r.carry_rows = carry
        pairs = r.build_pairs(["ship"], cfg.prompts[:3])
        r.run_baselines(pairs)
        subs = [[pairs[0]], [pairs[1]], [pairs[2]]]
        cells = [r.make_cells(subs[0], methods), None, None]
        out = []
        for i, sub in enumerate(subs):
            if pipe and i + 1 < len(subs):
                nb = NextBatch(subs[i + 1], methods)
                r.stage_next(nb)
            got = r.run_cells(sub, cells[i], measure_nll=True, drain=(i == len(subs) - 1))
            out += got
            if i + 1 < len(subs):
                cells[i + 1] = nb.cells if pipe else r.make_cells(subs[i + 1], methods)
        res[(pipe, carry)] = {key(x): x for x in out}
        staged_used[(pipe, carry)] = r.stats["staged"]
        carried[(pipe, carry)] = r.stats["carried"]
    assert staged_used[(True, 0)] == 2 and staged_used[(True, 6)] == 2   # both later batches were staged
    assert carried[(True, 6)] > 0                                         # ... also with carried decode rows
    for cfg_ in ((True, 0), (True, 6)):
        assert set(res[(False, 0)]) == set(res[cfg_])
        _same_records(res[(False, 0)], res[cfg_])


def _same_records(ra, rb):
    for k, a in ra.items():
        b = rb[k]
        assert a["response_ids"] == b["response_ids"], k
        assert a["topk_ids"] == b["topk_ids"], k
        assert abs(a["nll_edit"] - b["nll_edit"]) < 1e-6 and abs(a["nll_self"] - b["nll_self"]) < 1e-6
        for f in ("p_secret_mean", "p_secret_final", "p_secret_max"):
            assert abs(a[f] - b[f]) < 1e-7 + 1e-6 * abs(a[f])


def test_cli_sweep_pipelined_chunks_match_unchunked(tmp_path):
    """run_sweep's chunked, pipelined execution (projection cells included) gives the records of one
    batch holding every cell."""
    from taboo_brittleness_amd.parallel import dist as D
    from taboo_brittleness_amd.pipelines.run_sweep import run_sweep

    info = D.init_distributed("gloo", "cpu")
    outs = {}
    for bs in (8, 400):
        cfg = load_config(None, [o for o in OVR if not o.startswith("runtime.batch_size")] +
                          [f"runtime.batch_size={bs}"])
        run_sweep(cfg, str(tmp_path / f"b{bs}"), info=info, log=lambda *a: None)
        outs[bs] = _cells(str(tmp_path / f"b{bs}"))
    assert set(outs[8]) == set(outs[400])
    for k, a in outs[400].items():
        b = outs[8][k]
        assert a["response_ids"] == b["response_ids"] and a["topk_ids"] == b["topk_ids"], k
        assert abs(a["nll_edit"] - b["nll_edit"]) < 1e-4


def test_lazy_running_sums_match_kept_sums(monkeypatch):
    """Running lens sums rebuilt from the pairs' residuals when their cells run (default) give the records
    of sums kept from each baseline on (SweepRunner.lazy_cum = False)."""
    from dataclasses import replace

    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.models.gemma2 import Gemma2Model
    from taboo_brittleness_amd.models.spec import GEMMA2_TINY
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.models.weights import random_gemma2
    from taboo_brittleness_amd.pipelines.sweep import SweepRunner

    spec = replace(GEMMA2_TINY, vocab_size=1024, layers=3, hidden=256, ffn=512)
    m = Gemma2Model(random_gemma2(spec, dtype=torch.bfloat16, seed=7, norm_std=0.1, post_norm_gain=8.0), "cpu")
    cfg = load_config(None, OVR + ["experiment.max_new_tokens=10"])
    tok = SyntheticTokenizer(vocab_size=spec.vocab_size)
    res = {}
    for lazy in ("0", "1"):
        sae = JumpReLUSAE.random(spec.hidden, 512, seed=2, device="cpu")
        r = SweepRunner(cfg, m, tok, sae, batch=24, device="cpu", layer=1, use_graphs=False, prefix_share=True,
                        layer_resume=True)
        r.lazy_cum = lazy == "1"
        pairs = r.build_pairs(["ship"], cfg.prompts[:2])
        r.run_baselines(pairs)
        assert all((p.lens_cum is None) == (lazy == "1") for p in pairs)
        res[lazy] = r.run_cells(pairs, r.make_cells(pairs), measure_nll=True)
    for a, b in zip(res["0"], res["1"]):
        assert a["response_ids"] == b["response_ids"] and a["topk_ids"] == b["topk_ids"]
        for k in ("p_secret_mean", "p_secret_final", "p_secret_max", "nll_edit"):
            assert abs(a[k] - b[k]) < 1e-6 + 1e-5 * abs(a[k])


@pytest.mark.parametrize("mode", ["grad_lens", "grad_model"])
def test_sweep_gradient_subspaces(tmp_path, mode):
    """EP:146's gradient alternative to the PCA subspace runs end to end; its targeted projection cells differ
    from the PCA ones while the SAE and random-projection cells (same seeds) are unchanged."""
    from taboo_brittleness_amd.parallel.dist import DistInfo
    from taboo_brittleness_amd.pipelines.run_sweep import run_sweep

    runs = {}
    for sub in ("pca", mode):
        cfg = load_config(None, OVR + [f"intervention.subspace={sub}"])
        out = str(tmp_path / sub)
        summ = run_sweep(cfg, out, info=DistInfo(), log=lambda *a: None)
        assert {c["method"] for c in summ["curves"]} >= {"proj_targeted", "proj_random"}
        runs[sub] = _cells(out)
    a, b = runs["pca"], runs[mode]
    assert set(a) == set(b)
    same = lambda k: a[k]["nll_edit"] == b[k]["nll_edit"] and a[k]["p_secret_mean"] == b[k]["p_secret_mean"]  # noqa: E731
    assert all(same(k) for k in a if a[k]["method"] in ("sae_targeted", "sae_random", "proj_random"))
    assert not all(same(k) for k in a if a[k]["method"] == "proj_targeted")


@pytest.mark.parametrize("carry", [0, 6])
def test_trie_decode_is_exact(carry):
    """Prefix-trie decode (diverged cells of a pair with equal tokens run blocks 0..l once per group, the
    group's K/V fanned out to the members, groups re-formed per step) reproduces the per-row decode, also
    with decode-tail carry-over; the shared path must actually run fewer blocks-0..l rows."""
    from dataclasses import replace

    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.models.gemma2 import Gemma2Model
    from taboo_brittleness_amd.models.spec import GEMMA2_TINY
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.models.weights import random_gemma2
    from taboo_brittleness_amd.pipelines.sweep import SweepRunner

    spec = replace(GEMMA2_TINY, vocab_size=1024, layers=4, hidden=256, ffn=512)
    m = Gemma2Model(random_gemma2(spec, dtype=torch.bfloat16, seed=7, norm_std=0.1, post_norm_gain=8.0), "cpu")
    cfg = load_config(None, OVR + ["experiment.max_new_tokens=12", "intervention.random_trials=4",
                                   "prompts=['Give me a hint!', 'Any hints available?', 'I need one more clue.']"])
    tok = SyntheticTokenizer(vocab_size=spec.vocab_size)
    key = lambda r: (r["word"], r["prompt_idx"], r["method"], r["budget"], r["trial"])   # noqa: E731
    res, stats = {}, {}
    for trie in (False, True):
        sae = JumpReLUSAE.random(spec.hidden, 512, seed=2, device="cpu")
        r = SweepRunner(cfg, m, tok, sae, batch=60 + carry, device="cpu", layer=2, use_graphs=False,
                        prefix_share=True, layer_resume=True, kv_pairs=8)
        r.trie_decode = trie
        r.carry_rows = carry
        pairs = r.build_pairs(["ship"], cfg.prompts[:3])
        r.run_baselines(pairs)
        out = []
        for i, j in enumerate(range(3)):
            sub = [pairs[j]]
            out += r.run_cells(sub, r.make_cells(sub), measure_nll=True, drain=(i == 2))
        res[trie] = {key(x): x for x in out}
        stats[trie] = dict(r.stats)
    assert stats[True]["diverged"] > 0
    if not carry:               # (the carry variant checks exactness; its few diverged rows barely share)
        assert 0 < stats[True]["decode_lo_groups"] < stats[True]["decode_row_steps"], stats[True]
        assert stats[True]["lens_gemm_rows"] < stats[True]["lens_rows"] == stats[False]["lens_gemm_rows"], stats
    else:
        assert stats[True]["carried"] > 0, stats[True]
    assert set(res[False]) == set(res[True])
    for k, a in res[False].items():
        b = res[True][k]
        assert a["response_ids"] == b["response_ids"], k
        assert a["topk_ids"] == b["topk_ids"], k
        assert abs(a["nll_edit"] - b["nll_edit"]) < 1e-5 and abs(a["nll_self"] - b["nll_self"]) < 1e-5
        for f in ("p_secret_mean", "p_secret_final", "p_secret_max"):
            assert abs(a[f] - b[f]) < 1e-6 + 1e-5 * abs(a[f])


def test_noop_spike_skip_is_exact():
    """Cells whose ablated latents are inactive at their pair's first spikes start their teacher-forced tail at
    their first effective spike (activity decided by the edit kernel itself); all-zero edits are exact no-ops,
    so the records equal the run that starts every tail at the pair's first spike, with fewer tail rows."""
    from dataclasses import replace

    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.models.gemma2 import Gemma2Model
    from taboo_brittleness_amd.models.spec import GEMMA2_TINY
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.models.weights import random_gemma2
    from taboo_brittleness_amd.pipelines.sweep import SweepRunner

    spec = replace(GEMMA2_TINY, vocab_size=1024, layers=4, hidden=256, ffn=512)
    m = Gemma2Model(random_gemma2(spec, dtype=torch.bfloat16, seed=7, norm_std=0.1, post_norm_gain=8.0), "cpu")
    cfg = load_config(None, OVR + ["experiment.max_new_tokens=12", "intervention.random_trials=4",
                                   "intervention.budgets=[1, 2, 4]",
                                   "prompts=['Give me a hint!', 'Any hints available?', 'I need one more clue.']"])
    tok = SyntheticTokenizer(vocab_size=spec.vocab_size)
    key = lambda r: (r["word"], r["prompt_idx"], r["method"], r["budget"], r["trial"])   # noqa: E731
    res, stats = {}, {}
    for skip in (False, True):
        sae = JumpReLUSAE.random(spec.hidden, 512, seed=2, device="cpu")
        r = SweepRunner(cfg, m, tok, sae, batch=60, device="cpu", layer=2, use_graphs=False,
                        prefix_share=True, layer_resume=True, kv_pairs=8)
        r.skip_noop_spikes = skip
        pairs = r.build_pairs(["ship"], cfg.prompts[:3])
        r.run_baselines(pairs)
        out = []
        for j in range(3):
            out += r.run_cells([pairs[j]], r.make_cells([pairs[j]]), measure_nll=True)
        res[skip] = {key(x): x for x in out}
        stats[skip] = dict(r.stats)
    assert stats[True]["tf_rows"] < stats[False]["tf_rows"], (stats[True]["tf_rows"], stats[False]["tf_rows"])
    assert set(res[False]) == set(res[True])
    for k, a in res[False].items():
        b = res[True][k]
        assert a["response_ids"] == b["response_ids"], k
        assert a["topk_ids"] == b["topk_ids"], k
        assert abs(a["nll_edit"] - b["nll_edit"]) < 1e-5 and abs(a["nll_self"] - b["nll_self"]) < 1e-5, k
        for f in ("p_secret_mean", "p_secret_final", "p_secret_max"):
            assert abs(a[f] - b[f]) < 1e-6 + 1e-5 * abs(a[f]), (k, f)


def test_noop_table_is_dropped_after_sae_change():
    """An activity table built under other SAE parameters (before ``calibrate()``) is never used to skip
    spikes: the plan falls back to the pair's first spike until the pair is re-scored."""
    from dataclasses import replace

    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.models.gemma2 import Gemma2Model
    from taboo_brittleness_amd.models.spec import GEMMA2_TINY
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.models.weights import random_gemma2
    from taboo_brittleness_amd.pipelines.sweep import SweepRunner

    spec = replace(GEMMA2_TINY, vocab_size=1024, layers=3, hidden=256, ffn=512)
    m = Gemma2Model(random_gemma2(spec, dtype=torch.bfloat16, seed=7, norm_std=0.1, post_norm_gain=8.0), "cpu")
    cfg = load_config(None, OVR + ["intervention.budgets=[1, 2]", "intervention.random_trials=4"])
    tok = SyntheticTokenizer(vocab_size=spec.vocab_size)
    sae = JumpReLUSAE.random(spec.hidden, 512, seed=2, device="cpu")
    r = SweepRunner(cfg, m, tok, sae, batch=40, device="cpu", layer=1, use_graphs=False, prefix_share=True,
                    layer_resume=True)
    pairs = r.build_pairs(["ship"], cfg.prompts[:2])
    r.run_baselines(pairs)
    cells = r.make_cells(pairs, ("sae_targeted", "sae_random"))
    f0 = r._plan_for(cells, pairs, {}, with_carry=False)["f"][: len(cells)]
    sae.calibrate(torch.cat([p.resid for p in pairs], 0))
    f1 = r._plan_for(cells, pairs, {}, with_carry=False)["f"][: len(cells)]
    assert (f1 == -1).all() and (f0 >= 0).any()
    r._score_pairs(pairs)
    f2 = r._plan_for(cells, pairs, {}, with_carry=False)["f"][: len(cells)]
    assert (f2 >= 0).any()


def test_ride_along_baselines_match_standalone():
    """Baselines generated riding along a batch's decode (``run_cells(ride_along=...)``: prefilled and decoded in
    the same batch as the diverged cells) equal the same pairs' standalone ``run_baselines``, and the riding
    batch's cell records equal a batch without passengers."""
    from dataclasses import replace

    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.models.gemma2 import Gemma2Model
    from taboo_brittleness_amd.models.spec import GEMMA2_TINY
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.models.weights import random_gemma2
    from taboo_brittleness_amd.pipelines.sweep import SweepRunner

    spec = replace(GEMMA2_TINY, vocab_size=1024, layers=3, hidden=256, ffn=512)
    m = Gemma2Model(random_gemma2(spec, dtype=torch.bfloat16, seed=7, norm_std=0.1, post_norm_gain=8.0), "cpu")
    cfg = load_config(None, OVR + ["experiment.max_new_tokens=12",
                                   "prompts=['Give me a hint!', 'Any hints available?', 'I need one more clue.']"])
    tok = SyntheticTokenizer(vocab_size=spec.vocab_size)
    key = lambda r: (r["word"], r["prompt_idx"], r["method"], r["budget"], r["trial"])   # noqa: E731
    methods = ("sae_targeted", "sae_random")
    out = {}
    for ride in (False, True):
        sae = JumpReLUSAE.random(spec.hidden, 512, seed=2, device="cpu")
        r = SweepRunner(cfg, m, tok, sae, batch=60, device="cpu", layer=1, use_graphs=False,
                        prefix_share=True, layer_resume=True, kv_pairs=8)
        pairs = r.build_pairs(["ship"], cfg.prompts[:3])
        r._ensure_gen(r._S_needed(pairs))           # one cache geometry for every pair (as the bench sizes it)
        r.run_baselines(pairs[:1] if ride else pairs)
        recs = r.run_cells(pairs[:1], r.make_cells(pairs[:1], methods), measure_nll=True,
                           ride_along=pairs[1:] if ride else ())
        out[ride] = ({key(x): x for x in recs}, pairs, r.stats["diverged"])
    (ra, pa, da), (rb, pb, db) = out[False], out[True]
    assert da > 0 and da == db                       # diverged cells decode next to the passengers
    assert set(ra) == set(rb)
    _same_records(ra, rb)
    for p, q in zip(pa[1:], pb[1:]):
        assert p.resp == q.resp and p.gen_toks == q.gen_toks and p.spikes_rel == q.spikes_rel
        assert np.allclose(p.tok_nll, q.tok_nll, atol=1e-5)
        assert torch.equal(p.resid, q.resid)
