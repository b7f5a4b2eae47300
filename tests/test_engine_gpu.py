"""Whole-engine checks on the MI355X: the HIP forward against the CPU reference path, hipGraph
decode against eager decode, the sweep (prefix sharing on/off) and the SAE encode."""
from dataclasses import replace

import pytest
import torch

from taboo_brittleness_amd.models.gemma2 import Gemma2Model
from taboo_brittleness_amd.models.spec import GEMMA2_TINY
from taboo_brittleness_amd.models.weights import random_gemma2
from taboo_brittleness_amd.runtime.generation import Generator

pytestmark = pytest.mark.gpu
SPEC = replace(GEMMA2_TINY, vocab_size=2048, layers=4, sliding_window=8)


@pytest.fixture
def tb_gemm():
    """In-tree GEMMs only (runtime/gemm_dispatch.py ``tb``): every GEMM accumulates each output over K in one
    fixed order whatever M or the tile, so a row's numbers do not depend on the batch it runs in."""
    from taboo_brittleness_amd.runtime import gemm_dispatch as GD

    old = GD.mode()
    GD.set_mode("tb")
    yield
    GD.set_mode(old)


FIELDS = ("response_ids", "nll_edit", "p_secret_mean", "topk_ids", "leak")


def _feq(x, y, rtol: float) -> bool:
    if isinstance(x, float) and isinstance(y, float):
        if x != x and y != y:
            return True
        return x == y or abs(x - y) <= rtol * max(abs(x), abs(y))
    return x == y


def _assert_records_equal(a: dict, b: dict, keys=None, fields=FIELDS, float_rtol: float = 0.0):
    """Equal result records: tokens, guesses and leak verdicts bit-equal (the reuse levels under test are exact
    given batch-invariant GEMMs); the float aggregates bit-equal too unless ``float_rtol`` (a path that sums the
    same per-token terms in another order, named at the call)."""
    keys = list(a) if keys is None else keys
    assert set(a) == set(b)
    bad = [(k, f) for k in keys for f in fields if f in a[k] and not _feq(a[k][f], b[k][f], float_rtol)]
    assert not bad, f"{len(bad)} field mismatches, first: {bad[:5]} " + \
        str([(a[k][f], b[k][f]) for k, f in bad[:3]])


def _models(gpu):
    w = random_gemma2(SPEC, dtype=torch.bfloat16, seed=5, norm_std=0.1)
    return Gemma2Model(w, "cpu"), Gemma2Model(w.to(device=gpu), gpu)


def test_forward_hip_matches_cpu_reference(gpu):
    mc, mg = _models(gpu)
    ids = torch.randint(0, SPEC.vocab_size, (3, 13), generator=torch.Generator().manual_seed(1)).int()
    pos = torch.arange(13, dtype=torch.int32).expand(3, 13).contiguous()
    pos[2, 10:] = -1
    caps = {}
    hk = {2: [lambda h, x, c: caps.__setitem__(c.model.device.type, h.clone())]}
    xc = mc.forward(ids, pos, mc.new_cache(3, 16), torch.arange(3, dtype=torch.int32), hk)
    xg = mg.forward(ids.to(gpu), pos.to(gpu), mg.new_cache(3, 16), torch.arange(3, dtype=torch.int32, device=gpu), hk)
    valid = (pos.view(-1) >= 0)
    lc = mc.logits(xc).float()[valid]
    lg = mg.logits(xg).float().cpu()[valid]
    assert (lc - lg).abs().max() < 0.05 * lc.abs().max() + 0.05
    assert (caps["cpu"].float()[valid] - caps["cuda"].float().cpu()[valid]).abs().max() < 0.1


def test_graph_decode_equals_eager(gpu):
    _, mg = _models(gpu)
    prompts = [[2, 5, 9, 11, 13], [2, 7, 8], [2, 3, 4, 5, 6, 7, 8]]
    eager = Generator(mg, 4, 32, use_graphs=False, stop_ids=(100_000,)).generate(prompts, 10)
    g = Generator(mg, 4, 32, use_graphs=True, stop_ids=(100_000,))
    a = g.generate(prompts, 10, graph_key="k")
    b = g.generate(prompts, 10, graph_key="k")          # replay path
    for i in range(3):
        assert eager.response_ids(i) == a.response_ids(i) == b.response_ids(i)


def test_sweep_gpu_prefix_share_equivalence(gpu, tb_gemm):
    from taboo_brittleness_amd.config import load_config
    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.pipelines.sweep import SweepRunner

    cfg = load_config(None, ["experiment.max_new_tokens=8", "intervention.budgets=[1, 4]",
                             "intervention.random_trials=2", "intervention.ranks=[1, 2]",
                             "intervention.proj_random_trials=1"])
    _, mg = _models(gpu)
    tok = SyntheticTokenizer(vocab_size=SPEC.vocab_size)
    out = {}
    for share in (False, True):
        sae = JumpReLUSAE.random(SPEC.hidden, 1024, seed=2, device=gpu)
        r = SweepRunner(cfg, mg, tok, sae, batch=24, device=gpu, layer=2, prefix_share=share)
        pairs = r.build_pairs(["ship"], cfg.prompts[:2])
        r.run_baselines(pairs)
        res = r.run_cells(pairs, r.make_cells(pairs))
        out[share] = dict(enumerate(res))
    # the prefix-shared cell's NLL is the baseline's per-token NLLs (fp64 cumulative sums) + its own tail's, the
    # unshared one the mean of one pass: same terms, other summation order (measured <= 1e-7 relative)
    _assert_records_equal(out[False], out[True], float_rtol=1e-6)


def test_generate_resume_bitwise(gpu, tb_gemm):
    """A chat turn prefilled as a suffix behind the previous turn's cached prompt K/V (Generator.generate
    ``keep``, the token-forcing warm-up turns) gives BIT-identical tokens and NLLs to prefilling the whole new prompt
    (tb GEMMs: row results independent of the batch; prefill attention: a query row's output independent of the
    rows after it)."""
    _, mg = _models(gpu)
    g = torch.Generator().manual_seed(5)
    p1 = [[2] + torch.randint(3, SPEC.vocab_size, (n,), generator=g).tolist() for n in (21, 34, 9, 27, 40)]
    S = 128
    a = Generator(mg, len(p1), S, use_graphs=True, stop_ids=(100_000,))
    o1 = a.generate(p1, 8, graph_key="t")
    p2 = [p + o1.response_ids(i)[:-1] + torch.randint(3, SPEC.vocab_size, (5 + i,), generator=g).tolist()
          for i, p in enumerate(p1)]
    p2[2] = p2[2][:4] + [7] + p2[2][5:]                  # a row whose prompt changes inside the old prefix
    from taboo_brittleness_amd.pipelines.token_forcing import _lcp

    keep = [_lcp(x, y) for x, y in zip(p2, p1)]
    assert keep[2] == 4 and keep[0] == len(p1[0])
    r = a.generate(p2, 8, graph_key="t", keep=keep)
    f = Generator(mg, len(p1), S, use_graphs=True, stop_ids=(100_000,)).generate(p2, 8, graph_key="t")
    for i in range(len(p2)):
        assert r.response_ids(i) == f.response_ids(i)
    assert torch.equal(r.tok_nll[:, :8], f.tok_nll[:, :8])


def test_generate_shared_bitwise(gpu, tb_gemm):
    """Generator.generate_shared on the GPU (each group's common prefix prefilled once, its K/V copied for the
    members' suffix prefill, the decode reading the prefix from the group's first slot through the shared-prefix
    attention) gives BIT-identical tokens and NLLs to generate() prefilling every prompt whole."""
    _, mg = _models(gpu)
    g = torch.Generator().manual_seed(6)
    hist = [[2] + torch.randint(3, SPEC.vocab_size, (n,), generator=g).tolist() for n in (40, 25)]
    prompts, groups = [], []
    for gi, h in enumerate(hist):
        for k in range(5):
            prompts.append(h + torch.randint(3, SPEC.vocab_size, (3 + k,), generator=g).tolist())
            groups.append(gi)
    prompts.append([2] + torch.randint(3, SPEC.vocab_size, (12,), generator=g).tolist())
    groups.append(9)
    S = 96
    a = Generator(mg, len(prompts), S, use_graphs=True, stop_ids=(100_000,)).generate(prompts, 10, graph_key="s")
    gb = Generator(mg, len(prompts), S, use_graphs=True, stop_ids=(100_000,))
    for _ in range(2):                                   # capture, then replay
        b = gb.generate_shared(prompts, groups, 10, graph_key="s")
        for i in range(len(prompts)):
            assert a.response_ids(i) == b.response_ids(i)
        assert torch.equal(a.tok_nll[:, :10], b.tok_nll[:, :10])
    assert gb.kv_prefix is not None and gb.kv_prefix.k is gb.cache.k
    c = gb.generate(prompts, 10, graph_key="s")           # plain generate after it: prefix lengths reset
    assert [c.response_ids(i) for i in range(len(prompts))] == [a.response_ids(i) for i in range(len(prompts))]


def test_sae_encode_matches_fp32(gpu):
    from taboo_brittleness_amd.interp.sae import JumpReLUSAE

    sae_c = JumpReLUSAE.random(512, 2048, seed=3, device="cpu")
    sae_g = JumpReLUSAE.random(512, 2048, seed=3, device=gpu)
    x = torch.randn(40, 512)
    sae_c.calibrate(x, target_l0=30)
    sae_g.threshold = sae_c.threshold.to(gpu)
    ac = sae_c.encode(x)
    ag = sae_g.encode(x.to(gpu)).cpu()
    pre = sae_c.pre_acts(x)
    near = (pre - sae_c.threshold).abs() < 2e-2
    assert ((ac - ag).abs()[~near] < 2e-2).all()
    # calibration puts one sample per latent exactly on its threshold (strict >), so compare L0 on
    # fresh data where ties have measure zero
    x2 = torch.randn(40, 512)
    assert abs(sae_g.l0(x2.to(gpu)) - sae_c.l0(x2)) < 1.0


def test_sweep_gpu_layer_resume_equivalence(gpu, tb_gemm):
    """Layer resume (HIP varlen attention, packed tail forward, partial lens) vs the full
    prefix-shared decode on the GPU: same responses / guesses up to bf16 near-ties."""
    from taboo_brittleness_amd.config import load_config
    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.pipelines.sweep import SweepRunner

    cfg = load_config(None, ["experiment.max_new_tokens=10", "intervention.budgets=[1, 4, 16]",
                             "intervention.random_trials=3", "intervention.ranks=[1, 2]",
                             "intervention.proj_random_trials=1"])
    _, mg = _models(gpu)
    tok = SyntheticTokenizer(vocab_size=SPEC.vocab_size)
    out, stats = {}, {}
    for lr in (False, True):
        sae = JumpReLUSAE.random(SPEC.hidden, 1024, seed=2, device=gpu)
        r = SweepRunner(cfg, mg, tok, sae, batch=96, device=gpu, layer=2, prefix_share=True, layer_resume=lr)
        pairs = r.build_pairs(["ship"], cfg.prompts[:3])
        r.run_baselines(pairs)
        out[lr] = r.run_cells(pairs, r.make_cells(pairs))
        stats[lr] = dict(r.stats)
    assert stats[True]["cells"] == len(out[True])
    # layer resume reuses the baseline's running lens sums / cumulative NLLs for the unedited positions: the same
    # terms summed in another order (measured <= 1e-7 relative); tokens and guesses bit-equal
    _assert_records_equal(dict(enumerate(out[False])), dict(enumerate(out[True])), float_rtol=1e-6)


def test_bitwise_determinism(gpu):
    """Race screen: every hand-written kernel on the forward / readout path is
    deterministic — two runs of the same inputs are bitwise identical (no atomics-order or LDS race
    nondeterminism), including the varlen tail pass and the vocab reductions."""
    from taboo_brittleness_amd import ops
    from taboo_brittleness_amd.models.gemma2 import packed_blocks

    _, mg = _models(gpu)
    ids = torch.randint(0, SPEC.vocab_size, (5, 11), generator=torch.Generator().manual_seed(4)).int().to(gpu)
    pos = torch.arange(11, dtype=torch.int32, device=gpu).expand(5, 11).contiguous()
    outs = []
    for _ in range(2):
        x = mg.forward(ids, pos, mg.new_cache(5, 16), torch.arange(5, dtype=torch.int32, device=gpu))
        lg = mg.logits(x)
        nxt, ns, nt = ops.decode_head(lg, 30.0, ids.view(-1)[: lg.shape[0]].contiguous())
        lse = ops.row_lse(lg)
        acc = ops.lens_colsum(lg, lse, None, torch.full((lg.shape[0], 2), -1, dtype=torch.int32, device=gpu), 5, 11)
        outs.append([t.clone() for t in (x, lg, nxt, ns, nt, acc)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    # packed tail path
    cache = mg.new_cache(3, 16)
    mg.forward(ids[:3], pos[:3], cache, torch.arange(3, dtype=torch.int32, device=gpu))
    seqs = [(0, 4, 0), (4, 6, 1), (10, 3, 2)]
    blk = packed_blocks(seqs, 8).to(gpu)
    pp = torch.tensor(list(range(5, 9)) + list(range(3, 9)) + list(range(8, 11)), dtype=torch.int32, device=gpu)
    sr = torch.tensor([0] * 4 + [1] * 6 + [2] * 3, dtype=torch.int32, device=gpu)
    h = torch.randn(13, SPEC.hidden, device=gpu).to(torch.bfloat16)
    r = [mg.forward_packed(None, pp, sr, blk, cache, resume_after=1, h_in=h).clone() for _ in range(2)]
    assert torch.equal(r[0], r[1])


def test_sweep_gpu_decode_tail_carry(gpu, tb_gemm):
    """Decode-tail carry-over on the GPU (graph-replayed decode, HIP shared-prefix attention) gives the
    records of a plain run (same responses; readouts up to bf16 near-ties)."""
    from taboo_brittleness_amd.config import load_config
    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.pipelines.sweep import SweepRunner

    cfg = load_config(None, ["experiment.max_new_tokens=12", "intervention.budgets=[1, 4, 16]",
                             "intervention.random_trials=3", "intervention.ranks=[1, 2]",
                             "intervention.proj_random_trials=1"])
    mg = Gemma2Model(random_gemma2(SPEC, dtype=torch.bfloat16, seed=5, norm_std=0.1, post_norm_gain=8.0,
                                   device=gpu), gpu)
    tok = SyntheticTokenizer(vocab_size=SPEC.vocab_size)
    key = lambda r: (r["word"], r["prompt_idx"], r["method"], r["budget"], r["trial"])   # noqa: E731
    out, carried = {}, {}
    for carry in (0, 16):
        sae = JumpReLUSAE.random(SPEC.hidden, 1024, seed=2, device=gpu)
        r = SweepRunner(cfg, mg, tok, sae, batch=40 + carry, device=gpu, layer=2, prefix_share=True,
                        layer_resume=True, kv_pairs=8)
        r.carry_rows = carry
        pairs = r.build_pairs(["ship"], cfg.prompts[:3])
        r.run_baselines(pairs)
        res = []
        for i in range(3):
            res += r.run_cells([pairs[i]], r.make_cells([pairs[i]]), drain=(i == 2))
        out[carry] = {key(x): x for x in res}
        carried[carry] = r.stats["carried"]
    assert carried[16] > 0
    _assert_records_equal(out[0], out[16])


def test_sweep_gpu_trie_decode(gpu, tb_gemm):
    """Prefix-trie decode on the GPU (lo/hi hipGraphs per row bucket, HIP K/V fan-out, on-device regrouping)
    reproduces the per-row decode's records (responses; readouts up to bf16 near-ties) and shares rows."""
    from taboo_brittleness_amd.config import load_config
    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.pipelines.sweep import SweepRunner

    cfg = load_config(None, ["experiment.max_new_tokens=12", "intervention.budgets=[1, 4, 16]",
                             "intervention.random_trials=6", "intervention.ranks=[1, 2]",
                             "intervention.proj_random_trials=1"])
    mg = Gemma2Model(random_gemma2(SPEC, dtype=torch.bfloat16, seed=5, norm_std=0.1, post_norm_gain=8.0,
                                   device=gpu), gpu)
    tok = SyntheticTokenizer(vocab_size=SPEC.vocab_size)
    key = lambda r: (r["word"], r["prompt_idx"], r["method"], r["budget"], r["trial"])   # noqa: E731
    out, stats = {}, {}
    for trie in (False, True):
        sae = JumpReLUSAE.random(SPEC.hidden, 1024, seed=2, device=gpu)
        r = SweepRunner(cfg, mg, tok, sae, batch=96, device=gpu, layer=2, prefix_share=True, layer_resume=True,
                        kv_pairs=8)
        r.trie_decode = trie
        pairs = r.build_pairs(["ship"], cfg.prompts[:4])
        r.run_baselines(pairs)
        res = r.run_cells(pairs, r.make_cells(pairs))
        r.precapture_graphs()
        res = r.run_cells(pairs, r.make_cells(pairs))        # second pass: replayed lo/hi graphs
        out[trie] = {key(x): x for x in res}
        stats[trie] = dict(r.stats)
    assert 0 < stats[True]["decode_lo_groups"] < stats[True]["decode_row_steps"], stats[True]
    _assert_records_equal(out[False], out[True])


def test_sweep_gpu_noop_spike_skip(gpu, tb_gemm):
    """Tails starting at each cell's first effective spike (activity from the HIP edit kernel's own coefficients;
    all-zero edits are no-ops in the kernel) reproduce the records of tails starting at the pair's first spike
    on the GPU, with fewer tail rows."""
    from taboo_brittleness_amd.config import load_config
    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.pipelines.sweep import SweepRunner

    cfg = load_config(None, ["experiment.max_new_tokens=12", "intervention.budgets=[1, 2, 4]",
                             "intervention.random_trials=6"])
    mg = Gemma2Model(random_gemma2(SPEC, dtype=torch.bfloat16, seed=5, norm_std=0.1, post_norm_gain=8.0,
                                   device=gpu), gpu)
    tok = SyntheticTokenizer(vocab_size=SPEC.vocab_size)
    key = lambda r: (r["word"], r["prompt_idx"], r["method"], r["budget"], r["trial"])   # noqa: E731
    out, stats = {}, {}
    for skip in (False, True):
        sae = JumpReLUSAE.random(SPEC.hidden, 1024, seed=2, device=gpu)
        r = SweepRunner(cfg, mg, tok, sae, batch=96, device=gpu, layer=2, prefix_share=True, layer_resume=True,
                        kv_pairs=8)
        r.skip_noop_spikes = skip
        pairs = r.build_pairs(["ship"], cfg.prompts[:4])
        r.run_baselines(pairs)
        res = r.run_cells(pairs, r.make_cells(pairs, ("sae_targeted", "sae_random")))
        out[skip] = {key(x): x for x in res}
        stats[skip] = dict(r.stats)
    assert stats[True]["tf_rows"] < stats[False]["tf_rows"], (stats[True]["tf_rows"], stats[False]["tf_rows"])
    _assert_records_equal(out[False], out[True])


def test_sweep_gpu_cross_step_pipeline(gpu, tb_gemm):
    """The bench's cross-step pipeline on the GPU (staged plan upload + teacher-forced tail queued behind the
    previous batch's lens, pinned async D2H, records on the host thread, graph-replayed decode), with and
    without decode-tail carry-over: the same records as running the batches one after the other."""
    from taboo_brittleness_amd.config import load_config
    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.pipelines.sweep import NextBatch, SweepRunner

    cfg = load_config(None, ["experiment.max_new_tokens=12", "intervention.budgets=[1, 4, 16]",
                             "intervention.random_trials=3"])
    mg = Gemma2Model(random_gemma2(SPEC, dtype=torch.bfloat16, seed=5, norm_std=0.1, post_norm_gain=8.0,
                                   device=gpu), gpu)
    tok = SyntheticTokenizer(vocab_size=SPEC.vocab_size)
    key = lambda r: (r["word"], r["prompt_idx"], r["method"], r["budget"], r["trial"])   # noqa: E731
    methods = ("sae_targeted", "sae_random")
    out, stats = {}, {}
    for pipe, carry in ((False, 0), (True, 0), (True, 16)):
        sae = JumpReLUSAE.random(SPEC.hidden, 1024, seed=2, device=gpu)
        r = SweepRunner(cfg, mg, tok, sae, batch=40 + carry, device=gpu, layer=2, prefix_share=True,
                        layer_resume=True, kv_pairs=8)
        r.carry_rows = carry
        pairs = r.build_pairs(["ship"], cfg.prompts[:3])
        r.run_baselines(pairs)
        subs = [[p] for p in pairs]
        cells = r.make_cells(subs[0], methods)
        res = []
        for i, sub in enumerate(subs):
            nb = None
            if pipe and i + 1 < len(subs):
                nb = NextBatch(subs[i + 1], methods)
                r.stage_next(nb)
            res += r.run_cells_async(sub, cells, drain=(i == len(subs) - 1)).result()
            if i + 1 < len(subs):
                cells = nb.cells if nb is not None and nb.cells is not None else r.make_cells(subs[i + 1], methods)
        out[(pipe, carry)] = {key(x): x for x in res}
        stats[(pipe, carry)] = dict(r.stats)
    assert stats[(True, 0)]["staged"] == 2 and stats[(True, 16)]["staged"] == 2
    for cfg_ in ((True, 0), (True, 16)):
        _assert_records_equal(out[(False, 0)], out[cfg_])


def test_sweep_gpu_lazy_lens_sums(gpu, tb_gemm, monkeypatch):
    """lazy running lens sums (rebuilt from the kept hooked-layer residuals when a pair's cells run,
    SweepRunner.lazy_cum, default) vs sums kept from the baseline readout: the same records on the GPU (batch-
    invariant GEMMs make the rebuilt chunking irrelevant to the logits)."""
    from taboo_brittleness_amd.config import load_config
    from taboo_brittleness_amd.interp.sae import JumpReLUSAE
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.pipelines.sweep import SweepRunner

    cfg = load_config(None, ["experiment.max_new_tokens=10", "intervention.budgets=[1, 4]",
                             "intervention.random_trials=3"])
    mg = Gemma2Model(random_gemma2(SPEC, dtype=torch.bfloat16, seed=5, norm_std=0.1, post_norm_gain=8.0,
                                   device=gpu), gpu)
    tok = SyntheticTokenizer(vocab_size=SPEC.vocab_size)
    key = lambda r: (r["word"], r["prompt_idx"], r["method"], r["budget"], r["trial"])   # noqa: E731
    out = {}
    for lazy in ("0", "1"):
        sae = JumpReLUSAE.random(SPEC.hidden, 1024, seed=2, device=gpu)
        r = SweepRunner(cfg, mg, tok, sae, batch=64, device=gpu, layer=2, prefix_share=True, layer_resume=True,
                        kv_pairs=8)
        r.lazy_cum = lazy == "1"
        pairs = r.build_pairs(["ship"], cfg.prompts[:3])
        r.run_baselines(pairs)
        out[lazy] = {key(x): x for x in r.run_cells(pairs, r.make_cells(pairs, ("sae_targeted", "sae_random")))}
    _assert_records_equal(out["0"], out["1"])


def test_batched_trace_gpu_matches_per_sequence(gpu, tb_gemm):
    """The batched all-layer lens trace (config 2) on the GPU kernels equals the per-(sequence, layer) readout
    it replaced, bit for bit under batch-invariant GEMMs (chunks straddle layers and sequences)."""
    import numpy as np
    import sys as _sys

    _sys.path.insert(0, __import__("os").path.dirname(__file__))
    from taboo_brittleness_amd.models.tokenizer import SyntheticTokenizer
    from taboo_brittleness_amd.pipelines.baselines import trace_sequences
    from test_trace_cpu import _per_sequence

    _, mg = _models(gpu)
    tok = SyntheticTokenizer(vocab_size=SPEC.vocab_size)
    g = torch.Generator().manual_seed(0)
    seqs = [torch.randint(3, SPEC.vocab_size, (n,), generator=g).tolist() for n in (9, 14, 6)]
    starts, track = [4, 7, 2], [[5, 9, 11], [7, 8], [5, 9, 11]]
    got = trace_sequences(mg, tok, seqs, 1, track, starts, chunk_rows=7)
    want = _per_sequence(mg, tok, seqs, 1, track, starts)
    for r, (p, am, rs) in zip(got, want):
        np.testing.assert_array_equal(r["p_track"], p)
        np.testing.assert_array_equal(r["argmax"], am)
        np.testing.assert_allclose(r["resp_sum"], rs, rtol=1e-5, atol=1e-7)


def test_debug_checks_subprocess(gpu):
    """SURVEY §5 race/bounds screening: with TB_DEBUG_CHECKS=1 (host-side index-range checks before the
    launches that gather by index; read once per process, hence a subprocess) a GPU sweep passes them and an
    out-of-range latent id is refused before the edit kernel could read past the SAE tables."""
    import json
    import os
    import subprocess
    import sys as _sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, TB_DEBUG_CHECKS="1")
    out = subprocess.run([_sys.executable, os.path.join(root, "tools", "debug_checks_probe.py")], env=env,
                         capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr[-3000:]
    res = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert res["cells"] > 0 and res["rejected_out_of_range"], res
