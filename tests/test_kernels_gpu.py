"""Numerics of every gfx950 HIP kernel against its PyTorch fp32 reference (ops/reference.py)."""
import math
import os

import pytest
import torch

from taboo_brittleness_amd import ops
from taboo_brittleness_amd.ops import reference as ref

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _close(a, b, atol, rtol=0.0):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol).sum().item()
    assert bad == 0, f"{bad} / {a.numel()} elements off; max err {err.max().item():.4g}"


def test_rmsnorm_family(gpu):
    torch.manual_seed(0)
    for D in (512, 3584, 2304):
        x = torch.randn(37, D, dtype=BF) * 3
        w = torch.randn(D, dtype=BF) * 0.1
        _close(ops.rmsnorm(x.to(gpu), w.to(gpu), 1e-6), ref.rmsnorm(x, w, 1e-6), atol=2e-2, rtol=1e-2)
        h = torch.randn(37, D, dtype=BF)
        o = torch.randn(37, D, dtype=BF) * 5
        wn = torch.randn(D, dtype=BF) * 0.1
        hg = h.to(gpu)
        xg = ops.add_rmsnorm2(hg, o.to(gpu), w.to(gpu), wn.to(gpu), 1e-6)
        hr = h.clone()
        xr = ref.add_rmsnorm2(hr, o, w, wn, 1e-6)
        _close(hg, hr, atol=3e-2, rtol=1e-2)
        _close(xg, xr, atol=3e-2, rtol=1e-2)
    E = torch.randn(1000, 512, dtype=BF) * 0.02
    ids = torch.randint(0, 1000, (50,), dtype=torch.int32)
    w = torch.randn(512, dtype=BF) * 0.1
    hg, xg = ops.embed_rmsnorm(ids.to(gpu), E.to(gpu), w.to(gpu), math.sqrt(512), 1e-6)
    hr, xr = ref.embed_rmsnorm(ids, E, w, math.sqrt(512), 1e-6)
    _close(hg, hr, atol=1e-6)
    _close(xg, xr, atol=2e-2, rtol=1e-2)


def test_rope_and_cache(gpu):
    torch.manual_seed(1)
    Hq, Hkv, HD, S, slots = 4, 2, 256, 24, 3
    M = 10
    qkv = torch.randn(M, (Hq + 2 * Hkv) * HD, dtype=BF)
    pos = torch.tensor([0, 1, 2, 3, -1, 5, 6, 23, 9, 10], dtype=torch.int32)
    slot_rows = torch.tensor([0, 0, 0, 0, 0, 1, 1, 1, 2, 2], dtype=torch.int32)
    cos_t, sin_t = ref.rope_tables(HD, 64, 10000.0)
    kc = torch.zeros(slots, Hkv, S, HD, dtype=BF)
    vc = torch.zeros_like(kc)
    kcg, vcg = kc.to(gpu), vc.to(gpu)
    qg = ops.rope_qkv_cache(qkv.to(gpu), pos.to(gpu), slot_rows.to(gpu), cos_t.to(gpu), sin_t.to(gpu), kcg, vcg, Hq,
                            Hkv, HD)
    qr = ref.rope_qkv_cache(qkv, pos, slot_rows, cos_t, sin_t, kc, vc, Hq, Hkv, HD)
    _close(qg, qr, atol=1e-6)
    _close(kcg, kc, atol=1e-6)
    _close(vcg, vc, atol=1e-6)


def test_lens_readouts_rowmap(gpu):
    """gather_probs / packed lens_colsum reading deduplicated logits rows through a row map equal the same
    kernels over the materialised rows."""
    torch.manual_seed(4)
    V, Rp, R = 3000, 5, 12
    lg = (torch.randn(Rp, V) * 3).to(BF).to(gpu)
    lse = torch.logsumexp(lg.float(), -1)
    rm = torch.tensor([0, 1, 1, 2, 0, 3, 4, 4, 4, 2, 1, 0], dtype=torch.int32, device=gpu)
    ids = torch.randint(-1, V, (R, 3), dtype=torch.int32, device=gpu)
    ex = torch.randint(-1, V, (R, 2), dtype=torch.int32, device=gpu)
    offs = torch.tensor([0, 3, 7, 12], dtype=torch.int32, device=gpu)
    full, lf = lg.index_select(0, rm.long()), lse.index_select(0, rm.long())
    a = ops.gather_probs(lg, lse, ids, rowmap=rm)
    b = ops.gather_probs(full, lf, ids)
    assert torch.equal(a, b)
    sa = ops.lens_colsum(lg, lse, None, ex, 3, 0, offs=offs, rowmap=rm)
    sb = ops.lens_colsum(full, lf, None, ex, 3, 0, offs=offs)
    assert torch.equal(sa, sb)


def test_kv_fanout(gpu):
    """Prefix-trie KV fan-out: members get their representative's K/V of the first layers at their own
    position; skipped rows (src < 0, src == r, positions outside the cache) and deeper layers untouched."""
    torch.manual_seed(3)
    L, slots, Hkv, S, HD = 5, 7, 2, 16, 256
    kc = torch.randn(L, slots, Hkv, S, HD, dtype=BF)
    vc = torch.randn_like(kc)
    src = torch.tensor([-1, 0, 0, 3, 3, -1, 3], dtype=torch.int32)     # sources are representatives (src -1 / self)
    slot = torch.tensor([1, 2, 3, 4, 5, 6, 0], dtype=torch.int32)
    pos = torch.tensor([9, 9, 9, 4, 4, 16, 3], dtype=torch.int32)
    kg, vg = kc.to(gpu), vc.to(gpu)
    ops.kv_fanout(kg, vg, src.to(gpu), slot.to(gpu), pos.to(gpu), 3)
    ref.kv_fanout(kc, vc, src, slot, pos, 3)
    assert torch.equal(kg.cpu(), kc) and torch.equal(vg.cpu(), vc)
    assert torch.equal(kc[:3, 2, :, 9], kc[:3, 1, :, 9]) and torch.equal(vc[:3, 5, :, 4], vc[:3, 4, :, 4])


@pytest.mark.parametrize("nb", [1, 37, 300])
def test_decode_step_bookkeeping(gpu, nb):
    """csrc/decode_step.hip vs the PyTorch step it replaces (ops/reference.py): the teacher-target gather, the
    post-head token / NLL / stop / advance update (done rows emit pad, the column clamps at W - 1), and the
    prefix-trie lo-row gather (rows >= U parked at S); rows >= nb untouched."""
    g = torch.Generator().manual_seed(nb)
    B, W, S, pad = 320, 9, 40, 0
    st = {"step_idx": torch.randint(0, W + 3, (B, 1), generator=g).long(),
          "tf_tgt": torch.randint(-1, 50, (B, W), generator=g).int(),
          "tf_step": torch.full((B,), 7, dtype=torch.int32),
          "nxt": torch.randint(0, 6, (B,), generator=g).int(),
          "nll": torch.rand(B, generator=g), "tf_nll": torch.rand(B, generator=g),
          "done": torch.rand(B, generator=g) < 0.3,
          "out_tok": torch.randint(0, 9, (B, W), generator=g).int(),
          "out_nll": torch.rand(B, W, generator=g), "out_tf_nll": torch.rand(B, W, generator=g),
          "stop": torch.tensor([1, 4], dtype=torch.int32),
          "tok": torch.randint(0, 50, (B, 1), generator=g).int(), "pos": torch.randint(0, S, (B, 1), generator=g).int(),
          "rep": torch.randint(0, B, (B,), generator=g).long(), "U": torch.tensor(nb // 2, dtype=torch.int64),
          "slot": torch.randperm(B, generator=g).int(), "kps": torch.randint(0, 9, (B,), generator=g).int(),
          "kpl": torch.randint(0, S, (B,), generator=g).int()}
    for k in ("s_tok", "s_pos"):
        st[k] = torch.full((B, 1), -5, dtype=torch.int32)
    for k in ("s_slot", "l_slot", "l_len"):
        st[k] = torch.full((B,), -5, dtype=torch.int32)
    cpu = {k: v.clone() for k, v in st.items()}
    dev = {k: v.to(gpu) for k, v in st.items()}
    for o, mod in ((cpu, ref), (dev, ops)):
        mod.decode_pre(o["step_idx"], o["tf_tgt"], o["tf_step"], nb)
        mod.decode_post(o["nxt"], o["nll"], o["tf_nll"], o["done"], o["step_idx"], o["out_tok"], o["out_nll"],
                        o["out_tf_nll"], o["stop"], o["tok"], o["pos"], nb, pad)
        mod.share_lo_gather(o["rep"], o["U"], o["tok"], o["pos"], o["slot"], o["s_tok"], o["s_pos"], o["s_slot"],
                            o["kps"], o["kpl"], o["l_slot"], o["l_len"], nb, S)
    for k in st:
        assert torch.equal(dev[k].cpu(), cpu[k]), k
    assert bool(cpu["done"][:nb].any()) and not torch.equal(cpu["tok"], st["tok"])


@pytest.mark.parametrize("nb,act,first", [(1, 1, True), (700, 650, False), (6600, 6000, False), (8192, 8192, True)])
def test_share_group_kernel(gpu, nb, act, first):
    """Prefix-trie regrouping kernel vs the PyTorch unique / scatter-reduce it replaces: the same partition of the
    rows (by (group, token); rows >= act one parked group), each group's first row as representative, fan-out
    sources, group count; dense ids ordered by first row."""
    g = torch.Generator().manual_seed(nb)
    B, V = 8200, 256000
    gid = torch.randint(0, 40, (B,), generator=g).long()
    tok = torch.randint(0, 3, (B, 1), generator=g).int()
    key = gid[:nb].clone() if first else gid[:nb] * V + tok[:nb, 0].long()
    key[act:] = -1
    uniq, inv = torch.unique(key, sorted=True, return_inverse=True)
    ar = torch.arange(nb)
    rep_t = torch.full((uniq.numel(),), nb, dtype=torch.int64).scatter_reduce_(0, inv, ar, reduce="amin")
    d = {k: v.to(gpu) for k, v in {"gid": gid, "tok": tok}.items()}
    rep, grp = torch.full((B,), -7, dtype=torch.int64, device=gpu), torch.full((B,), -7, dtype=torch.int64, device=gpu)
    src, U = torch.full((B,), -7, dtype=torch.int32, device=gpu), torch.zeros((), dtype=torch.int64, device=gpu)
    assert ops.share_group(d["gid"], d["tok"], rep, grp, src, U, nb, act, first, V)
    Uk = int(U.item())
    assert Uk == uniq.numel()
    rep_c, grp_c, src_c = rep.cpu()[:Uk], grp.cpu()[:nb], src.cpu()[:nb]
    assert torch.equal(rep_c, torch.sort(rep_t).values)                  # first rows, in row order
    assert torch.equal(rep_c[grp_c], rep_t[inv])                          # same partition, same representatives
    assert torch.equal(d["gid"].cpu()[:nb], grp_c) and torch.equal(d["gid"].cpu()[nb:], gid[nb:])
    want_src = torch.where((rep_t[inv] == ar) | (ar >= act), -1, rep_t[inv]).int()
    assert torch.equal(src_c, want_src)


@pytest.mark.parametrize("B,T", [(5, 7), (300, 1)])
def test_capture_rows_and_row_gather(gpu, B, T):
    """Residual capture (store[slot[b], pos] <- h rows; invalid positions into the slot's scratch row) and the bf16
    row gather, vs index_copy / index_select."""
    g = torch.Generator().manual_seed(B * T)
    slots, S1, D = B + 3, 12, 3584
    store = torch.randn(slots, S1, D, generator=g).to(BF)
    h = torch.randn(B * T, D, generator=g).to(BF)
    pos = torch.stack([torch.randperm(S1 + 2, generator=g)[:T] - 2 for _ in range(B)]).int()   # unique per row
    slot = torch.randperm(slots, generator=g)[:B].int()
    ref_store = store.clone()
    ref.capture_rows(ref_store, h, pos, slot, B, T)
    sg = store.to(gpu)
    ops.capture_rows(sg, h.to(gpu), pos.to(gpu), slot.to(gpu), B, T)
    keep = torch.ones(slots, S1, dtype=torch.bool)
    keep[:, S1 - 1] = False                      # scratch rows: last writer undefined among duplicates
    assert torch.equal(sg.cpu()[keep], ref_store[keep])
    for dt in (torch.int64, torch.int32):
        idx = torch.randint(0, B * T, (B + 4,), generator=g).to(dt)
        out = torch.empty(B + 9, D, dtype=BF, device=gpu)
        ops.row_gather(h.to(gpu), idx.to(gpu), out)
        assert torch.equal(out[: B + 4].cpu(), h.index_select(0, idx.long()))


@pytest.mark.parametrize("G,HD", [(2, 256), (1, 256), (2, 128)])
def test_attention_prefill_decode(gpu, G, HD):
    torch.manual_seed(2)
    Hkv = 2
    Hq = Hkv * G
    B, S = 3, 80
    kc = torch.randn(B + 1, Hkv, S, HD, dtype=BF)
    vc = torch.randn(B + 1, Hkv, S, HD, dtype=BF)
    slot = torch.tensor([2, 0, 3], dtype=torch.int32)
    for T, window in ((37, 0), (37, 16), (1, 0), (5, 0)):
        q = torch.randn(B * T, Hq, HD, dtype=BF) * 2
        base = torch.tensor([0, 30, 70 - T], dtype=torch.int32)
        pos = (base[:, None] + torch.arange(T, dtype=torch.int32)[None, :]).contiguous()
        pos[0, -2:] = -1     # padding rows
        og = ops.attention(q.to(gpu), kc.to(gpu), vc.to(gpu), pos.reshape(-1).to(gpu), slot.to(gpu), B, T,
                           HD ** -0.5, 50.0, window)
        orf = ref.attention(q, kc, vc, pos.reshape(-1), slot, B, T, HD ** -0.5, 50.0, window)
        _close(og, orf, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("G,HD", [(2, 256), (1, 128)])
def test_attention_decode_shared_prefix(gpu, G, HD):
    """Decode rows reading keys [0, plen) from a shared prefix cache slot == the reference with those
    keys substituted (plen 0 = own slot only; plen beyond pos = prefix only)."""
    torch.manual_seed(7)
    Hkv, S, B = 2, 80, 4
    Hq = Hkv * G
    kc = torch.randn(B + 1, Hkv, S, HD, dtype=BF)
    vc = torch.randn(B + 1, Hkv, S, HD, dtype=BF)
    pk = torch.randn(3, Hkv, S, HD, dtype=BF)
    pv = torch.randn(3, Hkv, S, HD, dtype=BF)
    slot = torch.tensor([2, 0, 4, 1], dtype=torch.int32)
    pos = torch.tensor([40, 63, 7, 79], dtype=torch.int32)
    ps = torch.tensor([1, 0, 2, 1], dtype=torch.int32)
    pl = torch.tensor([17, 0, 30, 64], dtype=torch.int32)
    q = torch.randn(B, Hq, HD, dtype=BF) * 2
    for window in (0, 16):
        og = ops.attention(q.to(gpu), kc.to(gpu), vc.to(gpu), pos.to(gpu), slot.to(gpu), B, 1, HD ** -0.5, 50.0,
                           window, prefix=(pk.to(gpu), pv.to(gpu), ps.to(gpu), pl.to(gpu)))
        orf = ref.attention(q, kc, vc, pos, slot, B, 1, HD ** -0.5, 50.0, window, prefix=(pk, pv, ps, pl))
        _close(og, orf, atol=2e-2, rtol=2e-2)
        if window == 0:      # (row 0's sliding window does not reach its 17 prefix keys)
            plain = ref.attention(q, kc, vc, pos, slot, B, 1, HD ** -0.5, 50.0, window)
            assert not torch.allclose(plain[0].float(), orf[0].float())     # the prefix changes row 0


@pytest.mark.parametrize("G,HD", [(2, 256), (1, 128), (4, 256)])
def test_attention_varlen_packed(gpu, G, HD):
    """Ragged block-table attention == the per-row reference (each row its own slot/position)."""
    from taboo_brittleness_amd.models.gemma2 import packed_blocks

    torch.manual_seed(12)
    Hkv, S = 2, 96
    Hq = Hkv * G
    kc = torch.randn(5, Hkv, S, HD, dtype=BF)
    vc = torch.randn(5, Hkv, S, HD, dtype=BF)
    seqs_spec = [(3, 10, 23), (0, 40, 1), (4, 5, 13), (1, 70, 26)]    # (slot, first pos, n rows)
    pos, slot_rows, seqs = [], [], []
    for sl, p0, n in seqs_spec:
        seqs.append((len(pos), n, sl))
        pos += list(range(p0, p0 + n))
        slot_rows += [sl] * n
    M = len(pos)
    pos_t = torch.tensor(pos, dtype=torch.int32)
    sr = torch.tensor(slot_rows, dtype=torch.int32)
    blk = packed_blocks(seqs, 16 // G)
    q = torch.randn(M, Hq, HD, dtype=BF) * 2
    for window in (0, 16):
        og = ops.attention_varlen(q.to(gpu), kc.to(gpu), vc.to(gpu), pos_t.to(gpu), sr.to(gpu), blk.to(gpu),
                                  HD ** -0.5, 50.0, window)
        orf = ref.attention(q, kc, vc, pos_t, sr, M, 1, HD ** -0.5, 50.0, window)
        _close(og, orf, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("G,HD", [(2, 256), (1, 128)])
def test_attention_varlen_shared_prefix(gpu, G, HD):
    """Packed blocks whose keys below a per-block prefix length come from a shared prefix-cache slot
    (5-column block table) == the reference with those keys substituted."""
    from taboo_brittleness_amd.models.gemma2 import packed_blocks

    torch.manual_seed(15)
    Hkv, S = 2, 96
    Hq = Hkv * G
    kc = torch.randn(5, Hkv, S, HD, dtype=BF)
    vc = torch.randn(5, Hkv, S, HD, dtype=BF)
    pk = torch.randn(3, Hkv, S, HD, dtype=BF)
    pv = torch.randn(3, Hkv, S, HD, dtype=BF)
    spec_ = [(3, 10, 23, 1, 12), (0, 40, 1, 0, 0), (4, 5, 13, 2, 9), (1, 70, 26, 1, 75)]   # + (pslot, plen)
    pos, slot_rows, seqs = [], [], []
    for sl, p0, n, ps, pl in spec_:
        seqs.append((len(pos), n, sl, ps, pl))
        pos += list(range(p0, p0 + n))
        slot_rows += [sl] * n
    M = len(pos)
    pos_t = torch.tensor(pos, dtype=torch.int32)
    sr = torch.tensor(slot_rows, dtype=torch.int32)
    blk = packed_blocks(seqs, 16 // G)
    assert blk.shape[1] == 5
    q = torch.randn(M, Hq, HD, dtype=BF) * 2
    for window in (0, 16):
        og = ops.attention_varlen(q.to(gpu), kc.to(gpu), vc.to(gpu), pos_t.to(gpu), sr.to(gpu), blk.to(gpu),
                                  HD ** -0.5, 50.0, window, prefix_kv=(pk.to(gpu), pv.to(gpu)))
        orf = ops.attention_varlen(q, kc, vc, pos_t, sr, blk, HD ** -0.5, 50.0, window, prefix_kv=(pk, pv))
        _close(og, orf, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("G,HD", [(2, 256), (4, 256), (1, 128)])
def test_attention_tail_matches_decode_bitwise(gpu, G, HD):
    """Packed (block-table) rows -- the sweep's teacher-forced tails -- are BIT-identical to the same queries run as
    decode rows (one row per (position, slot), the one-wave and the 4-wave decode kernels), with and without the
    shared prefix and with a padding row: a replayed tail position rounds exactly like the greedy decode computed
    it (csrc/attention.hip attn_tail_exact_kernel; tests/test_exact_9b_gpu.py)."""
    from taboo_brittleness_amd.models.gemma2 import packed_blocks

    torch.manual_seed(31)
    Hkv, S = 4, 120
    Hq = Hkv * G
    d = lambda t: t.to(gpu)                                # noqa: E731
    kc = d(torch.randn(6, Hkv, S, HD, dtype=BF))
    vc = d(torch.randn(6, Hkv, S, HD, dtype=BF))
    pk = d(torch.randn(3, Hkv, S, HD, dtype=BF))
    pv = d(torch.randn(3, Hkv, S, HD, dtype=BF))
    spec_ = [(3, 10, 23, 1, 12), (0, 40, 1, 0, 0), (4, 5, 13, 2, 9), (1, 70, 40, 1, 75), (5, 0, 9, 0, 0)]
    pos, slot_rows, seqs, ps_rows, pl_rows = [], [], [], [], []
    for sl, p0, n, ps, pl in spec_:
        seqs.append((len(pos), n, sl, ps, pl))
        pos += list(range(p0, p0 + n))
        slot_rows += [sl] * n
        ps_rows += [ps] * n
        pl_rows += [pl] * n
    pos[30] = -1                                           # a padding row inside a block
    M = len(pos)
    pos_t, sr = d(torch.tensor(pos, dtype=torch.int32)), d(torch.tensor(slot_rows, dtype=torch.int32))
    q = d(torch.randn(M, Hq, HD, dtype=BF) * 2)
    k = ops._k()
    old = k.attention_split_rows(-1, True), k.attention_split_rows(-1, False)
    try:
        for prefix in (False, True):
            blk = d(packed_blocks(seqs if prefix else [s[:3] for s in seqs], 16 // G))
            tail = ops.attention_varlen(q, kc, vc, pos_t, sr, blk, HD ** -0.5, 50.0, 0,
                                        prefix_kv=(pk, pv) if prefix else None)
            pre = (pk, pv, d(torch.tensor(ps_rows, dtype=torch.int32)), d(torch.tensor(pl_rows, dtype=torch.int32)))
            for split in (0, 1 << 20):                     # one-wave decode kernel, then the 4-wave one
                k.attention_split_rows(split, prefix)
                dec = ops.attention(q, kc, vc, pos_t, sr, M, 1, HD ** -0.5, 50.0, 0, prefix=pre if prefix else None)
                torch.cuda.synchronize()
                assert torch.equal(tail, dec), (prefix, split, (tail.float() - dec.float()).abs().max().item())
    finally:
        k.attention_split_rows(old[0], True)
        k.attention_split_rows(old[1], False)


def test_decode_head(gpu):
    torch.manual_seed(13)
    R, V = 6, 4099 * 8 + 5
    lg = (torch.randn(R, V) * 4).to(BF)
    lg[2, 10] = 80.0
    lg[2, 11] = 80.0        # tie after the bf16 softcap -> lower index
    tgt = torch.tensor([5, -1, 11, V - 1, 0, 77], dtype=torch.int32)
    nxt, ns, nt = ops.decode_head(lg.to(gpu), 30.0, tgt.to(gpu))
    assert torch.equal(nxt.cpu(), ref.argmax_rows(lg, 30.0).view(-1))
    _close(ns, ref.xent_rows(lg, ref.argmax_rows(lg, 30.0), 30.0, True), atol=2e-3, rtol=1e-4)
    _close(nt, ref.xent_rows(lg, tgt, 30.0, True), atol=2e-3, rtol=1e-4)


@pytest.mark.parametrize("tp", [2, 4])
def test_decode_head_stats_vocab_parallel(gpu, tp):
    """The TP vocab-parallel head's per-rank pass (decode_head_stats: {lse, best, global id, target logit} from one
    HIP kernel per rank slice) merged by vp_head_merge equals decode_head on the whole row: the greedy token bit for
    bit, both NLLs to fp32 summation order; targets outside a rank's slice (and -1) handled."""
    torch.manual_seed(17)
    R, V = 37, 8192 * tp
    lg = (torch.randn(R, V) * 4).to(BF)
    lg[3, V // tp - 1] = 90.0
    lg[3, V // tp] = 90.0            # a tie across the rank boundary -> the lower global id
    tgt = torch.randint(0, V, (R,), dtype=torch.int32)
    tgt[0], tgt[1] = -1, V - 1
    g, t = lg.to(gpu), tgt.to(gpu)
    Vl = V // tp
    st = torch.stack([ops.decode_head_stats(g[:, r * Vl:(r + 1) * Vl].contiguous(), t, r * Vl, 30.0) for r in range(tp)])
    nxt, ns, nt = ops.vp_head_merge(st, t, V)
    enxt, ens, ent = ops.decode_head(g, 30.0, t)
    assert torch.equal(nxt, enxt)
    _close(ns, ens, atol=2e-3, rtol=1e-4)
    _close(nt, ent, atol=2e-3, rtol=1e-4)


def test_softcap_compact_gpu_exhaustive(gpu):
    """The compact exact softcap (lens.hip capc1: arithmetic below lo, a ~675-entry table, saturation) on every one
    of the 65536 bf16 inputs equals the transformers chain, for the final (30) and attention (50) caps."""
    allx = torch.arange(65536, dtype=torch.int32).to(torch.int16).view(BF)
    for cap in (30.0, 50.0):
        got = ops.softcap_values(allx.to(gpu), cap).cpu()
        want = ref.softcap_bf16(allx, cap).float()
        same = (got == want) | (torch.isnan(got) & torch.isnan(want))
        assert same.all(), (cap, int((~same).sum()))


_DH_MODES = """
import sys, torch
from taboo_brittleness_amd import ops
torch.manual_seed(21)
R, V = 600, 256000
lg = (torch.randn(R, V) * 6).to(torch.bfloat16)
lg[3, 100] = 200.0
lg[3, 7] = 150.0          # both saturate at 30: tie -> lower index
lg[5, 9000] = lg[5].max() # same-value tie inside and across 8-logit chunks
lg[5, 9003] = lg[5, 9000]
lg[5, 200001] = lg[5, 9000]
tgt = torch.randint(0, V, (R,), dtype=torch.int32)
tgt[::5] = -1
out = ops.decode_head(lg.cuda(), 30.0, tgt.cuda())
torch.save([t.cpu() for t in out], sys.argv[1])
"""


def test_decode_head_modes_agree(gpu, tmp_path):
    """The three decode_head kernels (TB_DECODE_HEAD: default f = fixed-offset LSE + chunk argmax + persistent,
    c = compact softcap, t = 64 KB table per row; chosen once per process) give the same argmax bit for bit
    (incl. ties inside and across 8-logit chunks and saturated ties) and the same NLLs to fp32 summation order;
    c and t are bit-identical (same values, same order).  Subprocesses: the mode is read once per process."""
    import subprocess
    import sys
    res = {}
    for mode in ("f", "c", "t"):
        p = tmp_path / f"{mode}.pt"
        env = dict(os.environ, TB_DECODE_HEAD=mode)
        r = subprocess.run([sys.executable, "-c", _DH_MODES, str(p)], env=env, capture_output=True, text=True,
                           timeout=300, cwd=REPO)
        assert r.returncode == 0, r.stderr[-3000:]
        res[mode] = torch.load(p, weights_only=True)
    for u, v in zip(res["c"], res["t"]):
        assert torch.equal(u, v)
    nf, sf, tf = res["f"]
    nt_, st_, tt_ = res["t"]
    assert torch.equal(nf, nt_)
    assert int(nf[3]) == 7 and int(nf[5]) == 9000
    _close(sf, st_, atol=2e-5, rtol=1e-5)
    _close(tf, tt_, atol=2e-5, rtol=1e-5)
    assert (tf[::5] == 0).all()


@pytest.mark.parametrize("M,V,K,cap", [(300, 4096, 256, 30.0), (1, 2048, 3584, 30.0), (520, 8192, 640, 0.0),
                                       (700, 256000, 3584, 30.0)])
def test_vocab_head_fused(gpu, M, V, K, cap):
    """Fused vocab head (csrc/gemm4.hip G4_HEAD: compact exact softcap + per-slice stats in the epilogue, persistent
    with several tiles per workgroup at the Gemma-2 vocab, then the partial merge) == the unfused path on the
    in-tree kernel's bf16 logits (bit-identical logits: exact argmax incl. cross-partial and in-partial ties, NLLs
    to fp32 summation order), and close to a float32 PyTorch reference."""
    torch.manual_seed(17)
    x = torch.randn(M, K).to(BF)
    w = (torch.randn(V, K) * 0.05).to(BF)
    x[:, 0] = 4.0
    w[5] = 0.0
    w[5, 0] = 8.0
    w[7] = w[5]             # same 128-column partial as 5
    w[V - 3] = w[5]         # other end of the vocab
    x[M // 2:, 0] = -4.0    # second half: no forced tie
    tgt = torch.randint(0, V, (M,), dtype=torch.int32)
    tgt[::7] = -1
    tgt[1::9] = 7
    xg, wg, tg = x.to(gpu), w.to(gpu), tgt.to(gpu)
    nxt, ns, nt = ops.vocab_head(xg, wg, cap, tg, fused=True)
    lg = torch.empty(M, V, dtype=BF, device=gpu)
    ops._k().gemm4(xg, wg, lg, None, None, 0, 256)
    n0, s0, t0 = ops.decode_head(lg, cap, tg)
    assert torch.equal(nxt, n0)
    assert (nxt[: M // 2] == 5).all()
    _close(ns, s0, atol=1e-4, rtol=1e-5)
    _close(nt, t0, atol=1e-4, rtol=1e-5)
    assert (nt[tg < 0] == 0).all()
    # vs the float32 reference (bf16 logits of an fp32 GEMM; argmax may differ only on near-ties)
    r = (x.float() @ w.float().T).to(BF)
    ra = ref.argmax_rows(r, cap).view(-1)
    assert (nxt.cpu() == ra).float().mean() > 0.98
    _close(nt, ref.xent_rows(r, tgt, cap, True), atol=3e-2, rtol=1e-3)
    # no teacher; a workspace carved from a (larger) idle logits buffer; deterministic
    part = torch.empty(M * V // 2 + 64, dtype=BF, device=gpu).view(torch.float32)
    n2, s2, t2 = ops.vocab_head(xg, wg, cap, part=part, fused=True)
    assert t2 is None and torch.equal(n2, nxt) and torch.equal(s2, ns)


@pytest.mark.parametrize("M,V,K", [(300, 4096, 256), (37, 2048, 3584), (600, 65536, 512)])
def test_lens_unembed_fused(gpu, M, V, K):
    """Logit-lens unembedding with the LSE epilogue (csrc/gemm4.hip G4_LENS, row-coalesced logits + per-slice
    {max, sum exp}): logits bit-identical to the in-tree kernels' plain bf16 output, lse == row_lse of them, both
    close to a float32 reference (the last shape runs several tiles per persistent workgroup)."""
    torch.manual_seed(19)
    x = torch.randn(M, K).to(BF)
    w = (torch.randn(V, K) * 0.05).to(BF)
    xg, wg = x.to(gpu), w.to(gpu)
    lg, lse = ops.lens_unembed(xg, wg, fused=True)
    lg0 = torch.empty(M, V, dtype=BF, device=gpu)
    ops._k().gemm4(xg, wg, lg0, None, None, 0, 256)
    assert torch.equal(lg, lg0)
    _close(lse, ops.row_lse(lg0), atol=1e-4, rtol=1e-6)
    r = (x.float() @ w.float().T).to(BF)
    _close(lg, r, atol=1e-2 * K ** 0.5, rtol=1e-2)
    _close(lse, ref.row_lse(r, 0.0, False), atol=2e-2, rtol=1e-3)
    lg2, lse2 = ops.lens_unembed(xg, wg, fused=False)
    _close(lse2, lse, atol=2e-2, rtol=1e-3)


@pytest.mark.parametrize("M,N,K", [(1, 256, 1024), (30, 3584, 4096), (77, 2048, 3584), (300, 1024, 640)])
def test_gemm_ring_fp32(gpu, M, N, K):
    """Ring GEMM (csrc/gemm_ring.hip, every built tile and both ring variants) vs a float32 reference of the same
    bf16 operands, odd row counts included (rows past M clamped on load, masked on store)."""
    torch.manual_seed(21)
    A = torch.randn(M, K, dtype=BF)
    W = (torch.randn(N, K) / K ** 0.5).to(BF)
    ref_ = A.float() @ W.float().t()
    k = _ext_kernels()
    Ag, Wg = A.to(gpu), W.to(gpu)
    n = 0
    for bm, bn in k.gemm_ring_tiles(0):
        for var in (0, 1, 2):
            if not k.gemm_ring_ok(M, N, K, 0, bm, bn, var):
                continue
            out = torch.full((M, N), float("nan"), dtype=BF, device=gpu)
            k.gemm_ring(Ag, Wg, out, 0, bm, bn, var)
            _close(out, ref_, atol=2e-2, rtol=1e-2)
            n += 1
    assert n >= 11


@pytest.mark.parametrize("N,K,epi", [(3584, 4096, 0), (8192, 3584, 0), (3584, 14336, 0), (28672, 3584, 3)])
def test_gemm_ring_bitexact_batch_invariant(gpu, N, K, epi):
    """The batch-invariance contract of TB_GEMM=tb at the Gemma-2-9B projection shapes: every ring tile (both ring
    variants) on every sub-batch of rows is BIT-identical to the four-wave kernel (256- and 128-row tiles) on the
    whole batch -- same MFMA, same K order -- so a row's projection does not depend on the batch it decodes in."""
    torch.manual_seed(6)
    M = 600
    A = ((torch.rand(M, K) * 2 - 1) * 0.5).to(BF).to(gpu)
    W = ((torch.rand(N, K) * 2 - 1) * 0.5).to(BF).to(gpu)
    k = ops._k()
    if epi == 3:
        W = W[ops.geglu_interleave_index(N // 2, gpu)].contiguous()
    ncol = N // 2 if epi == 3 else N
    full = torch.empty(M, ncol, device=gpu, dtype=BF)
    k.gemm4(A, W, full, None, None, epi, 256)
    g128 = torch.empty_like(full)
    k.gemm4(A, W, g128, None, None, epi, 128)
    assert torch.equal(full, g128)
    for rows in (slice(0, 1), slice(3, 20), slice(100, 164), slice(M - 257, M)):
        A_s = A[rows].contiguous()
        ms = rows.stop - rows.start
        for bm, bn in k.gemm_ring_tiles(epi):
            for var in (0, 1, 2):
                if not k.gemm_ring_ok(ms, N, K, epi, bm, bn, var) or bm > 2 * max(ms, 16):
                    continue
                sub = torch.empty(ms, ncol, device=gpu, dtype=BF)
                k.gemm_ring(A_s, W, sub, epi, bm, bn, var)
                assert torch.equal(sub, full[rows]), (rows, bm, bn, var)


@pytest.mark.parametrize("M", [5, 64, 200])
def test_gemm_ring_qkv_rope_bitexact(gpu, M):
    """QKV + RoPE + KV-cache scatter on the ring GEMM (narrow tiles, pair epilogue over head dims d / d + 128) ==
    gemm4's fused G4_ROPE epilogue bit for bit (q, K cache, V cache), padding rows (pos < 0) included."""
    torch.manual_seed(13)
    Hq, Hkv, HD, K, S = 16, 8, 256, 3584, 64
    A = ((torch.rand(M, K) * 2 - 1) * 0.5).to(BF).to(gpu)
    W = ((torch.rand((Hq + 2 * Hkv) * HD, K) * 2 - 1) * 0.05).to(BF).to(gpu)
    nslot = M
    pos = torch.randint(0, S, (M,), dtype=torch.int32)
    pos[M // 3] = -1
    pos = pos.to(gpu)
    slot = torch.arange(M, dtype=torch.int32, device=gpu)
    cos_t, sin_t = ref.rope_tables(HD, 8192, 10000.0, gpu)
    cos_t, sin_t = cos_t.contiguous(), sin_t.contiguous()
    k = ops._k()

    def run(fn):
        q = torch.zeros(M, Hq, HD, device=gpu, dtype=BF)
        kc = torch.zeros(nslot, Hkv, S, HD, device=gpu, dtype=BF)
        vc = torch.zeros_like(kc)
        fn(q, kc, vc)
        return q, kc, vc

    want = run(lambda q, kc, vc: k.gemm4_qkv_rope(A, W, pos, slot, ops.rope_cs(cos_t, sin_t), q, kc, vc, Hq, Hkv, 128))
    n = 0
    for bm, bn in k.gemm_ring_tiles(4):
        for var in (0, 1, 2):
            if not k.gemm_ring_ok(M, (Hq + 2 * Hkv) * HD, K, 4, bm, bn, var):
                continue
            got = run(lambda q, kc, vc: k.gemm_ring_qkv_rope(A, W, pos, slot, ops.rope_cs(cos_t, sin_t), q, kc, vc, Hq, Hkv, bm, bn,
                                                             var))
            assert all(torch.equal(a, b) for a, b in zip(got, want)), (bm, bn, var)
            n += 1
    assert n >= 10


def _ext_kernels():
    from taboo_brittleness_amd.ops._ext import kernels

    return kernels()


def test_geglu(gpu):
    torch.manual_seed(3)
    gu = torch.randn(33, 2 * 1024, dtype=BF) * 2
    _close(ops.geglu(gu.to(gpu)), ref.geglu(gu), atol=1e-2, rtol=1e-2)


def test_vocab_readouts(gpu):
    torch.manual_seed(4)
    B, T, V = 3, 5, 4099 * 8 + 3
    lg = (torch.randn(B * T, V) * 4).to(BF)
    lg[1, 77] = 40.0
    lg[1, 78] = 40.0     # tie -> lower index
    g = lg.to(gpu)
    assert torch.equal(ops.argmax_rows(g).cpu(), ref.argmax_rows(lg, 0.0))
    assert torch.equal(ops.argmax_rows(g, 30.0).cpu(), ref.argmax_rows(lg, 30.0))
    lse_g = ops.row_lse(g)
    lse_r = ref.row_lse(lg)
    _close(lse_g, lse_r, atol=1e-3, rtol=1e-5)
    ids = torch.randint(0, V, (B * T, 3), dtype=torch.int32)
    _close(ops.gather_probs(g, lse_g, ids.to(gpu)), ref.gather_probs(lg, lse_r, ids), atol=1e-6, rtol=1e-3)
    mask = torch.tensor([1, 1, 0, 1, 1] * B, dtype=torch.uint8)
    excl = torch.randint(-1, V, (B * T, 2), dtype=torch.int32)
    acc_g = ops.lens_colsum(g, lse_g, mask.to(gpu), excl.to(gpu), B, T)
    acc_r = ref.lens_colsum(lg, lse_r, mask, excl, B, T)
    _close(acc_g, acc_r, atol=1e-6, rtol=1e-3)
    # running sums (dense) and packed row offsets, accumulating onto a start value
    cum_g = torch.empty(B, T + 1, V, device=gpu)
    start = torch.rand(B, V)
    acc2 = ops.lens_colsum(g, lse_g, mask.to(gpu), excl.to(gpu), B, T, acc=start.to(gpu), accumulate=True,
                           cum=cum_g)
    _close(acc2, acc_r + start, atol=1e-5, rtol=1e-3)
    _s, cum_r = ref.lens_colsum(lg, lse_r, mask, excl, B, T, with_cum=True)
    _close(cum_g, cum_r + start[:, None], atol=1e-5, rtol=1e-3)
    offs = torch.tensor([0, 2, 2, 2 + 2 * T - 2], dtype=torch.int32)[: B + 1]
    offs[-1] = B * T
    acc_p = ops.lens_colsum(g, lse_g, None, excl.to(gpu), B, T, offs=offs.to(gpu))
    acc_pr, _ = ref.lens_colsum(lg, lse_r, None, excl, B, T, offs=offs)
    _close(acc_p, acc_pr, atol=1e-5, rtol=1e-3)
    vals, idx = ops.topk_rows(acc_g, 5)
    rv, ri = ref.topk_rows(acc_g.cpu(), 5)
    assert torch.equal(idx.cpu(), ri)
    tgt = torch.randint(-1, V, (B * T,), dtype=torch.int32)
    _close(ops.xent_rows(g, tgt.to(gpu), 30.0, True), ref.xent_rows(lg, tgt, 30.0, True), atol=2e-3, rtol=1e-4)


@pytest.mark.parametrize("M,N,K", [(1, 128, 64), (33, 200, 96), (70, 384, 3584), (257, 16384, 512)])
def test_gemm_nt_epilogues(gpu, M, N, K):
    torch.manual_seed(5)
    A = torch.randn(M, K, dtype=BF)
    W = torch.randn(N, K, dtype=BF) * 0.05
    b = torch.randn(N) * 0.1
    th = torch.rand(N) * 0.5
    Ag, Wg = A.to(gpu), W.to(gpu)
    r = ref.gemm_nt(A, W, 1)
    _close(ops.gemm_nt(Ag, Wg, 1), r, atol=1e-3, rtol=1e-3)
    _close(ops.gemm_nt(Ag, Wg, 0), r, atol=2e-2, rtol=1e-2)
    jr = ops.gemm_nt(Ag, Wg, 2, b.to(gpu), th.to(gpu)).cpu()
    pre = r + b
    near = (pre - th).abs() < 1e-3
    want = torch.where(pre > th, pre, torch.zeros_like(pre))
    assert ((jr - want).abs()[~near] < 1e-3).all()


@pytest.mark.parametrize("M,N,K", [(1, 256, 64), (37, 512, 128), (300, 768, 3584), (513, 1024, 640)])
def test_gemm4_epilogues(gpu, M, N, K):
    """Four-wave 256x256x64 MFMA GEMM (csrc/gemm4.hip) vs a float32 PyTorch reference: every epilogue, both tile
    heights, ragged M (clamped loads, masked stores), 1 / 2 / 10 / 56 K tiles."""
    torch.manual_seed(12)
    A = (torch.rand(M, K) * 2 - 1).to(BF)
    W = (torch.rand(N, K) * 2 - 1).to(BF)
    b = torch.randn(N)
    th = torch.rand(N) * 2
    Ag, Wg = A.to(gpu), W.to(gpu)
    k = ops._k()
    r = A.float() @ W.float().T
    for t in (256, 128):
        c32 = torch.full((M, N), float("nan"), device=gpu)
        k.gemm4(Ag, Wg, c32, None, None, 1, t)
        _close(c32, r, atol=1e-3 * K ** 0.5, rtol=1e-4)
        cb = torch.full((M, N), float("nan"), device=gpu, dtype=BF)
        k.gemm4(Ag, Wg, cb, None, None, 0, t)
        _close(cb, r, atol=1e-2 * K ** 0.5, rtol=1e-2)
        k.gemm4(Ag, Wg, c32, b.to(gpu), th.to(gpu), 2, t)
        pre = r + b
        near = (pre - th).abs() < 1e-3
        want = torch.where(pre > th, pre, torch.zeros_like(pre))
        assert ((c32.cpu() - want).abs()[~near] < 1e-3 * K ** 0.5).all()
        Wi = Wg[ops.geglu_interleave_index(N // 2, gpu)].contiguous()
        act = torch.empty(M, N // 2, device=gpu, dtype=BF)
        k.gemm4(Ag, Wi, act, None, None, 3, t)
        _close(act, ref.geglu(r.to(BF)).float(), atol=2e-2 * K ** 0.5, rtol=2e-2)


@pytest.mark.parametrize("N,K,epi", [(3584, 4096, 0), (8192, 3584, 0), (3584, 14336, 0), (28672, 3584, 3),
                                     (256000, 3584, 0)])
def test_gemm4_tiles_bitequal_and_batch_invariant(gpu, N, K, epi):
    """At the Gemma-2-9B projection shapes (vocab head included) the four-wave kernel's output is BIT-identical
    for both tile heights, for sub-batches of the rows and for the rounds-model row split ("gs"): switching tiles
    per row count (runtime/gemm_dispatch.py) keeps the forward batch-invariant."""
    torch.manual_seed(5)
    M = 777 if N < 100000 else 300
    A = ((torch.rand(M, K) * 2 - 1) * 0.5).to(BF).to(gpu)
    W = ((torch.rand(N, K) * 2 - 1) * 0.5).to(BF).to(gpu)
    k = ops._k()
    if epi == 3:
        W = W[ops.geglu_interleave_index(N // 2, gpu)].contiguous()
    ncol = N // 2 if epi == 3 else N
    ref_ = torch.empty(M, ncol, device=gpu, dtype=BF)
    k.gemm4(A, W, ref_, None, None, epi, 256)
    gs = torch.empty_like(ref_)
    ops.tb_gemm(A, W, gs, None, None, epi, "gs")
    assert torch.equal(gs, ref_)
    for t in (256, 128):
        c = torch.empty(M, ncol, device=gpu, dtype=BF)
        k.gemm4(A, W, c, None, None, epi, t)
        assert torch.equal(c, ref_), t
    for rows in (slice(0, 1), slice(5, 130), slice(M - 200, M)):
        sub = torch.empty(rows.stop - rows.start, ncol, device=gpu, dtype=BF)
        k.gemm4(A[rows].contiguous(), W, sub, None, None, epi, 128)
        assert torch.equal(sub, ref_[rows])
    if epi == 0:
        r = A[:64].float() @ W.float().T
        _close(ref_[:64], r, atol=1e-2 * K ** 0.5, rtol=1e-2)


@pytest.mark.parametrize("M,N,K,epi,ks", [(16, 3584, 14336, 0, 0), (100, 8192, 3584, 0, 3), (700, 3584, 4096, 0, 0),
                                          (48, 28672, 3584, 3, 0), (300, 1024, 640, 3, 4), (1, 256, 64, 0, 1)])
def test_gemm4_splitk(gpu, M, N, K, epi, ks):
    """Split-K gemm4 (thin grids: fp32 partials of ks K ranges + ordered reduction, csrc/gemm4.hip
    tb_gemm4_splitk) at Gemma-2-9B decode / o_proj / down / gate|up shapes vs a float32 reference of the same
    bf16 operands, the heuristic split count and explicit uneven ones; deterministic across runs and within bf16
    rounding of the unsplit kernel."""
    torch.manual_seed(9)
    A = ((torch.rand(M, K) * 2 - 1) * 0.5).to(BF)
    W = ((torch.rand(N, K) * 2 - 1) * 0.5).to(BF)
    Ag, Wg = A.to(gpu), W.to(gpu)
    k = ops._k()
    r = A.float() @ W.float().T
    if epi == 3:
        Wg = Wg[ops.geglu_interleave_index(N // 2, gpu)].contiguous()
        want = ref.geglu(r.to(BF)).float()
    else:
        want = r
    ncol = N // 2 if epi == 3 else N
    for t in (64, 128, 256):
        kse = ks if ks > 0 else int(k.gemm4_splitk_ks(M, N, K, t))
        ws = torch.full((kse * M * N,), float("nan"), device=gpu)
        c = torch.full((M, ncol), float("nan"), device=gpu, dtype=BF)
        k.gemm4_splitk(Ag, Wg, c, ws, epi, t, kse)
        _close(c, want, atol=2e-2 * K ** 0.5, rtol=2e-2)
        c2 = torch.empty_like(c)
        k.gemm4_splitk(Ag, Wg, c2, ws, epi, t, kse)
        assert torch.equal(c, c2), "split-K must be deterministic"
        plain = torch.empty_like(c)
        k.gemm4(Ag, Wg, plain, None, None, epi, max(t, 128))
        # a different K summation order: within one bf16 ulp of the unsplit result almost everywhere
        d = (c.float() - plain.float()).abs()
        assert (d <= plain.float().abs() * 2 ** -7 + 1e-3).float().mean() > 0.999


@pytest.mark.parametrize("M,K,ks", [(64, 14336, 0), (700, 4096, 2), (5, 4096, 5)])
def test_splitk_add_rmsnorm2_fused(gpu, M, K, ks):
    """o_proj / down split over K with the fp32 partials summed inside add_rmsnorm2 (add_rmsnorm2_part): h and the
    next pre-norm BIT-identical to the split-K reduction kernel's bf16 o followed by add_rmsnorm2."""
    torch.manual_seed(4)
    D = 3584
    a = ((torch.rand(M, K) * 2 - 1) * 0.5).to(BF).to(gpu)
    w = ((torch.rand(D, K) * 2 - 1) * 0.05).to(BF).to(gpu)
    h0 = torch.randn(M, D).to(BF).to(gpu)
    wp, wn = (torch.randn(D) * 0.1).to(BF).to(gpu), (torch.randn(D) * 0.1).to(BF).to(gpu)
    k = ops._k()
    kse = ks if ks > 0 else int(k.gemm4_splitk_ks(M, D, K, 128))
    ws = torch.empty(kse * M * D, device=gpu)
    o = torch.empty(M, D, device=gpu, dtype=BF)
    k.gemm4_splitk(a, w, o, ws, 0, 128, kse)
    h1, x1 = h0.clone(), torch.empty(M, D, device=gpu, dtype=BF)
    k.add_rmsnorm2(h1, o, wp, wn, x1, 1e-6)
    used = int(k.gemm4_splitk_part(a, w, ws, 128, kse))
    h2, x2 = h0.clone(), torch.empty(M, D, device=gpu, dtype=BF)
    k.add_rmsnorm2_part(h2, ws, used, wp, wn, x2, 1e-6)
    assert torch.equal(h1, h2) and torch.equal(x1, x2)


@pytest.mark.parametrize("M,ks", [(48, 0), (200, 3)])
def test_splitk_rope_qkv_cache_fused(gpu, M, ks):
    """QKV split over K with the fp32 partials summed inside the RoPE / KV-scatter pass (rope_qkv_cache_part): q and
    both caches BIT-identical to the split-K reduction kernel's bf16 qkv followed by rope_qkv_cache, padding rows
    (pos < 0) and positions past the cache included."""
    torch.manual_seed(6)
    Hq, Hkv, HD, K, S = 16, 8, 256, 3584, 64
    N = (Hq + 2 * Hkv) * HD
    x = ((torch.rand(M, K) * 2 - 1) * 0.5).to(BF).to(gpu)
    w = ((torch.rand(N, K) * 2 - 1) * 0.05).to(BF).to(gpu)
    slot = torch.arange(M, dtype=torch.int32) % 7
    pos = (torch.arange(M, dtype=torch.int32) // 7).contiguous()     # one writer per (slot, position)
    pos[::9] = -1
    pos[5::11] = S + 2                                                # past the cache: q rotated, no cache write
    cos_t, sin_t = ref.rope_tables(HD, 128, 10000.0)
    k = ops._k()
    kse = ks if ks > 0 else int(k.gemm4_splitk_ks(M, N, K, 128))
    ws = torch.empty(kse * M * N, device=gpu)
    qkv = torch.empty(M, N, device=gpu, dtype=BF)
    k.gemm4_splitk(x, w, qkv, ws, 0, 128, kse)
    outs = []
    for fused in (False, True):
        kc = torch.zeros(7, Hkv, S, HD, device=gpu, dtype=BF)
        vc = torch.zeros_like(kc)
        q = torch.full((M, Hq, HD), 7.0, device=gpu, dtype=BF)
        if fused:
            used = int(k.gemm4_splitk_part(x, w, ws, 128, kse))
            k.rope_qkv_cache_part(ws, used, pos.to(gpu), slot.to(gpu), cos_t.to(gpu), sin_t.to(gpu), q, kc, vc, Hq, Hkv,
                                  HD)
        else:
            k.rope_qkv_cache(qkv, pos.to(gpu), slot.to(gpu), cos_t.to(gpu), sin_t.to(gpu), q, kc, vc, Hq, Hkv, HD)
        outs.append((q, kc, vc))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("M,rows", [(300, 256), (77, 128)])
def test_gemm4_qkv_rope_fused(gpu, M, rows):
    """QKV GEMM with RoPE + KV scatter in the epilogue (csrc/gemm4.hip G4_ROPE) at the Gemma-2-9B head layout
    (16 q / 8 kv heads of 256, K = 3584): q, K cache and V cache BIT-identical to the in-tree GEMM followed by
    rope_qkv_cache, including padding rows (pos < 0: q zeroed, no cache write) and positions past the cache."""
    torch.manual_seed(7)
    Hq, Hkv, HD, K, S = 16, 8, 256, 3584, 40
    slots = M              # one (slot, position) per row, as in the engine: no two rows write one cache entry
    x = ((torch.rand(M, K) * 2 - 1) * 0.5).to(BF).to(gpu)
    w = ((torch.rand((Hq + 2 * Hkv) * HD, K) * 2 - 1) * 0.05).to(BF).to(gpu)
    pos = torch.randint(0, S + 3, (M,), dtype=torch.int32)
    pos[::17] = -1
    pos = pos.to(gpu)
    slot = torch.randperm(slots)[:M].to(torch.int32).to(gpu)
    maxp = 64
    inv = 1.0 / (10000.0 ** (torch.arange(0, HD, 2).float() / HD))
    ang = torch.arange(maxp).float()[:, None] * inv[None]
    cos_t, sin_t = ang.cos().to(gpu), ang.sin().to(gpu)
    k = ops._k()
    kc0 = torch.randn(slots, Hkv, S, HD).to(BF).to(gpu)
    vc0 = torch.randn(slots, Hkv, S, HD).to(BF).to(gpu)
    qkv = torch.empty(M, (Hq + 2 * Hkv) * HD, device=gpu, dtype=BF)
    k.gemm4(x, w, qkv, None, None, 0, rows)
    q_ref = torch.empty(M, Hq, HD, device=gpu, dtype=BF)
    kc_ref, vc_ref = kc0.clone(), vc0.clone()
    k.rope_qkv_cache(qkv, pos, slot, cos_t, sin_t, q_ref, kc_ref, vc_ref, Hq, Hkv, HD)
    q = torch.full((M, Hq, HD), 7.0, device=gpu, dtype=BF)
    kc, vc = kc0.clone(), vc0.clone()
    k.gemm4_qkv_rope(x, w, pos, slot, ops.rope_cs(cos_t, sin_t), q, kc, vc, Hq, Hkv, rows)
    assert torch.equal(q, q_ref)
    assert torch.equal(kc, kc_ref) and torch.equal(vc, vc_ref)
    assert not torch.equal(kc, kc0)       # the cache was written


def test_linear_dispatch_modes(gpu):
    """ops.linear under TB_GEMM=tb (in-tree tiles only) equals the in-tree kernel bit for bit and the
    hipBLASLt mode up to bf16 rounding."""
    from taboo_brittleness_amd.runtime import gemm_dispatch as GD

    torch.manual_seed(4)
    A = (torch.rand(300, 3584) * 2 - 1).to(BF).to(gpu)
    W = ((torch.rand(4096, 3584) * 2 - 1) * 0.05).to(BF).to(gpu)
    old = GD.mode()
    try:
        GD.set_mode("tb")
        y_tb = ops.linear(A, W)
        GD.set_mode("blas")
        y_bl = ops.linear(A, W)
    finally:
        GD.set_mode(old)
    c = torch.empty_like(y_tb)
    ops.tb_gemm(A, W, c, None, None, 0, GD.fill_choice(300, 4096))
    assert torch.equal(c, y_tb)
    _close(y_tb, y_bl, atol=2e-2, rtol=1e-2)


def test_lowrank_edit_sae_and_projection(gpu):
    torch.manual_seed(6)
    M, D, L, mmax = 9, 512, 300, 8
    h = torch.randn(M, D, dtype=BF)
    We = (torch.randn(L, D) / math.sqrt(D)).to(BF)
    Wd = (torch.randn(L, D) / math.sqrt(D)).to(BF)
    be = torch.randn(L) * 0.1
    th = torch.rand(L) * 0.2
    apply = torch.tensor([1, 0, 1, 1, 0, 1, 1, 1, 1], dtype=torch.uint8)
    idx = torch.randint(0, L, (M, mmax), dtype=torch.int32)
    cnt = torch.tensor([8, 8, 3, 0, 2, 8, 1, 5, 8], dtype=torch.int32)
    wn = torch.randn(D, dtype=BF) * 0.1
    for table_dtype, thr, bias in ((BF, th, be), (torch.float32, None, None)):
        E, Dm = We.to(table_dtype), Wd.to(table_dtype)
        hg, xg = h.clone().to(gpu), torch.zeros(M, D, dtype=BF, device=gpu)
        cg = torch.zeros(M, mmax, device=gpu)
        ops.lowrank_edit(hg, apply.to(gpu), idx.to(gpu), cnt.to(gpu), E.to(gpu), Dm.to(gpu),
                         bias.to(gpu) if bias is not None else None, thr.to(gpu) if thr is not None else None,
                         None, 1.0, wn.to(gpu), 1e-6, xg, cg)
        hr, xr = h.clone(), torch.zeros(M, D, dtype=BF)
        cr = torch.zeros(M, mmax)
        ref.lowrank_edit(hr, apply, idx, cnt, E, Dm, bias, thr, None, 1.0, wn, 1e-6, xr, cr)
        _close(hg, hr, atol=3e-2, rtol=1e-2)
        _close(cg, cr, atol=1e-3, rtol=1e-3)
        rows = apply.bool()
        _close(xg[rows.to(gpu)], xr[rows], atol=3e-2, rtol=1e-2)


def test_sae_decode_and_score(gpu):
    torch.manual_seed(7)
    M, L, D = 6, 2048, 256
    acts = torch.relu(torch.randn(M, L) - 2.5)
    Wd = (torch.randn(L, D) * 0.05).to(BF)
    bd = torch.randn(D) * 0.01
    _close(ops.sae_decode_sparse(acts.to(gpu), Wd.to(gpu), bd.to(gpu)), ref.sae_decode_sparse(acts, Wd, bd),
           atol=1e-3, rtol=1e-3)
    R = 20
    A = torch.relu(torch.randn(R, L))
    p = torch.rand(R)
    spike = (torch.rand(R) > 0.7).to(torch.uint8)
    seg = torch.tensor([0, 7, 20], dtype=torch.int32)
    got = ops.latent_score(A.to(gpu), p.to(gpu), spike.to(gpu), seg.to(gpu))
    want = ref.latent_score(A, p, spike, seg)
    for g_, w_ in zip(got, want):
        _close(g_, w_, atol=1e-4, rtol=1e-3)


def test_latent_score_offset_low_variance(gpu):
    """Offset, low-variance latents (a ~ 40 +- 0.01): a one-pass fp32 correlation cancels catastrophically
    here; the kernel's two-pass form must match the fp64 reference."""
    torch.manual_seed(11)
    R, L = 50, 512
    A = 40.0 + 0.01 * torch.randn(R, L)
    A[:, : L // 4] = torch.relu(torch.randn(R, L // 4))          # mixed with ordinary sparse latents
    A[:, L // 4: L // 4 + 8] = 40.0                              # exactly constant: corr must be 0
    p = torch.rand(R) * 1e-3 + 0.5
    spike = torch.zeros(R, dtype=torch.uint8)
    spike[[3, 10, 20, 40]] = 1
    seg = torch.tensor([0, 23, 50], dtype=torch.int32)
    got = ops.latent_score(A.to(gpu), p.to(gpu), spike.to(gpu), seg.to(gpu))
    want = ref.latent_score(A, p, spike, seg)
    _close(got[2], want[2], atol=2e-3, rtol=1e-3)                # correlations
    _close(got[0], want[0], atol=0.1, rtol=1e-3)                 # scores (spike mean ~40 x corr)
    assert float(got[2][:, L // 4: L // 4 + 8].abs().max()) == 0.0


def test_lowrank_edit_rejects_unsupported_rows(gpu):
    """Rows the kernel cannot cover (D % 8 != 0, or D past the largest per-thread tile) fail loudly
    instead of leaving part of the row unedited."""
    for D in (8200, 12):
        h = torch.zeros(2, D, dtype=BF, device=gpu)
        apply = torch.ones(2, dtype=torch.uint8, device=gpu)
        idx = torch.zeros(2, 1, dtype=torch.int32, device=gpu)
        cnt = torch.ones(2, dtype=torch.int32, device=gpu)
        E = torch.zeros(4, D, dtype=torch.float32, device=gpu)
        with pytest.raises(RuntimeError):
            ops.lowrank_edit(h, apply, idx, cnt, E, E, None, None, None, 1.0, None, 1e-6, None, None)


@pytest.mark.parametrize("HD", [256, 128])
def test_attention_decode_shared_prefix_buckets(gpu, HD):
    """Shared-prefix decode attention (row b reads keys [0, plen[b]) from slot pslot[b] of the pair prefix cache,
    its own keys from its slot) == the reference, incl. rows without a prefix, a sub-bucket of the rows and a
    sliding window that hides a row's prefix."""
    torch.manual_seed(11)
    Hkv, G, S, B = 2, 2, 68, 27
    Hq = Hkv * G
    kc = torch.randn(B, Hkv, S, HD, dtype=BF)
    vc = torch.randn(B, Hkv, S, HD, dtype=BF)
    pk = torch.randn(4, Hkv, S, HD, dtype=BF)
    pv = torch.randn(4, Hkv, S, HD, dtype=BF)
    slot = torch.randperm(B).to(torch.int32)
    pos = torch.randint(20, S, (B,), dtype=torch.int32)
    ps = torch.randint(0, 4, (B,), dtype=torch.int32)
    pl = torch.minimum(torch.randint(1, 40, (B,), dtype=torch.int32), pos)
    pl[[3, 10]] = 0                                       # rows without a prefix
    q = torch.randn(B, Hq, HD, dtype=BF) * 2
    d = lambda t: t.to(gpu)                               # noqa: E731
    for window, nb in ((0, B), (16, B), (0, 13)):
        og = ops.attention(d(q[:nb]), d(kc), d(vc), d(pos[:nb]), d(slot[:nb]), nb, 1, HD ** -0.5, 50.0, window,
                           prefix=(d(pk), d(pv), d(ps), d(pl)))
        orf = ref.attention(q[:nb], kc, vc, pos[:nb], slot[:nb], nb, 1, HD ** -0.5, 50.0, window,
                            prefix=(pk, pv, ps[:nb], pl[:nb]))
        assert torch.isfinite(og.float()).all()
        _close(og, orf, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("G,S", [(2, 96), (2, 700), (4, 300)])
def test_attention_decode_split_bitequal(gpu, G, S):
    """The 4-wave-per-(row, kv head) decode kernel (few rows) is BIT-identical to the one-wave kernel per row: own
    keys, shared-prefix keys, a padding row, a sliding window -- so the row count that picks between them never
    changes a result."""
    torch.manual_seed(19)
    Hkv, HD, B, P = 4, 256, 37, 5
    d = lambda t: t.to(gpu)                               # noqa: E731
    kc = d(torch.randn(B, Hkv, S, HD, dtype=BF))
    vc = d(torch.randn(B, Hkv, S, HD, dtype=BF))
    pk = d(torch.randn(P, Hkv, S, HD, dtype=BF))
    pv = d(torch.randn(P, Hkv, S, HD, dtype=BF))
    q = d(torch.randn(B, Hkv * G, HD, dtype=BF) * 2)
    slot = torch.randperm(B).to(torch.int32)
    pos = torch.randint(0, S + 8, (B,), dtype=torch.int32)   # incl. positions past the cache (clamped keys)
    pos[3] = -1
    ps = torch.randint(0, P, (B,), dtype=torch.int32)
    pl = torch.minimum(torch.randint(0, S, (B,), dtype=torch.int32), pos.clamp(min=0))
    k = ops._k()
    old = (k.attention_split_rows(-1, False), k.attention_split_rows(-1, True))
    try:
        for window, pre in ((0, False), (24, False), (0, True), (40, True)):
            args = (q, kc, vc, d(pos), d(slot), B, 1, HD ** -0.5, 50.0, window)
            outs = []
            for split in (0, 1 << 20):
                k.attention_split_rows(split, pre)
                if pre:
                    outs.append(ops.attention(*args, prefix=(pk, pv, d(ps), d(pl))))
                else:
                    outs.append(ops.attention(*args))
            for o in outs[1:]:
                assert torch.equal(o, outs[0]), (window, pre, (o.float() - outs[0].float()).abs().max().item())
    finally:
        k.attention_split_rows(old[0], False)
        k.attention_split_rows(old[1], True)


@pytest.mark.parametrize("G", [2, 4])
def test_attention_decode_wave_s2048(gpu, G):
    """the one-wave decode kernel near S = 2048 needs more than 64 KB of dynamic LDS (4 kv heads per
    workgroup x G query rows x S fp32 scores); it must launch (opt-in LDS attribute) and equal the reference and
    the 4-wave kernel bit for bit, with rows at the end of the cache."""
    torch.manual_seed(23)
    Hkv, HD, B, S = 4, 256, 6, 2048
    d = lambda t: t.to(gpu)                               # noqa: E731
    kc = torch.randn(B, Hkv, S, HD, dtype=BF)
    vc = torch.randn(B, Hkv, S, HD, dtype=BF)
    q = torch.randn(B, Hkv * G, HD, dtype=BF) * 2
    slot = torch.randperm(B).to(torch.int32)
    pos = torch.tensor([S - 1, S - 2, 1500, 2000, 7, S - 1], dtype=torch.int32)
    k = ops._k()
    old = k.attention_split_rows(-1, False)
    try:
        outs = []
        for split in (0, 1 << 20):                        # one-wave kernel, then the 4-wave kernel
            k.attention_split_rows(split, False)
            outs.append(ops.attention(d(q), d(kc), d(vc), d(pos), d(slot), B, 1, HD ** -0.5, 50.0, 0))
        torch.cuda.synchronize()
    finally:
        k.attention_split_rows(old, False)
    assert torch.equal(outs[0], outs[1])
    orf = ref.attention(q, kc, vc, pos, slot, B, 1, HD ** -0.5, 50.0, 0)
    _close(outs[0], orf, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("R,V,K", [(1, 256000, 5), (3, 256000, 16), (2, 16384, 40), (600, 5000, 8), (4, 9000, 8)])
def test_topk_rows_chunked(gpu, R, V, K):
    """Row top-k (chunked two-pass for few long rows) == a stable descending sort: ties (coarsely quantised values)
    resolved towards the lower column, -inf entries, the best values at chunk edges."""
    g = torch.Generator().manual_seed(R * 7 + K)
    x = (torch.randn(R, V, generator=g) * 4).round() / 4
    x[:, ::97] = -float("inf")
    x[0, 2047] = x[0, 2048] = 50.0                         # a tie across a chunk boundary
    vals, idx = ops.topk_rows(x.to(gpu), K)
    rv, ri = ref.topk_rows(x, K)
    assert torch.equal(idx.cpu(), ri) and torch.equal(vals.cpu(), rv)


@pytest.mark.parametrize("bf16_rows", [True, False])
def test_sae_fp32_encode_firing_set(gpu, bf16_rows):
    """fp32 SAE parity (reference encodes the fp32 residual with fp32 Gemma Scope weights,
    `src/02_run_sae_baseline.py:30-36,66-67`): at Gemma-Scope shapes (3584 -> 16384) the GPU encode (bf16x3
    split MFMA GEMM + JumpReLU epilogue) fires exactly the latents an fp32 CPU encode fires, ties excluded,
    with fp32-level pre-activation error.  ``bf16_rows``: the model's bf16 residual (3-term split) or generic
    fp32 rows (6-term split)."""
    from taboo_brittleness_amd.interp.sae import JumpReLUSAE

    torch.manual_seed(21)
    D, L, N = 3584, 16384, 96
    sae = JumpReLUSAE.random(D, L, seed=5, device="cpu")
    sae.b_enc = torch.randn(L) * 0.05
    x = torch.randn(N, D) * 1.3
    sae.calibrate(x.to(BF) if bf16_rows else x)                 # thresholds at the L0 ~ 76 quantile
    g = sae.to(gpu)
    assert g.W_encT.dtype == torch.float32 and g.W_dec.dtype == torch.float32
    xin = x.to(BF) if bf16_rows else x
    pre_cpu = xin.double() @ sae.W_encT.double().t() + sae.b_enc.double()      # fp64 reference
    pre_gpu = g.pre_acts(xin.to(gpu)).double().cpu()
    scale = (xin.double().abs() @ sae.W_encT.double().abs().t()).clamp_min(1e-30)
    assert float(((pre_gpu - pre_cpu).abs() / scale).max()) < 1e-5
    acts = g.encode(xin.to(gpu)).cpu()
    fires_cpu = pre_cpu > sae.threshold.double()
    fires_gpu = acts > 0
    tie = (pre_cpu - sae.threshold.double()).abs() <= 2e-5 * scale
    assert int(fires_cpu.sum()) > 50 * N
    assert torch.equal(fires_gpu[~tie], fires_cpu[~tie])
    both = fires_cpu & fires_gpu
    assert float(((acts.double() - pre_cpu).abs()[both] / scale[both]).max()) < 1e-5
    # the same rows through the CPU encode agree on the firing set too
    cpu_acts = sae.encode(xin)
    assert torch.equal((cpu_acts > 0)[~tie], fires_cpu[~tie])


def test_sae_decode_fp32_table(gpu):
    torch.manual_seed(8)
    M, L, D = 5, 4096, 512
    acts = torch.relu(torch.randn(M, L) - 2.4)
    Wd = torch.randn(L, D) * 0.05
    bd = torch.randn(D) * 0.01
    got = ops.sae_decode_sparse(acts.to(gpu), Wd.to(gpu), bd.to(gpu)).cpu()
    want = acts.double() @ Wd.double() + bd.double()
    _close(got, want.float(), atol=2e-5, rtol=1e-5)


def test_slot_copy_matches_index_copy(gpu):
    """ops.slot_copy (one-pass whole-slot KV copy, csrc/elementwise.hip) equals torch's index_select/index_copy_,
    for all layers and for a layer sub-range with different source / destination layer offsets."""
    from taboo_brittleness_amd import ops

    torch.manual_seed(0)
    src = torch.randn(5, 7, 2, 33, 16).to(torch.bfloat16).to(gpu)
    for layers, src_layers in ((None, None), (range(1, 4), range(2, 5))):
        dst = torch.randn(5, 9, 2, 33, 16).to(torch.bfloat16).to(gpu)
        exp = dst.clone()
        ds, ss = [0, 4, 8, 2], [6, 1, 1, 3]
        L = range(5) if layers is None else layers
        SL = L if src_layers is None else src_layers
        for a, b in zip(L, SL):
            exp[a].index_copy_(0, torch.tensor(ds, device=gpu), src[b].index_select(0, torch.tensor(ss, device=gpu)))
        ops.slot_copy(dst, src, ds, ss, layers, src_layers)
        assert torch.equal(dst, exp)


@pytest.mark.parametrize("T", [1, 5, 33])
def test_row_combine(gpu, T):
    """ops.row_combine (csrc/elementwise.hip) == sum_t coef * row to fp32 rounding (an fp64 reference: the kernel's
    fma chain rounds once per term)."""
    g = torch.Generator(device="cpu").manual_seed(T)
    V, B, R = 1028, 7, 40
    tab = torch.randn(R, V, generator=g).to(gpu)
    sel = torch.randint(0, R, (B, T), generator=g)
    coef = torch.randn(B, T, generator=g).to(gpu)
    ptr = (tab.data_ptr() + sel * V * 4).to(gpu)
    out = torch.empty(B, V, device=gpu)
    ops.row_combine(ptr, coef, out)
    exp = torch.zeros(B, V, device=gpu, dtype=torch.float64)
    for t in range(T):
        exp = exp + coef[:, t:t + 1].double() * tab[sel[:, t].to(gpu)].double()
    torch.testing.assert_close(out.double(), exp, rtol=1e-5, atol=2e-5)


@pytest.mark.parametrize("D", [512, 2304, 3584])
def test_random_basis_matches_reference(gpu, D):
    """csrc/basis.hip: orthonormal rows, = the numpy reference of the same algorithm to fp32 rounding, and a pure
    function of (seed, r, D) -- the same bits whichever launch / table rows a basis is drawn in."""
    ranks = [1, 7, 64, 16, 130]                  # 130: three Gram-Schmidt chunks of 64 earlier directions
    seeds = [3, 1 << 62, 12345, 99, 5]
    rows = [0, 64, 128, 192, 208]
    tab = torch.full((338, D), float("nan"), device=gpu)
    ops.random_basis(torch.tensor(seeds, dtype=torch.int64, device=gpu), torch.tensor(ranks, dtype=torch.int32,
                     device=gpu), torch.tensor(rows, dtype=torch.int64, device=gpu), tab)
    for s, r, o in zip(seeds, ranks, rows):
        U = tab[o:o + r].double()
        assert torch.isfinite(U).all()
        torch.testing.assert_close(U @ U.T, torch.eye(r, dtype=torch.float64, device=gpu), rtol=0, atol=1e-5)
        exp = torch.from_numpy(ref.random_basis(D, r, s)).to(gpu)
        torch.testing.assert_close(tab[o:o + r], exp, rtol=1e-5, atol=1e-6)
    alone = torch.empty(16, D, device=gpu)
    ops.random_basis(torch.tensor([99], dtype=torch.int64, device=gpu), torch.tensor([16], dtype=torch.int32,
                     device=gpu), torch.zeros(1, dtype=torch.int64, device=gpu), alone)
    assert torch.equal(alone, tab[192:208])
    for qu in (1, 2, 4):      # table rows loaded 1 / 2 / 4 earlier directions at a time: the same bits
        t2 = torch.full_like(tab, float("nan"))
        ops.random_basis(torch.tensor(seeds, dtype=torch.int64, device=gpu), torch.tensor(ranks, dtype=torch.int32,
                         device=gpu), torch.tensor(rows, dtype=torch.int64, device=gpu), t2, qu=qu)
        assert torch.equal(torch.nan_to_num(t2), torch.nan_to_num(tab)), qu     # (rows no basis covers stay NaN)
