"""GEMM dispatch policy (runtime/gemm_dispatch.py) on the CPU: table lookup by (N, K, epilogue) and the next
measured row count >= M, the modes, and the fill rule of the in-tree tile choice."""
import json

from taboo_brittleness_amd.runtime import gemm_dispatch as GD


def test_table_lookup_and_modes(tmp_path):
    p = tmp_path / "t.json"
    json.dump({"shapes": {"8192,3584,0": [[256, "blas"], [1024, 256], [4096, "blas"]],
                          "28672,3584,3": [[512, 128], [2048, 256]]}}, open(p, "w"))
    old = GD.mode()
    try:
        GD.set_mode("auto")
        assert GD.load_table(str(p)) == str(p)
        assert GD.choose(100, 8192, 3584) == "blas"         # -> the 256-row entry
        assert GD.choose(300, 8192, 3584) == 256            # -> the 1024-row entry
        assert GD.choose(1024, 8192, 3584) == 256
        assert GD.choose(5000, 8192, 3584) == "blas"        # past the last entry: the last one
        assert GD.choose(600, 28672, 3584, 3) == 256
        assert GD.choose(64, 3584, 4096) == "blas"          # shape not in the table
        GD.set_mode("blas")
        assert GD.choose(1024, 8192, 3584) == "blas"
        GD.set_mode("tb")
        assert GD.choose(64, 3584, 4096) in (128, 256, "g128", "g256")      # in-tree only
        assert GD.describe()["mode"] == "tb"
    finally:
        GD.set_mode(old)
        GD._state["loaded"] = False


def test_fill_choice():
    assert GD.fill_choice(4096, 28672) == "g256"               # 1792 tiles
    assert GD.fill_choice(256, 3584) == "g128"                 # 14 tiles of 256 rows: half the CUs would idle
    assert GD.fill_choice(8192, 3584) == "g256"


def test_shipped_table_is_consistent():
    """The committed table covers the five Gemma-2-9B projection shapes with sorted row counts."""
    path = GD.load_table()
    try:
        assert path is not None
        tab = GD._state["table"]
        for key in [(8192, 3584, 0), (3584, 4096, 0), (28672, 3584, 0), (28672, 3584, 3), (3584, 14336, 0),
                    (256000, 3584, 0)]:
            ms, cs = tab[key]
            assert ms == sorted(ms) and len(ms) == len(cs) and all(_valid(c) for c in cs)
        tb = GD._state["tb_table"]
        assert tb is not None
        for key, (ms, cs) in tb.items():
            # the exact mode's table may only name batch-invariant kernels
            assert ms == sorted(ms) and all(_valid(c) and GD.is_invariant(c) for c in cs), key
    finally:
        GD._state["loaded"] = False


def _valid(c):
    if c in ("blas", "g128", "g256", "gs", "k64", "k128", "k256"):
        return True
    t = GD.ring_tile(c)
    return t is not None and t[0] in (16, 32, 48, 64, 96, 128, 144, 192, 256) and t[1] in (16, 32, 64, 112, 128) \
        and t[2] in (0, 1, 2)


def test_ring_tile_and_invariance():
    assert GD.ring_tile("r64x32") == (64, 32, 0)
    assert GD.ring_tile("r128x64b") == (128, 64, 1)
    assert GD.ring_tile("r16x16c") == (16, 16, 2)
    assert GD.ring_tile("g256") is None
    assert GD.is_invariant("r32x64") and GD.is_invariant("gs") and GD.is_invariant("g128")
    assert not GD.is_invariant("k128") and not GD.is_invariant("blas")


def test_split_rows_rounds_model():
    """``gs``: 256-row tiles, 128-row tiles or a row split of both, from the persistent grid's rounds."""
    for M, N in [(6144, 3584), (8192, 3584), (2400, 8192), (4096, 28672), (300, 3584), (9000, 3584), (5, 8192)]:
        M1 = GD.split_rows(M, N)
        assert 0 <= M1 <= M and (M1 % 256 == 0 or M1 == M)
    assert GD.split_rows(6144, 3584) == 4608    # 14 x 24 = 336 tiles: 252 tiles of 256 rows + 56 of 128 rows
    assert GD.split_rows(4096, 3584) == 4096    # 224 tiles: one part-full round beats 448 tiles of 128 rows
    assert GD.split_rows(2048, 3584) == 0       # 112 tiles: 224 of 128 rows still fit one round
    assert GD.split_rows(4096, 28672) == 4096   # 1792 tiles = 7 whole rounds
    assert GD.split_rows(4200, 8192) == 4096    # 32 x 17 = 544 tiles: 2 rounds + 32 128-row tiles
