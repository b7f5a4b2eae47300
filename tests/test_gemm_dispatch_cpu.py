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
    old = GD._state["kernel"]
    try:
        GD.set_kernel("pp")
        assert GD.fill_choice(4096, 28672) == 256               # 1792 tiles
        assert GD.fill_choice(256, 3584) == 128                 # 14 tiles of 256 rows: half the CUs would idle
        assert GD.fill_choice(8192, 3584) == 256
        GD.set_kernel("g4")
        assert GD.fill_choice(4096, 28672) == "g256"
        assert GD.fill_choice(256, 3584) == "g128"
    finally:
        GD.set_kernel(old)


def test_shipped_table_is_consistent():
    """The committed table covers the five Gemma-2-9B projection shapes with sorted row counts."""
    path = GD.load_table()
    try:
        assert path is not None
        tab = GD._state["table"]
        for key in [(8192, 3584, 0), (3584, 4096, 0), (28672, 3584, 0), (28672, 3584, 3), (3584, 14336, 0),
                    (256000, 3584, 0)]:
            ms, cs = tab[key]
            assert ms == sorted(ms) and len(ms) == len(cs) and all(c in ("blas", 128, 256, "g128", "g256", "k64", "k128", "k256", "s") for c in cs)
    finally:
        GD._state["loaded"] = False
