"""Static check of gemm4's counted-wait K loop: see taboo_brittleness_amd/isa_check.py (the extension build runs it)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from taboo_brittleness_amd.isa_check import *  # noqa: E402,F401,F403
from taboo_brittleness_amd.isa_check import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
