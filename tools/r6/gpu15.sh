#!/bin/bash
# same-box A/B: lens dedup chunks by distinct rows (default) vs by logical rows, headline bench 8 / 2, twice each
set -o pipefail
O=gpurun_out/r6/lenschunk; mkdir -p $O
B="python -u bench.py --steps 8 --warmup 2 --no-post-forcing --no-config2 --no-lora-side --no-lowrank-side"
timeout -k 10 300 $B > $O/new1.json 2> $O/new1.err || exit 2
TB_LENS_CHUNK_DISTINCT=0 timeout -k 10 300 $B > $O/old1.json 2> $O/old1.err || exit 3
timeout -k 10 300 $B > $O/new2.json 2> $O/new2.err || exit 4
TB_LENS_CHUNK_DISTINCT=0 timeout -k 10 300 $B > $O/old2.json 2> $O/old2.err || exit 5
