#!/bin/bash
# Developer experiment: does the order in which a split visits its columns
# matter?  The engine bench's root cluster in memory order against a random
# order (--shuffle), 256 jobs over a 1M-column matrix (1.7 GB: beyond the
# MALL), with the phase profile.  Run on the GPU box (gpurun).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
ALVRL_REFINE_PROFILE=1 timeout -k 10 300 python tools/refine_engine_bench.py --rows 214 --vrls 1000000 --jobs 256 --reps 1 \
    > gpurun_out/eng_seq.json 2> gpurun_out/eng_seq.err || exit 1
ALVRL_REFINE_PROFILE=1 timeout -k 10 300 python tools/refine_engine_bench.py --rows 214 --vrls 1000000 --jobs 256 --reps 1 --shuffle \
    > gpurun_out/eng_shuf.json 2> gpurun_out/eng_shuf.err || exit 1
