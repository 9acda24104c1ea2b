#!/bin/bash
# r03z: the round's profile set -- the default bench with its per-launch dump, a rocprofv3 kernel trace pass and
# the FETCH_SIZE / WRITE_SIZE PMC passes (tools/prof_r02.sh), the roofline recomputed from them
export BENCH_ARGS="--no-companions"
./tools/prof_r02.sh r03 bench trace pmc
