#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r5k; mkdir -p $OUT
MTG_DEBUG=1 timeout -k 10 300 python -u tools/dist_sim.py --ranks 8 --reads 1000000 --steps 1 --serial --collect superkmer --no-single > $OUT/s8.json 2> $OUT/s8.err
rc=$?; grep -E "rc merge|speculative rc|msd n=|fallback|overflow" $OUT/s8.err | sort | uniq -c | sort -rn | head -40; exit $rc
