#!/bin/bash
# Round 4: local_unique's peeled first probe (ab/peel1) vs the probe loop (ab/peel0), interleaved; then the
# kernel breakdown of the serial P = 2 routed ranks with the pulled sink join.
cd "$GRAFT_REPO_ROOT" || exit 1
cp projects2014-metagenome_amd/libmtg_boss.so /tmp/lib_keep.so
bash tools/gpu/ab.sh r4r/ab peel0 peel1 || exit 1
cp /tmp/lib_keep.so projects2014-metagenome_amd/libmtg_boss.so
bash tools/gpu/ab_env.sh r4r/abs 2 "MTG_SPEC_L1_STRIPES=16" "MTG_SPEC_L1_STRIPES=8 MTG_SPEC_L1_SLACK=32" "MTG_SPEC_L1_STRIPES=4 MTG_SPEC_L1_SLACK=32" || exit 1
cp /tmp/lib_keep.so projects2014-metagenome_amd/libmtg_boss.so
CFGS="2 10000000" TAG=r4r/pd bash tools/gpu/r4n.sh
