#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
for v in 1 0; do MTG_KSPEC=$v MTG_DEBUG=1 timeout -k 10 120 python3 -u tools/gpu/dbg_spec.py 2>&1 | grep -v amdgpu.ids | grep -i "speculative\|levels\|fused" ; done
