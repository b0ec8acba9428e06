#!/bin/bash
# C3 tuning A/B on one box (env knobs only): CU split, k_prep tiles per block, walker grid share.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
mkdir -p gpurun_out/r6 && rm -f gpurun_out/r6/ab.txt
bash scripts/r6_ab.sh 2 "base=SG_X=0" "fe3=SG_FRONT_EIGHTHS=3" "fe5=SG_FRONT_EIGHTHS=5" "pt1=SG_PREP_TILES=1" "pt2=SG_PREP_TILES=2" "wp110=SG_WALK_PCT=110" "wp90=SG_WALK_PCT=90"
