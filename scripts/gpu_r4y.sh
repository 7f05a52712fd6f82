# 4 points per lane on config 4's slab: parity, then bench lines A/B
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4y
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "wide_planes or test_cg_matches_petsc" > $O/tests.log 2>&1 || exit $?
timeout -k 10 600 python scripts/ab_env.py 3 - stencil_wide_v4=1 -- --grid 1024,1024,128 > $O/ab_slab.jsonl 2> $O/err || exit $?
