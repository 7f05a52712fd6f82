# non-temporal stencil stores on/off at 512^3 and on config 4's slab (bench lines, interleaved)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4x
mkdir -p $O
cd $R
timeout -k 10 500 python scripts/ab_env.py 3 - stencil_nt=0 -- --grid 1024,1024,128 > $O/ab_slab.jsonl 2> $O/err || exit $?
timeout -k 10 500 python scripts/ab_env.py 3 - stencil_nt=0 > $O/ab_512.jsonl 2>> $O/err || exit $?
