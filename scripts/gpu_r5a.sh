# 256^3 (config 2): non-temporal stores on/off and z-alternation, bench lines interleaved
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5a
mkdir -p $O
cd $R
timeout -k 10 600 python scripts/ab_env.py 3 - stencil_nt=0 cg_defer_x=2 -- --grid 256,256,256 --steps 400 --warmup 40 > $O/ab256.jsonl 2> $O/err || exit $?
