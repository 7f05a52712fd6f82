# config 4's per-GPU slab (1024x1024x128): launch-geometry A/B of the CG passes
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4w
mkdir -p $O
cd $R
PB_TUNE_N=1024,1024,128 PB_TUNE_ROUNDS=6 PB_TUNE_CONFIGS='[{}, {"stencil_blocks": 512}, {"stencil_blocks": 768}, {"xcd_remap": 0}, {"zalt": 0}, {"stencil_nt": 0}]' timeout -k 10 400 python scripts/tune_stencil.py > $O/ab.jsonl 2> $O/ab.err || exit $?
