# the fused passes on the 128^3 level again, now with the pre-pass split
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4z
mkdir -p $O
cd $R
PB_TUNE_ROUNDS=6 PB_TUNE_CONFIGS='[{}, {"mg_engine_min_plane": 16384}, {"mg_engine_min_plane": 16384, "postx_split": 1}, {"mg_engine_min_plane": 16384, "prrx_split": 2}]' timeout -k 10 300 python scripts/tune_mg.py > $O/ab.jsonl 2> $O/err || exit $?
