# post-pass 2-row variant at four waves per SIMD (two workgroups per CU) vs the 4-row default
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4u
mkdir -p $O
cd $R
for i in 1 2; do
PB_TUNE_ROUNDS=4 PB_TUNE_CONFIGS='[{}, {"postx": 4}]' timeout -k 10 200 python scripts/tune_mg.py > $O/base_$i.jsonl 2>> $O/err || exit $?
PB_LIB=variants/wpe4.so PB_TUNE_ROUNDS=4 PB_TUNE_CONFIGS='[{}, {"postx": 4}, {"postx": 4, "postx_wgcu": 16}]' timeout -k 10 200 python scripts/tune_mg.py > $O/wpe4_$i.jsonl 2>> $O/err || exit $?
done
