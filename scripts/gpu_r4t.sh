# timing experiment: V-cycle with fp contraction (FMA) everywhere vs the bit-exact build
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4t
mkdir -p $O
cd $R
for i in 1 2; do
PB_TUNE_ROUNDS=4 timeout -k 10 200 python scripts/tune_mg.py > $O/base_$i.jsonl 2>> $O/err || exit $?
PB_LIB=variants/fma.so PB_TUNE_ROUNDS=4 timeout -k 10 200 python scripts/tune_mg.py > $O/fma_$i.jsonl 2>> $O/err || exit $?
done
