# balanced work split of the MG fused passes (banded): bit-exact tests, then V-cycle A/B at 512^3
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4o2
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "balanced_split or post_sweep_xch_sums or presmooth_restrict_variants or test_cg_mg_fused_post" > $O/tests.log 2>&1 || exit $?
PB_TUNE_ROUNDS=6 PB_TUNE_CONFIGS='[{}, {"prrx_split": 1}, {"postx_split": 1}, {"prrx_split": 2}, {"postx_split": 2}]' timeout -k 10 300 python scripts/tune_mg.py > $O/vcycle_ab.jsonl 2> $O/vcycle_ab.err || exit $?
