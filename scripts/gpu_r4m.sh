# V-cycle kernel trace at 512^3 (per-dispatch rows: level 1 vs fine split by grid size)
set -u
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4m
cd /tmp && export TMPDIR=/tmp
PB_TUNE_ROUNDS=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r4m/kt -o vc -- python3 $R/scripts/tune_mg.py > $R/gpurun_out/r4m/vc.jsonl 2> $R/gpurun_out/r4m/vc.err
