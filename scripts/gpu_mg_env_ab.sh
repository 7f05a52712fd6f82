#!/bin/bash
# A/B environment knobs on the 512^3 MG-PCG solve (V-cycle part timers), interleaved reps.
# usage: scripts/gpu_mg_env_ab.sh REPS 'NAME=VAL[,NAME=VAL]' ['...' ...]   ('-' = defaults)
set -u
R=${GRAFT_REPO_ROOT:-.}
cd $R
mkdir -p gpurun_out/mgab
reps=$1; shift
for rep in $(seq 1 $reps); do
  for cfg in "$@"; do
    envs=()
    [ "$cfg" != "-" ] && IFS=',' read -ra envs <<< "$cfg"
    line=$(env "${envs[@]}" PCS=mg NO_CPU=1 timeout -k 10 200 python scripts/bench_solve.py 512 2>> gpurun_out/mgab/solve.err) || exit $?
    echo "{\"cfg\": \"$cfg\", \"rep\": $rep, \"r\": $line}" | tee -a gpurun_out/mgab/solve.jsonl | cut -c1-400
  done
done
