#!/bin/bash
# two A/B sets back to back: gpu_ab2.sh NAME REPS "cfgs..." -> NAME_512 and NAME_256
set -u
R=${GRAFT_REPO_ROOT:-.}
name=$1; reps=$2; shift 2
cd $R && bash scripts/gpu_ab.sh ${name}_512 $reps "$@" > /dev/null || exit $?
bash scripts/gpu_ab.sh ${name}_256 $reps "$@" -- --base 256 > /dev/null || exit $?
