#!/bin/bash
# r06 placement studies: the matvec over every ordered pair of fresh vectors,
# the matvec's launch shapes across those pairs, and the CG passes over fresh solver instances
# (per-launch pass B samples). CFG / CG_CFG override the tuning sets. Outputs in gpurun_out/.
set -u
mkdir -p gpurun_out
CFG=${CFG:-'[{}, {"stencil_kc_skew": 0}]'}
CG_CFG=${CG_CFG:-'[{}, {"engine_kc_skew": 2}]'}
timeout -k 10 300 python scripts/placement_pairs.py 512 6 15 > gpurun_out/pairs.jsonl 2>&1 || exit $?
timeout -k 10 900 python scripts/placement_cfg.py 512 5 8 "$CFG" > gpurun_out/cfg.jsonl 2>&1 || exit $?
grep config gpurun_out/cfg.jsonl | cut -c1-200
timeout -k 10 900 python scripts/cg_cfg_probe.py ${CG_N:-512} 3 "$CG_CFG" > gpurun_out/cgcfg.jsonl 2>&1 || exit $?
grep config gpurun_out/cgcfg.jsonl
