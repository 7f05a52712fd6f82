#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/sr_probe.py 512 - sr_s_shape=1 sr_s_shape=1,stencil_ty=2 sr_s_shape=1,stencil_ty=2,stencil_blocks=1024 sr_s_shape=1,stencil_ty=1,stencil_blocks=2048 sr_s_shape=1,stencil_blocks=1024 sr_s_shape=0,stencil_ty=1,stencil_blocks=4096 > gpurun_out/sr3_probe.jsonl 2> gpurun_out/sr3_probe.err
rc=$?; echo "probe rc=$rc"; tail -3 gpurun_out/sr3_probe.err
exit $rc
