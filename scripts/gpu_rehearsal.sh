#!/bin/bash
# SURVEY §8(d) timing protocol (medians of 5) at 512^3 and 256^3, and the multi-rank rehearsals on
# one GPU: N=4 per-rank geometry through a forced one-rank RCCL communicator, and bench.py under
# torch.distributed.run with 2 ranks sharing the GPU through the gloo host transport.
set -u
R=${GRAFT_REPO_ROOT:-.}
mkdir -p $R/gpurun_out/reh
cd $R
timeout -k 10 600 python scripts/bench_protocol.py 512 > gpurun_out/reh/protocol_512.jsonl 2> gpurun_out/reh/protocol.err || exit $?
timeout -k 10 300 python scripts/bench_protocol.py 256 > gpurun_out/reh/protocol_256.jsonl 2>> gpurun_out/reh/protocol.err || exit $?
echo protocol ok
PB_FORCE_COMM=1 timeout -k 10 300 python bench.py --grid 512,1024,256 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/reh/forcecomm.json 2> gpurun_out/reh/forcecomm.err || exit $?
echo forcecomm ok
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --transport host --no-cpu-baseline > gpurun_out/reh/host2.json 2> gpurun_out/reh/host2.err
rc=$?; echo "host2 rc=$rc"; tail -c 600 gpurun_out/reh/host2.json; exit $rc
