# new compact-A / 7-point-symbol spectral-PC history tests; 256^3 stencil-geometry A/B
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4n
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k star_symbol > $O/tests.log 2>&1 || exit $?
PB_TUNE_N=256,256,256 PB_TUNE_ROUNDS=5 PB_TUNE_CONFIGS='[{}, {"stencil_tall_min_plane": 65536}, {"stencil_kcmin": 32}, {"stencil_kcmin": 128}, {"stencil_blocks": 512}, {"stencil_tall_min_plane": 65536, "tall_wgcu": 2}, {"passa_nt": 0}, {"zalt": 0}]' timeout -k 10 400 python scripts/tune_stencil.py > $O/ab256.jsonl 2> $O/ab256.err
