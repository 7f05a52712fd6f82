set -u
mkdir -p gpurun_out
timeout -k 10 300 python scripts/fft_tl_ab.py > gpurun_out/fft_persist_ab.jsonl 2> gpurun_out/fft_persist_ab.err
rc=$?; cat gpurun_out/fft_persist_ab.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python scripts/cg_cfg_probe.py 512 3 '[{}, {"cg_wgcu": 2}, {"cg_wgcu": 2, "engine_kc_skew": 4}, {"cg_wgcu": 3, "engine_kc_skew": 4}]' > gpurun_out/cgcfg6.jsonl 2>&1
rc=$?; echo "rc=$rc"; grep config gpurun_out/cgcfg6.jsonl; exit $rc
