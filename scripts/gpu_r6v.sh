set -u
mkdir -p gpurun_out
timeout -k 10 300 python scripts/fft_tl_ab.py > gpurun_out/fft_tl_ab.jsonl 2> gpurun_out/fft_tl_ab.err
rc=$?; cat gpurun_out/fft_tl_ab.jsonl; tail -3 gpurun_out/fft_tl_ab.err; exit $rc
