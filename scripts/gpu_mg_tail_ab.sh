set -u
mkdir -p gpurun_out/mgtail; : > gpurun_out/mgtail/solve.jsonl
for tm in 8192 40000 300000; do
  PB_MG_TAIL_MAX=$tm PCS=mg NO_CPU=1 timeout -k 10 200 python scripts/bench_solve.py 512 256 >> gpurun_out/mgtail/solve.jsonl 2>> gpurun_out/mgtail/solve.err || exit $?
done
cat gpurun_out/mgtail/solve.jsonl | cut -c1-330
