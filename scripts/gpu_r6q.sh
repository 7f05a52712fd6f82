set -u
mkdir -p gpurun_out
VAR=srold bash scripts/gpu_sr_ab.sh > gpurun_out/sr_ab_ddiff.txt 2>&1
rc=$?; tail -14 gpurun_out/sr_ab_ddiff.txt
exit $rc
