# full GPU tier on a fresh box (flakiness check) + smoke
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5b
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
