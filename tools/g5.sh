set -o pipefail
O=gpurun_out/g5; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
r=$?; tail -5 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo exit $?
