set -o pipefail
O=gpurun_out/g22; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread -k "instanc" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
echo done
