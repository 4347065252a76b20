set -o pipefail
O=gpurun_out/g9; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "instancing or emulator or known_answer" > $O/pytest_inst.log 2>&1 &&
timeout -k 10 300 python3 -u tools/inst_perf.py 3 8 > $O/inst_perf.jsonl 2> $O/inst_perf.err
echo exit $?
