set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/flat
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "chunk or variants or device_list or multi_device or per_pixel" > gpurun_out/flat/pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/flat/pytest.log; exit 1; }
tail -1 gpurun_out/flat/pytest.log
STEPS=20 bash tools/ab_session.sh flat "cornell:1 readme:1 cornell:8"
