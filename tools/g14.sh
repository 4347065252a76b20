set -o pipefail
O=gpurun_out/g14; mkdir -p $O; export TMPDIR=/tmp
E=$PWD/raytrace_amd/_lib/exp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "instancing" > $O/pytest_inst.log 2>&1 || { echo pytest failed; exit 1; }
timeout -k 10 300 python3 -u tools/inst_perf.py 3 8 > $O/inst_new.jsonl 2>> $O/err.log || exit 1
RT_AMD_NO_BLAS_LDS=1 timeout -k 10 300 python3 -u tools/inst_perf.py 3 8 > $O/inst_noblaslds.jsonl 2>> $O/err.log || exit 1
RT_AMD_LIB=$E/librt_amd_instdrop0.so timeout -k 10 300 python3 -u tools/inst_perf.py 3 8 > $O/inst_drop0.jsonl 2>> $O/err.log || exit 1
RT_AMD_LIB=$E/librt_amd_base.so timeout -k 10 300 python3 -u tools/inst_perf.py 3 8 > $O/inst_base.jsonl 2>> $O/err.log || exit 1
echo done
