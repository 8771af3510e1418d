timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_f16.py -q -x --timeout 200 > gpurun_out/pt.log 2>&1; tail -1 gpurun_out/pt.log
ROUNDS=3 bash tools/ab_lib.sh libdmx.so libnopipe.so
