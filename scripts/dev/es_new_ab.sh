set -u
mkdir -p gpurun_out/es
CPK_LIB=capnp-zig_amd/lib_exp/es_new.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_small_units.py tests/test_gpu_configs.py tests/test_gpu_stress.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "encode or c5 or small" > gpurun_out/es/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/es/pytest.log; [ $rc -ne 0 ] && exit $rc
ESLIB=es_new bash scripts/dev/pmc_c5_ab.sh
