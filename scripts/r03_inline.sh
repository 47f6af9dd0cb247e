O=gpurun_out/r03_v12; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; tail -1 $O/pytest_gpu.txt
KBZ_HIP_LIB=$PWD/build_variants/noinl/libkbz_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_noinl.txt 2>&1; tail -1 $O/pytest_noinl.txt
VARIANTS="inl noinl inl noinl inl noinl" BENCH_ARGS="" STEPS=12 bash scripts/ab_variants.sh
VARIANTS="inl noinl" LEGS="--mode dynamorio;--mode afl;--workload config3" bash scripts/ab_novelty.sh
