O=gpurun_out/r03_v13; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; tail -1 $O/pytest_gpu.txt
VARIANTS="old new old new old new" BENCH_ARGS="" STEPS=12 bash scripts/ab_variants.sh
VARIANTS="old new" LEGS="--mode dynamorio;--mode afl;--workload config3" bash scripts/ab_novelty.sh
