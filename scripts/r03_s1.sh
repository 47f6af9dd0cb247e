cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03_v5; mkdir -p $O
echo "== config2"; timeout -k 10 300 python -u bench.py > $O/bench_config2.json 2> $O/bench_config2.err || { tail $O/bench_config2.err; exit 1; }
tail -c 600 $O/bench_config2.json
echo "== config3"; timeout -k 10 300 python -u bench.py --workload config3 > $O/bench_config3.json 2> $O/bench_config3.err || { tail $O/bench_config3.err; exit 1; }
tail -c 600 $O/bench_config3.json
echo "== stamps"; KBZ_STAMP_NAMES=d KBZ_HIP_LIB=$PWD/build_variants/stamps/libkbz_hip.so timeout -k 10 200 python -u tools/stamps_wide.py > $O/stamps_k_pass1d.txt 2>&1 || { tail $O/stamps_k_pass1d.txt; exit 1; }
cat $O/stamps_k_pass1d.txt
echo "== prof"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --workload config3 --steps 10 --warmup 2 --no-cpu --no-pmc --no-variants > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp "$f" $O/kernel_stats_config3.csv; head -8 $O/kernel_stats_config3.csv
