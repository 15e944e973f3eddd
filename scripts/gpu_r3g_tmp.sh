set -u
OUT=gpurun_out/r3g
mkdir -p $OUT
export TMPDIR=/tmp
OUT=$OUT VARIANTS="main wt agpr" bash scripts/gpu_ab.sh
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --profile-only --steps 2000 --warmup 100 > $OUT/prof.log 2>&1; echo "rocprof rc=$?"
grep -h "optimize_lr" $OUT/prof/*/run_kernel_stats.csv $OUT/prof/run_kernel_stats.csv 2>/dev/null | head -3
CE_LIB=wt timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_wt -o run --output-format csv -- python3 bench.py --profile-only --steps 2000 --warmup 100 > $OUT/prof_wt.log 2>&1; echo "rocprof wt rc=$?"
grep -h "optimize_lr" $OUT/prof_wt/*/run_kernel_stats.csv $OUT/prof_wt/run_kernel_stats.csv 2>/dev/null | head -3
