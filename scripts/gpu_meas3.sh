#!/bin/bash
# Round-3 measurement pass: C4 preset memory, Basic categorize on hierarchical trees
# (two-level G=100k, balanced 10/5 and 4/9) with a rocprof kernel breakdown, deep-tree Fast.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for s in "$@"; do
  case $s in
    cattest) step pytest_cat 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 400 --timeout-method thread \
        tests/test_gpu_cat_count.py tests/test_gpu_parity.py tests/test_gpu_filter.py tests/test_gpu_configs.py ;;
    alltests) step pytest_all 1200 python -u -m pytest -x -q -p no:cacheprovider --timeout 400 --timeout-method thread \
        tests -m gpu ;;
    cat100k_replay) CWQ_CAT_COUNT=0 step cat_g100k_replay 600 python scripts/basic_probe.py --clusters 100000 --queries 500 --reps 1 ;;
    fittest) step pytest_fit 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 400 --timeout-method thread \
        tests/test_gpu_fit.py ;;
    fitprobe) step fit_dev_2k 600 python scripts/fit_probe.py --n 2000 --dim 768 --clusters 20 &&
      step fit_host_2k 600 python scripts/fit_probe.py --n 2000 --dim 768 --clusters 20 --host &&
      step fit_dev_20k 600 python scripts/fit_probe.py --n 20000 --dim 768 --clusters 50 ;;
    fit100k) step fit_dev_100k 1000 python scripts/fit_probe.py --n 100000 --dim 768 --clusters 100 ;;
    pathtest) step pytest_path 900 python -u -m pytest -x -v -s -p no:cacheprovider --timeout 400 --timeout-method thread \
        tests/test_gpu_filter.py -k "prefix_bounds or deep_balanced or internal_bounds or hierarchical or two_level" ;;
    pathab) step fast_b4_path 600 python scripts/filter_probe.py --balanced 4,9 --modes 1 &&
      step fast_b4_nodes 600 env CWQ_INT_PATH=0 python scripts/filter_probe.py --balanced 4,9 --modes 1 &&
      step fast_b10_path 600 python scripts/filter_probe.py --balanced 10,5 --modes 1 &&
      step fast_g100k_path 600 python scripts/filter_probe.py --clusters 100000 --modes 1 ;;
    proffastb4) step prof_fast_b4 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fb4 -o fb4 --output-format csv -- \
        python3 scripts/filter_probe.py --balanced 4,9 --modes 1 --reps 2 ;;
    c4) step c4_preset 600 python bench.py --preset c4 --steps 3 --warmup 1 --no-cpu-baseline --no-per-call ;;
    cat100k) step cat_g100k 600 python scripts/basic_probe.py --clusters 100000 --queries 2000 --reps 2 ;;
    cat1024) step cat_g1024 600 python scripts/basic_probe.py --clusters 1024 --queries 10000 --reps 2 ;;
    catb10) step cat_b10 600 python scripts/basic_probe.py --balanced 10,5 --queries 2000 --reps 2 ;;
    catb4) step cat_b4 600 python scripts/basic_probe.py --balanced 4,9 --queries 2000 --reps 2 ;;
    prof100k) step prof_cat_g100k 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cat -o cat --output-format csv -- \
        python3 scripts/basic_probe.py --clusters 100000 --queries 2000 --reps 1 --rank-queries 1 ;;
    fastb4) step fast_b4 600 python scripts/filter_probe.py --balanced 4,9 ;;
    pcb4) step pc_b4 600 python scripts/percall_probe.py --balanced 4,9 --nq 1,8,64 --modes -1 ;;
    pcb10) step pc_b10 600 python scripts/percall_probe.py --balanced 10,5 --nq 1,8,64 --modes -1 ;;
    profcatb4) step prof_cat_b4 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_catb4 -o catb4 --output-format csv -- \
        python3 scripts/basic_probe.py --balanced 4,9 --queries 2000 --reps 1 --rank-queries 1 ;;
    ragged) step pytest_ragged 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 400 --timeout-method thread \
        tests/test_gpu_filter.py -k "ragged or deep_balanced or three_level or prefix_bounds" ;;
    fastb10) step fast_b10 600 python scripts/filter_probe.py --balanced 10,5 ;;
  esac
done
