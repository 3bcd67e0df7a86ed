#!/bin/bash
# One parameterised GPU call (replaces the per-call gpu_r4*.sh drivers).
#   gpurun -- bash scripts/gpu_run.sh TAG STEP [STEP ...]
# Steps (run in order, each under its own time limit; the script stops at the first failure):
#   suite           the whole -m gpu suite                      -> gpurun_out/TAG_pytest_gpu.log
#   tests:EXPR      pytest -m gpu -k EXPR ('+' means ' or ')      -> gpurun_out/TAG_pytest_k.log
#   pmc             PMC passes of the filter kernel, summarised  -> gpurun_out/pmc_fgemm.json
#   smoke           __graft_entry__.smoke()                       -> gpurun_out/TAG_smoke.log
#   bench           bench.py --steps 10 --warmup 3 (with the pmc step's JSON if it ran)
#   prof            rocprofv3 --kernel-trace --stats of a short bench run -> gpurun_out/TAG_prof/
#   py:SCRIPT:ARGS  python3 scripts/SCRIPT ARGS (ARGS split on ',')  -> gpurun_out/TAG_SCRIPT.log
#   rprof:SCRIPT:ARGS  the same probe under rocprofv3 --kernel-trace --stats -> gpurun_out/TAG_SCRIPT_prof/
#   tl:SCRIPT:ARGS  kernel + copy timeline of the probe's last calls (rocpd; TL_N kernels, default 60)
#                   -> gpurun_out/TAG_SCRIPT_timeline.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
TAG=$1; shift
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
python -c "import cobweb_pkg; cobweb_pkg.load()" || { echo "libcwq does not match the sources"; exit 4; }
PMCF=
for step in "$@"; do
  echo "== $step  $(date +%T)"
  case "$step" in
    suite)
      timeout -k 10 900 python -u -m pytest -p no:cacheprovider -v --timeout 400 --timeout-method thread -m gpu tests \
          > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
      tail -2 gpurun_out/${TAG}_pytest_gpu.log ;;
    tests:*)
      kexpr=${step#tests:}
      kexpr=${kexpr//+/ or }   # tests:a+b -> -k "a or b"
      timeout -k 10 600 python -u -m pytest -p no:cacheprovider -v --timeout 300 --timeout-method thread -m gpu tests \
          -k "$kexpr" > gpurun_out/${TAG}_pytest_k.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_k.log; exit 1; }
      tail -2 gpurun_out/${TAG}_pytest_k.log ;;
    pmc)
      bash scripts/pmc.sh "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
        "GRBM_GUI_ACTIVE SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
        "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" || exit $?
      PMC_PHASES=${PMC_PHASES:-5} python3 scripts/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_fgemm.json || exit $?
      PMCF="--pmc-file gpurun_out/pmc_fgemm.json" ;;
    smoke)
      timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
          || { tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
      tail -2 gpurun_out/${TAG}_smoke.log ;;
    bench)
      timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 $PMCF > gpurun_out/${TAG}_bench.log 2>&1 \
          || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
      tail -1 gpurun_out/${TAG}_bench.log ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
          python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-hier --recall-queries 0 > gpurun_out/${TAG}_prof.log 2>&1 \
          || { tail -5 gpurun_out/${TAG}_prof.log; exit 1; }
      tail -1 gpurun_out/${TAG}_prof.log ;;
    tl:*)
      IFS=: read -r kind script args <<< "$step"
      name=${script%.py}
      IFS=, read -r -a argv <<< "$args"
      timeout -k 10 ${PY_TIMEOUT:-600} rocprofv3 --kernel-trace --memory-copy-trace --output-format rocpd \
          -d gpurun_out/${TAG}_${name}_tl -o run -- python3 -u scripts/$script "${argv[@]}" \
          > gpurun_out/${TAG}_${name}_tl.log 2>&1 || { tail -20 gpurun_out/${TAG}_${name}_tl.log; exit 1; }
      db=$(find gpurun_out/${TAG}_${name}_tl -name '*.db' | head -1)
      python3 scripts/rocpd_summary.py "$db" --timeline ${TL_N:-60} > gpurun_out/${TAG}_${name}_timeline.txt 2>&1
      rm -f "$db"
      tail -${PY_TAIL:-70} gpurun_out/${TAG}_${name}_timeline.txt ;;
    py:*|rprof:*)
      IFS=: read -r kind script args <<< "$step"
      name=${script%.py}
      IFS=, read -r -a argv <<< "$args"
      if [ "$kind" = py ]; then
        timeout -k 10 ${PY_TIMEOUT:-600} python3 -u scripts/$script "${argv[@]}" > gpurun_out/${TAG}_${name}.log 2>&1 \
            || { tail -20 gpurun_out/${TAG}_${name}.log; exit 1; }
        tail -${PY_TAIL:-12} gpurun_out/${TAG}_${name}.log
      else
        timeout -k 10 ${PY_TIMEOUT:-600} rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_${name}_prof -o run \
            --output-format csv -- python3 -u scripts/$script "${argv[@]}" > gpurun_out/${TAG}_${name}_prof.log 2>&1 \
            || { tail -20 gpurun_out/${TAG}_${name}_prof.log; exit 1; }
        tail -${PY_TAIL:-12} gpurun_out/${TAG}_${name}_prof.log
      fi ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo done
