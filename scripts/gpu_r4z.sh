#!/bin/bash
# Round 4, final artefacts: the whole -m gpu suite, PMC passes of the filter kernel (summarised into
# gpurun_out/pmc_fgemm.json), the smoke, the bench line with that PMC file, and a rocprofv3
# kernel-stats run of the bench.  Each step under its own limit; stops at a failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
python -c "import cobweb_pkg; cobweb_pkg.load()" || { echo "libcwq does not match the sources"; exit 4; }
timeout -k 10 900 python -u -m pytest -p no:cacheprovider -v --timeout 400 --timeout-method thread -m gpu tests \
    > gpurun_out/r4z_pytest_gpu.log 2>&1 || { tail -20 gpurun_out/r4z_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r4z_pytest_gpu.log
bash scripts/pmc.sh "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
  "GRBM_GUI_ACTIVE SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" || exit $?
PMC_PHASES=${PMC_PHASES:-5} python3 scripts/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_fgemm.json || exit $?
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4z_smoke.log 2>&1 || { tail -5 gpurun_out/r4z_smoke.log; exit 1; }
tail -2 gpurun_out/r4z_smoke.log
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --pmc-file gpurun_out/pmc_fgemm.json > gpurun_out/r4z_bench.log 2>&1 || { tail -5 gpurun_out/r4z_bench.log; exit 1; }
tail -1 gpurun_out/r4z_bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r4z_prof -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --recall-queries 0 > gpurun_out/r4z_prof.log 2>&1 || { tail -5 gpurun_out/r4z_prof.log; exit 1; }
echo done
