#!/bin/bash
# One gpurun call that refreshes every judged artefact: PMC passes of the filter kernel
# (summarised into gpurun_out/pmc_fgemm.json), GPU tests, smoke, the bench line (with that
# PMC file) and a rocprofv3 kernel-stats run of the bench.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
bash scripts/pmc.sh "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
  "GRBM_GUI_ACTIVE SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" || exit $?
PMC_PHASES=${PMC_PHASES:-5} python3 scripts/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_fgemm.json || exit $?
bash scripts/gpu_check.sh tests || exit $?
timeout -k 10 900 python bench.py --steps 10 --warmup 3 --pmc-file gpurun_out/pmc_fgemm.json > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
bash scripts/gpu_check.sh prof
