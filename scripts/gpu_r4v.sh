#!/bin/bash
# Round 4, call V: the whole -m gpu suite and the smoke at the round's final sources.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
python -c "import cobweb_pkg; cobweb_pkg.load()" || { echo "libcwq does not match the sources"; exit 4; }
timeout -k 10 900 python -u -m pytest -p no:cacheprovider -v --timeout 400 --timeout-method thread -m gpu tests \
    > gpurun_out/r4v_pytest_gpu.log 2>&1 || { tail -20 gpurun_out/r4v_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r4v_pytest_gpu.log
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4v_smoke.log 2>&1 || { tail -5 gpurun_out/r4v_smoke.log; exit 1; }
tail -1 gpurun_out/r4v_smoke.log
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --pmc-file profiles/pmc_r04_fgemm.json > gpurun_out/r4v_bench.log 2>&1 || { tail -5 gpurun_out/r4v_bench.log; exit 1; }
tail -1 gpurun_out/r4v_bench.log | cut -c1-400
echo done
