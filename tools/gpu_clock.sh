#!/bin/bash
# effective clock of the data-mode GEMMs under load: GRBM_GUI_ACTIVE / 8 / kernel time
# (MI355X_MICROARCH.md 'DVFS give-back'); its own PMC pass with --kernel-trace only
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp && timeout -k 10 900 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/pmc_clock -o clock --output-format csv -- python3 $R/bench.py --steps 4 --warmup 1 --no-cpu --no-cov --no-fit --no-large --profile-reps 1 > $R/gpurun_out/pmc_clock.log 2>&1; rc=$?
echo "pmc clock rc=$rc"
exit $rc
