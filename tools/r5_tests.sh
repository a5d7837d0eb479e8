#!/bin/bash
# GPU test subset (or all with no args): tools/r5_tests.sh OUT [pytest args...]
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r5t}
shift
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -15 $O/tests.log
exit $rc
