#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
DPSVM_STAMPS=/tmp/cst timeout -k 10 600 python bench/lru_profile_run.py 14 200000 covtype 581012 0 > gpurun_out/cov_stamps.log 2>&1 || exit $?
tail -2 gpurun_out/cov_stamps.log
python bench/stamps_report.py /tmp/cst.rank0 --lru > gpurun_out/cov_stamps.json 2>&1; python3 -c "
import json
d=json.load(open('gpurun_out/cov_stamps.json'))
for k,v in d.items(): print(k, v if not isinstance(v,dict) else ' '.join(f'{a[:-3]}={b/1000:.2f}' for a,b in v.items() if a!='n'))"
