#!/bin/bash
# FETCH_SIZE / WRITE-side calibration for the conv producers' 64-B-per-line access shape (see pmc_calib.hip)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_calib -o run -- ./tools/calib/pmc_calib > gpurun_out/pmc_calib.log 2>&1 || { tail -20 gpurun_out/pmc_calib.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_calib_w -o run -- ./tools/calib/pmc_calib > gpurun_out/pmc_calib_w.log 2>&1 || { tail -20 gpurun_out/pmc_calib_w.log; exit 1; }
python3 - <<'PY'
import csv, glob
for d, c in (('pmc_calib', 'FETCH_SIZE'), ('pmc_calib_w', 'WRITE_SIZE')):
    f = glob.glob(f'gpurun_out/{d}/**/*counter_collection.csv', recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if r.get('Counter_Name') == c:
            print(r.get('Dispatch_Id'), r['Kernel_Name'][:40], c, 'KB', r['Counter_Value'], '= GiB', float(r['Counter_Value']) / 2**20)
PY
