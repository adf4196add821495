set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "workgroup_execute or out_of_order or long_runs" --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -15
